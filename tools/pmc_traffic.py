#!/usr/bin/env python3
"""HBM traffic per launch from rocprofv3 PMC passes (MI355X_MICROARCH.md §HBM recipe).

Separate --pmc passes give FETCH_SIZE and WRITE_SIZE (KiB) per dispatch. On gfx950
FETCH_SIZE reports half the bytes of 16-B/lane streaming reads, so the guide's correction
is traffic = (2 * FETCH_SIZE + WRITE_SIZE) * 1024. Our row kernels mix 16-B/lane streams
(columns, values) with 8-B/lane x gathers (uncalibrated width), so the corrected figure is
an upper bound; the raw counters are kept next to it.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv --kernel 'k_rows_tile2<2' > traffic.json
"""
import argparse
import collections
import csv
import json
import re


def load(path, counter):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "").replace("void ", "")
        name = re.sub(r"\(.*", "", name)
        blocks = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
        agg[(name, blocks)].append(float(r["Counter_Value"]))
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--kernel", default="k_rows_tile2<2")
    a = ap.parse_args()
    F, W = load(a.fetch, "FETCH_SIZE"), load(a.write, "WRITE_SIZE")
    out = []
    for (name, blocks), fv in sorted(F.items(), key=lambda kv: -kv[0][1]):
        if not name.startswith(a.kernel) or (name, blocks) not in W:
            continue
        f = sum(fv) / len(fv)
        w = sum(W[(name, blocks)]) / len(W[(name, blocks)])
        out.append({"kernel": name, "blocks": blocks, "fetch_kib": f, "write_kib": w,
                    "traffic_bytes": (2 * f + w) * 1024.0,
                    "note": "(2*FETCH_SIZE + WRITE_SIZE)*1024 per MI355X_MICROARCH.md §HBM; "
                            "upper bound: 8-B/lane x gathers are doubled too"})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
