#!/usr/bin/env python3
"""Per-kernel counter anatomy from any number of rocprofv3 --pmc passes (one -d directory each).

Every counter of every pass is averaged per launch shape (kernel name, blocks) and the derived
figures the DESIGN.md tables quote are added where their counters are present:

* read bytes by request size (TCC_EA0_RDREQ_{32,64,128}B: what leaves L2 for the fabric),
  L2 hit rate, write requests (64 B);
* waves per launch, wave-cycles, and the split of those cycles into issuing (ACTIVE_INST_ANY),
  issue-stalled (WAIT_INST_ANY) and parked on s_waitcnt / barriers (WAIT_ANY);
* mean L1->L2 read latency in cycles (TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ).

    python tools/pmc_anatomy.py DIR1 DIR2 ... [--kernel k_rows] > anatomy.json
"""
import argparse
import collections
import csv
import glob
import json
import os
import re


def load(path, prefix):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "").replace("void ", "")
            name = re.sub(r"\(.*", "", name)
            if not name.startswith(prefix):
                continue
            blocks = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
            agg[(name, blocks)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="k_")
    a = ap.parse_args()
    merged = collections.defaultdict(dict)
    for d in a.dirs:
        for key, cs in load(d, a.kernel).items():
            for c, v in cs.items():
                merged[key][c] = sum(v) / len(v)
    out = []
    for (name, blocks), c in sorted(merged.items(), key=lambda kv: -kv[0][1]):
        g = lambda k: c.get(k)  # noqa: E731
        rec = {"kernel": name, "blocks": blocks, "counters": c}
        n32, n64, n128 = (c.get(f"TCC_EA0_RDREQ_{s}B_sum") for s in (32, 64, 128))
        if None not in (n32, n64, n128):
            rec["read_bytes_by_size"] = 32 * n32 + 64 * n64 + 128 * n128
        if g("TCC_HIT_sum") is not None and g("TCC_MISS_sum") is not None:
            t = g("TCC_HIT_sum") + g("TCC_MISS_sum")
            rec["l2_hit_rate"] = g("TCC_HIT_sum") / t if t else None
        if g("TCC_EA0_WRREQ_sum") is not None:
            rec["write_bytes_64B"] = 64 * g("TCC_EA0_WRREQ_sum")
        wc = g("SQ_WAVE_CYCLES")
        if wc:
            for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if g(k) is not None:
                    rec[k.lower() + "_frac"] = g(k) / wc
        if g("SQ_WAVES"):
            rec["waves"] = g("SQ_WAVES")
            if wc:
                rec["cycles_per_wave"] = wc / g("SQ_WAVES")
        if g("TCP_TCC_READ_REQ_sum") and g("TCP_TCC_READ_REQ_LATENCY_sum") is not None:
            rec["l1_l2_read_latency_cycles"] = g("TCP_TCC_READ_REQ_LATENCY_sum") / g("TCP_TCC_READ_REQ_sum")
        out.append(rec)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
