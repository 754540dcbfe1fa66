#!/usr/bin/env python3
"""Per-kernel read-request anatomy from the rocprofv3 passes of tools/pmc_requests.sh.

For every row kernel launch shape (name, blocks): TCC read requests to the memory side by size
(32 / 64 / 128 B) and their byte sum, DRAM-bound read requests, L2 hit rate and write requests
(WRITE requests are 64 B). The byte sum by size is the read traffic without FETCH_SIZE's
gfx950 64-B tally (MI355X_MICROARCH.md §HBM: FETCH_SIZE counts a 128-B request as 64 B).
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def load(path):
    hits = sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(hits[0])):
        name = r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "").replace("void ", "")
        name = re.sub(r"\(.*", "", name)
        if not name.startswith("k_rows"):
            continue
        blocks = int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"]))
        agg[(name, blocks)][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main():
    p1, p2 = load(sys.argv[1]), load(sys.argv[2])
    out = []
    for key in sorted(set(p1) & set(p2), key=lambda k: -k[1]):
        c = {k: sum(v) / len(v) for k, v in {**p1[key], **p2[key]}.items()}
        n32, n64, n128 = (c.get(f"TCC_EA0_RDREQ_{s}B_sum", 0.0) for s in (32, 64, 128))
        tot = c.get("TCC_EA0_RDREQ_sum", 0.0)
        hit, miss = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
        out.append({"kernel": key[0], "blocks": key[1], "rdreq": tot, "rdreq_32B": n32, "rdreq_64B": n64,
                    "rdreq_128B": n128, "read_bytes_by_size": 32 * n32 + 64 * n64 + 128 * n128,
                    "fetch_size_equiv_bytes": 64 * tot, "rdreq_dram": c.get("TCC_EA0_RDREQ_DRAM_sum"),
                    "wrreq": c.get("TCC_EA0_WRREQ_sum"), "write_bytes_64B": 64 * c.get("TCC_EA0_WRREQ_sum", 0.0),
                    "l2_hit_rate": hit / (hit + miss) if hit + miss else None})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
