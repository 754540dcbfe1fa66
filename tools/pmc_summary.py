#!/usr/bin/env python3
"""Per-kernel mean of every counter in rocprofv3 --pmc output directories (counter_collection.csv),
plus derived fractions: VALU / LDS instruction shares, wait split, HBM bytes ((2 FETCH + WRITE) KiB).
    python tools/pmc_summary.py gpurun_out/TAG/p1 gpurun_out/TAG/p2 ..."""
import collections
import csv
import glob
import json
import re
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("pamg::(anonymous namespace)::", ""))
            agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, c in agg.items():
    if n.startswith("__amd"):
        continue
    m = {k: sum(v) / len(v) for k, v in c.items()}
    out = {"kernel": n, **{k: round(v) for k, v in m.items()}}
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in m:
                out[k + "_frac"] = round(m[k] / wc, 3)
    if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
        out["hbm_GB"] = round((2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024 / 1e9, 3)
    print(json.dumps(out))
