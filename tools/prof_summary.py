#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (CSV) per (kernel, grid size): calls and average
duration. The level of a row-op launch is identified by its grid size (tiles), so the
level-0 Jacobi average can be compared with bench.py's roofline.ms_per_launch.

    python tools/prof_summary.py gpurun_out/prof_kt/kt_kernel_trace.csv [--top 20]
"""
import argparse
import collections
import csv
import json
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=25)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        name = (r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "")
                .replace("(anonymous namespace)::", "").replace("void ", ""))
        name = re.sub(r"\(.*", "", name)
        key = (name, int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(agg.items(), key=lambda kv: -sum(kv[1]))
    out = []
    for (name, grid), d in rows[: a.top]:
        out.append({"kernel": name, "blocks": grid, "calls": len(d), "avg_us": round(sum(d) / len(d), 2),
                    "min_us": round(min(d), 2), "total_ms": round(sum(d) / 1e3, 3)})
    if a.json:
        print(json.dumps(out, indent=1))
    else:
        print(f"{'kernel':58s} {'blocks':>9s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'total_ms':>9s}")
        for o in out:
            print(f"{o['kernel'][:58]:58s} {o['blocks']:9d} {o['calls']:6d} {o['avg_us']:10.2f} {o['min_us']:10.2f} {o['total_ms']:9.3f}")


if __name__ == "__main__":
    main()
