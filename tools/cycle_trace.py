#!/usr/bin/env python3
"""One V-cycle out of a rocprofv3 kernel trace: every dispatch of the cycle in launch order
with its duration and the idle gap before it, so latency-bound coarse levels and launch
gaps can be read off (dev tool).

A cycle starts at a level-0 row kernel whose grid equals the largest grid in the trace and
that follows a dispatch of a different kernel (the previous cycle's post-smoothing tail).
The cycle picked is the `--which`-th such start (default: the middle one of the graph
replays, away from warm-up and the eager profiling pass).

    python tools/cycle_trace.py gpurun_out/kt/kt_kernel_trace.csv [--which N]
"""
import argparse
import csv
import re


def short(name):
    name = (name.replace("pamg::(anonymous namespace)::", "")
            .replace("(anonymous namespace)::", "").replace("void ", ""))
    return re.sub(r"\(.*", "", name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--which", type=int, default=-1)
    ap.add_argument("--len", type=int, default=0, help="dispatches per cycle (0: up to the next start)")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                     int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    rows = [r for r in rows if r[2].startswith(("k_", "__amd"))]
    gmax = max(r[3] for r in rows if r[2].startswith("k_rows"))
    starts = [i for i, r in enumerate(rows)
              if r[2].startswith("k_rows") and r[3] == gmax and "<2," in r[2]
              and i > 0 and rows[i - 1][3] != gmax]
    if not starts:
        raise SystemExit("no cycle start found")
    k = starts[len(starts) // 2] if a.which < 0 else starts[a.which]
    nxt = [s for s in starts if s > k]
    end = k + a.len if a.len else (nxt[0] if nxt else len(rows))
    t0 = rows[k][0]
    tot_busy = 0
    print(f"{'#':>3s} {'kernel':60s} {'blocks':>8s} {'start_us':>9s} {'dur_us':>9s} {'gap_us':>7s}")
    for i in range(k, end):
        s, e, n, g = rows[i]
        gap = (s - rows[i - 1][1]) / 1e3 if i > k else 0.0
        tot_busy += e - s
        print(f"{i - k:3d} {n[:60]:60s} {g:8d} {(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.2f} {gap:7.2f}")
    span = (rows[end - 1][1] - t0) / 1e3
    print(f"cycle span {span:.1f} us, busy {tot_busy / 1e3:.1f} us, idle {span - tot_busy / 1e3:.1f} us, "
          f"{end - k} dispatches")


if __name__ == "__main__":
    main()
