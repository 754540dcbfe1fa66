#!/usr/bin/env python3
"""Where the 512^3 upload's time goes: the bench's hierarchy set up, then
AMGSolver (every level operator through pamg_mat_upload) with PAMG_TRACE_UPLOAD=1, whose per-phase
lines go to stderr; one JSON line with the wall times on stdout.

    PAMG_TRACE_UPLOAD=1 python tools/upload_trace.py --n 512 > up.json 2> up.log
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import parallel_amg_amd as pa  # noqa: E402
from parallel_amg_amd.partitioned import Context  # noqa: E402
from parallel_amg_amd.solver import AMGSolver  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    a = ap.parse_args()
    os.environ.setdefault("PAMG_TRACE_UPLOAD", "1")
    ctx = Context(0)
    be = pa.SequentialBackend(1)
    t0 = time.time()
    A, offs, xs = pa.generate_problem(be, "poisson3d", a.n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    del A
    t1 = time.time()
    print(f"# setup {t1 - t0:.1f}s", file=sys.stderr, flush=True)
    if os.environ.get("UPLOAD_PROFILE"):
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        S = AMGSolver(ctx, H)
        ctx.sync()
        pr.disable()
        pstats.Stats(pr, stream=sys.stderr).sort_stats("cumulative").print_stats(25)
    else:
        S = AMGSolver(ctx, H)
        ctx.sync()
    t2 = time.time()
    print(json.dumps({"n": a.n, "setup_s": round(t1 - t0, 2), "upload_s": round(t2 - t1, 2), "levels": S.L}))
    del S


if __name__ == "__main__":
    main()
