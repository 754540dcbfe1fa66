#!/usr/bin/env python3
"""Same-box A/B of a launch-time libpamg option on the bench's timed region: one 512^3 setup and
upload, then alternating values (a, b, a, b, ...), each timed as bench.py times it (graph replay
of --steps pipelined V-cycles, synchronised on both sides; the graphs are re-captured after every
switch) and checked for the same bits of x.

    python tools/cycle_ab.py --ab chain_store_x=1,0 --rounds 3 > ab.jsonl
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import parallel_amg_amd as pa  # noqa: E402
from parallel_amg_amd import _lib  # noqa: E402
from parallel_amg_amd.partitioned import Context, PVector, mul  # noqa: E402
from parallel_amg_amd.solver import AMGSolver  # noqa: E402


def set_opt(k, v):
    _lib.call("pamg_set_option", k.encode(), int(v))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--kind", default="poisson3d")
    ap.add_argument("--ab", required=True, help="KEY=a,b")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    key, vals = a.ab.split("=")
    va, vb = (int(v) for v in vals.split(","))
    t0 = time.time()
    ctx = Context(0)
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, a.kind, a.n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    del A
    S = AMGSolver(ctx, H, graph=True)
    Af = S.fine_operator()
    b = PVector(ctx, Af.nrows)
    mul(b, Af, PVector(ctx, Af.n_own_cols, Af.n_ghost, xs[0]))
    print(f"# setup + upload {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    ref = None
    for r in range(a.rounds):
        for v in (va, vb):
            set_opt(key, v)
            S.set_graph(False)
            S.set_graph(True)
            x = S.new_vector()
            S.vcycle(x, b, 3)  # warm-up + capture
            x = S.new_vector()
            ctx.sync()
            ts = time.perf_counter()
            S.vcycle_async(x, b, a.steps)
            ctx.sync()
            dt = time.perf_counter() - ts
            bits = x.own_values().view(np.int64)
            same = None if ref is None else bool(np.array_equal(bits, ref))
            if ref is None:
                ref = bits.copy()
            print(json.dumps({key: v, "round": r, "ms_per_cycle": round(dt / a.steps * 1e3, 4),
                              "vcycles_per_s": round(a.steps / dt, 2), "same_bits_as_first": same}), flush=True)
    set_opt(key, va)


if __name__ == "__main__":
    main()
