#!/usr/bin/env python3
"""Kernel micro-benchmark: row-operation kernels of libpamg on the hierarchy matrices.

For each tuning configuration (pamg_set_option) the level operators are re-uploaded and every
row op is timed with HIP events (pamg_bench_rowop); prints one JSON line per measurement with
the algorithmic bytes (SURVEY.md §8d CSR model) and the achieved GB/s, plus the rate on the
bytes the uploaded layout actually streams (format_GBps). Dev tool, not part of the ABI.

    python tools/kbench.py --n 512 --levels 1      # fine matrix only (no setup)
    python tools/kbench.py --n 256 --levels 3      # hierarchy levels 0..2 (A, R, P)
"""
from __future__ import annotations

import argparse
import ctypes as C
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import parallel_amg_amd as pa  # noqa: E402
from parallel_amg_amd._lib import call, layout_of  # noqa: E402
from parallel_amg_amd.partitioned import Context, PSparseMatrix, PVector  # noqa: E402
from parallel_amg_amd.solver import AMGSolver  # noqa: E402

OPNAME = {0: "spmv", 1: "residual", 2: "jacobi", 3: "prolong", 4: "jacobi_residual_tb", 5: "chain3_tb"}


def set_opts(**kw):
    for k, v in kw.items():
        call("pamg_set_option", k.encode(), int(v))


def bench(ctx, M, op, reps):
    x = PVector(ctx, M.n_own_cols, M.n_ghost, np.random.default_rng(1).standard_normal(M.n_own_cols))
    b = PVector(ctx, M.nrows, 0, np.ones(M.nrows))
    y = PVector(ctx, M.nrows)
    ms = C.c_double()
    call("pamg_bench_rowop", ctx.handle, M.handle, op, x.handle, b.handle, y.handle, 0.6, reps,
         C.byref(ms))
    extra = {0: 0, 1: 1, 2: 1, 3: 1, 4: 2, 5: 3}[op]  # fused: b + the other outputs, matrix once
    return ms.value, AMGSolver.csr_bytes(M, extra), AMGSolver.rowsum_bytes(M, extra)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--kind", default="poisson3d", choices=["poisson2d", "poisson3d", "aniso3d", "elastic3d"])
    ap.add_argument("--permute", type=int, default=None, metavar="SEED",
                    help="seeded random symmetric renumbering before setup (the irregular path)")
    ap.add_argument("--levels", type=int, default=1)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--configs", default="1024:1,1024:0",
                    help="tile_nnz:tile_order:col24:value_dict:long_tiles:row_len8:col_dict:tile_major:col_dict_anchor:"
                         "col_dict_tile:x_stage:tm_tile_dicts,...")
    ap.add_argument("--ops", default="0,2")
    ap.add_argument("--mats", default=None, help="comma list of level matrices to run (e.g. R0,A1); default all")
    ap.add_argument("--ab", default=None,
                    help="launch-time option to A/B on the same upload: KEY (values 0,1,0,1) or KEY=a,b "
                         "(a,b,a,b; e.g. symd_chunks=1,2)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="extra pamg_set_option before the uploads (e.g. band_pct=50)")
    ap.add_argument("--sweep", default=None, metavar="KEY=V1,V2,...",
                    help="an upload-time option swept over values: every matrix re-uploaded per value "
                         "(e.g. band_pct_restrict=25,50,100)")
    args = ap.parse_args()
    ab_vals = (0, 1, 0, 1)
    if args.ab and "=" in args.ab:
        args.ab, vs = args.ab.split("=")
        a_, b_ = (int(v) for v in vs.split(","))
        ab_vals = (a_, b_, a_, b_)
    for kv in args.set:
        k, v = kv.split("=")
        set_opts(**{k: int(v)})
    ctx = Context(0)
    be = pa.SequentialBackend(1)
    t = time.time()
    A, offs, xs = pa.generate_problem(be, args.kind, args.n)
    if args.permute is not None:
        A, xs = pa.permute_problem(A, xs, args.permute)
    mats = {"A0": (A[0], None)}
    if args.levels > 1:
        H = pa.build_hierarchy(be, A, offs, device=ctx)
        for l in range(min(args.levels, H.nlevels - 1)):
            lp = H.levels[l][0]
            mats[f"A{l}"] = (lp.A, lp.planA)
            mats[f"R{l}"] = (lp.R, lp.planR)
            mats[f"P{l}"] = (lp.P, lp.planP)
    print(f"# setup {time.time() - t:.1f}s", file=sys.stderr, flush=True)
    ops = [int(o) for o in args.ops.split(",")]
    # the grid operator first: a prolongation over its grid may take the neighbour-coded layout
    # (PncSet: the upload looks the grid up on the context)
    grid_op = PSparseMatrix(ctx, *mats["A0"])  # noqa: F841 (kept alive: its grid stays registered)
    sweep_key, sweep_vals = (args.sweep.split("=")[0], [int(v) for v in args.sweep.split("=")[1].split(",")]) \
        if args.sweep else (None, [None])
    for sv, cfg in itertools.product(sweep_vals, args.configs.split(",")):
        if sweep_key:
            set_opts(**{sweep_key: sv})
        given = [int(v) for v in cfg.split(":")]
        vals = given + [1024, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1][len(given):]  # library defaults for missing fields
        tnnz, order, c24, vd, lt, rl8, cd, tm, anc, ptd, xst, tmpt = vals[:12]
        set_opts(tile_nnz=tnnz, tile_order=order, col24=c24, value_dict=vd, long_tiles=lt, row_len8=rl8,
                 col_dict=cd, tile_major=tm, col_dict_anchor=anc, col_dict_tile=ptd, x_stage=xst, tm_tile_dicts=tmpt)
        for name, (M, plan) in mats.items():
            if args.mats and name not in args.mats.split(","):
                continue
            D = PSparseMatrix(ctx, M, plan)
            for op in ops:
                if op in (2, 4, 5) and not name.startswith("A"):
                    continue
                if op >= 4 and not layout_of(D).get("jr_fused"):
                    continue
                if op == 3 and not name.startswith("P"):
                    continue
                for abv in (ab_vals if args.ab else (None,)):
                    if abv is not None:
                        set_opts(**{args.ab: abv})
                    ms, byt, fbyt = bench(ctx, D, op, args.reps)
                    # GBps: SURVEY §8(d) CSR bytes; format_GBps: the bytes the uploaded layout streams
                    rec = {"cfg": cfg + "".join(f"+{kv}" for kv in args.set), "mat": name, "op": OPNAME[op], "rows": D.nrows, "nnz": D.nnz,
                           "ms": round(ms, 4), "GBps": round(byt / ms / 1e6, 1),
                           "format_GBps": round(fbyt / ms / 1e6, 1), "layout": layout_of(D)}
                    if abv is not None:
                        rec[args.ab] = abv
                    if sweep_key:
                        rec[sweep_key] = sv
                    print(json.dumps(rec), flush=True)
                if args.ab:
                    set_opts(**{args.ab: ab_vals[0]})
            del D


if __name__ == "__main__":
    main()
