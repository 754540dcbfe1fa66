#!/usr/bin/env python3
"""One part's kernels of an N-part hierarchy, timed alone on one GPU.

The driver's 8-GPU run measures the multi-GPU cycle; this measures what the T_N model of
DESIGN.md needs from one part: the 512^3 problem is set up as N z-slab parts (SequentialBackend,
the global-view operators, SPEC §S7), part p's level operators are uploaded into an in-process
world's context p (so its exchange plans address the real neighbour ranks), and each row
operation of the cycle is timed with HIP events through pamg_bench_rowop — the part's interior
and boundary rows, no exchange (exchanges are timed by bench.py N > 1). Level 0's cross-cycle
chain (op 5) runs the part's blocked pass on its inner planes plus the separate sweeps on the
planes next to its neighbours and the boundary rows (sweeps_part without exchanges).

    python tools/part_bench.py --n 512 --parts 8 --part 3 > part.json
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import parallel_amg_amd as pa  # noqa: E402
from parallel_amg_amd._lib import call, layout_of  # noqa: E402
from parallel_amg_amd.partitioned import LocalWorld, PSparseMatrix, PVector  # noqa: E402

OPNAME = {0: "spmv", 1: "residual", 2: "jacobi", 3: "prolong", 4: "jacobi_residual_tb", 5: "chain3_tb"}


def time_op(ctx, M, op, reps):
    print(f"#   op {OPNAME[op]} ({M.nrows} rows)", file=sys.stderr, flush=True)
    x = PVector(ctx, M.n_own_cols, M.n_ghost, np.random.default_rng(1).standard_normal(M.n_own_cols))
    b = PVector(ctx, M.nrows, 0, np.ones(M.nrows))
    # (the blocked passes of a part feed y to the next stage's boundary rows: ghost slots too)
    y = PVector(ctx, M.n_own_cols, M.n_ghost) if op >= 4 else PVector(ctx, M.nrows)
    ms = C.c_double()
    call("pamg_bench_rowop", ctx.handle, M.handle, op, x.handle, b.handle, y.handle, 0.6, reps, C.byref(ms))
    return ms.value


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--kind", default="poisson3d")
    ap.add_argument("--parts", type=int, default=8)
    ap.add_argument("--part", type=int, default=3)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--agglomerate", type=int, default=32768)
    a = ap.parse_args()
    t0 = time.time()
    W = LocalWorld(a.parts)
    ctx = W.ctxs[a.part]
    be = pa.SequentialBackend(a.parts)
    A, offs, xs = pa.generate_problem(be, a.kind, a.n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000, agglomerate=a.agglomerate), device=ctx)
    del A
    print(f"# setup {time.time() - t0:.1f}s, {H.nlevels} levels, replicated from {H.rep_level}", file=sys.stderr,
          flush=True)
    p = a.part
    out = []
    for l in range(H.nlevels - 1):
        lp = H.levels[l][p]
        whole = lp.whole
        rec = {"level": l, "rows": int(lp.A.nrows), "nnz": int(lp.A.nnz), "whole": bool(whole), "ms": {}}
        Ad = PSparseMatrix(ctx, lp.A, None if whole else lp.planA)
        lay = layout_of(Ad)
        rec["A_layout"] = {k: lay[k] for k in ("sym", "sym_vd", "jr_fused", "tm", "ell", "tile_nnz")}
        for op in ((1, 2, 4, 5) if l == 0 and lay["jr_fused"] else (1, 2)):
            rec["ms"][f"A_{OPNAME[op]}"] = round(time_op(ctx, Ad, op, a.reps), 4)
        del Ad
        rep_next = l + 1 >= H.rep_level
        Rd = PSparseMatrix(ctx, lp.R, lp.planR)
        rec["ms"]["R_spmv"] = round(time_op(ctx, Rd, 0, a.reps), 4)
        rec["R_layout"] = {k: v for k, v in layout_of(Rd).items() if k in ("rpat", "ell", "tm", "tile_nnz")}
        del Rd
        Pd = PSparseMatrix(ctx, lp.P, None if rep_next else lp.planP)
        rec["ms"]["P_prolong"] = round(time_op(ctx, Pd, 3, a.reps), 4)
        rec["P_layout"] = {k: v for k, v in layout_of(Pd).items() if k in ("pnc", "pnc_compact", "tm", "tile_nnz")}
        del Pd
        out.append(rec)
        print(json.dumps(rec), file=sys.stderr, flush=True)
    print(json.dumps({"n": a.n, "kind": a.kind, "parts": a.parts, "part": p, "levels": out,
                      "note": "one part's row operations alone (no exchange), HIP events, ms per launch"}))


if __name__ == "__main__":
    main()
