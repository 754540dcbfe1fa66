#!/usr/bin/env python3
"""Row-length sweep of the row-operation kernels (dev tool): random sparse matrices with a
fixed number of nonzeros per row (columns uniform over a small x, as on the coarse levels),
timed with pamg_bench_rowop for each tuning configuration. Separates the per-row cost (the
in-order LDS sum of SPEC §S3) from the per-nonzero cost.

    python tools/rowlen_bench.py [--nnz 200000] [--lens 4,16,64,256,432] [--configs ...]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from parallel_amg_amd._lib import call  # noqa: E402
from parallel_amg_amd.hcsr import HCSR  # noqa: E402
from parallel_amg_amd.partitioned import Context, PSparseMatrix, PVector  # noqa: E402


def random_rows(nrows, ncols, per_row, seed=0):
    rng = np.random.default_rng(seed)
    # sorted uniform columns (repeats allowed: a row sum does not care)
    col = np.sort(rng.integers(0, ncols, (nrows, per_row)), axis=1).astype(np.int32)
    rp = np.arange(nrows + 1, dtype=np.int64) * per_row
    val = rng.standard_normal(nrows * per_row)
    return HCSR.from_arrays(rp, col.reshape(-1), val, ncols)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nnz", type=int, default=200000)
    ap.add_argument("--ncols", type=int, default=2000)
    ap.add_argument("--lens", default="4,8,16,32,64,128,256,432,800")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--ops", default="0,1")
    ap.add_argument("--opts", default="", help="semicolon-separated option sets: name=v,name=v;...")
    a = ap.parse_args()
    ctx = Context(0)
    for optset in (a.opts.split(";") if a.opts else [""]):
        for kv in filter(None, optset.split(",")):
            k, v = kv.split("=")
            call("pamg_set_option", k.encode(), int(v))
        for L in (int(v) for v in a.lens.split(",")):
            nrows = max(1, a.nnz // L)
            M = random_rows(nrows, a.ncols, min(L, a.ncols))
            D = PSparseMatrix(ctx, M)
            x = PVector(ctx, a.ncols, 0, np.random.default_rng(1).standard_normal(a.ncols))
            b = PVector(ctx, nrows, 0, np.ones(nrows))
            y = PVector(ctx, nrows)
            for op in (int(o) for o in a.ops.split(",")):
                ms = C.c_double()
                call("pamg_bench_rowop", ctx.handle, D.handle, op, x.handle, b.handle, y.handle, 0.6,
                     a.reps, C.byref(ms))
                print(json.dumps({"opts": optset, "len": L, "rows": nrows, "nnz": M.nnz, "op": op,
                                  "us": round(ms.value * 1e3, 2)}), flush=True)
            del D, x, b, y


if __name__ == "__main__":
    main()
