#!/usr/bin/env python3
"""Diagnostic (round 5): the 512^3 level-0 one-sweep ops (k_sym_zm) and the ELL level-1 / R0 ops
against the oracle on random vectors; prints one JSON line per op with the number of differing
entries. Dev tool."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import parallel_amg_amd as pa  # noqa: E402
from oracle import oracle as O  # noqa: E402
from parallel_amg_amd.partitioned import Context, PSparseMatrix, PVector, jacobi, mul, residual  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
ctx = Context(0)
be = pa.SequentialBackend(1)
A, offs, xs = pa.generate_problem(be, "poisson3d", n)
M = A[0]
Mo = O.CSR(M.rowptr, M.col.astype(np.int64), M.val, M.ncols)
D = PSparseMatrix(ctx, M)
N = M.nrows
rng = np.random.default_rng(5)
xh, bh = rng.standard_normal(N), rng.standard_normal(N)
x, b, y = PVector(ctx, N, 0, xh), PVector(ctx, N, 0, bh), PVector(ctx, N)


def rep(name, got, ref):
    d = np.flatnonzero(got.view(np.int64) != ref.view(np.int64))
    print(json.dumps({"op": name, "n": int(N), "differ": int(d.size), "first": d[:5].tolist(),
                      "got": got[d[:3]].tolist(), "ref": ref[d[:3]].tolist()}), flush=True)


mul(y, D, x)
rep("spmv", y.own_values(), O.spmv(Mo, xh))
residual(y, D, x, b)
rep("residual", y.own_values(), O.residual(Mo, xh, bh))
t = PVector(ctx, N)
jacobi(x, D, b, t, 2.0 / 3.0, 1)
rep("jacobi", x.own_values(), O.jacobi(Mo, xh, bh, 2.0 / 3.0))
# zero-scaled inputs like a preconditioner's late iterations
xs_, bs_ = xh * 1e-6, bh * 1e-6
x2, b2 = PVector(ctx, N, 0, xs_), PVector(ctx, N, 0, bs_)
residual(y, D, x2, b2)
rep("residual_small", y.own_values(), O.residual(Mo, xs_, bs_))
# PCG pieces: one preconditioner application z = V(r) from zero against the oracle's, then PCG
from parallel_amg_amd.solver import AMGSolver  # noqa: E402
H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
S = AMGSolver(ctx, H)
lv = [H.levels[l][0] for l in range(H.nlevels)]
Ho = O.hierarchy_from_levels([p.A for p in lv], [p.P for p in lv[:-1]], [p.R for p in lv[:-1]],
                             [p.omega for p in lv], H.ainv)
bb = PVector(ctx, N)
mul(bb, S.A[0], PVector(ctx, N, 0, xs[0]))
bo = bb.own_values()
for maxit in (1, 2, 3):
    xg = S.new_vector()
    k, hg = S.pcg(xg, bb, 1e-30, maxit)
    xo, ko, ho = Ho.pcg(bo, 1e-30, maxit)
    rep(f"pcg_it{maxit}", xg.own_values(), xo)
    print(json.dumps({"hist_gpu": np.asarray(hg).tolist(), "hist_oracle": np.asarray(ho).tolist()}), flush=True)
# one stationary cycle from zero through the eager path (graph off) and with the graph
for g in (False, True):
    S.set_graph(g)
    xg = S.new_vector()
    S.vcycle(xg, bb, 1)
    rep(f"vcycle1_graph{int(g)}", xg.own_values(), Ho.solve(bo, 1))
