"""Hierarchy dump/load (SURVEY §5 checkpoint/resume): a saved and reloaded hierarchy equals the
original array for array (every level, part, plan; agglomerated tails too), and on the GPU
the reloaded one runs the same V-cycles bit for bit."""
import numpy as np
import pytest

import parallel_amg_amd as pa


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def same_csr(A, B):
    if A is None or B is None:
        assert A is None and B is None
        return
    assert A.ncols == B.ncols and np.array_equal(A.rowptr, B.rowptr) and np.array_equal(A.col, B.col)
    assert np.array_equal(bits(A.val), bits(B.val))


def same_plan(P, Q):
    if P is None or Q is None:
        assert P is None and Q is None
        return
    assert (P.n_own, P.col0, P.nbrs, P.recv_counts, P.send_counts) == (Q.n_own, Q.col0, Q.nbrs, Q.recv_counts, Q.send_counts)
    assert np.array_equal(P.ghost_ids, Q.ghost_ids) and np.array_equal(P.send_idx, Q.send_idx)
    assert P._recv == Q._recv and sorted(P._send) == sorted(Q._send)
    for q in P._send:
        assert np.array_equal(P._send[q], Q._send[q])


@pytest.mark.parametrize("kind,n,nparts,agglomerate", [("poisson3d", 14, 1, 32768), ("aniso3d", 12, 3, 0),
                                                       ("poisson2d", 48, 2, 400)])
def test_roundtrip(tmp_path, built, kind, n, nparts, agglomerate):
    be = pa.SequentialBackend(nparts)
    A, offs, _ = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=50, agglomerate=agglomerate))
    path = str(tmp_path / "h.npz")
    pa.save_hierarchy(H, path)
    G = pa.load_hierarchy(path)
    assert (G.nparts, G.nlevels, G.n_coarse, G.rep_level) == (H.nparts, H.nlevels, H.n_coarse, H.rep_level)
    assert np.array_equal(G.rep_offsets, H.rep_offsets) and np.array_equal(bits(G.ainv), bits(H.ainv))
    for l in range(H.nlevels):
        for p in range(nparts):
            a, b = H.levels[l][p], G.levels[l][p]
            assert np.array_equal(a.offsets, b.offsets)
            assert (a.omega, a.rho, a.whole) == (b.omega, b.rho, b.whole)
            assert (a.agg is None) == (b.agg is None) and (a.agg is None or np.array_equal(a.agg, b.agg))
            for w in "APR":
                same_csr(getattr(a, w), getattr(b, w))
            for w in ("planA", "planP", "planR"):
                same_plan(getattr(a, w), getattr(b, w))


@pytest.mark.gpu
def test_reloaded_hierarchy_solves_identically(tmp_path, ctx):
    from parallel_amg_amd.partitioned import PVector, mul
    from parallel_amg_amd.solver import AMGSolver
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 20)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100), device=ctx)
    path = str(tmp_path / "h.npz")
    pa.save_hierarchy(H, path)
    out = []
    for h in (H, pa.load_hierarchy(path)):
        S = AMGSolver(ctx, h)
        b = PVector(ctx, S.A[0].nrows)
        mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
        x = S.new_vector()
        S.vcycle(x, b, 5)
        out.append(x.own_values())
    assert np.array_equal(bits(out[0]), bits(out[1]))
