"""Pin the CPU oracle (oracle/pamg_oracle.c) before trusting it.

The reference ships no fixtures (parity with the reference is unpinned), so
the oracle is pinned by (a) independent implementations (scipy.sparse products, numpy
linear algebra), (b) hand-derived known answers, (c) the SPEC's own size formulas, and
(d) the committed golden fixtures (tests/golden/make_golden.py) against drift."""
import glob
import hashlib
import os

import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
EPS = 2.0 ** -53


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


@pytest.mark.parametrize("kind,n,nnz", [("poisson2d", 256, 326_656), ("poisson3d", 128, 14_581_760),
                                        ("poisson3d", 16, 16**3 * 7 - 3 * 2 * 16**2)])
def test_generator_nnz_formula(kind, n, nnz):
    # nnz = n(1+2d) - sum_k 2n/N_k
    A = O.generate(kind, *O.grid_shape(kind, n))
    assert A.nnz == nnz
    assert np.all(np.diff(A.rowptr) > 0)
    for i in range(0, A.nrows, max(1, A.nrows // 50)):
        c = A.col[A.rowptr[i]:A.rowptr[i + 1]]
        assert np.all(np.diff(c) > 0) and i in c


def test_generator_values():
    A = O.generate("aniso3d", 4, 4, 4, eps=1e-3).to_scipy()
    d = A.diagonal()
    assert np.all(d == 4.0 + 2.0 * 1e-3)
    assert A[0, 16] == -1e-3 and A[0, 1] == -1.0 and A[0, 4] == -1.0
    assert (A - A.T).nnz == 0


@pytest.mark.parametrize("kind,n", [("poisson2d", 40), ("poisson3d", 14), ("aniso3d", 12)])
def test_spmv_against_scipy(kind, n):
    A = O.generate(kind, *O.grid_shape(kind, n))
    rng = np.random.default_rng(0)
    x = rng.standard_normal(A.nrows)
    y = O.spmv(A, x)
    S = A.to_scipy()
    bound = 8 * EPS * (abs(S) @ np.abs(x))
    assert np.all(np.abs(y - S @ x) <= bound)
    # SPEC §S3 order: a sequential left-to-right sum of rounded products
    for i in (0, A.nrows // 2, A.nrows - 1):
        s = 0.0
        for k in range(A.rowptr[i], A.rowptr[i + 1]):
            s = s + A.val[k] * x[A.col[k]]
        assert y[i] == s


def test_jacobi_known_answer():
    A = O.CSR(np.array([0, 2, 5, 7]), np.array([0, 1, 0, 1, 2, 1, 2]),
              np.array([4.0, -1, -1, 4, -1, -1, 4]), 3)
    b = np.array([1.0, 2.0, 3.0])
    x1 = O.jacobi(A, np.zeros(3), b, 1.0)
    assert np.array_equal(x1, [0.25, 0.5, 0.75])
    x2 = O.jacobi(A, x1, b, 1.0)
    assert np.array_equal(x2, [0.375, 0.75, 0.875])
    assert np.array_equal(O.residual(A, x1, b), [0.5, 1.0, 0.5])


def _chain(n):
    rp = [0]
    col, val = [], []
    for i in range(n):
        for j, v in ((i - 1, -1.0), (i, 2.0), (i + 1, -1.0)):
            if 0 <= j < n:
                col.append(j)
                val.append(v)
        rp.append(len(col))
    return O.CSR(np.array(rp), np.array(col), np.array(val), n)


def test_aggregation_known_answer_chain():
    # hand-derived (SPEC §S4.3): pass 1 -> {0,1}, {2,3,4}, {5,6,7}; pass 2 puts 8 with 7
    H = O.setup(_chain(9), max_coarse=3)
    assert H.agg[0].tolist() == [0, 0, 1, 1, 1, 2, 2, 2, 2]


def test_aggregation_known_answer_grid4x4():
    # hand-derived: pass 1 -> {0,1,4} {3,2,7} {9,5,8,10,13} {15,11,14}; pass 2: 6->agg1, 12->agg2
    H = O.setup(O.generate("poisson2d", 4, 4, 1), max_coarse=4)
    assert H.agg[0].tolist() == [0, 0, 1, 1, 0, 2, 1, 1, 2, 2, 2, 3, 2, 2, 3, 3]


def test_aggregation_semicoarsening_aniso():
    # theta = 0.02 keeps the eps = 1e-3 z-links weak: aggregates never span two z-planes
    n = 8
    H = O.setup(O.generate("aniso3d", n, n, n), max_coarse=50)
    agg, z = H.agg[0], np.arange(n**3) // (n * n)
    for a in np.unique(agg):
        assert len(np.unique(z[agg == a])) == 1


@pytest.mark.parametrize("kind,n,nparts", [("poisson2d", 48, 1), ("poisson3d", 12, 2), ("aniso3d", 10, 3)])
def test_galerkin_and_prolongator_against_scipy(kind, n, nparts):
    A = O.generate(kind, *O.grid_shape(kind, n))
    H = O.setup(A, nparts=nparts, max_coarse=20, agglomerate=0)
    for l in range(H.nlevels - 1):
        Al, P, R = H.A[l].to_scipy(), H.P[l].to_scipy(), H.R[l].to_scipy()
        assert (R - P.T).nnz == 0 and np.array_equal((R - P.T).toarray(), np.zeros(R.shape))
        # P = (I - omega D^-1 A) T with T from the aggregates (SPEC §S4.4-6)
        agg = H.agg[l]
        nc = H.A[l + 1].nrows
        cnt = np.bincount(agg[agg >= 0], minlength=nc)
        rows = np.nonzero(agg >= 0)[0]
        T = sp.csr_matrix((1.0 / np.sqrt(cnt[agg[rows]]), (rows, agg[rows])), shape=(Al.shape[0], nc))
        Pref = T - sp.diags(H.omega[l] / Al.diagonal()) @ (Al @ T)
        assert abs(P - Pref).max() <= 1e-14
        Ac = (R @ Al @ P).toarray()
        assert np.abs(Ac - H.A[l + 1].to_scipy().toarray()).max() <= 1e-13 * np.abs(Ac).max()
        # decoupled aggregation: aggregates never cross part boundaries
        o = H.offsets[l]
        for p in range(nparts):
            ap = agg[o[p]:o[p + 1]]
            ap = ap[ap >= 0]
            if len(ap):
                oc = H.offsets[l + 1]
                assert ap.min() >= oc[p] and ap.max() < oc[p + 1]


def test_coarse_inverse():
    A = O.generate("poisson3d", 10, 10, 10)
    H = O.setup(A, max_coarse=200)
    Ac = H.A[-1].to_scipy().toarray()
    np.testing.assert_allclose(H.ainv @ Ac, np.eye(len(Ac)), atol=1e-10)


def test_vcycle_converges_to_manufactured_solution():
    A = O.generate("poisson2d", 64, 64, 1)
    xs = O.xstar(A.nrows)
    b = O.spmv(A, xs)
    H = O.setup(A, max_coarse=100)
    x, hist = H.solve(b, 40, res_hist=True)
    assert np.all(np.diff(hist) < 0)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8
    r = b - A.to_scipy() @ x
    assert abs(np.linalg.norm(r) - hist[-1]) <= 1e-9 * max(hist[-1], 1e-300) + 1e-15


def test_oracle_from_levels_equals_setup():
    A = O.generate("poisson3d", 12, 12, 12)
    H = O.setup(A, max_coarse=50)

    class M:  # int32-column view, as the product's host CSR exposes it
        def __init__(s, c):
            s.nrows, s.ncols, s.rowptr, s.col, s.val = c.nrows, c.ncols, c.rowptr, c.col.astype(np.int32), c.val

    H2 = O.hierarchy_from_levels([M(a) for a in H.A], [M(p) for p in H.P], [M(r) for r in H.R], H.omega,
                                 H.ainv.T.reshape(-1).copy())
    b = O.spmv(A, O.xstar(A.nrows))
    assert np.array_equal(bits(H.solve(b, 3)), bits(H2.solve(b, 3)))


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))), ids=os.path.basename)
def test_golden_fixtures(path):
    g = np.load(path, allow_pickle=False)
    kind, n, nparts = str(g["kind"]), int(g["n"]), int(g["nparts"])
    A = O.generate(kind, *O.grid_shape(kind, n))
    b = O.spmv(A, O.xstar(A.nrows))
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
    assert sha(b) == str(g["b_sha"])
    H = O.setup(A, nparts=nparts, max_coarse=int(g["max_coarse"]), agglomerate=0)
    assert H.nlevels == int(g["nlevels"])
    assert np.array_equal(bits(H.omega), bits(g["omega"]))
    for l in range(H.nlevels):
        assert np.array_equal(H.offsets[l], g[f"offsets_{l}"])
        mats = [("A", H.A[l])] + ([("P", H.P[l]), ("R", H.R[l])] if l < H.nlevels - 1 else [])
        for tag, M in mats:
            for part in ("rowptr", "col", "val"):
                assert sha(getattr(M, part)) == str(g[f"{tag}{l}_{part}_sha"]), (tag, l, part)
        if l < H.nlevels - 1:
            assert np.array_equal(H.agg[l], g[f"agg_{l}"])
    x, hist = H.solve(b, int(g["ncycles"]), res_hist=True)
    assert sha(x) == str(g["x_sha"])
    np.testing.assert_allclose(hist, g["res_hist"], rtol=1e-12)


def test_oracle_setup_is_thread_count_independent():
    """The oracle's setup runs rows of its Gustavson products, transpose, strength and Gershgorin
    loops on OpenMP threads (round 6, so the 512^3 setups finish in about a minute): every level's
    A, P, R and aggregates must have the same bits on 1 and on 8 threads (each row is computed as
    the serial loop computes it)."""
    L = O.lib()
    A = O.generate("aniso3d", 24, 24, 24)
    got = []
    for threads in (1, 8):
        L.orc_set_threads(threads)
        H = O.setup(A, nparts=3, max_coarse=40, agglomerate=0)
        h = hashlib.sha256()
        for l in range(H.nlevels):
            for M in [H.A[l]] + ([H.P[l], H.R[l]] if l < H.nlevels - 1 else []):
                for a in (M.rowptr, M.col, M.val):
                    h.update(np.ascontiguousarray(a).tobytes())
            if l < H.nlevels - 1:
                h.update(H.agg[l].tobytes())
        got.append(h.hexdigest())
    L.orc_set_threads(os.cpu_count() or 1)
    assert got[0] == got[1]
