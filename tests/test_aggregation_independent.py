"""An independent pin for the aggregation indices.

The oracle's aggregation (``oracle/pamg_oracle.c`` aggregate()) and the product's
(``csrc/setup.cpp`` pamg_setup_aggregate) share one formulation, so their bit-exact agreement
proves the port, not the algorithm. ``oracle.aggregate_sets`` restates SPEC §S4.2-3 a second
way — a scipy strength matrix built with whole-array numpy operations, and the three passes as
set operations on neighbour lists — and both C implementations must give its indices exactly:
hand-derived answers, the SPEC grids (every level of their hierarchies, 1-3 decoupled parts),
random graphs with weak links and isolated rows, and the BASELINE grids up to 128^3.
CPU only: no GPU is involved."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import oracle as O


def _chain(n):
    rp, col, val = [0], [], []
    for i in range(n):
        for j, v in ((i - 1, -1.0), (i, 2.0), (i + 1, -1.0)):
            if 0 <= j < n:
                col.append(j)
                val.append(v)
        rp.append(len(col))
    return O.CSR(np.array(rp), np.array(col), np.array(val), n)


def _product_agg(A, offs, theta=0.02):
    """The product's pamg_setup_aggregate, part by part (each part's rows, global columns),
    numbered globally like the oracle (part coarse offset + local number)."""
    from parallel_amg_amd import hcsr as HC
    out, base = np.empty(A.nrows, np.int64), 0
    for p in range(len(offs) - 1):
        a, b = int(offs[p]), int(offs[p + 1])
        sl = slice(A.rowptr[a], A.rowptr[b])
        M = HC.HCSR.from_arrays(A.rowptr[a:b + 1] - A.rowptr[a], A.col[sl].astype(np.int32), A.val[sl], A.ncols)
        agg, na = HC.aggregate(M, a, theta)
        out[a:b] = np.where(agg >= 0, agg.astype(np.int64) + base, -1)
        base += na
    return out


def test_strength_matrix_against_dense_definition():
    """SPEC §S4.2 evaluated entry by entry on a small operator with weak links (aniso3d)."""
    A = O.generate("aniso3d", 5, 4, 3)
    S = O.strength_matrix(A, 0.02)
    D = A.to_scipy().toarray()
    want = np.zeros_like(D, bool)
    for i in range(A.nrows):
        for j in range(A.nrows):
            if i != j and D[i, j] != 0.0:
                want[i, j] = abs(D[i, j]) >= 0.02 * np.sqrt(abs(D[i, i] * D[j, j]))
    assert np.array_equal(S.toarray() != 0, want)
    assert 0 < S.nnz < A.nnz - A.nrows  # the z-links are weak, the x/y links strong


def test_known_answers():
    # hand-derived (SPEC §S4.3; the same answers tests/test_oracle.py pins the C oracle with)
    agg, c = O.aggregate_sets(_chain(9))
    assert agg.tolist() == [0, 0, 1, 1, 1, 2, 2, 2, 2] and c.tolist() == [0, 3]
    agg, c = O.aggregate_sets(O.generate("poisson2d", 4, 4, 1))
    assert agg.tolist() == [0, 0, 1, 1, 0, 2, 1, 1, 2, 2, 2, 3, 2, 2, 3, 3] and c.tolist() == [0, 4]
    # decoupled over two parts: the chain split 5 | 4 aggregates each half on its own
    agg, c = O.aggregate_sets(_chain(9), offsets=[0, 5, 9])
    assert agg.tolist() == [0, 0, 1, 1, 1, 2, 2, 3, 3] and c.tolist() == [0, 2, 4]


@pytest.mark.parametrize("kind,n,nparts", [("poisson2d", 64, 1), ("poisson2d", 64, 2), ("poisson3d", 24, 1),
                                           ("poisson3d", 32, 3), ("aniso3d", 24, 2), ("elastic3d", 12, 1),
                                           ("elastic3d", 12, 2)])
def test_both_implementations_every_level(built, kind, n, nparts):
    """Every level of the oracle's hierarchy (its coarse operators have longer, irregular rows):
    the C oracle's aggregates, the product's, and the set restatement agree exactly."""
    A = O.generate(kind, *O.grid_shape(kind, n))
    H = O.setup(A, nparts=nparts, max_coarse=20, agglomerate=0)
    assert H.nlevels >= 2
    for l in range(H.nlevels - 1):
        offs = H.offsets[l]
        ref, coffs = O.aggregate_sets(H.A[l], offsets=offs)
        assert np.array_equal(coffs, H.offsets[l + 1]), (l, coffs, H.offsets[l + 1])
        assert np.array_equal(H.agg[l], ref), f"level {l}: the C oracle differs from the set restatement"
        assert np.array_equal(_product_agg(H.A[l], offs), ref), f"level {l}: the product differs"


def _random_graph(seed, n, density, weak_frac, iso_frac):
    rng = np.random.default_rng(seed)
    M = sp.random(n, n, density=density, random_state=rng, format="coo")
    v = -np.abs(rng.standard_normal(M.nnz))
    v[rng.random(M.nnz) < weak_frac] *= 1e-4  # below theta: weak
    M = sp.coo_matrix((v, (M.row, M.col)), shape=(n, n)).tocsr()
    M = (M + M.T).tolil()
    for i in np.nonzero(rng.random(n) < iso_frac)[0]:
        M[i, :] = 0
        M[:, i] = 0
    M = M.tocsr()
    M.setdiag(0)
    M.eliminate_zeros()
    M = (M + sp.diags(np.asarray(abs(M).sum(axis=1)).ravel() + 1.0 + rng.random(n))).tocsr()
    M.sort_indices()
    return O.CSR(M.indptr.astype(np.int64), M.indices.astype(np.int64), M.data.copy(), n)


@pytest.mark.parametrize("seed", range(8))
def test_random_graphs(built, seed):
    """Irregular patterns, weak couplings and isolated rows (aggregate -1), 1-4 parts with
    random offsets."""
    rng = np.random.default_rng(100 + seed)
    n = int(rng.integers(50, 1500))
    A = _random_graph(seed, n, float(rng.uniform(0.002, 0.03)), 0.3, 0.05)
    nparts = int(rng.integers(1, 5))
    offs = np.concatenate([[0], np.sort(rng.choice(np.arange(1, n), nparts - 1, replace=False)), [n]])
    ref, coffs = O.aggregate_sets(A, offsets=offs)
    H = O.setup(A, offsets=offs, max_coarse=max(1, n // 1000), agglomerate=0, max_levels=2)
    assert np.array_equal(H.agg[0], ref)
    assert np.array_equal(H.offsets[1], coffs)
    assert np.array_equal(_product_agg(A, offs), ref)


@pytest.mark.parametrize("kind,n,nparts", [("poisson3d", 128, 1), ("poisson2d", 256, 2), ("aniso3d", 64, 4)])
def test_baseline_grids(built, kind, n, nparts):
    """BASELINE.json configs at (or scaled to) CPU size: 3D 128^3 one part (configs[1]), 2D 256^2
    on 2 parts (configs[0]), anisotropic 64^3 on 4 parts (configs[3]'s operator and part count):
    level 0 and level 1 of the C oracle's hierarchy and the product's aggregates equal the set
    restatement."""
    A = O.generate(kind, *O.grid_shape(kind, n))
    H = O.setup(A, nparts=nparts, agglomerate=0)
    for l in range(min(2, H.nlevels - 1)):
        ref, coffs = O.aggregate_sets(H.A[l], offsets=H.offsets[l])
        assert np.array_equal(H.agg[l], ref)
        assert np.array_equal(coffs, H.offsets[l + 1])
        assert np.array_equal(_product_agg(H.A[l], H.offsets[l]), ref)
