"""Matrix Market input (BASELINE.json configs[4]: SuiteSparse Flan_1565, not in the image) and
the elastic3d stand-in generator: libpamg's reader against scipy.io.mmread (an independent
parser) and the product generator against the oracle, bit for bit."""
import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp

import parallel_amg_amd as pa
from oracle import oracle as O
from parallel_amg_amd import hcsr as HC


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def _write(tmp_path, M, name, symmetry="general", field="real"):
    p = tmp_path / name
    scipy.io.mmwrite(str(p), M, symmetry=symmetry, field=field)
    return str(p)


@pytest.mark.parametrize("symmetry", ["general", "symmetric"])
def test_reader_matches_scipy(tmp_path, symmetry, built):
    rng = np.random.default_rng(4)
    A = O.generate("elastic3d", 4, 4, 3).to_scipy()
    A = A + sp.diags(np.round(rng.standard_normal(A.shape[0]), 6))  # non-integer values too
    path = _write(tmp_path, A.tocoo(), "a.mtx", symmetry)
    ref = scipy.io.mmread(path).tocsr()
    ref.sort_indices()
    M, n = HC.read_mtx(path)
    assert n == A.shape[0] and M.nrows == n
    assert np.array_equal(M.rowptr, ref.indptr) and np.array_equal(M.col, ref.indices)
    assert np.array_equal(bits(M.val), bits(ref.data))
    # row ranges (what each part of a partitioned run reads)
    for r0, r1 in ((0, 7), (7, 100), (100, n)):
        Mp, _ = HC.read_mtx(path, r0, r1)
        assert np.array_equal(Mp.rowptr, ref.indptr[r0:r1 + 1] - ref.indptr[r0])
        assert np.array_equal(Mp.col, ref.indices[ref.indptr[r0]:ref.indptr[r1]])


def test_reader_duplicates_and_pattern(tmp_path, built):
    p = tmp_path / "d.mtx"
    p.write_text("%%MatrixMarket matrix coordinate real general\n% comment\n3 3 5\n"
                 "1 1 1.5\n3 2 2\n1 1 0.25\n2 2 4\n3 3 1e-3\n")
    M, n = HC.read_mtx(str(p))
    assert n == 3 and M.rowptr.tolist() == [0, 1, 2, 4]
    assert M.col.tolist() == [0, 1, 1, 2] and M.val.tolist() == [1.75, 4.0, 2.0, 1e-3]
    q = tmp_path / "p.mtx"
    q.write_text("%%MatrixMarket matrix coordinate pattern symmetric\n2 2 2\n1 1\n2 1\n")
    M, _ = HC.read_mtx(str(q))
    assert M.col.tolist() == [0, 1, 0] and M.val.tolist() == [1.0, 1.0, 1.0]
    r = tmp_path / "bad.mtx"
    r.write_text("%%MatrixMarket matrix array real general\n2 2\n1\n2\n3\n4\n")
    with pytest.raises(Exception):
        HC.read_mtx(str(r))


def test_elastic_generator_and_setup_bit_exact(built):
    be = pa.SequentialBackend(2)
    A, offs, xs = pa.generate_problem(be, "elastic3d", 7)
    Ao = O.generate("elastic3d", 7, 7, 7)
    a = A[0]
    assert a.nrows + A[1].nrows == Ao.nrows
    assert np.array_equal(np.concatenate([A[0].col, A[1].col]), Ao.col)
    assert np.array_equal(bits(np.concatenate([A[0].val, A[1].val])), bits(Ao.val))
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=60))
    Ho = O.setup(Ao, nparts=2, max_coarse=60)
    assert H.nlevels == Ho.nlevels
    for l in range(H.nlevels):
        full = np.concatenate([M.val for M in H.part_rows(l)])
        assert np.array_equal(bits(full), bits(Ho.A[l].val))


def _irregular_spd(seed=0):
    rng = np.random.default_rng(seed)
    A = O.generate("poisson2d", 40, 40, 1).to_scipy().tolil()
    for i in range(200):  # a dense-ish corner: rows 0..199 get ~40 extra couplings
        for j in rng.choice(200, 40, replace=False):
            if j != i:
                A[i, j] = A[j, i] = -0.01
    A = A.tocsr()
    A.setdiag(A.diagonal() + abs(A).sum(axis=1).A1)   # strictly diagonally dominant -> SPD
    A.sort_indices()
    return A


def test_nnz_balanced_partition(tmp_path, built):
    A = _irregular_spd()
    path = _write(tmp_path, A.tocoo(), "irr.mtx", "symmetric")
    counts = HC.mtx_row_counts(path)
    assert np.array_equal(counts, np.diff(A.indptr))
    be = pa.SequentialBackend(3)
    Ap, offs, xs = pa.load_problem(be, path, partition="nnz")
    per = [Ap[p].nnz for p in range(3)]
    assert max(per) - min(per) <= max(np.diff(A.indptr)) + 2      # balanced to one row
    assert offs[1] < A.shape[0] // 3                              # the dense corner is split off
    H = pa.build_hierarchy(be, Ap, offs, pa.SAParams(max_coarse=50))
    Ao = O.CSR(A.indptr.astype(np.int64), A.indices.astype(np.int64), A.data.copy(), A.shape[1])
    Ho = O.setup(Ao, offsets=offs, max_coarse=50)
    assert H.nlevels == Ho.nlevels
    for l in range(H.nlevels):
        full = np.concatenate([M.val for M in H.part_rows(l)])
        assert np.array_equal(bits(full), bits(Ho.A[l].val))
        assert np.array_equal(H.offsets(l), Ho.offsets[l])


def test_load_problem_partitions_like_the_generator(tmp_path, built):
    Ao = O.generate("poisson3d", 6, 6, 6)
    path = _write(tmp_path, Ao.to_scipy().tocoo(), "p.mtx", "symmetric")
    be = pa.SequentialBackend(3)
    A, offs, xs = pa.load_problem(be, path)
    G, goffs, gxs = pa.generate_problem(be, "poisson3d", 6)
    assert np.array_equal(offs, goffs)
    for p in range(3):
        assert np.array_equal(A[p].rowptr, G[p].rowptr) and np.array_equal(A[p].col, G[p].col)
        assert np.array_equal(bits(A[p].val), bits(G[p].val)) and np.array_equal(xs[p], gxs[p])
