"""Product host setup (libpamg C++ routines driven by parallel_amg_amd.hierarchy) against the
oracle: every integer and every floating-point array bit-exact, for 1..4 in-process parts
(the PartitionedArrays debug-backend shape), plus the golden fixtures incl. BASELINE.json
configs[0] (2D 256^2, 2 parts on CPU)."""
import glob
import hashlib
import os

import numpy as np
import pytest

import parallel_amg_amd as pa
from oracle import oracle as O
from parallel_amg_amd import hcsr as HC

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _rows(M, a, b):
    sl = slice(M.rowptr[a], M.rowptr[b])
    return M.rowptr[a:b + 1] - M.rowptr[a], M.col[sl], M.val[sl]


def check_against_oracle(kind, n, nparts, max_coarse, agglomerate=32768):
    be = pa.SequentialBackend(nparts)
    A, offs, xs = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=max_coarse, agglomerate=agglomerate))
    Ao = O.generate(kind, *O.grid_shape(kind, n))
    Ho = O.setup(Ao, nparts=nparts, max_coarse=max_coarse, agglomerate=agglomerate)
    assert H.nlevels == Ho.nlevels
    assert np.array_equal(np.concatenate([xs[p] for p in range(nparts)]), O.xstar(Ao.nrows))
    for l in range(H.nlevels):
        assert np.array_equal(H.offsets(l), Ho.offsets[l])
        for p in range(nparts):
            lp, o = H.levels[l][p], Ho.offsets[l]
            # an agglomerated (whole) level: every part holds all rows
            a, b = (0, int(o[-1])) if lp.whole else (int(o[p]), int(o[p + 1]))
            rp, c, v = _rows(Ho.A[l], a, b)
            assert np.array_equal(lp.A.rowptr, rp) and np.array_equal(lp.A.col, c)
            assert np.array_equal(bits(lp.A.val), bits(v))
            assert lp.omega == Ho.omega[l] and lp.rho == Ho.rho[l]
            if l < H.nlevels - 1:
                rp, c, v = _rows(Ho.P[l], a, b)
                assert np.array_equal(lp.P.rowptr, rp) and np.array_equal(lp.P.col, c)
                assert np.array_equal(bits(lp.P.val), bits(v))
                # rows of R = the next level's rows as this level's aggregation numbered them
                co = H.rep_offsets if l + 1 == H.rep_level else Ho.offsets[l + 1]
                ca, cb = (0, int(co[-1])) if lp.whole else (int(co[p]), int(co[p + 1]))
                rp, c, v = _rows(Ho.R[l], ca, cb)
                assert np.array_equal(lp.R.rowptr, rp) and np.array_equal(lp.R.col, c)
                assert np.array_equal(bits(lp.R.val), bits(v))
                assert np.array_equal(np.where(lp.agg >= 0, lp.agg + ca, -1), Ho.agg[l][a:b])
    assert np.array_equal(bits(H.ainv), bits(Ho.ainv.T.reshape(-1)))
    return H


@pytest.mark.parametrize("kind,n,nparts,max_coarse", [
    ("poisson2d", 50, 1, 100), ("poisson3d", 18, 1, 60), ("aniso3d", 14, 1, 100),
    ("poisson3d", 18, 2, 60), ("poisson2d", 41, 3, 80), ("aniso3d", 13, 4, 120),
])
@pytest.mark.parametrize("agglomerate", [0, 32768, 400])
def test_host_setup_bit_exact(kind, n, nparts, max_coarse, agglomerate, built):
    H = check_against_oracle(kind, n, nparts, max_coarse, agglomerate)
    if nparts > 1:
        whole = [H.levels[l][0].whole for l in range(H.nlevels)]
        first = whole.index(True) if any(whole) else H.nlevels
        assert not any(whole[:first]) and all(whole[first:])
        if agglomerate == 0:
            assert first == H.nlevels and H.rep_level == H.nlevels - 1
        else:
            assert H.rep_level == first or (first == H.nlevels and H.rep_level == H.nlevels - 1)


def test_exchange_plans_are_consistent(built):
    """Every ghost a part receives from q is exactly what q sends to it (PRange invariant)."""
    be = pa.SequentialBackend(3)
    A, offs, _ = pa.generate_problem(be, "poisson3d", 12)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=40))
    for l in range(H.nlevels):
        for attr, nxt in (("planA", False), ("planR", False), ("planP", True)):
            for p in range(3):
                P = getattr(H.levels[l][p], attr)
                if P is None:
                    continue
                o = (H.rep_offsets if nxt and l + 1 == H.rep_level else H.offsets(l + 1 if nxt else l))
                for k, q in enumerate(P.nbrs):
                    Q = getattr(H.levels[l][q], attr)
                    mine = P.ghost_ids[(P.ghost_ids >= o[q]) & (P.ghost_ids < o[q + 1])]
                    assert len(mine) == P.recv_counts[k]
                    assert np.array_equal(Q._send.get(p, np.zeros(0, np.int64)) + o[q], mine)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "*.npz"))), ids=os.path.basename)
def test_host_setup_golden(path, built):
    g = np.load(path, allow_pickle=False)
    nparts = int(g["nparts"])
    be = pa.SequentialBackend(nparts)
    A, offs, _ = pa.generate_problem(be, str(g["kind"]), int(g["n"]))
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=int(g["max_coarse"]), agglomerate=0))
    assert H.nlevels == int(g["nlevels"])
    for l in range(H.nlevels):
        tags = ["A"] + (["P", "R"] if l < H.nlevels - 1 else [])
        for tag in tags:
            parts = [getattr(H.levels[l][p], tag) for p in range(nparts)]
            base = np.cumsum([0] + [int(m.rowptr[-1]) for m in parts[:-1]])
            rp = np.concatenate([parts[0].rowptr] + [m.rowptr[1:] + base[i] for i, m in enumerate(parts) if i > 0])
            col = np.concatenate([m.col for m in parts]).astype(np.int64)
            val = np.concatenate([m.val for m in parts])
            assert sha(rp) == str(g[f"{tag}{l}_rowptr_sha"]), (tag, l)
            assert sha(col) == str(g[f"{tag}{l}_col_sha"]), (tag, l)
            assert sha(val) == str(g[f"{tag}{l}_val_sha"]), (tag, l)
    assert sha(H.ainv.reshape(int(np.sqrt(len(H.ainv))), -1).T.copy()) == str(g["ainv_sha"])


def test_hcsr_roundtrip_and_rows(built):
    rng = np.random.default_rng(2)
    rp = np.array([0, 3, 3, 7, 8], np.int64)
    col = rng.integers(0, 50, 8).astype(np.int32)
    val = rng.standard_normal(8)
    M = HC.HCSR.from_arrays(rp, col, val, 50)
    assert M.nrows == 4 and M.nnz == 8 and M.ncols == 50
    assert np.array_equal(M.rowptr, rp) and np.array_equal(M.col, col) and np.array_equal(M.val, val)
    r, c, v = M.rows([2, 0])
    assert r.tolist() == [0, 4, 7] and np.array_equal(c, np.concatenate([col[3:7], col[0:3]]))
    with pytest.raises(OverflowError):
        HC.HCSR.from_arrays(rp, np.full(8, 2**31 - 1, np.int64), val, 2**31)


def test_dense_coarse_solve_refuses_oversized_levels(built):
    """A coarsest level above PAMG_MAX_DENSE_COARSE rows is refused before any n^2 allocation
    (a max_levels cap can leave 10^5+ rows there: 10^11 doubles)."""
    import ctypes

    import pytest
    from parallel_amg_amd import hcsr as HC
    from parallel_amg_amd._lib import PamgError, call
    n = HC.MAX_DENSE_COARSE + 1
    idx = np.arange(n, dtype=np.int64)
    M = HC.HCSR.from_arrays(np.arange(n + 1, dtype=np.int64), idx.astype(np.int32), np.full(n, 2.0), n)
    with pytest.raises(PamgError, match="dense-solve limit"):
        HC.cholinv(M)
    one = (ctypes.c_double * 1)()
    with pytest.raises(PamgError, match="dense-solve limit"):  # the C entry point checks too
        call("pamg_setup_cholinv", M.handle, one)
