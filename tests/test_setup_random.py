"""Property tests (hypothesis) of the product setup against the oracle on random sparse SPD
matrices: irregular patterns, weak and strong couplings (strength threshold §S4.2), isolated
rows (aggregate -1), 1..4 parts with random offsets — every level's A, P, R and aggregates
bit-exact, with and without agglomeration."""
import numpy as np
import pytest
import scipy.sparse as sp
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import parallel_amg_amd as pa
from oracle import oracle as O
from parallel_amg_amd.hcsr import HCSR


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def random_spd(seed, n, density, weak_frac, isolated_frac):
    rng = np.random.default_rng(seed)
    M = sp.random(n, n, density=density, random_state=rng, format="coo")
    vals = -np.abs(rng.standard_normal(M.nnz))
    weak = rng.random(M.nnz) < weak_frac
    vals[weak] *= 1e-4                       # below theta = 0.02: not strong
    M = sp.coo_matrix((vals, (M.row, M.col)), shape=(n, n)).tocsr()
    M = (M + M.T).tolil()
    iso = rng.random(n) < isolated_frac       # rows with no off-diagonal couplings at all
    for i in np.nonzero(iso)[0]:
        M[i, :] = 0
        M[:, i] = 0
    M = M.tocsr()
    M.setdiag(0)
    M.eliminate_zeros()
    d = np.asarray(abs(M).sum(axis=1)).ravel() + 1.0 + rng.random(n)
    M = (M + sp.diags(d)).tocsr()
    M.sort_indices()
    return M


@settings(max_examples=80, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(seed=st.integers(0, 2**31 - 1), n=st.integers(30, 700), density=st.floats(0.002, 0.05),
       weak=st.floats(0.0, 0.6), iso=st.floats(0.0, 0.1), nparts=st.integers(1, 4),
       agglomerate=st.sampled_from([0, 200, 32768]))
def test_random_spd_setup_matches_oracle(built, seed, n, density, weak, iso, nparts, agglomerate):
    M = random_spd(seed, n, density, weak, iso)
    rng = np.random.default_rng(seed ^ 0x5A5A)
    cuts = np.sort(rng.choice(np.arange(1, n), size=nparts - 1, replace=False)) if nparts > 1 else []
    offs = np.array([0, *cuts, n], np.int64)
    be = pa.SequentialBackend(nparts)
    A = {p: HCSR.from_arrays(M.indptr[offs[p]:offs[p + 1] + 1] - M.indptr[offs[p]],
                             M.indices[M.indptr[offs[p]]:M.indptr[offs[p + 1]]].astype(np.int32),
                             M.data[M.indptr[offs[p]]:M.indptr[offs[p + 1]]], n) for p in range(nparts)}
    prm = pa.SAParams(max_coarse=20, agglomerate=agglomerate)
    H = pa.build_hierarchy(be, A, offs, prm)
    Ao = O.CSR(M.indptr.astype(np.int64), M.indices.astype(np.int64), M.data.copy(), n)
    Ho = O.setup(Ao, offsets=offs, max_coarse=20, agglomerate=agglomerate)
    assert H.nlevels == Ho.nlevels
    for l in range(H.nlevels):
        assert np.array_equal(H.offsets(l), Ho.offsets[l])
        full = np.concatenate([m.val for m in H.part_rows(l)])
        assert np.array_equal(bits(full), bits(Ho.A[l].val))
        if l < H.nlevels - 1:
            Pv = np.concatenate([m.val for m in H.part_rows(l, "P")])
            assert np.array_equal(bits(Pv), bits(Ho.P[l].val))
            # aggregate ids: local per part, numbered after the parts before (the next level's
            # row offsets as this aggregation produced them); a whole level is one part
            lv = H.levels[l]
            if lv[0].whole:
                agg = lv[0].agg
            else:
                co = H.rep_offsets if l + 1 == H.rep_level else Ho.offsets[l + 1]
                agg = np.concatenate([np.where(lv[p].agg >= 0, lv[p].agg + co[p], -1) for p in range(nparts)])
            assert np.array_equal(agg, Ho.agg[l])
    assert np.array_equal(bits(H.ainv), bits(Ho.ainv.T.reshape(-1)))
