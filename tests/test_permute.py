"""bench --permute: the seeded symmetric permutation Q A Q^T (hierarchy.permute_problem)
against scipy's row/column indexing, on CPU."""
import numpy as np
import pytest
import scipy.sparse as sp

import parallel_amg_amd as pa
from parallel_amg_amd.hierarchy import permutation


@pytest.mark.parametrize("kind,n", [("poisson3d", 7), ("elastic3d", 4), ("poisson2d", 20)])
def test_permute_problem_matches_scipy(kind, n):
    be = pa.SequentialBackend(1)
    A, _offs, xs = pa.generate_problem(be, kind, n)
    P, xp = pa.permute_problem(A, xs, 11)
    M = sp.csr_matrix((A[0].val, A[0].col, A[0].rowptr), shape=(A[0].nrows, A[0].ncols))
    Q = sp.csr_matrix((P[0].val, P[0].col, P[0].rowptr), shape=(P[0].nrows, P[0].ncols))
    perm = permutation(M.shape[0], 11)
    R = M[perm][:, perm].tocsr()
    R.sort_indices()
    assert np.array_equal(Q.indptr, R.indptr) and np.array_equal(Q.indices, R.indices)
    assert np.array_equal(Q.data, R.data)
    # the permuted system has the permuted solution: Q (x*[perm]) == (A x*)[perm]
    np.testing.assert_allclose(Q @ xp[0], (M @ xs[0])[perm], rtol=1e-13, atol=1e-13)
    with pytest.raises(ValueError):
        pa.permute_problem({0: A[0], 1: A[0]}, xs, 1)
