"""The roofline's algorithmic byte model on the metric's workload, CPU only.

bench.py's `roofline.achieved` divides AMGSolver.csr_bytes by the measured launch time; these
are the per-launch figures DESIGN.md quotes for the 512^3 fine level (937,951,232 nonzeros,
134,217,728 rows), from the SPEC §S2 nonzero formula.
"""
from types import SimpleNamespace

from parallel_amg_amd.solver import AMGSolver


def _nnz_grid(n, d):
    # SPEC §S2: nnz = N (1 + 2d) - sum_k 2 N / n_k on an n^d grid, Dirichlet rows eliminated
    N = n ** d
    return N * (1 + 2 * d) - d * 2 * N // n


def test_nnz_formula_matches_survey():
    assert _nnz_grid(256, 2) == 326_656
    assert _nnz_grid(128, 3) == 14_581_760
    assert _nnz_grid(256, 3) == 117_047_296
    assert _nnz_grid(512, 3) == 937_951_232


def test_level0_bytes_per_launch_512():
    n = 512 ** 3
    A0 = SimpleNamespace(nnz=_nnz_grid(512, 3), nrows=n, n_own_cols=n, n_ghost=0)
    # Jacobi / residual: 12 B/nnz + 4 B/row pointer (+1) + x once + y + b
    assert AMGSolver.csr_bytes(A0, 1) == 15_013_511_172
    # SpMV: without b
    assert AMGSolver.csr_bytes(A0, 0) == 15_013_511_172 - 8 * n
    # the format model starts from the uploaded layout's matrix stream instead
    A0.stream_bytes = 11_342_721_568 - 3 * 8 * n
    assert AMGSolver.rowsum_bytes(A0, 1) == 11_342_721_568


def test_per_part_bytes_scale_with_the_slab():
    # 8 slabs of 64 planes: each part reads its own rows and two ghost planes of x
    n, parts = 512 ** 3, 8
    rows = n // parts
    plane = 512 * 512
    full = AMGSolver.csr_bytes(SimpleNamespace(nnz=_nnz_grid(512, 3), nrows=n, n_own_cols=n, n_ghost=0), 0)
    mid = AMGSolver.csr_bytes(SimpleNamespace(nnz=rows * 7 - 4 * 512 * 64 * 2, nrows=rows,
                                              n_own_cols=rows, n_ghost=2 * plane), 0)
    assert parts * mid > full  # ghosts are re-read by both neighbours
    assert abs(parts * mid - full) / full < 0.01


def test_chain_bytes_per_launch_512():
    """The pipelined chain's algorithmic bytes (bench.py roofline for k_sym_zc<3>): the matrix
    once, in0 and b, and the outputs it stores — the pre-smoothed iterate and the residual
    (chain_store_x 0, the default), plus the post-smoothed iterate with chain_store_x 1."""
    n = 512 ** 3
    A0 = SimpleNamespace(nnz=_nnz_grid(512, 3), nrows=n, n_own_cols=n, n_ghost=0)
    two = AMGSolver.csr_bytes(A0, 2)
    three = AMGSolver.csr_bytes(A0, 3)
    assert two == 12 * A0.nnz + 36 * n + 4 == 16_087_252_996
    assert three - two == 8 * n
