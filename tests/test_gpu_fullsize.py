"""Full-size checks (BASELINE.json sizes) through properties that need no oracle run:

* 512^3 fine matrix (the metric's workload): A*1 on the GPU equals the exact integer row sums
  6 - (#neighbours) for all 134M rows; A*x* matches the host's SPEC §S3 row sums on sampled rows;
  one Jacobi sweep gives the same bits in all four upload layouts.
* 256^3 hierarchy: a V-cycle is linear and scaling by 2 is exact in binary floating point, so
  V(2x, 2b) must equal 2 V(x, b) bit for bit; two runs are bit-identical (determinism); the
  residual falls every cycle; graph replay equals eager launches.
"""
import numpy as np
import pytest

import parallel_amg_amd as pa
from parallel_amg_amd.partitioned import PSparseMatrix, PVector, axpby, mul
from parallel_amg_amd.solver import AMGSolver

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def test_fine_512_rowsums(ctx):
    n = 512
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", n)
    A0 = A[0]
    assert A0.nnz == 937_951_232
    D = PSparseMatrix(ctx, A0)
    N = A0.nrows
    ones = PVector(ctx, N, 0, np.ones(N))
    y = PVector(ctx, N)
    mul(y, D, ones)
    got = y.own_values()
    cnt = np.diff(A0.rowptr)                 # 1 + #neighbours
    assert np.array_equal(got, 6.0 - (cnt - 1).astype(np.float64))
    # A x* on sampled rows against the SPEC row sum computed on the host
    x = PVector(ctx, N, 0, xs[0])
    mul(y, D, x)
    got = y.own_values()
    rng = np.random.default_rng(1)
    for i in rng.integers(0, N, 2000):
        s = 0.0
        for k in range(A0.rowptr[i], A0.rowptr[i + 1]):
            s = s + A0.val[k] * xs[0][A0.col[k]]
        assert got[i] == s


def test_fine_512_layouts_agree(ctx):
    """The metric's level-0 Jacobi gives the same bits in every upload layout at full size:
    the symmetric diagonal-class layout with its row-class dictionary (default) and without it,
    tile-major slots + 4-bit column dictionary
    (+ x staging), variant 1 with the dictionary, 24-bit columns + 8-bit row lengths, plain
    32-bit CSR tiles, the tile path's default (8-bit per-tile value dictionaries) and the sliced-ELL
    layout."""
    import ctypes
    from parallel_amg_amd._lib import call, layout_of
    from parallel_amg_amd.partitioned import jacobi
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 512)
    A0 = A[0]
    N = A0.nrows
    rng = np.random.default_rng(3)
    xh = rng.standard_normal(N)
    bh = rng.standard_normal(N)
    b = PVector(ctx, N, 0, bh)
    layouts = [{}, {"sym_vd": 0}, {"sym_dia": 0, "value_dict": 0, "ell": 0},
               {"sym_dia": 0, "tile_major": 0, "value_dict": 0, "ell": 0},
               {"sym_dia": 0, "tile_major": 0, "col_dict": 0, "value_dict": 0, "ell": 0},
               {"sym_dia": 0, "tile_major": 0, "col_dict": 0, "col24": 0, "row_len8": 0, "value_dict": 0, "ell": 0},
               {"sym_dia": 0, "ell": 0},  # the tile path's default: 8-bit per-tile value dictionaries in tile-major slots
               {"sym_dia": 0}]  # the sliced-ELL layout (what a square operator without the stencil layout takes)
    keys = ("sym_dia", "tile_major", "col_dict", "col24", "row_len8", "value_dict", "sym_vd", "ell")
    old = []
    for k in keys:
        v = ctypes.c_int64()
        call("pamg_get_option", k.encode(), ctypes.byref(v))
        old.append(v.value)
    ref, seen = None, []
    try:
        for lay in layouts:
            for k, v in zip(keys, old):
                call("pamg_set_option", k.encode(), lay.get(k, v))
            D = PSparseMatrix(ctx, A0)
            seen.append(layout_of(D))
            x, t = PVector(ctx, N, 0, xh), PVector(ctx, N)
            jacobi(x, D, b, t, 2.0 / 3.0, 1)
            got = bits(x.own_values())
            del D, x, t
            if ref is None:
                ref = got
            else:
                assert np.array_equal(got, ref), lay
    finally:
        for k, v in zip(keys, old):
            call("pamg_set_option", k.encode(), v)
    assert seen[0]["sym"] and seen[0]["cd_offsets"] == 3 and seen[0]["sym_vd"]
    assert seen[1]["sym"] and not seen[1]["sym_vd"]
    seen = seen[1:]
    assert seen[1]["tm"] and seen[1]["cd"] == 4 and seen[1]["x_stage"] and not seen[2]["tm"] and seen[2]["cd"] == 4
    assert seen[3]["cd"] == 0 and seen[3]["c24"] and not seen[4]["c24"]
    assert seen[5]["tm"] and seen[5]["tm_vd"]
    assert seen[6]["ell"] and not seen[5]["ell"]


@pytest.fixture(scope="module")
def h256(ctx):
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 256)
    H = pa.build_hierarchy(be, A, offs)
    S = AMGSolver(ctx, H)
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    return S, b


def test_vcycle_scaling_by_two_is_exact(ctx, h256):
    S, b = h256
    n = S.A[0].nrows
    rng = np.random.default_rng(7)
    x0 = rng.standard_normal(n)
    x1 = PVector(ctx, n, 0, x0)
    S.vcycle(x1, b, 2)
    b2 = PVector(ctx, n)
    axpby(2.0, b, 0.0, b2)                   # exact: 2*b + 0*b2
    x2 = PVector(ctx, n, 0, 2.0 * x0)
    S.vcycle(x2, b2, 2)
    assert np.array_equal(bits(x2.own_values()), bits(2.0 * x1.own_values()))


def test_vcycle_deterministic_and_converging(ctx, h256):
    S, b = h256
    out = []
    for graph in (True, False, True):
        S.set_graph(graph)
        x = S.new_vector()
        hist = S.vcycle(x, b, 4, res_hist=True)
        out.append((x.own_values(), hist))
        assert np.all(np.diff(hist) < 0)
    S.set_graph(True)
    assert np.array_equal(bits(out[0][0]), bits(out[1][0]))
    assert np.array_equal(bits(out[0][0]), bits(out[2][0]))
    np.testing.assert_array_equal(out[0][1], out[2][1])


def _stencil27(m, seed=3):
    """27-point operator on an m^3 grid (random off-diagonal values, dominant diagonal) in CSR
    with columns ascending: ~26 nonzeros per row, built vectorised."""
    N = m ** 3
    idx = np.arange(N, dtype=np.int64)
    z, y, x = idx // (m * m), (idx // m) % m, idx % m
    cols, valid = [], []
    for dz in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dx in (-1, 0, 1):
                ok = (z + dz >= 0) & (z + dz < m) & (y + dy >= 0) & (y + dy < m) & (x + dx >= 0) & (x + dx < m)
                cols.append(idx + dz * m * m + dy * m + dx)
                valid.append(ok)
    C = np.stack(cols, axis=1)
    V = np.stack(valid, axis=1)
    del cols, valid
    rowptr = np.zeros(N + 1, np.int64)
    np.cumsum(V.sum(axis=1), out=rowptr[1:])
    col = C[V]
    del C
    rng = np.random.default_rng(seed)
    val = rng.standard_normal(col.size)
    rows = np.repeat(idx, np.diff(rowptr))
    val[col == rows] = 40.0
    return rowptr, col, val, N


def test_long_row_operator_full_size(ctx):
    """A square operator of >= 64 M nonzeros at ~26 per row (the 512^3 A1 regime): the upload
    takes 2048-nonzero tiles (long_tiles_min; 4096 before round 3's A/B) and SpMV / Jacobi give
    the oracle's bits, the same bits as the 1024-nonzero tiles."""
    import ctypes
    from oracle import oracle as O
    from parallel_amg_amd._lib import call, layout_of
    from parallel_amg_amd.hcsr import HCSR
    from parallel_amg_amd.partitioned import jacobi
    rowptr, col, val, N = _stencil27(140)
    assert col.size >= 64 << 20 and col.size >= 24 * N
    M = HCSR.from_arrays(rowptr, col.astype(np.int32), val, N)
    rng = np.random.default_rng(9)
    xh, bh = rng.standard_normal(N), rng.standard_normal(N)
    Mo = O.CSR(rowptr, col, val, N)
    ref = O.spmv(Mo, xh)
    refj = O.jacobi(Mo, xh, bh, 0.6)
    outs = []
    for ltm in (24, 48):
        old = ctypes.c_int64()
        call("pamg_get_option", b"long_tiles_min", ctypes.byref(old))
        try:
            call("pamg_set_option", b"long_tiles_min", ltm)
            D = PSparseMatrix(ctx, M)
        finally:
            call("pamg_set_option", b"long_tiles_min", old.value)
        assert layout_of(D)["tile_nnz"] == (2048 if ltm == 24 else 1024)
        x, b, y, t = PVector(ctx, N, 0, xh), PVector(ctx, N, 0, bh), PVector(ctx, N), PVector(ctx, N)
        mul(y, D, x)
        assert np.array_equal(bits(y.own_values()), bits(ref))
        jacobi(x, D, b, t, 0.6, 1)
        assert np.array_equal(bits(x.own_values()), bits(refj))
        outs.append(x.own_values())
        del D
    assert np.array_equal(bits(outs[0]), bits(outs[1]))
