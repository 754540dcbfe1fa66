"""GPU parity: libpamg's HIP kernels (through the C-ABI) against the CPU oracle (SPEC.md).

Bit-exact for every row-sum op and for whole V-cycles (SPEC §S3 fixes the summation order);
norms/dots within 1e-12 relative (tree reductions)."""
import numpy as np
import pytest

import parallel_amg_amd as pa
from oracle import oracle as O
from parallel_amg_amd._lib import PamgError
from parallel_amg_amd.hcsr import HCSR
from parallel_amg_amd.partitioned import PSparseMatrix, PVector, axpby, dot, jacobi, mul, norm, residual
from parallel_amg_amd.solver import AMGSolver

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


@pytest.fixture
def novd():
    """Value dictionaries off (the library default is on): for tests that assert which column
    layout an upload picks on matrices with few distinct values."""
    import ctypes
    from parallel_amg_amd._lib import call
    v = ctypes.c_int64()
    call("pamg_get_option", b"value_dict", ctypes.byref(v))
    call("pamg_set_option", b"value_dict", 0)
    yield
    call("pamg_set_option", b"value_dict", v.value)


def random_csr(rng, lengths, ncols, square=False, palette=None):
    rows, cols, vals = [0], [], []
    for i, m in enumerate(lengths):
        m = min(max(m, 1) if square else m, ncols)
        c = rng.choice(ncols, size=m, replace=False)
        if square and m > 0 and i not in c:
            c[0] = i
        c = np.sort(c)
        v = rng.standard_normal(m) if palette is None else rng.choice(palette, m)
        if square and m > 0:
            v[c == i] = 4.0 + abs(v[c == i]) + m
        cols.append(c)
        vals.append(v)
        rows.append(rows[-1] + m)
    rp = np.asarray(rows, np.int64)
    col = np.concatenate(cols).astype(np.int64) if cols else np.zeros(0, np.int64)
    val = np.concatenate(vals) if vals else np.zeros(0)
    return O.CSR(rp, col, val, ncols)


def upload(ctx, M: O.CSR):
    h = HCSR.from_arrays(M.rowptr, M.col.astype(np.int32), M.val, M.ncols)
    return PSparseMatrix(ctx, h), h


LENGTHS = {
    "stencil7": [7] * 3000,
    "ragged": [0, 1, 7, 27, 73, 0, 500, 3, 2049, 64, 1, 0] * 40,
    "long": [5000, 1, 2047, 2048, 2049, 0, 9000],
    "budget_edge": [1021, 1022, 1023, 1024, 1, 2045, 2046, 2047, 2048, 3, 4093, 4094, 4095, 4096, 2, 511] * 3,
    "one_row": [13],
    "empty_rows": [0] * 100,
    # short rows on average (8-bit row lengths in use) with the longest row at the limit...
    "len8_edge": ([255, 254] + [1, 0, 3, 7] * 10) * 8,
    # ... and one past it (32-bit row pointers)
    "len8_over": ([256] + [2] * 40) * 4,
}

# (tile_nnz, tile_order, col24, value_dict, long_tiles, row_len8, col_dict, tile_major): every
# layout the upload can produce and the kernel that runs it (kernels.hip launch_tile):
TILE_CONFIGS = [
    (1024, 1, 0, 0, 1, 0, 0, 0, 0),  # k_rows_tile2, 32-bit columns + row pointers
    (2048, 1, 0, 0, 1, 0, 0, 0, 0),
    (4096, 0, 0, 0, 0, 0, 0, 0, 0),  #   natural tile order, 4096-nonzero tiles everywhere
    (1024, 1, 1, 0, 1, 0, 0, 0, 0),  # k_rows_tile2 <C24>
    (1024, 1, 1, 0, 1, 1, 0, 0, 0),  # k_rows_tile2 <C24, RL8>
    (1024, 1, 1, 1, 1, 0, 0, 0, 0),  # k_rows_tile2 <C24, VD> (opt-in value dictionaries)
    (2048, 1, 1, 1, 1, 1, 0, 0, 0),
    (1024, 1, 1, 0, 1, 1, 1, 0, 0),  # k_rows_tile2 <RL8, CD 4/8>
    (1024, 1, 0, 0, 1, 0, 1, 0, 0),  #   column dictionaries without the 24-bit stream
    (1024, 1, 1, 0, 1, 1, 1, 1, 1),  # default: k_rows_sym on symmetric stencils, k_rows_tm on
    #   dictionary / slot-filling sets
    (1024, 1, 1, 0, 1, 1, 1, 1, 0),  # the same without the symmetric layout
    (1024, 0, 1, 0, 0, 1, 1, 1, 0),  #   natural order, no long tiles
    (2048, 1, 1, 0, 1, 1, 1, 1, 0),
    (4096, 1, 1, 0, 1, 1, 1, 1, 0),
    (1024, 1, 1, 0, 1, 1, 1, 2, 0),  # k_rows_tm on every eligible set (24-bit tile-major too)
    (1024, 1, 1, 0, 1, 0, 0, 2, 0),  #   24-bit tile-major only
    (4096, 1, 1, 0, 1, 1, 1, 2, 0),
]
OPT_KEYS = ("tile_nnz", "tile_order", "col24", "value_dict", "long_tiles", "row_len8", "col_dict", "tile_major",
            "sym_dia")


@pytest.fixture(params=TILE_CONFIGS,
                ids=lambda c: "t{}_ord{}_c24{}_vd{}_lt{}_rl{}_cd{}_tm{}_sym{}".format(*c))
def tile_cfg(request, built):
    import ctypes
    from parallel_amg_amd._lib import call
    old = []
    for k in OPT_KEYS:
        v = ctypes.c_int64()
        call("pamg_get_option", k.encode(), ctypes.byref(v))
        old.append(v.value)
    for k, v in zip(OPT_KEYS, request.param):
        call("pamg_set_option", k.encode(), v)
    yield request.param
    for k, v in zip(OPT_KEYS, old):
        call("pamg_set_option", k.encode(), v)


# value palettes: None = all distinct (no tile fits a value dictionary); a few repeated
# values incl. +-0.0 (every tile fits one); 17 values (tiles straddle the 16-value limit)
PALETTES = {"distinct": None, "few": [-1.0, 2.5, 0.0, -0.0, 6.0, 1e-300],
            "seventeen": [float(v) for v in range(-8, 9)]}


@pytest.mark.parametrize("palette", list(PALETTES))
@pytest.mark.parametrize("case", list(LENGTHS))
def test_spmv_residual_bit_exact(ctx, case, palette, tile_cfg):
    rng = np.random.default_rng(11)
    lengths = LENGTHS[case]
    ncols = max(max(lengths) + 1, len(lengths) + 7)
    M = random_csr(rng, lengths, ncols, palette=PALETTES[palette])
    A, _h = upload(ctx, M)
    xh = rng.standard_normal(ncols)
    bh = rng.standard_normal(len(lengths))
    x = PVector(ctx, ncols, 0, xh)
    y = PVector(ctx, len(lengths))
    mul(y, A, x)
    ref = O.spmv(M, xh)
    assert np.array_equal(bits(y.own_values()), bits(ref))
    b = PVector(ctx, len(lengths), 0, bh)
    r = PVector(ctx, len(lengths))
    residual(r, A, x, b)
    assert np.array_equal(bits(r.own_values()), bits(O.residual(M, xh, bh)))
    # prolongate-add: y <- y + A x (the op the V-cycle applies with P)
    import ctypes
    from parallel_amg_amd._lib import call
    ms = ctypes.c_double()
    yy = PVector(ctx, len(lengths), 0, bh)
    call("pamg_bench_rowop", ctx.handle, A.handle, 3, x.handle, None, yy.handle, 0.0, 1, ctypes.byref(ms))
    # two launches (warm-up + 1 timed): bh + s + s, in that order
    assert np.array_equal(bits(yy.own_values()), bits((bh + ref) + ref))


@pytest.mark.parametrize("palette", ["distinct", "few"])
@pytest.mark.parametrize("case", ["stencil7", "ragged", "long", "budget_edge", "one_row"])
def test_jacobi_bit_exact(ctx, case, palette, tile_cfg):
    rng = np.random.default_rng(5)
    lengths = LENGTHS[case]
    n = max(max(lengths) + 1, len(lengths))
    lengths = lengths + [3] * (n - len(lengths))
    M = random_csr(rng, lengths, n, square=True, palette=PALETTES[palette])
    A, _h = upload(ctx, M)
    xh, bh = rng.standard_normal(n), rng.standard_normal(n)
    x, b, t = PVector(ctx, n, 0, xh), PVector(ctx, n, 0, bh), PVector(ctx, n)
    jacobi(x, A, b, t, 0.7, 3)
    ref = xh
    for _ in range(3):
        ref = O.jacobi(M, ref, bh, 0.7)
    assert np.array_equal(bits(x.own_values()), bits(ref))


def offset_csr(rng, n, offsets, lengths, palette=None, diag_from_palette=False):
    """Square matrix whose row i holds the diagonal plus columns i + o for o drawn from
    `offsets` (those inside [0, n)): at most len(offsets) + 1 distinct row-relative offsets,
    the layout the column dictionaries (col_dict) compress. The diagonal is 4 + row length +
    |value| (dominant), or with diag_from_palette a palette value too, so that every value of
    the matrix is one of the palette's."""
    offsets = np.asarray(offsets, np.int64)
    rows, cols, vals = [0], [], []
    for i in range(n):
        m = lengths[i % len(lengths)]
        cand = i + offsets
        cand = cand[(cand >= 0) & (cand < n) & (cand != i)]
        c = np.sort(np.concatenate([[i], rng.choice(cand, size=min(max(m - 1, 0), len(cand)), replace=False)]))
        v = rng.standard_normal(len(c)) if palette is None else rng.choice(palette, len(c))
        if not diag_from_palette:
            v[c == i] = 4.0 + len(c) + abs(v[c == i])
        cols.append(c)
        vals.append(v)
        rows.append(rows[-1] + len(c))
    return O.CSR(np.asarray(rows, np.int64), np.concatenate(cols).astype(np.int64), np.concatenate(vals), n)


# (name, number of distinct off-diagonal offsets, row lengths): 4-bit tables (<= 16 offsets
# with the diagonal), 8-bit (17..256), no dictionary (> 256); ragged rows up to the 255 limit
COLDICT_CASES = [("stencil7", None, [7]), ("d15", 15, [1, 16, 5, 9]), ("d16", 16, [17, 2]),
                 ("d200", 200, [30, 1, 7, 255, 3]), ("d255", 255, [64, 9]), ("d256", 256, [40, 2]),
                 ("ragged4", 12, [1, 2, 13, 1, 1, 9, 4]), ("rows256", 3, [1, 1, 1, 4, 1, 1, 1, 2])]


@pytest.mark.parametrize("name,ndist,lengths", COLDICT_CASES, ids=[c[0] for c in COLDICT_CASES])
@pytest.mark.parametrize("tnnz", [1024, 4096])
def test_column_dictionary_bit_exact(ctx, novd, name, ndist, lengths, tnnz):
    """col_dict: columns rebuilt as row + table[index] give the very bits of the oracle for
    SpMV, residual, prolongate-add and Jacobi (in-tile diagonal and stored diagonal), and the
    layout engages exactly when the matrix has <= 256 distinct row-relative offsets."""
    import ctypes
    from parallel_amg_amd._lib import call, layout_of
    rng = np.random.default_rng(len(name) * 7 + tnnz)
    n = 4000
    if ndist is None:
        offs = [-289, -17, -1, 1, 17, 289]
    else:
        offs = rng.choice(np.arange(-n // 2, n // 2), size=ndist + 1, replace=False)
        offs = offs[offs != 0][:ndist]
    M = offset_csr(rng, n, offs, lengths)
    rows = np.repeat(np.arange(n), np.diff(M.rowptr))
    distinct = len(np.unique(M.col - rows))
    dist_anc = len(np.unique(M.col - np.repeat(M.col[np.minimum(M.rowptr[:-1], max(M.nnz - 1, 0))], np.diff(M.rowptr))))
    keys = ("col_dict", "tile_nnz", "tile_major", "col_dict_anchor", "col_dict_tile")
    old = []
    for k in keys:
        v = ctypes.c_int64()
        call("pamg_get_option", k.encode(), ctypes.byref(v))
        old.append(v.value)
    try:
        call("pamg_set_option", b"col_dict_anchor", 1)
        call("pamg_set_option", b"col_dict_tile", 0)  # set-wide tables only (per-tile: below)
        call("pamg_set_option", b"tile_nnz", tnnz)
        call("pamg_set_option", b"col_dict", 0)
        call("pamg_set_option", b"tile_major", 0)
        plain = upload(ctx, M)[0].stream_bytes
        for tm in (0, 2):
            call("pamg_set_option", b"col_dict", 1)
            call("pamg_set_option", b"tile_major", tm)
            A, _h = upload(ctx, M)
            if not tm:
                assert (A.stream_bytes < plain) == (distinct <= 256), (A.stream_bytes, plain, distinct)
            lay = layout_of(A)
            assert lay["tm"] == bool(tm)
            # row-relative where <= 256 offsets; else (tile-major only) anchored where <= 256
            nd = distinct if distinct <= 256 else (dist_anc if tm and dist_anc <= 256 else 0)
            assert lay["anchored"] == (distinct > 256 and nd > 0), (lay, distinct, dist_anc)
            assert lay["cd"] == (4 if 0 < nd <= 16 else 8 if nd else 0), (lay, distinct, dist_anc)
            assert lay["cd_offsets"] == nd
            xh, bh = rng.standard_normal(n), rng.standard_normal(n)
            x, b = PVector(ctx, n, 0, xh), PVector(ctx, n, 0, bh)
            y = PVector(ctx, n)
            mul(y, A, x)
            ref = O.spmv(M, xh)
            assert np.array_equal(bits(y.own_values()), bits(ref))
            r = PVector(ctx, n)
            residual(r, A, x, b)
            assert np.array_equal(bits(r.own_values()), bits(O.residual(M, xh, bh)))
            ms = ctypes.c_double()
            yy = PVector(ctx, n, 0, bh)
            call("pamg_bench_rowop", ctx.handle, A.handle, 3, x.handle, None, yy.handle, 0.0, 1, ctypes.byref(ms))
            assert np.array_equal(bits(yy.own_values()), bits((bh + ref) + ref))
            t = PVector(ctx, n)
            jacobi(x, A, b, t, 0.7, 3)
            rj = xh
            for _ in range(3):
                rj = O.jacobi(M, rj, bh, 0.7)
            assert np.array_equal(bits(x.own_values()), bits(rj))
    finally:
        for k, v in zip(keys, old):
            call("pamg_set_option", k.encode(), v)


def test_blas1(ctx):
    rng = np.random.default_rng(3)
    n = 100_003
    xh, yh = rng.standard_normal(n), rng.standard_normal(n)
    x, y = PVector(ctx, n, 0, xh), PVector(ctx, n, 0, yh)
    assert dot(x, y) == pytest.approx(float(np.dot(xh, yh)), rel=1e-12)
    assert norm(x) == pytest.approx(float(np.linalg.norm(xh)), rel=1e-12)
    axpby(2.5, x, -0.5, y)
    assert np.array_equal(bits(y.own_values()), bits(2.5 * xh + (-0.5) * yh))


def test_shape_errors_raise(ctx):
    M = O.generate("poisson2d", 8, 8, 1)
    A, _h = upload(ctx, M)
    x = PVector(ctx, 63)
    y = PVector(ctx, 64)
    with pytest.raises(PamgError):
        mul(y, A, x)


CONFIGS = [("poisson2d", 64, 300), ("poisson3d", 24, 100), ("aniso3d", 20, 300), ("poisson3d", 12, 1000),
           ("elastic3d", 10, 200)]


@pytest.mark.parametrize("kind,n,max_coarse", CONFIGS)
def test_vcycle_bit_exact(ctx, kind, n, max_coarse, tile_cfg):
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=max_coarse))
    S = AMGSolver(ctx, H)
    xst = PVector(ctx, S.A[0].nrows, 0, xs[0])
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], xst)
    Ao = O.generate(kind, *O.grid_shape(kind, n))
    bo = O.spmv(Ao, O.xstar(Ao.nrows))
    assert np.array_equal(bits(b.own_values()), bits(bo))
    Ho = O.setup(Ao, max_coarse=max_coarse)
    assert Ho.nlevels == H.nlevels
    x = S.new_vector()
    hist = S.vcycle(x, b, 6, res_hist=True)
    xo, ho = Ho.solve(bo, 6, res_hist=True)
    assert np.array_equal(bits(x.own_values()), bits(xo))
    np.testing.assert_allclose(hist, ho, rtol=1e-12)
    assert hist[-1] < hist[0]


@pytest.mark.parametrize("kind,n,max_coarse", [("poisson3d", 24, 100), ("aniso3d", 20, 300), ("poisson2d", 96, 200)])
def test_pcg_matches_oracle(ctx, kind, n, max_coarse):
    """SPEC §S8: same iteration count, iterates within 1e-8 (dots are reductions)."""
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=max_coarse))
    S = AMGSolver(ctx, H)
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    Ao = O.generate(kind, *O.grid_shape(kind, n))
    bo = O.spmv(Ao, O.xstar(Ao.nrows))
    Ho = O.setup(Ao, max_coarse=max_coarse)
    xo, ko, ho = Ho.pcg(bo, 1e-10, 60)
    x = S.new_vector()
    k, h = S.pcg(x, b, 1e-10, 60)
    assert k == ko and k < 30
    np.testing.assert_allclose(h, ho, rtol=1e-6)
    xg = x.own_values()
    assert np.linalg.norm(xg - xo) <= 1e-8 * np.linalg.norm(xo)
    assert np.linalg.norm(xg - xs[0]) <= 1e-8 * np.linalg.norm(xs[0])


def test_pcg_equals_primitive_sequence(ctx):
    """pamg_pcg (fused x / r update + r.r in one kernel) gives the bits of the same CG written
    with the separate C-ABI primitives (mul, dot, axpby, V-cycle from zero)."""
    from parallel_amg_amd.partitioned import copy
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 20)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100))
    S = AMGSolver(ctx, H)
    A0 = S.A[0]
    b = PVector(ctx, A0.nrows)
    mul(b, A0, PVector(ctx, A0.nrows, 0, xs[0]))
    x1 = S.new_vector()
    k1, h1 = S.pcg(x1, b, 1e-9, 40)

    x = S.new_vector()
    r, z, p, q = S.new_vector(), S.new_vector(), S.new_vector(), S.new_vector()
    residual(r, A0, x, b)
    nr0 = np.sqrt(dot(r, r))
    hist = [nr0]
    z.fill(0.0)
    S.vcycle(z, r, 1)
    copy(p, z)
    rz = dot(r, z)
    k = 0
    while k < 40:
        k += 1
        mul(q, A0, p)
        alpha = rz / dot(p, q)
        axpby(alpha, p, 1.0, x)
        axpby(-alpha, q, 1.0, r)
        hist.append(np.sqrt(dot(r, r)))
        if hist[-1] <= 1e-9 * nr0:
            break
        z.fill(0.0)
        S.vcycle(z, r, 1)
        rz_new = dot(r, z)
        beta = rz_new / rz
        rz = rz_new
        axpby(1.0, z, beta, p)
    assert k == k1
    assert np.array_equal(bits(np.asarray(hist)), bits(h1))
    assert np.array_equal(bits(x.own_values()), bits(x1.own_values()))


def test_graph_equals_eager(ctx):
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 20)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100))
    S = AMGSolver(ctx, H)
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    out = []
    for g in (True, False):
        S.set_graph(g)
        x = S.new_vector()
        S.vcycle(x, b, 5)
        out.append(x.own_values())
    assert np.array_equal(bits(out[0]), bits(out[1]))
    prof = S.profile(S.new_vector(), b, 2)
    assert prof.shape == (H.nlevels, 6) and prof[0, 4] > 0


@pytest.mark.parametrize("nu1,nu2", [(2, 1), (1, 2), (2, 2), (3, 1), (3, 4)])
def test_vcycle_sweeps_bit_exact(ctx, nu1, nu2):
    """SPEC §S6 V(nu1, nu2): pre/post sweep ping-pong on the device vs the oracle's loops."""
    kind, n, mc = "poisson3d", 16, 100
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=mc))
    S = AMGSolver(ctx, H)
    S.set_sweeps(nu1, nu2)
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    Ao = O.generate(kind, n, n, n)
    bo = O.spmv(Ao, O.xstar(Ao.nrows))
    Ho = O.setup(Ao, max_coarse=mc)
    Ho.set_sweeps(nu1, nu2)
    xo, ho = Ho.solve(bo, 4, res_hist=True)
    for graph in (True, False):
        S.set_graph(graph)
        x = S.new_vector()
        hist = S.vcycle(x, b, 4, res_hist=True)
        assert np.array_equal(bits(x.own_values()), bits(xo))
        np.testing.assert_allclose(hist, ho, rtol=1e-12)
    # more smoothing per cycle converges faster per cycle than V(1,1)
    Ho.set_sweeps(1, 1)
    _, h11 = Ho.solve(bo, 4, res_hist=True)
    assert ho[-1] < h11[-1]
    with pytest.raises(PamgError):
        S.set_sweeps(0, 1)


def test_stream_bytes_layout(ctx, novd):
    """pamg_mat_stream_bytes: 12 B/nnz + row pointers + 16-B tile descriptors in the 32-bit
    layout; 3-B columns (+ a 4-B base per tile) in the 24-bit one; 1 B per row instead of a
    4-B row pointer with 8-bit row lengths (roofline byte model)."""
    from parallel_amg_amd._lib import call
    M = O.generate("poisson3d", 16, 16, 16)
    n, nnz = M.nrows, len(M.col)

    def stream_bytes(**opts):
        for k, v in opts.items():
            call("pamg_set_option", k.encode(), v)
        try:
            A, _h = upload(ctx, M)
            return A.stream_bytes
        finally:
            for k in opts:
                call("pamg_set_option", k.encode(), 0 if k == "value_dict" else 1)

    from parallel_amg_amd._lib import layout_of
    # the symmetric diagonal-class layout with its row-class dictionary (default): a 1-B class id
    # per row + 27 classes of (diagonal, 3 upper values, mask); without it: 1-B mask + diagonal +
    # 3 upper values per row
    A, _h = upload(ctx, M)
    assert layout_of(A)["sym"] and layout_of(A)["sym_vd"] and A.stream_bytes == n + 27 * (32 + 4) + 4
    A, _h = _with_options({"sym_vd": 0}, lambda: upload(ctx, M))
    assert layout_of(A)["sym"] and A.stream_bytes == n * (1 + 8 + 24) + 4
    call("pamg_set_option", b"sym_dia", 0)
    try:
        _stream_bytes_tiles(ctx, M, stream_bytes)
    finally:
        call("pamg_set_option", b"sym_dia", 1)


def _stream_bytes_tiles(ctx, M, stream_bytes):
    from parallel_amg_amd._lib import layout_of
    n, nnz = M.nrows, len(M.col)
    got0 = stream_bytes(col24=0, row_len8=0, col_dict=0, tile_major=0)
    nt, rem = divmod(got0 - 12 * nnz - 4 * (n + 1), 16)
    assert rem == 0 and nt > 0
    assert stream_bytes(col24=1, row_len8=0, col_dict=0, tile_major=0) == 11 * nnz + 4 * (n + 1) + 20 * nt
    assert stream_bytes(col24=1, row_len8=1, col_dict=0, tile_major=0) == 11 * nnz + n + 4 + 20 * nt
    # 2 distinct values: a square operator keeps its column dictionary in tile-major slots and
    # takes 8-bit value dictionaries there (a byte per slot + a 4-entry table per tile instead
    # of 8 B per slot); 4-bit value dictionaries are for rectangular operators
    A1, _h1 = _with_options({"value_dict": 1}, lambda: upload(ctx, M))
    l1 = layout_of(A1)
    assert l1["tm"] and l1["tm_vd"] and not l1["vd"]
    tn = l1["tile_nnz"]
    assert stream_bytes() - A1.stream_bytes == l1["tiles"] * (8 * tn - (tn + 8 * 4))
    # column dictionary: 7 offsets -> 4-bit indices + the 28-B table, 8-bit row lengths, no
    # per-tile base
    assert stream_bytes(tile_major=0) == 8 * nnz + (nnz + 1) // 2 + 4 * 7 + n + 4 + 16 * nt
    # tile-major (default): whole padded slots of 1024 values + 512 B of indices + the
    # row-length slot per tile
    A, _h = upload(ctx, M)
    lay = layout_of(A)
    assert lay["tm"] and lay["cd"] == 4 and 0 < lay["tm_rs"] <= 256 and lay["tm_rs"] % 4 == 0
    assert A.stream_bytes == nt * (lay["tm_rs"] + 8 * 1024 + 512 + 16) + 4 * 7 + 4


def anchored_csr(rng, nrows, ncols, nshape, maxlen):
    """A restriction-shaped matrix: row i reads anchor_i + a subset (always holding 0) of one
    set of nshape offsets; anchors are unrelated to the row index (sorted, random gaps), so
    no row-relative dictionary fits but an anchored one does."""
    shape = np.concatenate([[0], np.sort(rng.choice(np.arange(1, 3000), nshape - 1, replace=False))])
    anchors = np.sort(rng.integers(0, ncols - 3001, nrows))
    rows, cols = [0], []
    for i in range(nrows):
        m = int(rng.integers(1, min(nshape, maxlen) + 1))
        sub = np.concatenate([[0], rng.choice(shape[1:], m - 1, replace=False)]) if m > 1 else np.array([0])
        cols.append(anchors[i] + np.sort(sub))
        rows.append(rows[-1] + m)
    col = np.concatenate(cols).astype(np.int64)
    return O.CSR(np.asarray(rows, np.int64), col, rng.standard_normal(len(col)), ncols)


@pytest.mark.parametrize("nshape,maxlen,tnnz", [(12, 12, 1024), (75, 40, 1024), (75, 255, 1024),
                                                (256, 60, 4096), (257, 60, 1024)])
def test_anchored_dictionary_bit_exact(ctx, novd, nshape, maxlen, tnnz):
    """Anchored column dictionaries (column = the row's first column + table[index], anchors in
    the tile-major slots; the layout of the level-0 restriction): SpMV, residual and
    prolongate-add give the oracle's bits; 257 offsets fall back to 24-bit columns."""
    import ctypes
    from parallel_amg_amd._lib import call, layout_of
    rng = np.random.default_rng(nshape * 31 + maxlen)
    nr, nc = 3000, 60000
    M = anchored_csr(rng, nr, nc, nshape, maxlen)
    old = ctypes.c_int64()
    call("pamg_get_option", b"tile_nnz", ctypes.byref(old))
    try:
        call("pamg_set_option", b"tile_nnz", tnnz)
        A, _h = upload(ctx, M)
    finally:
        call("pamg_set_option", b"tile_nnz", old.value)
    lay = layout_of(A)
    used = len(np.unique(M.col - np.repeat(M.col[M.rowptr[:-1]], np.diff(M.rowptr))))
    if used <= 256:  # one set-wide anchored table in tile-major slots
        assert lay["anchored"] and lay["tm"] and not lay["per_tile"]
        assert lay["cd"] == (4 if used <= 16 else 8), (lay, used)
    else:            # too many for one table: per-tile tables (if they pay) or 24-bit columns
        assert lay["per_tile"] or lay["cd"] == 0, lay
    xh, bh = rng.standard_normal(nc), rng.standard_normal(nr)
    x, b = PVector(ctx, nc, 0, xh), PVector(ctx, nr, 0, bh)
    y = PVector(ctx, nr)
    mul(y, A, x)
    ref = O.spmv(M, xh)
    assert np.array_equal(bits(y.own_values()), bits(ref))
    r = PVector(ctx, nr)
    residual(r, A, x, b)
    assert np.array_equal(bits(r.own_values()), bits(O.residual(M, xh, bh)))
    ms = ctypes.c_double()
    yy = PVector(ctx, nr, 0, bh)
    call("pamg_bench_rowop", ctx.handle, A.handle, 3, x.handle, None, yy.handle, 0.0, 1, ctypes.byref(ms))
    assert np.array_equal(bits(yy.own_values()), bits((bh + ref) + ref))



def _layout_ops_match_oracle(ctx, M, rng):
    """SpMV / residual / prolongate-add (and Jacobi on square M) of the uploaded M against
    the oracle, bit for bit."""
    import ctypes
    from parallel_amg_amd._lib import call
    A, _h = upload(ctx, M)
    nr, nc = M.nrows, M.ncols
    xh, bh = rng.standard_normal(nc), rng.standard_normal(nr)
    x, b = PVector(ctx, nc, 0, xh), PVector(ctx, nr, 0, bh)
    y = PVector(ctx, nr)
    mul(y, A, x)
    ref = O.spmv(M, xh)
    assert np.array_equal(bits(y.own_values()), bits(ref))
    r = PVector(ctx, nr)
    residual(r, A, x, b)
    assert np.array_equal(bits(r.own_values()), bits(O.residual(M, xh, bh)))
    ms = ctypes.c_double()
    yy = PVector(ctx, nr, 0, bh)
    call("pamg_bench_rowop", ctx.handle, A.handle, 3, x.handle, None, yy.handle, 0.0, 1, ctypes.byref(ms))
    assert np.array_equal(bits(yy.own_values()), bits((bh + ref) + ref))
    if nr == nc:
        t = PVector(ctx, nr)
        jacobi(x, A, b, t, 0.7, 2)
        rj = O.jacobi(M, O.jacobi(M, xh, bh, 0.7), bh, 0.7)
        assert np.array_equal(bits(x.own_values()), bits(rj))
    return A


def drift_csr(rng, n, ncols, anchored, nset=12, every=200, step=37):
    """Rows whose columns are (row | a slowly drifting anchor) + a subset of an offset set that
    shifts by `step` every `every` rows: far more than 256 offsets in the matrix, a few dozen
    per tile — the shape of the coarse operators (row-relative) and prolongators (anchored)."""
    base = np.sort(rng.choice(np.arange(-300, 300), nset, replace=False))
    rows, cols = [0], []
    for i in range(n):
        g = (i // every) % 30
        m = int(rng.integers(1, nset + 1))
        if anchored:  # 30 scaled copies of the set around a drifting anchor
            c = np.unique(3 * i + int(rng.integers(0, 4)) + (g + 1) * rng.choice(base, m, replace=False))
        else:         # 30 shifted copies of the set, relative to the row
            c = np.unique(i + g * step - 15 * step + rng.choice(base, m, replace=False))
        c = c[(c >= 0) & (c < ncols)]  # dropped, not clipped: no new offsets at the edges
        if not anchored:
            c = np.unique(np.concatenate([c, [i]]))  # square: keep the diagonal
        cols.append(c)
        rows.append(rows[-1] + len(c))
    col = np.concatenate(cols).astype(np.int64)
    val = rng.standard_normal(len(col))
    if not anchored:  # diagonally dominant rows for Jacobi
        rp = np.asarray(rows)
        for i in range(n):
            seg = slice(rp[i], rp[i + 1])
            val[seg][col[seg] == i] = 4.0 + (rp[i + 1] - rp[i])
    return O.CSR(np.asarray(rows, np.int64), col, val, ncols)


@pytest.mark.parametrize("anchored,tnnz,tm", [(False, 1024, 0), (False, 4096, 0), (True, 1024, 0), (True, 2048, 0),
                                             (False, 1024, 1), (False, 4096, 1), (True, 1024, 1)])
def test_per_tile_dictionaries_bit_exact(ctx, novd, anchored, tnnz, tm):
    """col_dict_tile: no table fits the whole matrix (> 256 offsets) but every tile's fits —
    per-tile row-relative tables (coarse-operator shape) or per-tile anchored ones with 16-bit
    anchors (prolongator shape) in the descriptor kernel; SpMV / residual / prolongate-add (and
    Jacobi for the square case) give the oracle's bits; tm_tile_dicts moves the row-relative
    ones into tile-major slots (the anchored ones stay in the descriptor kernel)."""
    import ctypes
    from parallel_amg_amd._lib import call, layout_of
    rng = np.random.default_rng(tnnz + anchored)
    n = 6000
    M = drift_csr(rng, n, 3 * n if anchored else n, anchored, nset=6 if anchored else 12)
    old = ctypes.c_int64()
    call("pamg_get_option", b"tile_nnz", ctypes.byref(old))
    try:
        call("pamg_set_option", b"tile_nnz", tnnz)
        D = _with_options({"tm_tile_dicts": tm}, lambda: _layout_ops_match_oracle(ctx, M, rng))
    finally:
        call("pamg_set_option", b"tile_nnz", old.value)
    lay = layout_of(D)
    assert lay["per_tile"] and lay["anchored"] == anchored and lay["tm"] == (tm == 1 and not anchored), lay
    assert lay["cd"] in (4, 8) and lay["cd_offsets"] in (16, 32, 64, 128, 256), lay


def test_hierarchy_operators_any_dictionary_bit_exact(ctx):
    """The level-1 operator and the level-0 prolongator of a real hierarchy, in whatever column
    format the upload picks (per-tile tables at 512^3, 24-bit or set-wide tables at this size),
    give the oracle's bits."""
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 48)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100))
    rng = np.random.default_rng(5)
    for M in (H.levels[1][0].A, H.levels[0][0].P, H.levels[1][0].P):
        Mo = O.CSR(M.rowptr.copy(), M.col.astype(np.int64), M.val.copy(), M.ncols)
        _layout_ops_match_oracle(ctx, Mo, rng)


@pytest.mark.parametrize("name,ndist,lengths", [("d300", 300, [30, 1, 7, 64]), ("d2000", 2000, [9, 3, 40]),
                                                ("wide_ragged", 600, [1, 255, 2, 17])])
def test_per_tile_dictionaries_random(ctx, novd, name, ndist, lengths):
    """Random offset patterns too wide for one table: per-tile tables where they stream less
    than 24-bit columns (else 24-bit), bit-exact either way."""
    from parallel_amg_amd._lib import layout_of
    rng = np.random.default_rng(len(name))
    n = 5000
    offs = rng.choice(np.arange(-n // 2, n // 2), size=ndist + 1, replace=False)
    offs = offs[offs != 0][:ndist]
    M = offset_csr(rng, n, offs, lengths)
    D = _layout_ops_match_oracle(ctx, M, rng)
    lay = layout_of(D)
    assert lay["per_tile"] or lay["cd"] == 0, lay

def _with_options(opts, fn):
    import ctypes
    from parallel_amg_amd._lib import call
    old = {}
    for k in opts:
        v = ctypes.c_int64()
        call("pamg_get_option", k.encode(), ctypes.byref(v))
        old[k] = v.value
    try:
        for k, v in opts.items():
            call("pamg_set_option", k.encode(), v)
        return fn()
    finally:
        for k, v in old.items():
            call("pamg_set_option", k.encode(), v)


# x_stage cases (name -> matrix, x staged?): clustered row-relative offsets — the stencils
# (7-point: 5 runs; 27-point and elastic: 9), ragged rows, offsets past both ends of the
# vector; 13 runs (more than kXsMaxClusters) and a run too wide for the lanes fall back to
# gathers
def _xs_case(name):
    rng = np.random.default_rng(11)
    if name == "poisson3d_24":
        return O.generate("poisson3d", 24, 24, 24), True
    if name == "poisson2d_64":
        return O.generate("poisson2d", 64, 64, 1), True
    if name == "aniso3d_20":
        return O.generate("aniso3d", 20, 20, 20), True
    if name == "elastic3d_12":
        return O.generate("elastic3d", 12, 12, 12), True
    if name == "ragged":
        offs = [-1500, -201, -200, -199, -1, 1, 199, 200, 201, 1500]
        return offset_csr(rng, 4000, offs, [1, 11, 6, 9, 12, 9, 8]), True  # <= 171 rows per tile: 5 runs fit
    if name == "clusters13":
        offs = [k * 400 + d for k in range(-6, 7) for d in (-1, 0, 1) if k * 400 + d != 0]
        return offset_csr(rng, 6000, offs, [20, 3, 39]), False
    assert name == "wide_run"  # one run 0..220 wide: rows + 220 > 256 lanes
    return offset_csr(rng, 3000, [-700, -1, 1, 60, 100, 140, 180, 220], [8, 2, 5]), False


@pytest.mark.parametrize("name", ["poisson3d_24", "poisson2d_64", "aniso3d_20", "elastic3d_12", "ragged",
                                  "clusters13", "wide_run"])
@pytest.mark.parametrize("x_stage", [1, 0])
def test_x_stage_bit_exact(ctx, novd, name, x_stage):
    """x_stage: row-relative dictionary tiles read x from LDS copies of the runs their offset
    clusters cover (loaded coalesced at entry) instead of gathering it; SpMV / residual /
    prolongate-add / Jacobi (diagonal = offset 0's entry) give the oracle's bits either way,
    and the layout stages x exactly where the runs fit."""
    from parallel_amg_amd._lib import layout_of
    M, staged = _xs_case(name)
    rng = np.random.default_rng(len(name))
    D = _with_options({"x_stage": x_stage, "tile_major": 2, "sym_dia": 0},
                      lambda: _layout_ops_match_oracle(ctx, M, rng))
    lay = layout_of(D)
    assert lay["tm"] and lay["cd"] in (4, 8) and not lay["anchored"], lay
    assert lay["x_stage"] == (staged and x_stage == 1), lay


def test_restriction_takes_anchored_dictionary(ctx, novd):
    """The level-0 restriction of the 7-point Poisson hierarchy (5x5x5 neighbourhoods of the
    aggregate roots) is uploaded with an anchored 8-bit dictionary in tile-major slots."""
    from parallel_amg_amd._lib import layout_of
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 24)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100), device=ctx)
    S = AMGSolver(ctx, H)
    lay = layout_of(S.R[0])
    assert lay["anchored"] and lay["tm"] and lay["cd"] == 8 and lay["cd_offsets"] <= 256, lay


@pytest.mark.parametrize("tnnz", [1024, 2048, 4096])
def test_restriction_anchored_tiles_bit_exact(ctx, tnnz):
    """The level-0 restriction (anchored 8-bit dictionary, 8-bit value dictionary, tile-major
    slots) on 1024-, 2048- (the 512^3 R0's budget since round 4) and 4096-nonzero tiles: SpMV,
    residual and prolongate-add bit-exact with the oracle."""
    from parallel_amg_amd._lib import layout_of
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 40)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100))
    R = H.levels[0][0].R
    M = O.CSR(R.rowptr.copy(), R.col.astype(np.int64), R.val.copy(), R.ncols)
    with _with_option("tile_nnz", tnnz):
        D = _layout_ops_match_oracle(ctx, M, np.random.default_rng(tnnz))
    lay = layout_of(D)
    assert lay["anchored"] and lay["tm"] and lay["tile_nnz"] == tnnz, lay


@pytest.mark.parametrize("seed,n,density,weak,iso", [(1, 3000, 0.003, 0.3, 0.02), (2, 5000, 0.001, 0.0, 0.0),
                                                     (3, 2500, 0.01, 0.6, 0.05), (4, 4000, 0.002, 0.2, 0.1)])
def test_vcycle_random_spd_bit_exact(ctx, seed, n, density, weak, iso):
    """Irregular matrices (random patterns, weak couplings, isolated rows) through the whole
    device path — GPU setup products, ragged tiles on every level, V-cycles — vs the oracle."""
    from test_setup_random import random_spd
    M = random_spd(seed, n, density, weak, iso)
    A = {0: HCSR.from_arrays(M.indptr, M.indices.astype(np.int32), M.data, n)}
    be = pa.SequentialBackend(1)
    H = pa.build_hierarchy(be, A, np.array([0, n], np.int64), pa.SAParams(max_coarse=60), device=ctx)
    S = AMGSolver(ctx, H)
    rng = np.random.default_rng(seed)
    bh = rng.standard_normal(n)
    b = PVector(ctx, n, 0, bh)
    Ao = O.CSR(M.indptr.astype(np.int64), M.indices.astype(np.int64), M.data.copy(), n)
    Ho = O.setup(Ao, max_coarse=60)
    assert Ho.nlevels == H.nlevels
    xo, ho = Ho.solve(bh, 5, res_hist=True)
    x = S.new_vector()
    hist = S.vcycle(x, b, 5, res_hist=True)
    assert np.array_equal(bits(x.own_values()), bits(xo))
    np.testing.assert_allclose(hist, ho, rtol=1e-12)


@pytest.mark.parametrize("kind,n,seed", [("poisson3d", 14, 1), ("elastic3d", 6, 2), ("aniso3d", 12, 3)])
def test_vcycle_permuted_bit_exact(ctx, kind, n, seed):
    """Randomly renumbered grid operators (bench --permute, the Flan_1565 proxy): the column
    dictionaries and the banded tile order no longer apply, so the fine level runs the
    24/32-bit column layouts; setup on the GPU and V-cycles stay bit-exact with the oracle run
    on the same permuted matrix."""
    from parallel_amg_amd._lib import layout_of
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, kind, n)
    A, xs = pa.permute_problem(A, xs, seed)
    M = A[0]
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100), device=ctx)
    S = AMGSolver(ctx, H)
    assert layout_of(S.A[0])["cd"] == 0  # no row-relative dictionary survives the shuffle
    b = PVector(ctx, M.nrows)
    mul(b, S.A[0], PVector(ctx, M.nrows, 0, xs[0]))
    Ao = O.CSR(M.rowptr.copy(), M.col.astype(np.int64), M.val.copy(), M.ncols)
    bo = O.spmv(Ao, xs[0])
    assert np.array_equal(bits(b.own_values()), bits(bo))
    Ho = O.setup(Ao, max_coarse=100)
    assert Ho.nlevels == H.nlevels
    xo, ho = Ho.solve(bo, 5, res_hist=True)
    x = S.new_vector()
    hist = S.vcycle(x, b, 5, res_hist=True)
    assert np.array_equal(bits(x.own_values()), bits(xo))
    np.testing.assert_allclose(hist, ho, rtol=1e-12)


def test_default_solver_fine_operator_is_caller_numbered(ctx):
    """with the default reorder="auto", a scattered problem of >= 4096 rows gets a
    locality-permuted level 0 inside the hierarchy, yet S.A[0] stays the caller's operator:
    b = S.A[0] x* through the default constructor equals the oracle's A x* on the caller's
    numbering, and the V-cycle from that b keeps the oracle's bits."""
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 20)
    A, xs = pa.permute_problem(A, xs, 5)
    M = A[0]
    assert M.nrows >= 4096
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100), device=ctx)
    S = AMGSolver(ctx, H)                      # default constructor (reorder="auto")
    assert 0 in S.reordered
    b = PVector(ctx, M.nrows)
    mul(b, S.A[0], PVector(ctx, M.nrows, 0, xs[0]))
    Ao = O.CSR(M.rowptr.copy(), M.col.astype(np.int64), M.val.copy(), M.ncols)
    bo = O.spmv(Ao, xs[0])
    assert np.array_equal(bits(b.own_values()), bits(bo))
    Ho = O.setup(Ao, max_coarse=100)
    xo = Ho.solve(bo, 4)
    x = S.new_vector()
    S.vcycle(x, b, 4)
    assert np.array_equal(bits(x.own_values()), bits(xo))


# ---------------------------------------------------------------- locality permutation (reorder)
def test_upload_perm_rows_and_columns_bit_exact(ctx):
    """pamg_mat_upload_perm: device row i = row perm[i], device column k = column perm[k], each
    row in its storage order — SpMV / residual / Jacobi of the permuted vectors are the
    unpermuted results, moved."""
    rng = np.random.default_rng(7)
    M = random_csr(rng, [7, 0, 3, 27, 1, 9] * 400, 2400, square=True)
    n = M.nrows
    h = HCSR.from_arrays(M.rowptr, M.col.astype(np.int32), M.val, M.ncols)
    perm = rng.permutation(n).astype(np.int64)
    A = PSparseMatrix(ctx, h, row_perm=perm, col_perm=perm)
    xh = rng.standard_normal(n)
    bh = rng.standard_normal(n)
    x, b, y = PVector(ctx, n, 0, xh[perm]), PVector(ctx, n, 0, bh[perm]), PVector(ctx, n)
    mul(y, A, x)
    assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)[perm]))
    residual(y, A, x, b)
    assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)[perm]))
    t = PVector(ctx, n)
    jacobi(x, A, b, t, 0.61, 2)
    xj = O.jacobi(M, O.jacobi(M, xh, bh, 0.61), bh, 0.61)
    assert np.array_equal(bits(x.own_values()), bits(xj[perm]))


@pytest.mark.parametrize("kind,n,seed", [("poisson3d", 20, 1), ("elastic3d", 14, 2), ("aniso3d", 18, 3),
                                         ("poisson2d", 96, 4)])
@pytest.mark.parametrize("reorder", ["auto", "on"])
def test_reorder_vcycle_bit_exact_caller_numbering(ctx, kind, n, seed, reorder):
    """a randomly renumbered problem (the Flan_1565 proxy) set up in the
    caller's numbering; the device layout carries a per-level locality permutation (reverse
    Cuthill-McKee of each A_l, P_l / R_l through the fine and coarse permutations, rows in
    storage order). The V-cycle takes and returns the caller's vectors and is bit-exact with the
    oracle run on the caller's (unpermuted) numbering; PCG matches the oracle's iterations."""
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, kind, n)
    A, xs = pa.permute_problem(A, xs, seed)
    M = A[0]
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100), device=ctx)
    S = AMGSolver(ctx, H, reorder=reorder)
    assert 0 in S.reordered, (S.reordered, S.span)   # the shuffled fine level is always permuted
    if reorder == "on":
        assert S.reordered == list(range(H.nlevels - 1))
    b = PVector(ctx, M.nrows)
    mul(b, S.fine_operator(), PVector(ctx, M.nrows, 0, xs[0]))
    Ao = O.CSR(M.rowptr.copy(), M.col.astype(np.int64), M.val.copy(), M.ncols)
    bo = O.spmv(Ao, xs[0])
    assert np.array_equal(bits(b.own_values()), bits(bo))
    Ho = O.setup(Ao, max_coarse=100)
    assert Ho.nlevels == H.nlevels
    xo, ho = Ho.solve(bo, 5, res_hist=True)
    x = S.new_vector()
    hist = S.vcycle(x, b, 5, res_hist=True)
    assert np.array_equal(bits(x.own_values()), bits(xo))
    np.testing.assert_allclose(hist, ho, rtol=1e-12)
    # stationary cycles without history (graph replay) continue from the same caller vector
    x2 = S.new_vector()
    S.vcycle(x2, b, 3)
    S.vcycle(x2, b, 2)
    assert np.array_equal(bits(x2.own_values()), bits(xo))
    xpo, ko, hpo = Ho.pcg(bo, 1e-10, 80)
    xp = S.new_vector()
    k, hp = S.pcg(xp, b, 1e-10, 80)
    assert k == ko
    np.testing.assert_allclose(hp, hpo, rtol=1e-6)
    assert np.linalg.norm(xp.own_values() - xpo) <= 1e-8 * np.linalg.norm(xpo)


@pytest.mark.parametrize("kind,n", [("poisson3d", 64), ("aniso3d", 48), ("elastic3d", 16)])
def test_aggregate_order_vcycle_bit_exact(ctx, kind, n):
    """reorder="agg" (VERDICT r4 next-4): levels 1 .. L-2 uploaded in the order of their coarse
    aggregates (each level-(l+1) aggregate's nodes contiguous), level 0 in its grid layout: the
    V-cycles (graph-replayed, pipelined) and the residual history are the oracle's bits."""
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100), device=ctx)
    S = AMGSolver(ctx, H, reorder="agg")
    assert S.reordered == list(range(1, H.nlevels - 1)), S.reordered
    M = A[0]
    b = PVector(ctx, M.nrows)
    mul(b, S.fine_operator(), PVector(ctx, M.nrows, 0, xs[0]))
    Ao = O.CSR(M.rowptr.copy(), M.col.astype(np.int64), M.val.copy(), M.ncols)
    bo = O.spmv(Ao, xs[0])
    Ho = O.setup(Ao, max_coarse=100)
    xo, ho = Ho.solve(bo, 5, res_hist=True)
    x = S.new_vector()
    hist = S.vcycle(x, b, 5, res_hist=True)
    assert np.array_equal(bits(x.own_values()), bits(xo))
    np.testing.assert_allclose(hist, ho, rtol=1e-12)
    x2 = S.new_vector()
    S.vcycle(x2, b, 3)
    S.vcycle(x2, b, 2)
    assert np.array_equal(bits(x2.own_values()), bits(xo))


def test_reorder_graph_equals_eager(ctx):
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 18)
    A, xs = pa.permute_problem(A, xs, 5)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100))
    S = AMGSolver(ctx, H, reorder="on")
    b = PVector(ctx, A[0].nrows, 0, xs[0])
    out = []
    for g in (True, False):
        S.set_graph(g)
        x = S.new_vector()
        S.vcycle(x, b, 4)
        out.append(x.own_values())
    assert np.array_equal(bits(out[0]), bits(out[1]))


# ---------------------------------------------------------------- symmetric diagonal-class layout
def _with_option(key, value):
    import contextlib
    import ctypes
    from parallel_amg_amd._lib import call

    @contextlib.contextmanager
    def cm():
        v = ctypes.c_int64()
        call("pamg_get_option", key.encode(), ctypes.byref(v))
        call("pamg_set_option", key.encode(), value)
        try:
            yield
        finally:
            call("pamg_set_option", key.encode(), v.value)
    return cm()


def _sym_grid(kind, n, seed=None):
    """The SPEC grid operator, or (seed) the same pattern with random symmetric values;
    "p9": the 2D 9-point pattern (9 offsets: 16-bit row masks)."""
    if kind == "p9":
        import scipy.sparse as sp
        t = sp.diags([1.0, 1.0, 1.0], [-1, 0, 1], shape=(n, n))
        P = sp.kron(t, t).tocsr()
        P.sort_indices()
        M = O.CSR(P.indptr.astype(np.int64), P.indices.astype(np.int64), P.data.copy(), n * n)
        seed = 9 if seed is None else seed
    else:
        M = O.generate(kind, *O.grid_shape(kind, n))
    if seed is None:
        return M
    import scipy.sparse as sp
    S = sp.csr_matrix((M.val, M.col, M.rowptr), shape=(M.nrows, M.ncols))
    R = S.copy()
    R.data = np.random.default_rng(seed).standard_normal(R.nnz)
    T = (R + R.T).tocsr()                       # bitwise symmetric: a + b == b + a
    T.setdiag(np.abs(T).sum(axis=1).A1 + 1.0)
    T.sort_indices()
    return O.CSR(T.indptr.astype(np.int64), T.indices.astype(np.int64), T.data.copy(), M.ncols)


@pytest.mark.parametrize("kind,n,seed", [("poisson3d", 24, None), ("poisson2d", 80, None), ("aniso3d", 20, None),
                                         ("poisson3d", 7, None), ("poisson3d", 19, 5), ("poisson2d", 33, 6),
                                         ("poisson3d", 40, None), ("p9", 45, None)])
@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("rows", [1, 2])
@pytest.mark.parametrize("vd", [0, 1])
def test_sym_dia_bit_exact(ctx, kind, n, seed, order, rows, vd):
    """k_rows_sym / k_rows_sym2 (diagonal + upper values per row, lower values read from their
    mirrors, no column stream; one or two rows per lane) and k_rows_symd (the row-class
    dictionary: a class id per row, values from the table; the SPEC grids, whose rows take a few
    tuples): SpMV, residual and Jacobi bit-exact with the oracle, natural and XCD-banded block
    orders, odd and even row counts."""
    from parallel_amg_amd._lib import layout_of
    M = _sym_grid(kind, n, seed)
    with _with_option("tile_order", order), _with_option("sym_rows", rows), _with_option("sym_vd", vd):
        A, _h = upload(ctx, M)
    lay = layout_of(A)
    assert lay["sym"] and lay["cd_offsets"] == {"poisson2d": 2, "p9": 4}.get(kind, 3), lay
    assert lay["sym_vd"] == bool(vd and rows == 2 and seed is None and kind != "p9"), lay
    rng = np.random.default_rng(n)
    xh, bh = rng.standard_normal(M.nrows), rng.standard_normal(M.nrows)
    x, b, y = PVector(ctx, M.nrows, 0, xh), PVector(ctx, M.nrows, 0, bh), PVector(ctx, M.nrows)
    mul(y, A, x)
    assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)))
    residual(y, A, x, b)
    assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)))
    t = PVector(ctx, M.nrows)
    jacobi(x, A, b, t, 0.57, 2)
    assert np.array_equal(bits(x.own_values()), bits(O.jacobi(M, O.jacobi(M, xh, bh, 0.57), bh, 0.57)))


@pytest.mark.parametrize("kind,n", [("poisson3d", 40), ("poisson2d", 80), ("aniso3d", 20), ("poisson3d", 7),
                                    ("poisson3d", 33)])
@pytest.mark.parametrize("order", [0, 1])
@pytest.mark.parametrize("ch", [1, 2, 4])
def test_symd_units_per_block_bit_exact(ctx, kind, n, order, ch):
    """k_rows_symd with CH 512-row units per block (symd_chunks; a unit count that CH does not
    divide leaves the last block's tail units idle): SpMV, residual, Jacobi bit-exact with the
    oracle."""
    from parallel_amg_amd._lib import layout_of
    M = _sym_grid(kind, n)
    with _with_option("tile_order", order), _with_option("sym_rows", 2), _with_option("sym_vd", 1):
        A, _h = upload(ctx, M)
    assert layout_of(A)["sym_vd"], layout_of(A)
    rng = np.random.default_rng(n + ch)
    xh, bh = rng.standard_normal(M.nrows), rng.standard_normal(M.nrows)
    x, b, y = PVector(ctx, M.nrows, 0, xh), PVector(ctx, M.nrows, 0, bh), PVector(ctx, M.nrows)
    with _with_option("symd_chunks", ch):
        mul(y, A, x)
        assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)))
        residual(y, A, x, b)
        assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)))
        t = PVector(ctx, M.nrows)
        jacobi(x, A, b, t, 0.57, 2)
    assert np.array_equal(bits(x.own_values()), bits(O.jacobi(M, O.jacobi(M, xh, bh, 0.57), bh, 0.57)))


@pytest.mark.parametrize("kind,shape", [("poisson3d", (64, 64, 64)), ("aniso3d", (64, 64, 64)),
                                        ("poisson3d", (128, 128, 128)), ("poisson3d", (64, 32, 40)),
                                        ("aniso3d", (192, 48, 7))])
@pytest.mark.parametrize("zch", [0, 1, 3, 8])
def test_sym_zm_bit_exact(ctx, kind, shape, zch):
    """k_sym_zm (the default one-sweep kernel of a whole one-part grid operator: marches along z,
    x and ids of planes k-1..k+1 in registers, plane k's in-plane neighbours through a
    double-buffered LDS plane; zm_chunks = z chunks per tile column, 0 = auto): SpMV, residual
    and two Jacobi sweeps bit-exact with the oracle, with chunk boundaries inside the grid (3, 8),
    one chunk per column (1) and the automatic split (0)."""
    from parallel_amg_amd._lib import layout_of
    M = O.generate(kind, *shape)
    Ad, _h = upload(ctx, M)
    lay = layout_of(Ad)
    assert lay["sym"] and lay["sym_vd"] and lay["jr_fused"], lay
    rng = np.random.default_rng(shape[2] + zch)
    xh, bh = rng.standard_normal(M.nrows), rng.standard_normal(M.nrows)
    x, b, y = PVector(ctx, M.nrows, 0, xh), PVector(ctx, M.nrows, 0, bh), PVector(ctx, M.nrows)
    with _with_option("zm_chunks", zch):
        mul(y, Ad, x)
        assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)))
        residual(y, Ad, x, b)
        assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)))
        t = PVector(ctx, M.nrows)
        jacobi(x, Ad, b, t, 0.57, 2)
    assert np.array_equal(bits(x.own_values()), bits(O.jacobi(M, O.jacobi(M, xh, bh, 0.57), bh, 0.57)))


def _ell_cases(kind):
    """Square operators for the sliced-ELL layout: a SPEC grid (7- / 5-point, ragged last group),
    a random SPD pattern, and a matrix with empty and single-entry rows."""
    if kind == "grid3d":
        return O.generate("poisson3d", 19, 19, 19)
    if kind == "grid2d":
        return O.generate("poisson2d", 150, 150, 1)
    if kind == "random":  # a 7-point pattern with values from a 24-entry palette, diagonal 10
        M = O.generate("poisson3d", 17, 17, 17)
        pal = np.random.default_rng(9).standard_normal(24)
        val = pal[np.random.default_rng(10).integers(0, 24, M.nnz)]
        rows = np.repeat(np.arange(M.nrows), np.diff(M.rowptr))
        val[M.col == rows] = 10.0
        return O.CSR(M.rowptr.copy(), M.col.copy(), val, M.ncols)
    n = 3000
    rng = np.random.default_rng(4)
    rows, cols, vals = [], [], []
    for i in range(n):
        if i % 97 == 0:
            continue  # an empty row
        k = 1 if i % 13 == 0 else int(rng.integers(2, 40))
        cs = np.unique(np.clip(i + rng.integers(-60, 60, k), 0, n - 1))
        rows += [i] * len(cs)
        cols += cs.tolist()
        vals += (rng.integers(1, 9, len(cs)) * 0.25).tolist()
    import scipy.sparse as sp
    T = sp.csr_matrix((vals, (rows, cols)), shape=(n, n))
    T.sort_indices()
    return O.CSR(T.indptr.astype(np.int64), T.indices.astype(np.int64), T.data.copy(), n)


@pytest.mark.parametrize("pair", [1, 0])
@pytest.mark.parametrize("kind", ["grid3d", "grid2d", "random", "ragged"])
def test_ell_bit_exact(ctx, kind, pair):
    """k_rows_ell (sliced ELL, per-group 8-bit offset and value dictionaries; round 5; round 6: one
    byte per nonzero naming an (offset, value) pair where a group has <= 256 of them, ell_pair):
    SpMV and residual bit-exact with the oracle, and two Jacobi sweeps where every row has its
    diagonal; the same results as the tile layouts on the same matrix."""
    from parallel_amg_amd._lib import layout_of
    M = _ell_cases(kind)
    with _with_option("ell_min_rows", 0), _with_option("sym_dia", 0), _with_option("ell_pair", pair):
        A, _h = upload(ctx, M)
        with _with_option("ell", 0):
            B, _h2 = upload(ctx, M)
    assert layout_of(A)["ell"] and not layout_of(B)["ell"], (layout_of(A), layout_of(B))
    if kind != "ragged":  # (the ragged rows' groups hold more than 256 pairs: separate tables)
        assert layout_of(A)["ell_pair"] == bool(pair), layout_of(A)
    rng = np.random.default_rng(3)
    xh, bh = rng.standard_normal(M.nrows), rng.standard_normal(M.nrows)
    for D in (A, B):
        x, b, y = PVector(ctx, M.nrows, 0, xh), PVector(ctx, M.nrows, 0, bh), PVector(ctx, M.nrows)
        mul(y, D, x)
        assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)))
        residual(y, D, x, b)
        assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)))
        if kind != "ragged":
            t = PVector(ctx, M.nrows)
            jacobi(x, D, b, t, 0.57, 2)
            assert np.array_equal(bits(x.own_values()), bits(O.jacobi(M, O.jacobi(M, xh, bh, 0.57), bh, 0.57)))


def test_ell_declines_what_does_not_fit(ctx):
    """More than 256 distinct values in a group (random values on a 7-point grid) or a row longer
    than 255: the tile layouts, still bit-exact."""
    from parallel_amg_amd._lib import layout_of
    M = O.generate("poisson3d", 12, 12, 12)
    M = O.CSR(M.rowptr.copy(), M.col.copy(), np.random.default_rng(1).standard_normal(M.nnz), M.ncols)
    n = 400
    dense = O.CSR(np.arange(0, n * n + 1, n, dtype=np.int64), np.tile(np.arange(n, dtype=np.int64), n),
                  np.ones(n * n), n)
    for Mx in (M, dense):
        with _with_option("ell_min_rows", 0), _with_option("sym_dia", 0):
            A, _h = upload(ctx, Mx)
        assert not layout_of(A)["ell"]
        xh = np.random.default_rng(2).standard_normal(Mx.nrows)
        x, y = PVector(ctx, Mx.nrows, 0, xh), PVector(ctx, Mx.nrows)
        mul(y, A, x)
        assert np.array_equal(bits(y.own_values()), bits(O.spmv(Mx, xh)))


def test_restriction_layouts_128(ctx):
    """The 128^3 hierarchy's restriction R_0 (263,552 coarse rows reading the 2.1M-entry fine vector,
    29 nonzeros per row): in the pattern-dictionary layout (58 aggregate-shape patterns; round 6), in
    the anchored sliced-ELL layout (rpat 0; offsets from each row's first column) and in tiles (rpat 0,
    ell_restrict 0): y = R r and b - R r bit-exact with the oracle in all three."""
    from parallel_amg_amd._lib import layout_of
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 128)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    R0 = H.levels[0][0].R
    D = PSparseMatrix(ctx, R0)
    lay = layout_of(D)
    assert lay["rpat"] and not lay["ell"] and lay["cd_offsets"] == 58, lay
    with _with_option("rpat", 0):
        D1 = PSparseMatrix(ctx, R0)
        with _with_option("ell_restrict", 0):
            D2 = PSparseMatrix(ctx, R0)
    assert layout_of(D1)["ell"] and not layout_of(D1)["rpat"]
    assert not layout_of(D2)["ell"] and not layout_of(D2)["rpat"]
    Mo = O.CSR(R0.rowptr.copy(), R0.col.astype(np.int64), R0.val.copy(), R0.ncols)
    rng = np.random.default_rng(12)
    rh, bh = rng.standard_normal(R0.ncols), rng.standard_normal(R0.nrows)
    r, b = PVector(ctx, R0.ncols, 0, rh), PVector(ctx, R0.nrows, 0, bh)
    for M in (D, D1, D2):
        y = PVector(ctx, R0.nrows)
        mul(y, M, r)
        assert np.array_equal(bits(y.own_values()), bits(O.spmv(Mo, rh)))
        residual(y, M, r, b)
        assert np.array_equal(bits(y.own_values()), bits(O.residual(Mo, rh, bh)))


def _rpat_case(npat, seed, ragged=True, nrows=6000):
    """A restriction-shaped matrix (nrows x 4 nrows + 64) whose rows copy npat patterns of
    (offset, value) pairs from their first column: lengths 1..40 (ragged) or 29, values from a
    12-entry palette, rows in runs of random length."""
    rng = np.random.default_rng(seed)
    pal = rng.standard_normal(12)
    pats = []
    for _ in range(npat):
        L = int(rng.integers(1, 41)) if ragged else 29
        offs = np.unique(np.concatenate([[0], rng.integers(1, 60, L - 1)]))
        pats.append((offs, pal[rng.integers(0, 12, len(offs))]))
    ncols = 4 * nrows + 64
    rows, cols, vals = [], [], []
    j = 0
    while j < nrows:
        p = int(rng.integers(0, npat))
        for _ in range(int(rng.integers(1, 90))):
            if j == nrows:
                break
            offs, v = pats[p]
            rows += [j] * len(offs)
            cols += (4 * j + offs).tolist()
            vals += v.tolist()
            j += 1
    import scipy.sparse as sp
    T = sp.csr_matrix((vals, (rows, cols)), shape=(nrows, ncols))
    T.sort_indices()
    return O.CSR(T.indptr.astype(np.int64), T.indices.astype(np.int64), T.data.copy(), ncols)


@pytest.mark.parametrize("npat,ragged", [(1, False), (7, True), (255, True)])
def test_rpat_bit_exact(ctx, npat, ragged):
    """k_rows_rpat (round 6): restrictions whose rows repeat 1, 7 or up to 255 patterns (ragged
    lengths 1..40): y = R r and b - R r bit-exact with the oracle, in this layout and in the tiles."""
    from parallel_amg_amd._lib import layout_of
    M = _rpat_case(npat, 20 + npat, ragged)
    A, _h = upload(ctx, M)
    with _with_option("rpat", 0):
        B, _h2 = upload(ctx, M)
    la = layout_of(A)
    assert la["rpat"] and la["cd_offsets"] <= npat and not layout_of(B)["rpat"], (la, layout_of(B))
    rng = np.random.default_rng(5)
    xh, bh = rng.standard_normal(M.ncols), rng.standard_normal(M.nrows)
    for D in (A, B):
        x, b, y = PVector(ctx, M.ncols, 0, xh), PVector(ctx, M.nrows, 0, bh), PVector(ctx, M.nrows)
        mul(y, D, x)
        assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)))
        residual(y, D, x, b)
        assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)))


def test_rpat_declines(ctx):
    """More than 255 patterns (a restriction whose every row has its own values) or a row longer
    than 128: ELL or the tiles, still bit-exact."""
    from parallel_amg_amd._lib import layout_of
    M = _rpat_case(7, 3)
    many = O.CSR(M.rowptr.copy(), M.col.copy(), np.random.default_rng(1).standard_normal(M.nnz), M.ncols)
    n, m = 50, 4000
    long_rows = O.CSR(np.arange(0, n * 200 + 1, 200, dtype=np.int64),
                      (np.arange(n)[:, None] * 40 + np.arange(200)[None, :]).ravel().astype(np.int64),
                      np.ones(n * 200), m)
    for Mx in (many, long_rows):
        A, _h = upload(ctx, Mx)
        assert not layout_of(A)["rpat"]
        xh = np.random.default_rng(2).standard_normal(Mx.ncols)
        x, y = PVector(ctx, Mx.ncols, 0, xh), PVector(ctx, Mx.nrows)
        mul(y, A, x)
        assert np.array_equal(bits(y.own_values()), bits(O.spmv(Mx, xh)))


def test_ell_level1_operator_128(ctx):
    """The level-1 operator of the 128^3 hierarchy (263,552 rows, 30 nonzeros per row: what the
    512^3 cycle runs per V-cycle twice) in the sliced-ELL layout: residual and Jacobi bit-exact with
    the oracle."""
    from parallel_amg_amd._lib import layout_of
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 128)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    M1 = H.levels[1][0].A
    D = PSparseMatrix(ctx, M1)
    assert layout_of(D)["ell"] and layout_of(D)["ell_pair"], layout_of(D)
    Mo = O.CSR(M1.rowptr.copy(), M1.col.astype(np.int64), M1.val.copy(), M1.ncols)
    rng = np.random.default_rng(8)
    xh, bh = rng.standard_normal(M1.nrows), rng.standard_normal(M1.nrows)
    x, b, y = PVector(ctx, M1.nrows, 0, xh), PVector(ctx, M1.nrows, 0, bh), PVector(ctx, M1.nrows)
    residual(y, D, x, b)
    assert np.array_equal(bits(y.own_values()), bits(O.residual(Mo, xh, bh)))
    t = PVector(ctx, M1.nrows)
    jacobi(x, D, b, t, 0.61, 1)
    assert np.array_equal(bits(x.own_values()), bits(O.jacobi(Mo, xh, bh, 0.61)))


def _cut_grid(n=64, cut=31):
    """poisson3d n^3 with the couplings between x = cut and x = cut + 1 removed (both directions):
    a tb_ok grid operator with absent entries INSIDE the grid (mask bits clear for in-grid
    neighbours), so the row-class kernels' maskless sums (zc_rows) meet +0.0 table values."""
    import scipy.sparse as sp
    M = O.generate("poisson3d", n, n, n)
    S = sp.csr_matrix((M.val, M.col, M.rowptr), shape=(M.nrows, M.ncols)).tocoo()
    xr, xc = S.row % n, S.col % n
    keep = ~(((S.col - S.row == 1) & (xr == cut)) | ((S.row - S.col == 1) & (xc == cut)))
    T = sp.csr_matrix((S.data[keep], (S.row[keep], S.col[keep])), shape=S.shape)
    T.sort_indices()
    return O.CSR(T.indptr.astype(np.int64), T.indices.astype(np.int64), T.data.copy(), M.ncols)


@pytest.mark.parametrize("zch", [0, 3])
def test_row_class_kernels_absent_in_grid_entries(ctx, zch):
    """k_sym_zm (SpMV, residual, Jacobi) and k_sym_zc (S = 2 through pamg_jacobi_residual; S = 3
    through pipelined V-cycles elsewhere) on a grid with a cut plane of removed couplings: bit-exact
    with the oracle, which sums present entries only."""
    from parallel_amg_amd._lib import layout_of
    from parallel_amg_amd.partitioned import jacobi_residual
    M = _cut_grid()
    Ad, _h = upload(ctx, M)
    lay = layout_of(Ad)
    assert lay["sym"] and lay["sym_vd"] and lay["jr_fused"], lay
    rng = np.random.default_rng(19 + zch)
    N = M.nrows
    xh, bh = rng.standard_normal(N), rng.standard_normal(N)
    x, b, y = PVector(ctx, N, 0, xh), PVector(ctx, N, 0, bh), PVector(ctx, N)
    with _with_option("zm_chunks", zch):
        mul(y, Ad, x)
        assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)))
        residual(y, Ad, x, b)
        assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)))
        t, r = PVector(ctx, N), PVector(ctx, N)
        assert jacobi_residual(t, r, Ad, x, b, 0.66)
    to = O.jacobi(M, xh, bh, 0.66)
    assert np.array_equal(bits(t.own_values()), bits(to))
    assert np.array_equal(bits(r.own_values()), bits(O.residual(M, to, bh)))


@pytest.mark.parametrize("breaker", ["asym_value", "signed_zero", "unsorted_row", "diagonal_only"])
def test_sym_dia_declines_what_it_cannot_reproduce(ctx, breaker):
    """A mirror that differs in one bit (or +0.0 against -0.0), a row whose storage order is
    not the ascending offset order, or an operator with no off-diagonal class at all (a part of
    isolated rows) keeps the rows in tiles — still bit-exact."""
    from parallel_amg_amd._lib import layout_of
    M = _sym_grid("poisson3d", 12)
    if breaker == "diagonal_only":
        n = M.nrows
        M = O.CSR(np.arange(n + 1, dtype=np.int64), np.arange(n, dtype=np.int64), 3.0 + np.arange(n) % 7, n)
    val, col = M.val.copy(), M.col.copy()
    i = 700
    a, e = int(M.rowptr[i]), int(M.rowptr[i + 1])
    if breaker == "asym_value":
        val[a] = np.nextafter(val[a], 0.0)             # a(i, i-n^2) one ulp off its mirror
    elif breaker == "signed_zero":
        val[a] = 0.0
        j = int(col[a])
        for k in range(M.rowptr[j], M.rowptr[j + 1]):
            if col[k] == i:
                val[k] = -0.0
    elif breaker == "unsorted_row":
        col[a:e] = col[a:e][::-1].copy()               # same entries, descending storage order
        val[a:e] = val[a:e][::-1].copy()
    M2 = O.CSR(M.rowptr.copy(), col, val, M.ncols)
    A, _h = upload(ctx, M2)
    assert not layout_of(A)["sym"]
    xh = np.random.default_rng(1).standard_normal(M.nrows)
    x, y = PVector(ctx, M.nrows, 0, xh), PVector(ctx, M.nrows)
    mul(y, A, x)
    assert np.array_equal(bits(y.own_values()), bits(O.spmv(M2, xh)))


def _row_classes(M):
    """The distinct (present offsets, diagonal, upper values) tuples of a square CSR matrix — what
    the row-class dictionary (sym_vd) counts, on the host."""
    keys = set()
    for i in range(M.nrows):
        a, e = int(M.rowptr[i]), int(M.rowptr[i + 1])
        offs = tuple(int(c) - i for c in M.col[a:e])
        vals = tuple(float(v).hex() for c, v in zip(M.col[a:e], M.val[a:e]) if c >= i)
        keys.add((offs, vals))
    return len(keys)


@pytest.mark.parametrize("npal", [1, 12, 13])
def test_sym_row_class_dictionary_limit(ctx, npal):
    """The row-class dictionary holds <= 64 tuples: 2D Poisson on a 30 x 30 grid (9 boundary
    cases: interior, 4 edges, 4 single-row corners) whose diagonal at grid point (r, c) is
    palette entry (r + c) % npal gives 5 npal + 4 classes — 9, 64 (dictionary, at the limit) and
    69 (f64 arrays) — and both layouts are bit-exact with the oracle (SpMV, residual, two Jacobi
    sweeps)."""
    from parallel_amg_amd._lib import layout_of
    M = _sym_grid("poisson2d", 30)
    val = M.val.copy()
    rows = np.repeat(np.arange(M.nrows), np.diff(M.rowptr))
    dg = M.col == rows
    pal = 4.0 + np.arange(npal) / 8.0
    i = np.arange(M.nrows)
    val[dg] = pal[(i // 30 + i % 30) % npal]
    M = O.CSR(M.rowptr.copy(), M.col.copy(), val, M.ncols)
    ncl = _row_classes(M)
    assert ncl == 5 * npal + 4
    A, _h = upload(ctx, M)
    lay = layout_of(A)
    assert lay["sym"] and lay["sym_vd"] == (ncl <= 64), (ncl, lay)
    rng = np.random.default_rng(npal)
    xh, bh = rng.standard_normal(M.nrows), rng.standard_normal(M.nrows)
    x, b, y = PVector(ctx, M.nrows, 0, xh), PVector(ctx, M.nrows, 0, bh), PVector(ctx, M.nrows)
    mul(y, A, x)
    assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)))
    residual(y, A, x, b)
    assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)))
    t = PVector(ctx, M.nrows)
    jacobi(x, A, b, t, 0.57, 2)
    assert np.array_equal(bits(x.own_values()), bits(O.jacobi(M, O.jacobi(M, xh, bh, 0.57), bh, 0.57)))


def test_sym_dia_vcycle_same_bits_either_layout(ctx):
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 28)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=200))
    out = []
    for on in (1, 0):
        with _with_option("sym_dia", on):
            S = AMGSolver(ctx, H)
        from parallel_amg_amd._lib import layout_of
        assert layout_of(S.A[0])["sym"] == bool(on)
        b = PVector(ctx, S.A[0].nrows, 0, xs[0])
        x = S.new_vector()
        h = S.vcycle(x, b, 4, res_hist=True)
        out.append((x.own_values(), h))
        del S
    assert np.array_equal(bits(out[0][0]), bits(out[1][0]))
    assert np.array_equal(bits(out[0][1]), bits(out[1][1]))


@pytest.mark.parametrize("npal,tnnz,lengths", [(40, 1024, [7, 31, 2]), (60, 4096, [31]), (17, 2048, [9]),
                                               (17, 2048, [31]), (60, 2048, [31]), (128, 2048, [31]),
                                               (129, 2048, [31]), (150, 2048, [31]), (256, 1024, [31]),
                                               (1000, 1024, [31, 7])])
def test_tile_major_value_dictionary_bit_exact(ctx, npal, tnnz, lengths):
    """8-bit per-tile value dictionaries in tile-major slots (value_dict, where the 4-bit ones do
    not fit and every tile has <= 256 distinct values — the 512^3 level-1 operator's case): SpMV,
    residual, Jacobi and prolongate-add bit-exact with the oracle. The rule (runtime.hip
    build_tile_major): the set takes them when its widest tile has 17..256 distinct values
    (bit patterns), <= 128 on 2048-nonzero tiles (the kernel's LDS table), rounded up to 4.
    Every value here (the diagonal too) is a palette value, and each tile draws ~2000 of them,
    so a tile holds the whole palette: npal is the widest tile's count, and the cases sit on
    both sides of each limit (128 / 129 on 2048-nonzero tiles, 256 on 1024)."""
    from parallel_amg_amd._lib import layout_of
    rng = np.random.default_rng(npal + tnnz)
    pal = rng.standard_normal(npal)
    M = offset_csr(rng, 3000, [-57, -9, -3, -1, 1, 2, 3, 9, 11, 57, 130, -130], lengths, palette=pal,
                   diag_from_palette=True)
    with _with_option("tile_nnz", tnnz), _with_option("tile_major", 2):
        A, _h = upload(ctx, M)
    lay = layout_of(A)
    limit = 128 if tnnz == 2048 else 256
    assert lay["tm"] and lay["tm_vd"] == (16 < npal <= limit), lay
    xh, bh, yh = (rng.standard_normal(M.nrows) for _ in range(3))
    x, b = PVector(ctx, M.nrows, 0, xh), PVector(ctx, M.nrows, 0, bh)
    y = PVector(ctx, M.nrows)
    mul(y, A, x)
    assert np.array_equal(bits(y.own_values()), bits(O.spmv(M, xh)))
    residual(y, A, x, b)
    assert np.array_equal(bits(y.own_values()), bits(O.residual(M, xh, bh)))
    t = PVector(ctx, M.nrows)
    jacobi(x, A, b, t, 0.61, 1)
    assert np.array_equal(bits(x.own_values()), bits(O.jacobi(M, xh, bh, 0.61)))


@pytest.mark.parametrize("rl8", [0, 1])
@pytest.mark.parametrize("lengths", [[3, 4, 1, 5, 0, 9, 2], [4], [255, 2, 1]])
def test_prolongator_value_dictionary_row_lengths_bit_exact(ctx, rl8, lengths):
    """Tall operators (the prolongators' shape) take 4-bit per-tile value dictionaries in the
    descriptor kernel, with 8-bit row lengths where the rows are short (row_len8) or row
    pointers: SpMV, residual and prolongate-add bit-exact with the oracle, ragged and empty
    rows and a 255-nonzero row included."""
    from parallel_amg_amd._lib import layout_of
    rng = np.random.default_rng(len(lengths) + 10 * rl8)
    M = random_csr(rng, (lengths * 6000)[:6000], 900, palette=PALETTES["few"])
    with _with_option("row_len8", rl8), _with_option("value_dict", 1), _with_option("col24", 1):
        A = _layout_ops_match_oracle(ctx, M, rng)
    lay = layout_of(A)
    short = M.rowptr[-1] <= 16 * M.nrows
    assert lay["vd"] and lay["c24"] and lay["rl8"] == bool(rl8 and short), lay


def _grid_prolongator(n, nvals, seed):
    """A prolongator of the 512^3 P0's shape on an n^3 grid: 2 x 2 x 2 aggregates in
    lexicographic order, each fine row reading its own aggregate and, per direction, the
    neighbour aggregate on its side (ascending columns, clipped at the boundary), values from a
    palette of nvals — <= 16 distinct values per tile (4-bit value dictionaries) and a few
    anchored column offsets per tile."""
    rng = np.random.default_rng(seed)
    m = n // 2
    z, y, x = np.meshgrid(np.arange(n), np.arange(n), np.arange(n), indexing="ij")
    X, Y, Z = x.ravel() // 2, y.ravel() // 2, z.ravel() // 2
    sx = np.where(x.ravel() % 2 == 0, -1, 1)
    sy = np.where(y.ravel() % 2 == 0, -1, 1)
    sz = np.where(z.ravel() % 2 == 0, -1, 1)
    cols = [Z * m * m + Y * m + X]
    for (ax, s_) in ((X, sx), (Y, sy), (Z, sz)):
        nb = ax + s_
        ok = (nb >= 0) & (nb < m)
        c = cols[0] + np.where(ax is X, s_, np.where(ax is Y, s_ * m, s_ * m * m))
        cols.append(np.where(ok, c, -1))
    C = np.stack(cols, axis=1)
    C.sort(axis=1)
    rowptr = np.zeros(n ** 3 + 1, np.int64)
    valid = C >= 0
    rowptr[1:] = np.cumsum(valid.sum(axis=1))
    col = C[valid].astype(np.int64)
    pal = 0.03125 * (1 + np.arange(nvals))
    val = pal[rng.integers(0, nvals, col.size)]
    return O.CSR(rowptr, col, val, m ** 3)


@pytest.mark.parametrize("n,nvals", [(64, 6), (48, 16), (32, 3)])
def test_prolongator_value_dictionaries_bit_exact(ctx, n, nvals):
    """A prolongator whose tiles hold <= 16 values (the 512^3 P0's layout: 4-bit value
    dictionaries beside 24-bit columns): SpMV, residual and prolongate-add bit-exact with the
    oracle."""
    from parallel_amg_amd._lib import layout_of
    M = _grid_prolongator(n, nvals, n)
    A0 = _layout_ops_match_oracle(ctx, M, np.random.default_rng(n))
    lay0 = layout_of(A0)
    assert lay0["vd"] and lay0["cd"] == 0, lay0


@pytest.mark.parametrize("kind,shape", [("poisson3d", (128, 128, 128)), ("aniso3d", (128, 128, 128)),
                                        ("poisson3d", (256, 256, 256)), ("poisson3d", (64, 32, 40)),
                                        ("aniso3d", (192, 48, 7))])
@pytest.mark.parametrize("vd", [1, 0])
def test_jacobi_residual_op_bit_exact(ctx, kind, shape, vd):
    """pamg_jacobi_residual: the temporally blocked pass (k_sym_tb, S = 2; k_sym_zc over the
    row-class dictionary) against the two separate sweeps on random x, b — t and r bit for bit,
    repeated, and the separate sweeps against the oracle; grids whose tiles split the planes into
    z chunks, and a grid with fewer planes than a chunk."""
    from parallel_amg_amd._lib import layout_of
    from parallel_amg_amd.partitioned import jacobi_residual
    Ao = O.generate(kind, *shape)
    with _with_option("sym_vd", vd):
        Ad, _h = upload(ctx, Ao)
    assert layout_of(Ad)["jr_fused"] and layout_of(Ad)["sym_vd"] == bool(vd)
    rng = np.random.default_rng(7)
    N = Ao.nrows
    x = PVector(ctx, N, 0, rng.standard_normal(N))
    b = PVector(ctx, N, 0, rng.standard_normal(N))
    out = {}
    for fuse in (0, 1):
        with _with_option("jr_fuse", fuse):
            for rep in range(3 if fuse else 1):
                t = PVector(ctx, N)
                r = PVector(ctx, N)
                f = jacobi_residual(t, r, Ad, x, b, 0.66)
                assert f == bool(fuse)
                out[(fuse, rep)] = (t.own_values(), r.own_values())
    t0, r0 = out[(0, 0)]
    to = O.jacobi(Ao, x.own_values(), b.own_values(), 0.66)
    assert np.array_equal(bits(t0), bits(to))
    assert np.array_equal(bits(r0), bits(O.residual(Ao, to, b.own_values())))
    for rep in range(3):
        t1, r1 = out[(1, rep)]
        bt = np.flatnonzero(bits(t1) != bits(t0))
        br = np.flatnonzero(bits(r1) != bits(r0))
        if br.size:  # the row sums of SPEC §S3 at the first differing rows (diagnostic)
            bh = b.own_values()
            for i in br[:2]:
                s = 0.0
                for k in range(Ao.rowptr[i], Ao.rowptr[i + 1]):
                    s = s + Ao.val[k] * t0[Ao.col[k]]
                print("row", i, "fused", r1[i].hex(), "unfused", r0[i].hex(), "spec", (bh[i] - s).hex(),
                      "cols", Ao.col[Ao.rowptr[i]:Ao.rowptr[i + 1]])
        assert bt.size == 0 and br.size == 0, (rep, bt.size, br.size, bt[:8], br[:8], r1[br[:4]], r0[br[:4]])


@pytest.mark.parametrize("kind,n", [("poisson3d", 128), ("aniso3d", 128)])
def test_fused_jacobi_residual_bit_exact(ctx, kind, n):
    """jr_fuse: the level-0 pre-smoothing sweep and residual pipelined in one persistent
    kernel (t handed between workgroups write-through) give the unfused cycle's bits — x and
    the residual history — and the oracle's."""
    from parallel_amg_amd._lib import layout_of
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    S = AMGSolver(ctx, H)
    assert layout_of(S.A[0])["jr_fused"]
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    out = []
    for fuse in (1, 0):
        with _with_option("jr_fuse", fuse):
            S.set_graph(False)   # re-capture with the option (read at capture)
            S.set_graph(True)
            x = S.new_vector()
            h = S.vcycle(x, b, 3, res_hist=True)
            x2 = S.new_vector()
            S.vcycle(x2, b, 3)    # graph replay
            out.append((x.own_values(), h, x2.own_values()))
    assert np.array_equal(bits(out[0][0]), bits(out[1][0]))
    assert np.array_equal(bits(out[0][1]), bits(out[1][1]))
    assert np.array_equal(bits(out[0][2]), bits(out[0][0]))
    Ao = O.generate(kind, n, n, n)
    Ho = O.setup(Ao, max_coarse=1000)
    xo, ho = Ho.solve(O.spmv(Ao, O.xstar(Ao.nrows)), 3, res_hist=True)
    assert np.array_equal(bits(out[0][0]), bits(xo))


@pytest.mark.parametrize("kind", ["poisson3d", "aniso3d"])
@pytest.mark.parametrize("vd", [1, 0])
def test_pipelined_cycles_bit_exact(ctx, kind, vd):
    """Stationary runs of K >= 2 cycles take the cross-cycle pipeline (one k_sym_chain launch per
    cycle boundary: the level-0 post-smoothing of cycle k, the pre-smoothing and residual of
    cycle k + 1; the iterate alternating between two level-0 buffers): x after K cycles has the
    bits of K separate unfused cycles and of the oracle, with graph replay and eagerly."""
    be = pa.SequentialBackend(1)
    n = 128
    A, offs, xs = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    with _with_option("sym_vd", vd):
        S = AMGSolver(ctx, H)
    from parallel_amg_amd._lib import layout_of
    assert layout_of(S.A[0])["sym_vd"] == bool(vd)
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    ref = {}
    with _with_option("jr_fuse", 0):
        S.set_graph(False)
        for K in (2, 3, 4, 5):
            x = S.new_vector()
            for _ in range(K):
                S.vcycle(x, b, 1)
            ref[K] = x.own_values()
    for graph in (True, False):
        with _with_option("jr_fuse", 1):
            S.set_graph(False)
            S.set_graph(graph)
            for K in (2, 3, 4, 5):
                x = S.new_vector()
                S.vcycle(x, b, K)
                assert np.array_equal(bits(x.own_values()), bits(ref[K])), (graph, K)
            # a continued run: 3 + 2 cycles == 5
            x = S.new_vector()
            S.vcycle(x, b, 3)
            S.vcycle(x, b, 2)
            assert np.array_equal(bits(x.own_values()), bits(ref[5]))
            assert S.graph_state()["captured"] == graph
    Ao = O.generate(kind, n, n, n)
    Ho = O.setup(Ao, max_coarse=1000)
    xo, _ho = Ho.solve(O.spmv(Ao, O.xstar(Ao.nrows)), 4, res_hist=True)
    assert np.array_equal(bits(ref[4]), bits(xo))


@pytest.fixture(scope="module")
def level1_128(ctx):
    """The level-1 operator of the 128^3 Poisson hierarchy (the 512^3 A1's kind: ~30 nonzeros per
    row, <= 73 distinct row-relative offsets per 2048-nonzero tile, a few hundred distinct values;
    64^3's level 1 is too irregular for per-tile 8-bit tables: up to 486 offsets per tile)."""
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 128)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    M = H.levels[1][0].A
    return O.CSR(M.rowptr.copy(), M.col.astype(np.int64), M.val.copy(), M.ncols)


@pytest.mark.parametrize("kind", ["poisson3d", "aniso3d"])
@pytest.mark.parametrize("key,val", [("chain_store_x", 1), ("tb_xfast", 0), ("tb_xfast", 1)])
def test_chain_variants_bit_exact(ctx, kind, key, val):
    """The chain's options — chain_store_x (the unread post-smoothed iterate stored too) and
    tb_xfast (tile order x- or y-fastest): the fused pre-smoothing pass (k_sym_zc<2, 2>) and
    pipelined cycles (k_sym_zc<3, 1>) keep the oracle's bits."""
    from parallel_amg_amd._lib import layout_of
    from parallel_amg_amd.partitioned import jacobi_residual
    be = pa.SequentialBackend(1)
    n = 128
    A, offs, xs = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    S = AMGSolver(ctx, H)
    assert layout_of(S.A[0])["sym_vd"]
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    Ao = O.generate(kind, n, n, n)
    rng = np.random.default_rng(2)
    xh, bh = rng.standard_normal(Ao.nrows), rng.standard_normal(Ao.nrows)
    with _with_option(key, val):
        t, r = PVector(ctx, Ao.nrows), PVector(ctx, Ao.nrows)
        assert jacobi_residual(t, r, S.A[0], PVector(ctx, Ao.nrows, 0, xh), PVector(ctx, Ao.nrows, 0, bh), 0.66)
        S.set_graph(False)
        S.set_graph(True)
        x = S.new_vector()
        S.vcycle(x, b, 5)
    to = O.jacobi(Ao, xh, bh, 0.66)
    assert np.array_equal(bits(t.own_values()), bits(to))
    assert np.array_equal(bits(r.own_values()), bits(O.residual(Ao, to, bh)))
    Ho = O.setup(Ao, max_coarse=1000)
    xo = Ho.solve(O.spmv(Ao, O.xstar(Ao.nrows)), 5)
    assert np.array_equal(bits(x.own_values()), bits(xo))


def _grid_hierarchy_P0(nx, ny, nz):
    """The level-0 prolongation of the SA hierarchy of a 7-point Poisson grid (host setup)."""
    M = O.generate("poisson3d", nx, ny, nz)
    n = M.nrows
    A = {0: HCSR.from_arrays(M.rowptr, M.col.astype(np.int32), M.val, n)}
    H = pa.build_hierarchy(pa.SequentialBackend(1), A, np.array([0, n], np.int64), pa.SAParams(max_coarse=100))
    lp = H.levels[0][0]
    P = lp.P
    return lp.A, O.CSR(P.rowptr.copy(), P.col.astype(np.int64), P.val.copy(), P.ncols)


@pytest.mark.parametrize("shape", [(64, 16, 12), (128, 32, 20), (64, 64, 64)])
def test_prolongation_neighbour_coded_bit_exact(ctx, shape):
    """k_rows_pnc (round 5: the prolongation's columns named by the grid neighbours whose anchors
    they are — 12 B per row; round 6: 6 B per row as 16-bit ids of the rows' (pattern, values)
    combinations, pnc_compact): a level-0 prolongation uploaded after its grid operator takes the
    layout, and its SpMV, residual and prolongate-add are bit-exact with the oracle; with the
    option off the tile layouts give the same bits."""
    from parallel_amg_amd._lib import layout_of
    A0, P = _grid_hierarchy_P0(*shape)
    Ad = PSparseMatrix(ctx, A0)
    assert layout_of(Ad)["jr_fused"], layout_of(Ad)  # (the grid is registered on the context)
    D = _layout_ops_match_oracle(ctx, P, np.random.default_rng(sum(shape)))
    lay = layout_of(D)
    # (compact records where the rows take <= 1024 (pattern, values) combinations: 128 x 32 x 20)
    assert lay["pnc"] and lay["pnc_compact"] == (shape == (128, 32, 20)), lay
    assert lay["cd"] <= 128 and lay["cd_offsets"] <= 1024, lay
    with _with_option("pnc_compact", 0):
        R = _layout_ops_match_oracle(ctx, P, np.random.default_rng(sum(shape)))
    assert layout_of(R)["pnc"] and not layout_of(R)["pnc_compact"]
    with _with_option("pnc", 0):
        T = _layout_ops_match_oracle(ctx, P, np.random.default_rng(sum(shape)))
    assert not layout_of(T)["pnc"]
    del Ad


def test_prolongation_compact_records_128(ctx):
    """The 128^3 level-0 prolongation (2.1M rows; its aggregates nearly all alike: 428 (pattern,
    values) combinations) takes the compact records — a 16-bit combination id per row (round 6) —
    and its SpMV, residual and prolongate-add are the oracle's bits, as with 64-bit records."""
    from parallel_amg_amd._lib import layout_of
    A0, P = _grid_hierarchy_P0(128, 128, 128)
    Ad = PSparseMatrix(ctx, A0)
    assert layout_of(Ad)["jr_fused"], layout_of(Ad)
    D = _layout_ops_match_oracle(ctx, P, np.random.default_rng(7))
    lay = layout_of(D)
    assert lay["pnc"] and lay["pnc_compact"] and lay["cd_offsets"] == 428, lay
    with _with_option("pnc_compact", 0):
        E = _layout_ops_match_oracle(ctx, P, np.random.default_rng(7))
    assert layout_of(E)["pnc"] and not layout_of(E)["pnc_compact"]
    del Ad


def test_prolongation_neighbour_coded_declines(ctx):
    """A column that is no neighbour's anchor, a row longer than 7, or no grid of the prolongation's
    row count on the context: the tile layouts, still bit-exact."""
    from parallel_amg_amd._lib import layout_of
    A0, P = _grid_hierarchy_P0(64, 16, 10)
    Ad = PSparseMatrix(ctx, A0)
    assert layout_of(Ad)["jr_fused"]
    # one entry of row 500 moved to a far column (kept sorted, values unchanged)
    col = P.col.copy()
    r0, r1 = P.rowptr[500], P.rowptr[501]
    far = P.ncols - 1 if col[r1 - 1] < P.ncols - 1 else 0
    if far > col[r1 - 1]:
        col[r1 - 1] = far
    else:
        col[r0] = far
    moved = O.CSR(P.rowptr.copy(), col, P.val.copy(), P.ncols)
    # row 700 given 8 entries (the first columns not in it)
    rows = [P.col[P.rowptr[i]:P.rowptr[i + 1]].tolist() for i in range(P.nrows)]
    vals = [P.val[P.rowptr[i]:P.rowptr[i + 1]].tolist() for i in range(P.nrows)]
    extra = [c for c in range(P.ncols) if c not in rows[700]][:8 - len(rows[700])]
    rows[700] = sorted(rows[700] + extra)
    vals[700] = (vals[700] + [0.125] * len(extra))[:8]
    rp = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.int64)
    long8 = O.CSR(rp, np.concatenate(rows).astype(np.int64), np.concatenate(vals), P.ncols)
    # a grid whose operator never took the blocked layout (nx = 40: not a multiple of the tile)
    A1, P1 = _grid_hierarchy_P0(40, 16, 10)
    for M in (moved, long8, P1):
        D = _layout_ops_match_oracle(ctx, M, np.random.default_rng(5))
        assert not layout_of(D)["pnc"]
    del Ad


def test_prolongation_neighbour_coded_same_size_grids(ctx):
    """Two 7-point grids of the same row count and different shapes registered on the context (the
    prolongation's own uploaded first, the other after): the upload tries each and finds its own."""
    from parallel_amg_amd._lib import layout_of
    A0, P = _grid_hierarchy_P0(64, 32, 12)          # 24576 rows
    own = PSparseMatrix(ctx, A0)
    decoy_M = O.generate("poisson3d", 128, 16, 12)  # 24576 rows too
    decoy = PSparseMatrix(ctx, HCSR.from_arrays(decoy_M.rowptr, decoy_M.col.astype(np.int32), decoy_M.val,
                                                decoy_M.nrows))
    assert layout_of(own)["jr_fused"] and layout_of(decoy)["jr_fused"]
    D = _layout_ops_match_oracle(ctx, P, np.random.default_rng(8))
    assert layout_of(D)["pnc"], layout_of(D)
    del own, decoy
