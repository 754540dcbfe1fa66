"""The bench's timed path at the bench's size: 3D 7-point Poisson 512^3, one
part, the library defaults.

bench.py times ``S.vcycle_async(x, b, K)``: with jr_fuse on, stationary runs of K >= 2 cycles
take the cross-cycle pipeline (``vcycle_pipe``: one ``k_sym_zc<3>`` launch per cycle boundary —
the level-0 post-smoothing of cycle k, the pre-smoothing and residual of cycle k + 1 — five
captured graphs, the iterate alternating between ``t[0]`` and ``u0``). At 512^3 that kernel runs
a geometry no smaller test reaches (8 x 32 xy tiles, one z chunk of all 512 planes per
workgroup, 256 workgroups), and the level-1 operator runs in the sliced-ELL layout, so these tests
pin the timed path at this size:

* K pipelined cycles through graph replay == K separate cycles (jr_fuse off, eager), bit for
  bit, from x = 0 and continued from a non-zero iterate (the bench's warm-up then timed runs);
* the temporally blocked pre-smoothing pass ``k_sym_zc<2>`` == Jacobi then residual, bit for bit;
* the oracle (oracle/pamg_oracle.c, OpenMP) run on the same 512^3 hierarchy (its level operators
  handed over by ``O.hierarchy_from_levels``, as bench.py's cpu_baseline does) for 3 V-cycles from
  x = 0 on the same b == the pipelined, graph-replayed cycles bench.py times, bit for bit
  (~4 s of oracle work on the box's 16 host threads);
* the oracle's OWN setup of the 512^3 problem (its generator, strength, aggregation, smoothing,
  transpose and Galerkin products) == the product's hierarchy: every level's aggregates, A, P, R
  and omega and the coarse inverse, bit for bit; and 3 oracle V-cycles on that independent
  hierarchy == the timed call (VERDICT r5 missing-3: setup parity at the metric's size).
"""
import contextlib
import ctypes

import numpy as np
import pytest

import parallel_amg_amd as pa
from parallel_amg_amd._lib import call, layout_of
from parallel_amg_amd.partitioned import PVector, jacobi_residual, mul
from parallel_amg_amd.solver import AMGSolver

pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


@contextlib.contextmanager
def option(key, value):
    v = ctypes.c_int64()
    call("pamg_get_option", key.encode(), ctypes.byref(v))
    call("pamg_set_option", key.encode(), int(value))
    try:
        yield
    finally:
        call("pamg_set_option", key.encode(), v.value)


@pytest.fixture(scope="module")
def h512(ctx):
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 512)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
    del A
    S = AMGSolver(ctx, H)
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    yield S, b
    del S, b


def test_timed_path_geometry(h512):
    """The 512^3 level-0 operator takes the symmetric layout with the blocked passes (the
    layout whose kernels the bench times)."""
    S, _b = h512
    lay = layout_of(S.A[0])
    assert lay["sym"] and lay["jr_fused"] and lay["cd_offsets"] == 3, lay
    assert S.L == 6
    assert layout_of(S.A_dev[1])["ell"] and layout_of(S.R[0])["rpat"], (layout_of(S.A_dev[1]), layout_of(S.R[0]))


def test_pipelined_cycles_512_bit_exact(ctx, h512):
    S, b = h512
    n = S.A[0].nrows
    ref = {}
    with option("jr_fuse", 0):
        S.set_graph(False)
        x = S.new_vector()
        for k in range(1, 6):
            S.vcycle(x, b, 1)
            if k in (3, 5):
                ref[k] = x.own_values()
    assert not np.array_equal(bits(ref[3]), bits(ref[5]))
    with option("jr_fuse", 1):
        S.set_graph(False)
        S.set_graph(True)
        x = S.new_vector()
        S.vcycle_async(x, b, 3)          # what bench.py times (graph replay, pipelined)
        ctx.sync()
        assert S.graph_state()["captured"]
        got3 = x.own_values()
        S.vcycle_async(x, b, 2)          # continued from a non-zero iterate
        ctx.sync()
        got5 = x.own_values()
    d3 = np.flatnonzero(bits(got3) != bits(ref[3]))
    assert d3.size == 0, (d3.size, d3[:8], n)
    d5 = np.flatnonzero(bits(got5) != bits(ref[5]))
    assert d5.size == 0, (d5.size, d5[:8], n)


def test_timed_path_512_matches_oracle(ctx, h512):
    """The bench's timed call (vcycle_async: graph replay of the cross-cycle pipeline) against the
    CPU oracle's V-cycle on the same 512^3 hierarchy, 3 cycles from x = 0, bit for bit."""
    from oracle import oracle as O
    S, b = h512
    H = S._H
    lv = [H.levels[l][0] for l in range(H.nlevels)]
    Ho = O.hierarchy_from_levels([p.A for p in lv], [p.P for p in lv[:-1]], [p.R for p in lv[:-1]],
                                 [p.omega for p in lv], H.ainv)
    bh = b.own_values()
    xo = Ho.solve(bh, 3)
    del Ho
    S.set_graph(False)
    S.set_graph(True)
    with option("jr_fuse", 1):
        x = S.new_vector()
        S.vcycle_async(x, b, 3)
        ctx.sync()
        assert S.graph_state()["captured"]
        got = x.own_values()
    d = np.flatnonzero(bits(got) != bits(xo))
    assert d.size == 0, (d.size, d[:8], np.abs(got - xo).max())


def test_blocked_pre_smoothing_512_bit_exact(ctx, h512):
    """k_sym_zc<2> (Jacobi -> residual in one pass) == the two separate sweeps (k_sym_zm), random x, b."""
    S, _b = h512
    A0 = S.A[0]
    n = A0.nrows
    rng = np.random.default_rng(11)
    x = PVector(ctx, n, 0, rng.standard_normal(n))
    b = PVector(ctx, n, 0, rng.standard_normal(n))
    out = []
    for fuse in (1, 0):
        t, r = PVector(ctx, n), PVector(ctx, n)
        with option("jr_fuse", fuse):
            ran = jacobi_residual(t, r, A0, x, b, S.omega[0])
        assert ran == bool(fuse)
        out.append((t.own_values(), r.own_values()))
        del t, r
    assert np.array_equal(bits(out[0][0]), bits(out[1][0]))
    assert np.array_equal(bits(out[0][1]), bits(out[1][1]))


def test_pcg_512_matches_oracle(ctx, h512):
    """Time to solution at the benchmarked size: PCG with one V-cycle as the preconditioner (SPEC
    §S8, bench.py's time_to_solution leg) against the oracle's PCG on the same 512^3 hierarchy —
    the same iteration count and residual history to 1e-6 (dot products reduce in a different
    order, so the iterates agree to rounding, not bit for bit)."""
    from oracle import oracle as O
    S, b = h512
    H = S._H
    lv = [H.levels[l][0] for l in range(H.nlevels)]
    Ho = O.hierarchy_from_levels([p.A for p in lv], [p.P for p in lv[:-1]], [p.R for p in lv[:-1]],
                                 [p.omega for p in lv], H.ainv)
    _xo, ko, ho = Ho.pcg(b.own_values(), 1e-8, 60)
    del Ho
    x = S.new_vector()
    k, hist = S.pcg(x, b, 1e-8, 60)
    assert k == ko, (k, ko, hist[-3:], ho[-3:])
    np.testing.assert_allclose(hist, ho, rtol=1e-6)


def _same_csr(got, want, what):
    """Product host CSR (int32 global columns) == oracle CSR (int64), bit for bit."""
    assert got.nrows == want.nrows and got.nnz == want.nnz, (what, got.nrows, want.nrows, got.nnz, want.nnz)
    assert np.array_equal(np.asarray(got.rowptr, np.int64), want.rowptr), what
    assert np.array_equal(np.asarray(got.col, np.int64), want.col), what
    d = np.flatnonzero(bits(got.val) != bits(want.val))
    assert d.size == 0, (what, d.size, d[:8])


@pytest.mark.timeout(900)
def test_setup_512_matches_oracle_setup(ctx, h512):
    """a10 at the metric's size: the oracle's own setup of 512^3 (serial aggregation, OpenMP
    rows elsewhere; ~1-2 min on 16 host threads) against the hierarchy the bench times."""
    from oracle import oracle as O
    S, b = h512
    H = S._H
    n = 512
    Ao = O.generate("poisson3d", n, n, n)
    bo = O.spmv(Ao, O.xstar(Ao.nrows))
    assert np.array_equal(bits(b.own_values()), bits(bo))
    Ho = O.setup(Ao, max_coarse=1000, fetch=False)
    del Ao
    assert Ho.nlevels == H.nlevels
    for l in range(H.nlevels):
        lp = H.levels[l][0]
        assert bits(lp.omega) == bits(Ho.omega[l]), l
        _same_csr(lp.A, Ho.csr(l, 0), f"A{l}")
        if l < H.nlevels - 1:
            assert np.array_equal(np.asarray(lp.agg, np.int64), Ho.aggregates(l)), f"aggregates of level {l}"
            _same_csr(lp.P, Ho.csr(l, 1), f"P{l}")
            _same_csr(lp.R, Ho.csr(l, 2), f"R{l}")
    nc = Ho.ainv.shape[0]
    assert np.array_equal(bits(np.asarray(H.ainv).reshape(nc, nc)), bits(Ho.ainv.T)), "coarse inverse"
    # the timed call against V-cycles on the oracle's own hierarchy
    xo = Ho.solve(bo, 3)
    del Ho
    S.set_graph(False)
    S.set_graph(True)
    with option("jr_fuse", 1):
        x = S.new_vector()
        S.vcycle_async(x, b, 3)
        ctx.sync()
        got = x.own_values()
    d = np.flatnonzero(bits(got) != bits(xo))
    assert d.size == 0, (d.size, d[:8])
