"""PartitionedArrays ``with_debug`` on the device: every part of a
``SequentialBackend(n)`` in ONE process on one GPU, one context per part registered in an
in-process world (pamg_world / pamg_comm_init_local), ghosts moved by device-to-device copies
from the sibling parts' vectors. The global-view oracle's multi-part setup (SPEC §S7) is the
reference: b = A x*, x after V-cycles (bit for bit), residual histories and PCG (1e-12), with
NaN-poisoned ghost slots before every exchange (a read before the copy landed would show)."""
import contextlib
import ctypes

import numpy as np
import pytest

import parallel_amg_amd as pa
from oracle import oracle as O
from parallel_amg_amd._lib import call, layout_of
from parallel_amg_amd.partitioned import LocalWorld, PVector, consistent, mul
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


@pytest.mark.parametrize("nparts,kind,n,max_coarse,agglomerate", [
    (2, "poisson3d", 20, 100, 0),         # decoupled on every level, the coarsest gathered
    (2, "poisson3d", 20, 100, 32768),     # agglomerated from level 1 on (one all-gather)
    (3, "poisson2d", 60, 200, 0),
    (4, "poisson3d", 24, 60, 0),          # interior parts with two neighbours
    (2, "poisson2d", 20, 1000, 0),        # one level: the distributed coarsest solve
    (2, "poisson2d", 256, 1000, 0),       # BASELINE.json configs[0] at its size (golden test below)
    (8, "poisson3d", 64, 1000, 0),        # BASELINE.json configs[2]'s part count; z-slabs: the
    (8, "aniso3d", 64, 1000, 32768),      # blocked level-0 passes run on every part (tb_part)
])
def test_local_world_vcycle_bit_exact(built, nparts, kind, n, max_coarse, agglomerate):
    ncycles = 4
    with option("poison_ghosts", 1):
        W = LocalWorld(nparts)
        try:
            be = pa.SequentialBackend(nparts)
            A, offs, xs = pa.generate_problem(be, kind, n)
            H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=max_coarse, agglomerate=agglomerate),
                                   device=W.ctxs[0])
            S = [AMGSolver(W.ctxs[p], H, part=p) for p in range(nparts)]
            assert all(not s.graph_state()["enabled"] for s in S)   # synchronous transport: eager
            A0 = [s.A[0] for s in S]
            xst = [PVector(W.ctxs[p], A0[p].n_own_cols, A0[p].n_ghost, xs[p]) for p in range(nparts)]
            b = [PVector(W.ctxs[p], A0[p].nrows) for p in range(nparts)]
            W.run(lambda p: mul(b[p], A0[p], xst[p]))
            x = [s.new_vector() for s in S]
            hist = W.run(lambda p: S[p].vcycle(x[p], b[p], ncycles, res_hist=True))
            # one stationary run of the same cycles (the cross-cycle pipeline where every part is
            # a z-slab of whole planes) gives the same bits
            xp = [s.new_vector() for s in S]
            W.run(lambda p: S[p].vcycle(xp[p], b[p], ncycles))
            same_pipe = [np.array_equal(bits(xp[p].own_values()), bits(x[p].own_values())) for p in range(nparts)]
            # consistent!(x): the owners' values in every part's ghost slots
            pl = [H.levels[0][p].planA for p in range(nparts)]
            v = [PVector(W.ctxs[p], pl[p].n_own, pl[p].n_ghost, x[p].own_values()) for p in range(nparts)]
            if A0[0].plan is not None:
                W.run(lambda p: consistent(v[p], A0[p].plan))
            pcg = W.run(lambda p: S[p].pcg(S[p].new_vector(), b[p], rtol=1e-8, maxit=60))
            # the same cycles through the all-parts entry point (one call; the library runs a
            # thread per part): what a single-threaded with_debug driver (Julia map) calls
            xw = [s.new_vector() for s in S]
            arr = lambda objs: (ctypes.c_void_p * nparts)(*[o.handle for o in objs])  # noqa: E731
            hw = np.zeros(ncycles)
            call("pamg_world_vcycle", W._h, arr(S), arr(xw), arr(b), ncycles, hw.ctypes.data_as(ctypes.c_void_p))
            same_world = [np.array_equal(bits(xw[p].own_values()), bits(x[p].own_values())) for p in range(nparts)]
            assert all(same_world) and np.array_equal(hw, hist[0]), same_world
            xq = [s.new_vector() for s in S]
            itw, hq = ctypes.c_int(), np.zeros(61)
            call("pamg_world_pcg", W._h, arr(S), arr(xq), arr(b), 1e-8, 60, ctypes.byref(itw),
                 hq.ctypes.data_as(ctypes.c_void_p))
            assert itw.value == pcg[0][0]
            assert np.array_equal(hq[:itw.value + 1], np.asarray(pcg[0][1])[:itw.value + 1])
            fused = [layout_of(a)["jr_fused"] for a in A0]
            pnc0 = [bool(s.P) and layout_of(s.P[0])["pnc"] for s in S]  # (a part's P0: interior rows neighbour-coded)
            got_b = np.concatenate([bb.own_values() for bb in b])
            got_x = np.concatenate([xx.own_values() for xx in x])
            ghosts = [(np.asarray(pl[p].ghost_ids, np.int64), v[p].ghost_values()) for p in range(nparts)]
        finally:
            del S
            W.close()
    Ao = O.generate(kind, *O.grid_shape(kind, n))
    bo = O.spmv(Ao, O.xstar(Ao.nrows))
    Ho = O.setup(Ao, nparts=nparts, max_coarse=max_coarse, agglomerate=agglomerate)
    xo, ho = Ho.solve(bo, ncycles, res_hist=True)
    _xpo, kpo, hpo = Ho.pcg(bo, rtol=1e-8, maxit=60)
    assert np.array_equal(bits(got_b), bits(bo))
    assert np.array_equal(bits(got_x), bits(xo))
    assert all(same_pipe), same_pipe
    if n == 64:
        assert all(fused), fused
        if kind == "poisson3d":
            assert any(pnc0), pnc0
    for p in range(nparts):
        np.testing.assert_allclose(hist[p], ho, rtol=1e-12)
        its, ph = pcg[p]
        assert its == kpo
        np.testing.assert_allclose(ph, hpo, rtol=1e-10)
        gid, gv = ghosts[p]
        if A0[0].plan is not None and len(gid):
            assert np.array_equal(bits(gv), bits(got_x[gid]))


# (a part takes ELL where >= 75 % of its rows are interior: 60 planes in 3 slabs leave the middle
# slab 18 of its 20 planes)
@pytest.mark.parametrize("nparts,kind,n", [(3, "poisson2d", 60), (3, "poisson3d", 60), (2, "aniso3d", 20)])
def test_local_world_ell_interior_rows_bit_exact(built, nparts, kind, n):
    """Several parts with the sliced-ELL layout on every level's interior rows (ell_min_rows 0,
    sym_dia 0: level 0 too; the boundary rows — ghost columns — stay in tiles and run after the
    exchange, marked skipped in the slices): b = A x* and x after 4 V-cycles are the oracle's
    multi-part bits, ghosts NaN-poisoned."""
    ncycles = 4
    with option("poison_ghosts", 1), option("ell_min_rows", 0), option("sym_dia", 0):
        W = LocalWorld(nparts)
        try:
            be = pa.SequentialBackend(nparts)
            A, offs, xs = pa.generate_problem(be, kind, n)
            H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=60, agglomerate=0), device=W.ctxs[0])
            S = [AMGSolver(W.ctxs[p], H, part=p) for p in range(nparts)]
            assert any(layout_of(s.A[0])["ell"] for s in S)
            if kind == "poisson2d":  # (a part's R_0 interior rows in the pattern-dictionary layout, boundary
                # rows skipped; the 60^3 slabs' aggregates take more than 255 shapes: ELL)
                assert any(layout_of(s.R[0])["rpat"] for s in S)
            A0 = [s.A[0] for s in S]
            xst = [PVector(W.ctxs[p], A0[p].n_own_cols, A0[p].n_ghost, xs[p]) for p in range(nparts)]
            b = [PVector(W.ctxs[p], A0[p].nrows) for p in range(nparts)]
            W.run(lambda p: mul(b[p], A0[p], xst[p]))
            x = [s.new_vector() for s in S]
            W.run(lambda p: S[p].vcycle(x[p], b[p], ncycles))
            got_b = np.concatenate([v.own_values() for v in b])
            got_x = np.concatenate([v.own_values() for v in x])
        finally:
            del S
            W.close()
    Ao = O.generate(kind, *O.grid_shape(kind, n))
    bo = O.spmv(Ao, O.xstar(Ao.nrows))
    Ho = O.setup(Ao, nparts=nparts, max_coarse=60, agglomerate=0)
    assert np.array_equal(bits(got_b), bits(bo))
    assert np.array_equal(bits(got_x), bits(Ho.solve(bo, ncycles)))


def test_baseline_config0_golden(built):
    """BASELINE.json configs[0] — 2D 5-pt Poisson 256 x 256, 2 parts, the PartitionedArrays
    sequential-backend shape — on the HIP path (both parts in one process, the device world) against
    the committed fixture tests/golden/poisson2d_256_p2.npz (tests/golden/make_golden.py: 10 V-cycles
    of the oracle's 2-part, decoupled hierarchy): b, x after 10 cycles by sha256, bit for bit, the
    leading 64 entries of x, and the residual history to 1e-12."""
    import hashlib
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "poisson2d_256_p2.npz"))
    kind, n, nparts = str(g["kind"]), int(g["n"]), int(g["nparts"])
    ncycles, max_coarse = int(g["ncycles"]), int(g["max_coarse"])
    assert (kind, n, nparts) == ("poisson2d", 256, 2)
    sha = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    with option("poison_ghosts", 1):
        W = LocalWorld(nparts)
        try:
            be = pa.SequentialBackend(nparts)
            A, offs, xs = pa.generate_problem(be, kind, n)
            H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=max_coarse, agglomerate=0),
                                   device=W.ctxs[0])
            assert H.nlevels == int(g["nlevels"])
            S = [AMGSolver(W.ctxs[p], H, part=p) for p in range(nparts)]
            A0 = [s.A[0] for s in S]
            xst = [PVector(W.ctxs[p], A0[p].n_own_cols, A0[p].n_ghost, xs[p]) for p in range(nparts)]
            b = [PVector(W.ctxs[p], A0[p].nrows) for p in range(nparts)]
            W.run(lambda p: mul(b[p], A0[p], xst[p]))
            x = [s.new_vector() for s in S]
            hist = W.run(lambda p: S[p].vcycle(x[p], b[p], ncycles, res_hist=True))
            got_b = np.concatenate([v.own_values() for v in b])
            got_x = np.concatenate([v.own_values() for v in x])
        finally:
            del S
            W.close()
    assert sha(got_b) == str(g["b_sha"])
    assert np.array_equal(bits(got_x[:64]), bits(g["x"]))
    assert sha(got_x) == str(g["x_sha"])
    for p in range(nparts):
        np.testing.assert_allclose(hist[p], g["res_hist"], rtol=1e-12)


def test_local_world_rejects_a_second_transport(built):
    """A context joins one transport only; a world rank is taken once."""
    from parallel_amg_amd._lib import PamgError
    from parallel_amg_amd.partitioned import Context
    W = LocalWorld(2)
    try:
        with pytest.raises(PamgError):
            call("pamg_comm_init_local", W.ctxs[0].handle, W._h, 1)
        c = Context(0)
        with pytest.raises(PamgError):
            call("pamg_comm_init_local", c.handle, W._h, 1)   # rank 1 is taken
        c.close()
        y = PVector(W.ctxs[0], 10, 0, np.arange(10.0))
        assert np.array_equal(y.own_values(), np.arange(10.0))
    finally:
        W.close()


def test_ranks_disagreeing_on_the_pipeline_bit_exact(built):
    """whether a rank pipelines its level-0 cycles (the blocked chain, SymDia::tb_part)
    depends on its part's shape. Here part 0 is a z-slab of whole planes (it pipelines) and parts
    1, 2 start or end inside a plane (separate cycles): the exchanges still pair up (both
    schedules issue them in the same order), and x, the residual history and a stationary run
    keep the oracle's bits."""
    from parallel_amg_amd.hcsr import HCSR
    n, plane = 64, 64 * 64
    offs = np.array([0, 20 * plane, 40 * plane + 1000, n ** 3], np.int64)
    whole, _o, wx = pa.generate_problem(pa.SequentialBackend(1), "poisson3d", n)
    M = whole[0]
    nparts = 3
    A, xs = {}, {}
    for p in range(nparts):
        a, c = int(offs[p]), int(offs[p + 1])
        lo, hi = int(M.rowptr[a]), int(M.rowptr[c])
        A[p] = HCSR.from_arrays(M.rowptr[a:c + 1] - lo, M.col[lo:hi].copy(), M.val[lo:hi].copy(), M.ncols)
        xs[p] = np.ascontiguousarray(wx[0][a:c])
    ncycles = 4
    with option("poison_ghosts", 1):
        W = LocalWorld(nparts)
        try:
            be = pa.SequentialBackend(nparts)
            H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000, agglomerate=0), device=W.ctxs[0])
            S = [AMGSolver(W.ctxs[p], H, part=p) for p in range(nparts)]
            fused = [layout_of(s.A[0])["jr_fused"] for s in S]
            A0 = [s.A[0] for s in S]
            xst = [PVector(W.ctxs[p], A0[p].n_own_cols, A0[p].n_ghost, xs[p]) for p in range(nparts)]
            b = [PVector(W.ctxs[p], A0[p].nrows) for p in range(nparts)]
            W.run(lambda p: mul(b[p], A0[p], xst[p]))
            x = [s.new_vector() for s in S]
            hist = W.run(lambda p: S[p].vcycle(x[p], b[p], ncycles, res_hist=True))
            xp = [s.new_vector() for s in S]
            W.run(lambda p: S[p].vcycle(xp[p], b[p], ncycles))
            got_x = np.concatenate([v.own_values() for v in x])
            got_xp = np.concatenate([v.own_values() for v in xp])
        finally:
            del S
            W.close()
    assert fused == [True, False, False], fused
    Ao = O.CSR(M.rowptr.copy(), M.col.astype(np.int64), M.val.copy(), M.ncols)
    Ho = O.setup(Ao, offsets=offs, max_coarse=1000, agglomerate=0)
    xo, ho = Ho.solve(O.spmv(Ao, wx[0]), ncycles, res_hist=True)
    assert np.array_equal(bits(got_x), bits(xo))
    assert np.array_equal(bits(got_xp), bits(xo))
    for p in range(nparts):
        np.testing.assert_allclose(hist[p], ho, rtol=1e-12)


def test_part_bench_rowop_stage_vectors_need_ghost_slots(built):
    """pamg_bench_rowop's blocked passes on one part (ops 4 / 5: sweeps_part without exchanges)
    feed each stage's output to the next stage's boundary rows, which read ghost slots: an output
    vector without them is refused (it once faulted the GPU at 512 x 512 x 64), one with them runs."""
    from parallel_amg_amd._lib import PamgError
    from parallel_amg_amd.partitioned import PSparseMatrix
    nparts = 4
    W = LocalWorld(nparts)
    try:
        be = pa.SequentialBackend(nparts)
        A, offs, xs = pa.generate_problem(be, "poisson3d", 64)
        H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=W.ctxs[0])
        ctx = W.ctxs[1]
        lp = H.levels[0][1]
        Ad = PSparseMatrix(ctx, lp.A, lp.planA)
        assert layout_of(Ad)["jr_fused"], layout_of(Ad)
        x = PVector(ctx, Ad.n_own_cols, Ad.n_ghost, xs[1])
        b = PVector(ctx, Ad.nrows, 0, np.ones(Ad.nrows))
        ms = ctypes.c_double()
        with pytest.raises(PamgError):
            call("pamg_bench_rowop", ctx.handle, Ad.handle, 4, x.handle, b.handle, PVector(ctx, Ad.nrows).handle,
                 0.6, 1, ctypes.byref(ms))
        y = PVector(ctx, Ad.n_own_cols, Ad.n_ghost)
        for op in (4, 5):
            call("pamg_bench_rowop", ctx.handle, Ad.handle, op, x.handle, b.handle, y.handle, 0.6, 2, ctypes.byref(ms))
            assert ms.value > 0
        del Ad
    finally:
        W.close()


def _two_plans(nparts=2, n_own=10):
    """Two exchange plans over the same 2-part index space with EQUAL counts between the parts
    (3 ghosts each way) but different ghost ids: tags 1 and 2."""
    from parallel_amg_amd.hierarchy import build_plans
    be = pa.SequentialBackend(nparts)
    offs = np.array([0, n_own, 2 * n_own], np.int64)
    pa_ = build_plans(be, {0: np.array([10, 11, 12]), 1: np.array([7, 8, 9])}, offs)
    pb_ = build_plans(be, {0: np.array([15, 16, 17]), 1: np.array([0, 1, 2])}, offs)
    return pa_, pb_


def test_local_world_mismatched_pairing_fails(built):
    """part 0 exchanging plan A while part 1 exchanges plan B (same counts
    between the two parts) must fail on both parts (PAMG_E_STATE, tags differ) instead of moving
    B's rows into A's ghost slots; after pamg_world_reset the correctly paired exchange runs and
    lands the owners' values."""
    from parallel_amg_amd.partitioned import DevicePlan
    hA, hB = _two_plans()
    W = LocalWorld(2)
    try:
        pA = [DevicePlan(W.ctxs[p], hA[p], tag=1) for p in range(2)]
        pB = [DevicePlan(W.ctxs[p], hB[p], tag=2) for p in range(2)]
        v = [PVector(W.ctxs[p], 10, 3, np.arange(10.0) + 10 * p) for p in range(2)]
        with pytest.raises(RuntimeError, match="schedules diverged|broken"):
            W.run(lambda p: consistent(v[p], pA[p] if p == 0 else pB[p]))
        # (a run over all the parts clears the break once they have all returned: ADVICE r5)
        assert not W.broken
        W.reset()
        assert not W.broken
        W.run(lambda p: consistent(v[p], pA[p]))
        assert np.array_equal(v[0].ghost_values(), [10.0, 11.0, 12.0])
        assert np.array_equal(v[1].ghost_values(), [7.0, 8.0, 9.0])
        W.run(lambda p: consistent(v[p], pB[p]))
        assert np.array_equal(v[0].ghost_values(), [15.0, 16.0, 17.0])
        assert np.array_equal(v[1].ghost_values(), [0.0, 1.0, 2.0])
        del pA, pB, v
    finally:
        W.close()


def test_local_world_failed_part_releases_siblings(built):
    """a part that fails before an exchange (here a Python exception) breaks the
    world at once, so its sibling's exchange fails within seconds instead of waiting 300 s."""
    import time
    from parallel_amg_amd.partitioned import DevicePlan
    hA, _hB = _two_plans()
    W = LocalWorld(2)
    try:
        pA = [DevicePlan(W.ctxs[p], hA[p], tag=1) for p in range(2)]
        v = [PVector(W.ctxs[p], 10, 3, np.arange(10.0)) for p in range(2)]

        def body(p):
            if p == 0:
                raise ValueError("part 0 gives up")
            consistent(v[p], pA[p])

        t = time.time()
        with pytest.raises(RuntimeError, match="part 0"):
            W.run(body)
        assert time.time() - t < 60
        assert not W.broken  # every part returned: the run reset the world itself
        W.run(lambda p: consistent(v[p], pA[p]))
        # a run over SOME parts leaves the break for the caller's reset (the others may be busy)
        with pytest.raises(RuntimeError, match="part 0"):
            W.run(body, parts=[0])
        assert W.broken
        W.reset()
        W.run(lambda p: consistent(v[p], pA[p]))
        del pA, v
    finally:
        W.close()


def test_world_call_argument_error_leaves_the_world_usable(built):
    """a pamg_world_* call whose part fails an argument check (here part 1
    passes no plan) fails that call — the sibling waiting in its exchange is released at once —
    and the world is reset before the call returns, so the next call runs."""
    import time
    from parallel_amg_amd._lib import PamgError
    from parallel_amg_amd.partitioned import DevicePlan
    hA, _hB = _two_plans()
    W = LocalWorld(2)
    try:
        pA = [DevicePlan(W.ctxs[p], hA[p], tag=1) for p in range(2)]
        v = [PVector(W.ctxs[p], 10, 3, np.arange(10.0) + 10 * p) for p in range(2)]
        vs = (ctypes.c_void_p * 2)(*[x.handle.value for x in v])
        bad = (ctypes.c_void_p * 2)(pA[0].handle.value, None)
        good = (ctypes.c_void_p * 2)(*[q.handle.value for q in pA])
        t = time.time()
        with pytest.raises(PamgError, match="part 1"):
            call("pamg_world_exchange", W._h, bad, vs)
        assert time.time() - t < 60
        assert not W.broken
        call("pamg_world_exchange", W._h, good, vs)
        assert np.array_equal(v[0].ghost_values(), [10.0, 11.0, 12.0])
        assert np.array_equal(v[1].ghost_values(), [7.0, 8.0, 9.0])
        del pA, v
    finally:
        W.close()


def test_local_world_zero_listed_neighbour_fails_fast(built):
    """part 0's plan expects 3 ghosts from part 1 and sends it 3, while part 1's
    plan (same tag) lists part 0 with zero counts. Part 0 must fail at once with the count
    mismatch, not after the 300 s pairing timeout."""
    import time
    from parallel_amg_amd.hierarchy import HostPlan
    from parallel_amg_amd.partitioned import DevicePlan
    hA, _hB = _two_plans()
    lonely = HostPlan(n_own=10, col0=10, ghost_ids=np.zeros(0, np.int64), nbrs=[0], recv_counts=[0],
                      send_counts=[0], send_idx=np.zeros(0, np.int64))
    W = LocalWorld(2)
    try:
        plans = [DevicePlan(W.ctxs[0], hA[0], tag=7), DevicePlan(W.ctxs[1], lonely, tag=7)]
        v = [PVector(W.ctxs[0], 10, 3, np.arange(10.0)), PVector(W.ctxs[1], 10, 0, np.arange(10.0))]
        t = time.time()
        with pytest.raises(RuntimeError, match="zero counts"):
            W.run(lambda p: consistent(v[p], plans[p]))
        assert time.time() - t < 60
        del plans, v
    finally:
        W.close()


def test_local_world_part_without_neighbours(built):
    """a part whose operator has no neighbour (a decoupled block) never meets
    the others at an exchange; the coupled parts still exchange, pairwise. Two decoupled 2D Poisson
    blocks, the first split over parts 0 and 1, the second all on part 2: b = A x* and x after 4
    V-cycles equal the oracle's 3-part setup bit for bit."""
    import scipy.sparse as sp
    from parallel_amg_amd.hcsr import HCSR
    nb = 20
    whole, _o, _x = pa.generate_problem(pa.SequentialBackend(1), "poisson2d", nb)
    M1 = whole[0]
    B = sp.csr_matrix((M1.val, M1.col, M1.rowptr), shape=(M1.nrows, M1.nrows))
    Mbd = sp.block_diag([B, B], format="csr")
    Mbd.sort_indices()
    n = Mbd.shape[0]
    rng = np.random.default_rng(3)
    xstar = rng.uniform(-1, 1, n)
    offs = np.array([0, n // 4, n // 2, n], np.int64)
    rp, col, val = Mbd.indptr.astype(np.int64), Mbd.indices.astype(np.int64), Mbd.data.copy()
    A, xs = {}, {}
    for p in range(3):
        a, c = int(offs[p]), int(offs[p + 1])
        lo, hi = int(rp[a]), int(rp[c])
        A[p] = HCSR.from_arrays(rp[a:c + 1] - lo, col[lo:hi].copy(), val[lo:hi].copy(), n)
        xs[p] = np.ascontiguousarray(xstar[a:c])
    ncycles = 4
    with option("poison_ghosts", 1):
        W = LocalWorld(3)
        try:
            be = pa.SequentialBackend(3)
            H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=40, agglomerate=0), device=W.ctxs[0])
            assert not H.levels[0][2].planA.nbrs and H.levels[0][0].planA.nbrs
            S = [AMGSolver(W.ctxs[p], H, part=p) for p in range(3)]
            A0 = [s.A[0] for s in S]
            assert A0[2].plan is None and A0[0].plan is not None
            xst = [PVector(W.ctxs[p], A0[p].n_own_cols, A0[p].n_ghost, xs[p]) for p in range(3)]
            b = [PVector(W.ctxs[p], A0[p].nrows) for p in range(3)]
            W.run(lambda p: mul(b[p], A0[p], xst[p]))
            x = [s.new_vector() for s in S]
            W.run(lambda p: S[p].vcycle(x[p], b[p], ncycles))
            got_b = np.concatenate([v.own_values() for v in b])
            got_x = np.concatenate([v.own_values() for v in x])
        finally:
            del S
            W.close()
    Ao = O.CSR(rp, col, val, n)
    bo = O.spmv(Ao, xstar)
    Ho = O.setup(Ao, offsets=offs, max_coarse=40, agglomerate=0)
    xo = Ho.solve(bo, ncycles)
    assert np.array_equal(bits(got_b), bits(bo))
    assert np.array_equal(bits(got_x), bits(xo))


def test_failed_create_keeps_the_context_reference_count(built):
    """a hierarchy / matrix create that fails after its object took the
    context must give back exactly the reference it took — never one it did not — so the
    context is torn down once, with its last user."""
    from parallel_amg_amd import hcsr as HC
    from parallel_amg_amd._lib import PamgError
    from parallel_amg_amd.partitioned import Context, PSparseMatrix
    c = Context(0)
    assert c.refcount() == 1
    v = PVector(c, 2, 0, np.ones(2))
    M = HC.HCSR.from_arrays(np.array([0, 2, 4]), np.array([0, 1, 0, 1], np.int32),
                            np.array([4.0, -1.0, -1.0, 4.0]), 2)
    A = PSparseMatrix(c, M)
    B = PSparseMatrix(c, HC.HCSR.from_arrays(np.array([0, 1, 2, 3]), np.array([0, 1, 2], np.int32),
                                             np.array([2.0, 2.0, 2.0]), 3))
    assert c.refcount() == 4
    arrPR = (ctypes.c_void_p * 1)(A.handle.value)
    om = np.array([2.0 / 3.0, 2.0 / 3.0])
    ainv = np.eye(3)
    h = ctypes.c_void_p()
    # a NULL level is refused before anything is made
    arrA = (ctypes.c_void_p * 2)(A.handle.value, None)
    with pytest.raises(PamgError, match="A\\[1\\] is NULL"):
        call("pamg_hier_create", c.handle, 2, arrA, arrPR, arrPR, om.ctypes.data_as(ctypes.c_void_p), 3,
             ainv.ctypes.data_as(ctypes.c_void_p), 1, None, ctypes.byref(h))
    assert c.refcount() == 4
    # R (2 rows) does not fit the 3-row coarse level: fails after the hierarchy took the context
    arrA = (ctypes.c_void_p * 2)(A.handle.value, B.handle.value)
    for _ in range(3):
        with pytest.raises(PamgError, match="shapes inconsistent"):
            call("pamg_hier_create", c.handle, 2, arrA, arrPR, arrPR, om.ctypes.data_as(ctypes.c_void_p), 3,
                 ainv.ctypes.data_as(ctypes.c_void_p), 1, None, ctypes.byref(h))
        assert c.refcount() == 4
    del B
    assert c.refcount() == 3
    one = (ctypes.c_void_p * 1)(A.handle.value)
    with pytest.raises(PamgError, match="n_coarse"):  # a one-level hierarchy with the wrong coarse size
        call("pamg_hier_create", c.handle, 1, one, None, None, om.ctypes.data_as(ctypes.c_void_p), 5,
             ainv.ctypes.data_as(ctypes.c_void_p), 0, None, ctypes.byref(h))
    assert c.refcount() == 3
    # a failed plan create (send index out of range) likewise
    from parallel_amg_amd.hierarchy import HostPlan
    from parallel_amg_amd.partitioned import DevicePlan
    with pytest.raises(PamgError):
        DevicePlan(c, HostPlan(n_own=2, col0=0, ghost_ids=np.zeros(1, np.int64), nbrs=[0], recv_counts=[1],
                               send_counts=[1], send_idx=np.array([9], np.int64)))
    assert c.refcount() == 3
    del A
    assert c.refcount() == 2
    assert np.array_equal(v.own_values(), np.ones(2))
    del v
    assert c.refcount() == 1


def test_context_outlives_its_handle(built):
    """Handles may be destroyed in any order (a garbage collector finalises the objects of a
    reference cycle in no particular order): a context whose handle is destroyed stays alive
    while a vector made on it exists, and is torn down with the last one."""
    from parallel_amg_amd.partitioned import Context
    c = Context(0)
    v = PVector(c, 16, 0, np.arange(16.0))
    raw = c._h
    call("pamg_ctx_destroy", raw)
    c._h = None
    out = np.empty(16)
    call("pamg_vec_download", raw, v.handle, out.ctypes.data_as(ctypes.c_void_p))
    assert np.array_equal(out, np.arange(16.0))
    del v
