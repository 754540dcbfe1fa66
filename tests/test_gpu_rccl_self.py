"""RCCL transport on one GPU: a one-rank RCCL communicator with self-exchange plans.

RCCL refuses several ranks on one device, so the multi-part tests of the one-GPU box use the
host debug transport. This test drives the RCCL code itself on the real device instead: every
operator of a single-part hierarchy is re-uploaded with some of its own columns moved into
ghost slots, and a plan whose only neighbour is the part itself (``nbrs = [0]``) fills those
slots by ``ncclSend``/``ncclRecv`` to self. The operator is unchanged (same values in the same
storage order, read through a ghost slot instead of the own entry), so every result must be
bit-identical to the plain single-part path — with the exchange on the comm stream overlapped
with the interior rows, and with the whole cycle (RCCL nodes included) captured as a hipGraph.

Covers: ncclGroupStart/Send/Recv/GroupEnd on the comm stream, the packed (scattered send list)
and direct (contiguous send run) send paths, the interior/boundary split around the join
event, and RCCL nodes inside hipGraph capture (V-cycles, residual histories, PCG).
"""
import ctypes as C
from dataclasses import replace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _self_plan(HostPlan, M, n_own, ghost_own_ids, square):
    """A plan of one part whose ghosts are copies of its own entries ``ghost_own_ids``; the
    entries of M that read one of them (its diagonal excepted: Jacobi finds a_ii by column id)
    go through the ghost slot."""
    g = np.asarray(ghost_own_ids, np.int64)
    rows = np.repeat(np.arange(M.nrows, dtype=np.int64), np.diff(M.rowptr))

    class SelfPlan(HostPlan):
        def localize(self, col):
            col = np.asarray(col, np.int64)
            out = col.copy()
            k = np.searchsorted(g, col)
            hit = (k < len(g)) & (g[np.minimum(k, len(g) - 1)] == col)
            if square:
                hit &= col != rows
            out[hit] = n_own + k[hit]
            return out.astype(np.int32)

    return SelfPlan(n_own=n_own, col0=0, ghost_ids=g, nbrs=[0], recv_counts=[len(g)],
                    send_counts=[len(g)], send_idx=g.copy())


def _pick(n, mode, rng):
    if n < 4:
        return np.zeros(0, np.int64)
    if mode == "stride":       # scattered: packed before the send
        return np.arange(1, n, 3, dtype=np.int64)
    if mode == "block":        # one contiguous run: sent straight from the vector
        return np.arange(n // 3, n // 3 + max(1, n // 4), dtype=np.int64)
    return np.unique(rng.integers(0, n, max(1, n // 5))).astype(np.int64)


def _selfify(H, HostPlan):
    rng = np.random.default_rng(7)
    modes = ["stride", "block", "random"]
    levels = []
    for l in range(H.nlevels):
        lp = H.levels[l][0]
        n = lp.A.nrows
        kw = {"planA": _self_plan(HostPlan, lp.A, n, _pick(n, modes[l % 3], rng), True)}
        if l < H.nlevels - 1:
            nc = H.levels[l + 1][0].A.nrows
            kw["planR"] = _self_plan(HostPlan, lp.R, n, _pick(n, modes[(l + 1) % 3], rng), False)
            kw["planP"] = _self_plan(HostPlan, lp.P, nc, _pick(nc, modes[(l + 2) % 3], rng), False)
        levels.append({0: replace(lp, **kw)})
    return replace(H, levels=levels)


def _run(kind, n, q):
    """The test body, in a fresh process that loads libpamg before anything imports torch, so
    libpamg's RCCL is /opt/rocm's 2.27.7 (in a process where torch came first it binds to the
    wheel's RCCL 2.26.6, which segfaults on this self-exchange: _lib.runtime_providers); a
    failure comes back as a message instead of ending the pytest run."""
    import os
    import sys
    import traceback
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        from parallel_amg_amd import _lib
        _lib.lib()
        assert "/torch/" not in _lib.runtime_providers().get("rccl", ""), _lib.runtime_providers()
        import parallel_amg_amd as pa
        from parallel_amg_amd._lib import call
        from parallel_amg_amd.hierarchy import HostPlan
        from parallel_amg_amd.partitioned import Context, PVector, mul
        from parallel_amg_amd.solver import AMGSolver

        ctx = Context(0)
        rccl_ctx = Context(0)
        uid = C.create_string_buffer(128)
        call("pamg_comm_unique_id", uid)
        call("pamg_comm_init", rccl_ctx.handle, 1, 0, uid.raw)

        be = pa.SequentialBackend(1)
        A, offs, xs = pa.generate_problem(be, kind, n)
        H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=40))
        assert H.nlevels >= 3
        Hs = _selfify(H, HostPlan)

        # reference: the plain single-part path (no communicator)
        S0 = AMGSolver(ctx, H, graph=False)
        xst0 = PVector(ctx, S0.A[0].n_own_cols, S0.A[0].n_ghost, xs[0])
        b0 = PVector(ctx, S0.A[0].nrows)
        mul(b0, S0.A[0], xst0)
        x0 = S0.new_vector()
        h0 = S0.vcycle(x0, b0, 3, res_hist=True)
        it0, ph0 = S0.pcg(S0.new_vector(), b0, rtol=1e-10, maxit=60)

        # consistent!(x) split (pamg_exchange_begin / _end) vs the synchronous exchange: same
        # ghost bits, with an SpMV of another vector overlapping the exchange in flight
        from parallel_amg_amd.partitioned import DevicePlan, consistent, consistent_async
        pl = Hs.levels[0][0].planA
        dp = DevicePlan(rccl_ctx, pl)
        own = np.random.default_rng(3).standard_normal(pl.n_own)
        va = PVector(rccl_ctx, pl.n_own, pl.n_ghost, own)
        vb = PVector(rccl_ctx, pl.n_own, pl.n_ghost, own)
        consistent(va, dp)
        S1 = AMGSolver(rccl_ctx, Hs, graph=False)
        u = PVector(rccl_ctx, S1.A[0].n_own_cols, S1.A[0].n_ghost, xs[0])
        yu = PVector(rccl_ctx, S1.A[0].nrows)
        t = consistent_async(vb, dp)
        mul(yu, S1.A[0], u)
        assert t.wait() is vb
        ga, gb = va.ghost_values(), vb.ghost_values()
        assert len(ga) == pl.n_ghost > 0 and np.array_equal(ga.view(np.int64), gb.view(np.int64))
        assert np.array_equal(ga, own[pl.send_idx])  # self-plan ghosts are copies of own entries
        assert np.array_equal(yu.own_values().view(np.int64), b0.own_values().view(np.int64))
        t2 = consistent_async(vb, dp)
        try:
            consistent_async(va, dp)  # one exchange in flight per plan
            raise AssertionError("second begin on a busy plan was accepted")
        except _lib.PamgError as e:
            assert e.code == -6, e
        t2.wait()
        del S1, u, yu
        for graph in (False, True):
            S = AMGSolver(rccl_ctx, Hs, graph=graph)
            assert S.A[0].n_ghost > 0 and S.R[0].n_ghost > 0
            # SpMV through the self-exchange (overlapped interior/boundary split)
            xst = PVector(rccl_ctx, S.A[0].n_own_cols, S.A[0].n_ghost, xs[0])
            b = PVector(rccl_ctx, S.A[0].nrows)
            mul(b, S.A[0], xst)
            assert np.array_equal(b.own_values().view(np.int64), b0.own_values().view(np.int64))
            x = S.new_vector()
            S.vcycle(x, b, 2)  # first call captures the graph (when enabled)
            S.vcycle(x, b, 1)
            h = S.vcycle(S.new_vector(), b, 3, res_hist=True)
            x3 = S.new_vector()
            S.vcycle(x3, b, 3)
            assert np.array_equal(x3.own_values().view(np.int64), x0.own_values().view(np.int64)), \
                f"graph={graph}: V-cycles through RCCL self-exchange differ from the plain path"
            np.testing.assert_allclose(h, h0, rtol=1e-12, atol=0)
            st = S.graph_state()
            assert st["captured"] == graph and not st["failed"], st
            it, ph = S.pcg(S.new_vector(), b, rtol=1e-10, maxit=60)
            assert it == it0
            np.testing.assert_allclose(ph, ph0, rtol=1e-9, atol=0)
            del S, xst, b, x, x3
        q.put("ok")
    except BaseException:
        q.put(traceback.format_exc())


@pytest.mark.parametrize("kind,n", [("poisson3d", 14), ("aniso3d", 12), ("poisson2d", 40)])
def test_rccl_self_exchange_vcycle_bits(built, kind, n):
    import multiprocessing as mp
    import queue
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_run, args=(kind, n, q))
    p.start()
    try:
        res = q.get(timeout=150)
    except queue.Empty:
        res = None
    p.join(timeout=60)
    assert res == "ok", res if res is not None else f"worker died (exit code {p.exitcode})"
