"""Hierarchy dump/load (SURVEY §5 checkpoint/resume): a saved and reloaded hierarchy equals the
original array for array (every level, part, plan; agglomerated tails too), and on the GPU
the reloaded one runs the same V-cycles bit for bit."""
import numpy as np
import pytest

import parallel_amg_amd as pa


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def same_csr(A, B):
    if A is None or B is None:
        assert A is None and B is None
        return
    assert A.ncols == B.ncols and np.array_equal(A.rowptr, B.rowptr) and np.array_equal(A.col, B.col)
    assert np.array_equal(bits(A.val), bits(B.val))


def same_plan(P, Q):
    if P is None or Q is None:
        assert P is None and Q is None
        return
    assert (P.n_own, P.col0, P.nbrs, P.recv_counts, P.send_counts) == (Q.n_own, Q.col0, Q.nbrs, Q.recv_counts, Q.send_counts)
    assert np.array_equal(P.ghost_ids, Q.ghost_ids) and np.array_equal(P.send_idx, Q.send_idx)
    assert P._recv == Q._recv and sorted(P._send) == sorted(Q._send)
    for q in P._send:
        assert np.array_equal(P._send[q], Q._send[q])


@pytest.mark.parametrize("kind,n,nparts,agglomerate", [("poisson3d", 14, 1, 32768), ("aniso3d", 12, 3, 0),
                                                       ("poisson2d", 48, 2, 400)])
def test_roundtrip(tmp_path, built, kind, n, nparts, agglomerate):
    be = pa.SequentialBackend(nparts)
    A, offs, _ = pa.generate_problem(be, kind, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=50, agglomerate=agglomerate))
    path = str(tmp_path / "h.npz")
    pa.save_hierarchy(H, path)
    G = pa.load_hierarchy(path)
    assert (G.nparts, G.nlevels, G.n_coarse, G.rep_level) == (H.nparts, H.nlevels, H.n_coarse, H.rep_level)
    assert np.array_equal(G.rep_offsets, H.rep_offsets) and np.array_equal(bits(G.ainv), bits(H.ainv))
    for l in range(H.nlevels):
        for p in range(nparts):
            a, b = H.levels[l][p], G.levels[l][p]
            assert np.array_equal(a.offsets, b.offsets)
            assert (a.omega, a.rho, a.whole) == (b.omega, b.rho, b.whole)
            assert (a.agg is None) == (b.agg is None) and (a.agg is None or np.array_equal(a.agg, b.agg))
            for w in "APR":
                same_csr(getattr(a, w), getattr(b, w))
            for w in ("planA", "planP", "planR"):
                same_plan(getattr(a, w), getattr(b, w))


@pytest.mark.gpu
def test_reloaded_hierarchy_solves_identically(tmp_path, ctx):
    from parallel_amg_amd.partitioned import PVector, mul
    from parallel_amg_amd.solver import AMGSolver
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", 20)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=100), device=ctx)
    path = str(tmp_path / "h.npz")
    pa.save_hierarchy(H, path)
    out = []
    for h in (H, pa.load_hierarchy(path)):
        S = AMGSolver(ctx, h)
        b = PVector(ctx, S.A[0].nrows)
        mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
        x = S.new_vector()
        S.vcycle(x, b, 5)
        out.append(x.own_values())
    assert np.array_equal(bits(out[0]), bits(out[1]))


def _ckpt_worker(rank, world, port, path, q):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import parallel_amg_amd as pa
        be = pa.DistributedBackend()
        A, offs, _ = pa.generate_problem(be, "poisson3d", 12)
        H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=40))
        try:  # a partial hierarchy needs the {rank} placeholder
            pa.save_hierarchy(H, path.replace("{rank}", "shared"))
            raise AssertionError("saved a partial hierarchy to a shared path")
        except ValueError:
            pass
        pa.save_hierarchy(H, path)
        dist.barrier()
        G = pa.load_hierarchy(path, backend=be)
        assert sorted(G.levels[0]) == [rank] and G.nlevels == H.nlevels
        for l in range(H.nlevels):
            same_csr(H.levels[l][rank].A, G.levels[l][rank].A)
            same_plan(H.levels[l][rank].planA, G.levels[l][rank].planA)
        other = pa.SequentialBackend(world)  # holds every part: the file of one rank must not load
        try:
            pa.load_hierarchy(path, backend=other)
            raise AssertionError("loaded one rank's file for all parts")
        except ValueError:
            pass
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_distributed_roundtrip_one_file_per_rank(tmp_path, built):
    """DistributedBackend (gloo, 2 ranks): each rank saves its own part under a '{rank}' path and
    loads it back; a shared path or a mismatching backend is refused."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "h_{rank}.npz")
    procs = [ctx.Process(target=_ckpt_worker, args=(r, 2, port, path, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
    assert sorted(f.name for f in tmp_path.iterdir()) == ["h_0.npz", "h_1.npz"]
