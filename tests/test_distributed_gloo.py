"""N>1 path on CPU: the distributed host setup (DistributedBackend over gloo, one part per
process) must produce, part for part, exactly the hierarchy of the global-view oracle with
the same partition (SPEC §S7), and the same exchange plans as the in-process backend."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, kind, n, max_coarse, agglomerate, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    import torch.distributed as dist

    import parallel_amg_amd as pa
    from oracle import oracle as O
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        be = pa.DistributedBackend()
        A, offs, xs = pa.generate_problem(be, kind, n)
        prm = pa.SAParams(max_coarse=max_coarse, agglomerate=agglomerate)
        H = pa.build_hierarchy(be, A, offs, prm)
        Ao = O.generate(kind, *O.grid_shape(kind, n))
        Ho = O.setup(Ao, nparts=world, max_coarse=max_coarse, agglomerate=agglomerate)
        bits = lambda a: np.asarray(a, np.float64).view(np.int64)
        assert H.nlevels == Ho.nlevels, (H.nlevels, Ho.nlevels)
        # same plans as the in-process (debug) backend
        Hs = pa.build_hierarchy(pa.SequentialBackend(world), *pa.generate_problem(pa.SequentialBackend(world), kind, n)[:2],
                                prm)
        for l in range(H.nlevels):
            lp = H.levels[l][rank]
            o = Ho.offsets[l]
            # agglomerated (whole) levels: every rank holds all rows
            a, b = (0, int(o[-1])) if lp.whole else (int(o[rank]), int(o[rank + 1]))
            assert np.array_equal(lp.offsets, o)
            Ar = Ho.A[l]
            sl = slice(Ar.rowptr[a], Ar.rowptr[b])
            assert np.array_equal(lp.A.rowptr, Ar.rowptr[a:b + 1] - Ar.rowptr[a])
            assert np.array_equal(lp.A.col, Ar.col[sl]) and np.array_equal(bits(lp.A.val), bits(Ar.val[sl]))
            assert lp.omega == Ho.omega[l]
            ps = Hs.levels[l][rank]
            for pl, pq in ((lp.planA, ps.planA), (lp.planP, ps.planP), (lp.planR, ps.planR)):
                if pl is None:
                    continue
                assert pl.nbrs == pq.nbrs and pl.recv_counts == pq.recv_counts and pl.send_counts == pq.send_counts
                assert np.array_equal(pl.ghost_ids, pq.ghost_ids) and np.array_equal(pl.send_idx, pq.send_idx)
            if l < H.nlevels - 1:
                Pr = Ho.P[l]
                sl = slice(Pr.rowptr[a], Pr.rowptr[b])
                assert np.array_equal(lp.P.col, Pr.col[sl]) and np.array_equal(bits(lp.P.val), bits(Pr.val[sl]))
                co = H.rep_offsets if l + 1 == H.rep_level else Ho.offsets[l + 1]
                ca, cb = (0, int(co[-1])) if lp.whole else (int(co[rank]), int(co[rank + 1]))
                Rr = Ho.R[l]
                sl = slice(Rr.rowptr[ca], Rr.rowptr[cb])
                assert np.array_equal(lp.R.col, Rr.col[sl]) and np.array_equal(bits(lp.R.val), bits(Rr.val[sl]))
                assert np.array_equal(np.where(lp.agg >= 0, lp.agg + ca, -1), Ho.agg[l][a:b])
        assert np.array_equal(bits(H.ainv), bits(Ho.ainv.T.reshape(-1)))
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("world,kind,n,max_coarse,agglomerate", [
    (2, "poisson2d", 48, 100, 0),     # BASELINE.json configs[0] shape (2 parts on CPU), reduced
    (2, "poisson2d", 48, 100, 32768),
    (2, "poisson3d", 14, 60, 0),
    (3, "aniso3d", 12, 80, 0),
    (3, "aniso3d", 12, 80, 200),      # agglomerated from level 2 on
])
def test_distributed_setup_matches_oracle(world, kind, n, max_coarse, agglomerate, built):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, n, max_coarse, agglomerate, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res.get(r) == "ok", res.get(r)


def _rcm_worker(rank, world, port, path, q):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="1")
    import torch.distributed as dist

    import parallel_amg_amd as pa
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        be = pa.DistributedBackend()
        A, offs, xs = pa.load_problem(be, path, partition="rcm")
        # the in-process path (whole matrix, renumbered once, split) gives the same parts
        As, offs_s, xs_s = pa.load_problem(pa.SequentialBackend(world), path, partition="rcm")
        assert np.array_equal(offs, offs_s)
        a, s = A[rank], As[rank]
        assert np.array_equal(a.rowptr, s.rowptr) and np.array_equal(a.col, s.col)
        assert np.array_equal(a.val.view(np.int64), s.val.view(np.int64))
        assert np.array_equal(xs[rank], xs_s[rank])
        q.put((rank, "ok"))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_rcm_partition_reads_only_own_rows(tmp_path, built):
    """partition="rcm" over gloo: rank 0 computes the reverse Cuthill-McKee order
    and the nnz-balanced blocks, broadcasts them, and every rank reads only its block's rows
    (pamg_read_mtx_rows) — the same parts as renumbering the whole matrix in one process."""
    import scipy.io
    import scipy.sparse as sp
    rng = np.random.default_rng(4)
    n = 900
    G = sp.random(n, n, density=0.006, random_state=5, format="csr")
    M = (G + G.T + sp.identity(n) * 10.0).tocoo()
    path = str(tmp_path / "r.mtx")
    scipy.io.mmwrite(path, M, symmetry="symmetric")
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rcm_worker, args=(r, world, port, path, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert res.get(r) == "ok", res.get(r)
