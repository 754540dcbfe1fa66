"""BASELINE.json configs at their stated sizes and part counts ("Next" item 1).

* configs[1] 3D 7-pt Poisson 128^3, one part: GPU setup + 6 V-cycles + PCG, bit-exact against
  the oracle's own setup and solve of the same 2,097,152-row problem.
* configs[3] anisotropic Poisson 256^3 as 4 parts: four processes on one GPU (host debug
  transport — RCCL refuses several ranks per device), distributed setup over gloo with GPU
  Galerkin products, 3 V-cycles; b, x and residual histories bit-exact / 1e-12 against the
  oracle's 4-part setup (SPEC §S7: same global operators, partitioned storage).
* configs[2] 3D 7-pt Poisson 512^3 as 8 parts: eight processes on one GPU (host transport).
  Level 0: every part's SpMV, residual and Jacobi rows are bit-identical to the one-part run
  of the same global operator (compared by SHA-256 of the row bits). Whole 8-part V-cycles
  (5 levels + agglomerated tail): deterministic (two runs, same bits), linear (V(2b) = 2 V(b)
  bit for bit: scaling by 2 is exact), and the residual falls every cycle. No oracle runs
  at this size (its setup would take ~10 min); the 8-part operators' parity at small sizes is
  tests/test_gpu_multipart.py.

Configs[4] (SuiteSparse Flan_1565) is not in the image (no network); its stand-in is
elastic3d, with and without a random renumbering (test_gpu_parity.py::test_vcycle_permuted_*).
"""
import hashlib
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

import parallel_amg_amd as pa
from parallel_amg_amd.partitioned import PVector, mul
from parallel_amg_amd.solver import AMGSolver

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(np.asarray(a, np.float64)).tobytes()).hexdigest()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def say(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------- configs[1]: 128^3, one part
def test_config_poisson3d_128_one_part(ctx):
    from oracle import oracle as O
    kind, n, mc = "poisson3d", 128, 1000
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, kind, n)
    assert A[0].nrows == 2_097_152 and A[0].nnz == 14_581_760
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=mc), device=ctx)
    S = AMGSolver(ctx, H)
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    Ao = O.generate(kind, n, n, n)
    bo = O.spmv(Ao, O.xstar(Ao.nrows))
    assert np.array_equal(bits(b.own_values()), bits(bo))
    Ho = O.setup(Ao, max_coarse=mc)
    assert Ho.nlevels == H.nlevels
    xo, ho = Ho.solve(bo, 6, res_hist=True)
    x = S.new_vector()
    hist = S.vcycle(x, b, 6, res_hist=True)
    assert np.array_equal(bits(x.own_values()), bits(xo))
    np.testing.assert_allclose(hist, ho, rtol=1e-12)
    # time-to-solution path (SPEC §S8): same iteration count as the oracle's PCG
    _xo, ko, hpo = Ho.pcg(bo, 1e-8, 60)
    k, hp = S.pcg(S.new_vector(), b, 1e-8, 60)
    assert k == ko and hp[-1] <= 1e-8 * hp[0]
    np.testing.assert_allclose(hp, hpo, rtol=1e-6)


# ------------------------------------------------------------ multi-process workers (spawn)
def _setup_worker(rank, world, port):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), OMP_NUM_THREADS="4")
    from parallel_amg_amd import _lib
    _lib.lib()  # before torch: /opt/rocm's HIP/RCCL (see _lib.runtime_providers)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _aniso_worker(rank, world, port, n, mc, agg, ncycles, q):
    dist = None
    try:
        dist = _setup_worker(rank, world, port)
        from parallel_amg_amd._lib import call
        from parallel_amg_amd.partitioned import Context
        call("pamg_set_option", b"poison_ghosts", 1)  # ghosts are NaN until their exchange lands
        be = pa.DistributedBackend()
        A, offs, xs = pa.generate_problem(be, "aniso3d", n)
        ctx = Context(0, be, transport="host")
        H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=mc, agglomerate=agg), device=ctx)
        S = AMGSolver(ctx, H, part=rank)
        A0 = S.A[0]
        b = PVector(ctx, A0.nrows)
        mul(b, A0, PVector(ctx, A0.n_own_cols, A0.n_ghost, xs[rank]))
        x = S.new_vector()
        hist = S.vcycle(x, b, ncycles, res_hist=True)
        q.put((rank, "ok", b.own_values(), x.own_values(), hist, H.nlevels))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None, None, None, None))
    finally:
        if dist is not None and dist.is_initialized():
            dist.destroy_process_group()


def _run(target, world, args, timeout=600):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    return procs, q


def _collect(procs, q, world, timeout=600):
    res = {}
    t0 = time.time()
    while len(res) < world:
        left = timeout - (time.time() - t0)
        if left <= 0:
            break
        r = q.get(timeout=left)
        res[r[0]] = r
    for p in procs:
        p.join(timeout=60)
    for p in procs:
        if p.is_alive():
            p.kill()
    errs = [f"rank {r}: {res[r][1]}" for r in res if res[r][1] != "ok"]
    assert len(res) == world and not errs, "\n".join(errs) or f"only {sorted(res)} answered"
    return res


# --------------------------------------------------------- configs[3]: aniso 256^3, 4 parts
def test_config_aniso3d_256_four_parts(built):
    from oracle import oracle as O
    world, n, mc, agg, ncycles = 4, 256, 1000, 32768, 3
    procs, q = _run(_aniso_worker, world, (n, mc, agg, ncycles))
    # the oracle's 4-part setup runs here while the ranks set up on the GPU
    say("oracle setup (4 parts, 16.8M rows)")
    Ao = O.generate("aniso3d", n, n, n)
    bo = O.spmv(Ao, O.xstar(Ao.nrows))
    Ho = O.setup(Ao, nparts=world, max_coarse=mc, agglomerate=agg)
    xo, ho = Ho.solve(bo, ncycles, res_hist=True)
    say("oracle done")
    res = _collect(procs, q, world)
    assert all(res[r][5] == Ho.nlevels for r in range(world))
    b = np.concatenate([res[r][2] for r in range(world)])
    x = np.concatenate([res[r][3] for r in range(world)])
    assert np.array_equal(bits(b), bits(bo))
    assert np.array_equal(bits(x), bits(xo))
    for r in range(world):
        np.testing.assert_allclose(res[r][4], ho, rtol=1e-12)
    assert ho[-1] < ho[0]


# ------------------------------------------------------ configs[2]: Poisson 512^3, 8 parts
SEED2 = 977


def _p512_worker(rank, world, port, n, q):
    dist = None
    try:
        dist = _setup_worker(rank, world, port)
        from parallel_amg_amd.hcsr import gen_xstar
        from parallel_amg_amd.partitioned import Context, jacobi, residual
        be = pa.DistributedBackend()
        A, offs, xs = pa.generate_problem(be, "poisson3d", n)
        ctx = Context(0, be, transport="host")
        H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000, agglomerate=32768), device=ctx)
        del A
        S = AMGSolver(ctx, H, part=rank)
        A0 = S.A[0]
        r0, r1 = int(offs[rank]), int(offs[rank + 1])
        out = {"nlevels": H.nlevels, "rep": int(S.rep_level)}
        # level 0, the metric's operator: SpMV / residual / Jacobi rows of this part
        u = PVector(ctx, A0.n_own_cols, A0.n_ghost, xs[rank])
        y = PVector(ctx, A0.nrows)
        mul(y, A0, u)
        out["spmv"] = digest(y.own_values())
        c = PVector(ctx, A0.nrows, 0, gen_xstar(r0, r1 - r0, SEED2))
        r = PVector(ctx, A0.nrows)
        residual(r, A0, u, c)
        out["resid"] = digest(r.own_values())
        t = A0.new_input_vector()
        jacobi(u, A0, c, t, S.omega[0], 1)
        out["jacobi"] = digest(u.own_values())
        # whole 8-part V-cycles: determinism, linearity (x 2 exact), falling residuals
        b = y
        x1, x2, x3 = S.new_vector(), S.new_vector(), S.new_vector()
        h1 = S.vcycle(x1, b, 3, res_hist=True)
        h2 = S.vcycle(x2, b, 3, res_hist=True)
        b2 = PVector(ctx, A0.nrows, 0, 2.0 * b.own_values())
        h3 = S.vcycle(x3, b2, 3, res_hist=True)
        v1, v2, v3 = x1.own_values(), x2.own_values(), x3.own_values()
        out["det"] = bool(np.array_equal(bits(v1), bits(v2)) and np.array_equal(h1, h2))
        out["lin"] = bool(np.array_equal(bits(2.0 * v1), bits(v3)) and np.array_equal(2.0 * h1, h3))
        out["hist"] = h1
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None))
    finally:
        if dist is not None and dist.is_initialized():
            dist.destroy_process_group()


def test_config_poisson3d_512_eight_parts(ctx):
    from parallel_amg_amd.hcsr import gen_xstar
    from parallel_amg_amd.partitioned import PSparseMatrix, jacobi, residual
    world, n = 8, 512
    procs, q = _run(_p512_worker, world, (n,))
    # the one-part level-0 rows of the same global operator, on this process's context
    say("one-part 512^3 level 0")
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, "poisson3d", n)
    N = A[0].nrows
    D = PSparseMatrix(ctx, A[0])
    from parallel_amg_amd.hcsr import gershgorin
    rho = gershgorin(A[0], 0)
    omega = 4.0 / (3.0 * rho)
    del A
    u = PVector(ctx, N, 0, xs[0])
    y = PVector(ctx, N)
    mul(y, D, u)
    yv = y.own_values()
    c = PVector(ctx, N, 0, gen_xstar(0, N, SEED2))
    r = PVector(ctx, N)
    residual(r, D, u, c)
    rv = r.own_values()
    del r
    t = PVector(ctx, N)
    jacobi(u, D, c, t, omega, 1)
    jv = u.own_values()
    del D, u, y, c, t
    say("one-part done")
    parts = [(N * p) // world for p in range(world + 1)]
    res = _collect(procs, q, world, timeout=900)
    outs = [res[p][2] for p in range(world)]
    assert len({o["nlevels"] for o in outs}) == 1 and outs[0]["nlevels"] >= 5
    for p, o in enumerate(outs):
        sl = slice(parts[p], parts[p + 1])
        assert o["spmv"] == digest(yv[sl]), f"part {p}: SpMV rows differ from the one-part run"
        assert o["resid"] == digest(rv[sl]), f"part {p}: residual rows differ"
        assert o["jacobi"] == digest(jv[sl]), f"part {p}: Jacobi rows differ"
        assert o["det"], f"part {p}: two 8-part V-cycle runs differ"
        assert o["lin"], f"part {p}: V(2b) != 2 V(b)"
        np.testing.assert_allclose(o["hist"], outs[0]["hist"], rtol=1e-12)
    h = outs[0]["hist"]
    assert np.all(np.diff(h) < 0) and h[-1] < 0.5 * h[0]
