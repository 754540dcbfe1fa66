"""BASELINE.json configs at their stated sizes and part counts ("Next" item 1).

* configs[1] 3D 7-pt Poisson 128^3, one part: GPU setup + 6 V-cycles + PCG, bit-exact against
  the oracle's own setup and solve of the same 2,097,152-row problem.
* configs[3] anisotropic Poisson 256^3 as 4 parts: four processes on one GPU (host debug
  transport — RCCL refuses several ranks per device), distributed setup over gloo with GPU
  Galerkin products, 3 V-cycles; b, x and residual histories bit-exact / 1e-12 against the
  oracle's 4-part setup (SPEC §S7: same global operators, partitioned storage).
* configs[2] 3D 7-pt Poisson 512^3 as 8 parts: eight processes on one GPU (host transport),
  against the oracle's own 8-part setup of the same problem (round 6; ~2 min of oracle setup
  on the box's host threads): every part's rows of every level's A, P, R and its aggregates,
  level-0 SpMV / residual / Jacobi rows, and x after 3 V-cycles bit for bit; residual
  histories 1e-12; plus determinism and linearity (V(2b) = 2 V(b) bit for bit).

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


def _csr_digest(rowptr, col, val):
    """SHA-256 of a block of CSR rows: row lengths, global columns (int64), value bits."""
    h = hashlib.sha256()
    rp = np.asarray(rowptr, np.int64)
    h.update(np.diff(rp).tobytes())
    h.update(np.ascontiguousarray(col, np.int64).tobytes())
    h.update(np.ascontiguousarray(val, np.float64).tobytes())
    return h.hexdigest()


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
        out = {"nlevels": H.nlevels, "rep": int(S.rep_level), "levels": []}
        # this part's rows of every level's operators and its aggregates (global coarse ids)
        for l in range(H.nlevels):
            lp = H.levels[l][rank]
            rec = {"A": _csr_digest(lp.A.rowptr, lp.A.col, lp.A.val), "omega": float(lp.omega),
                   "whole": bool(lp.whole)}
            if l < H.nlevels - 1:
                rec["agg"] = np.asarray(lp.agg, np.int64)  # local aggregate numbers, -1 isolated
                rec["P"] = _csr_digest(lp.P.rowptr, lp.P.col, lp.P.val)
                rec["R"] = _csr_digest(lp.R.rowptr, lp.R.col, lp.R.val)
                rec["R_rows"] = int(lp.R.nrows)  # this part's aggregates
            out["levels"].append(rec)
        # level 0, the metric's operator: SpMV / residual / Jacobi rows of this part
        u = PVector(ctx, A0.n_own_cols, A0.n_ghost, xs[rank])
        y = PVector(ctx, A0.nrows)
        mul(y, A0, u)
        out["spmv"] = y.own_values()
        c = PVector(ctx, A0.nrows, 0, gen_xstar(r0, r1 - r0, SEED2))
        r = PVector(ctx, A0.nrows)
        residual(r, A0, u, c)
        out["resid"] = r.own_values()
        t = A0.new_input_vector()
        jacobi(u, A0, c, t, S.omega[0], 1)
        out["jacobi"] = u.own_values()
        del u, c, r, t
        # whole 8-part V-cycles from x = 0 on b = A x*: against the oracle's below; also
        # determinism and linearity (x 2 is exact)
        b = y
        x1, x2, x3 = S.new_vector(), S.new_vector(), S.new_vector()
        h1 = S.vcycle(x1, b, 3, res_hist=True)
        h2 = S.vcycle(x2, b, 3, res_hist=True)
        b2 = PVector(ctx, A0.nrows, 0, 2.0 * b.own_values())
        h3 = S.vcycle(x3, b2, 3, res_hist=True)
        v1, v2, v3 = x1.own_values(), x2.own_values(), x3.own_values()
        out["det"] = bool(np.array_equal(bits(v1), bits(v2)) and np.array_equal(h1, h2))
        out["lin"] = bool(np.array_equal(bits(2.0 * v1), bits(v3)) and np.array_equal(2.0 * h1, h3))
        out["x"] = v1
        out["hist"] = h1
        q.put((rank, "ok", out))
    except Exception:
        import traceback
        q.put((rank, traceback.format_exc(), None))
    finally:
        if dist is not None and dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.timeout(1500)
def test_config_poisson3d_512_eight_parts(built):
    """configs[2] at its size and part count, against the ORACLE: eight
    processes on one GPU (host transport) set 512^3 up distributed (8 z-slab parts, decoupled
    aggregation, agglomerated tail) and run 3 V-cycles; then the oracle sets the same problem up
    globally with the same 8-part partition (its own generator, aggregation, products; ~2 min on
    the box's host threads) and runs its V-cycles. Required, bit for bit: every part's rows of
    every level's A, P, R, its aggregates and omega; b = A x*, a residual and a Jacobi sweep on
    level 0; x after 3 cycles. Residual histories 1e-12 (norms reduce in another order)."""
    from oracle import oracle as O
    world, n = 8, 512
    procs, q = _run(_p512_worker, world, (n,))
    # the oracle's 8-part setup runs here while the ranks set up on the GPU
    say("oracle setup (8 parts, 134M rows)")
    Ao = O.generate("poisson3d", n, n, n)
    N = Ao.nrows
    offs = O.uniform_offsets(N, world)
    xs = O.xstar(N)
    bo = O.spmv(Ao, xs)
    co = O.xstar(N, 0, SEED2)
    ro = O.residual(Ao, xs, co)
    Ho = O.setup(Ao, nparts=world, max_coarse=1000, agglomerate=32768, fetch=False)
    say("oracle setup done")
    jo = O.jacobi(Ao, xs, co, Ho.omega[0])
    del Ao
    res = _collect(procs, q, world, timeout=1200)
    outs = [res[p][2] for p in range(world)]
    say("ranks done")
    assert all(o["nlevels"] == Ho.nlevels for o in outs), ([o["nlevels"] for o in outs], Ho.nlevels)
    for p, o in enumerate(outs):
        sl = slice(offs[p], offs[p + 1])
        for name, want in (("spmv", bo), ("resid", ro), ("jacobi", jo)):
            d = np.flatnonzero(bits(o[name]) != bits(want[sl]))
            assert d.size == 0, f"part {p}: {name} rows differ ({d.size} entries)"
    for l in range(Ho.nlevels):
        Al = Ho.csr(l, 0)
        lo = Ho.offsets[l]
        if l < Ho.nlevels - 1:
            Pl, Rl, agg = Ho.csr(l, 1), Ho.csr(l, 2), Ho.aggregates(l)
        for p, o in enumerate(outs):
            rec = o["levels"][l]
            assert bits(rec["omega"]) == bits(Ho.omega[l]), (p, l)
            # a level held whole (the agglomerated tail) is all of the oracle's rows on every part
            a, e = (0, Al.nrows) if rec["whole"] else (int(lo[p]), int(lo[p + 1]))
            assert rec["A"] == _csr_digest(Al.rowptr[a:e + 1], Al.col[Al.rowptr[a]:Al.rowptr[e]],
                                           Al.val[Al.rowptr[a]:Al.rowptr[e]]), f"part {p}: A{l} rows differ"
            if l == Ho.nlevels - 1:
                continue
            # the part's aggregates are numbered after those of the parts before it (SPEC §S7)
            c0 = 0 if rec["whole"] else sum(outs[q]["levels"][l]["R_rows"] for q in range(p))
            c1 = c0 + rec["R_rows"]
            assert np.array_equal(np.where(rec["agg"] >= 0, rec["agg"] + c0, -1), agg[a:e]), \
                f"part {p}: aggregates of level {l}"
            assert rec["P"] == _csr_digest(Pl.rowptr[a:e + 1], Pl.col[Pl.rowptr[a]:Pl.rowptr[e]],
                                           Pl.val[Pl.rowptr[a]:Pl.rowptr[e]]), f"part {p}: P{l} rows differ"
            assert c1 <= Rl.nrows, (p, l, c0, c1, Rl.nrows)
            assert rec["R"] == _csr_digest(Rl.rowptr[c0:c1 + 1], Rl.col[Rl.rowptr[c0]:Rl.rowptr[c1]],
                                           Rl.val[Rl.rowptr[c0]:Rl.rowptr[c1]]), f"part {p}: R{l} rows differ"
        del Al
        if l < Ho.nlevels - 1:
            del Pl, Rl, agg
    xo, ho = Ho.solve(bo, 3, res_hist=True)
    del Ho
    for p, o in enumerate(outs):
        sl = slice(offs[p], offs[p + 1])
        d = np.flatnonzero(bits(o["x"]) != bits(xo[sl]))
        assert d.size == 0, f"part {p}: x after 3 V-cycles differs from the oracle's ({d.size} entries)"
        assert o["det"], f"part {p}: two 8-part V-cycle runs differ"
        assert o["lin"], f"part {p}: V(2b) != 2 V(b)"
        np.testing.assert_allclose(o["hist"], ho, rtol=1e-12)
    assert np.all(np.diff(ho) < 0) and ho[-1] < 0.5 * ho[0]
