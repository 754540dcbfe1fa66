#!/usr/bin/env python3
"""bench.py — V-cycle throughput of the MI355X AMG solve path (BASELINE.json metric).

Workload (BASELINE.json configs[2] / metric line): 3D 7-point Poisson, 512^3 = 134,217,728
fp64 unknowns, smoothed-aggregation hierarchy (SPEC.md §S4), V(1,1) weighted-Jacobi cycles
(SPEC.md §S6). A "step" is one V-cycle over the whole (global) problem; with N GPUs the
grid is row-partitioned into N slabs (strong scaling: total work fixed) and each V-cycle
exchanges ghosts over RCCL.

    python bench.py [--gpus N --steps K --warmup W]          # N=1
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints ONE JSON line. Timed region: device sync + barrier, K V-cycles (hipGraph
replay), device sync + barrier; max over ranks. Inputs are resident in HBM. libpamg is loaded
before torch, and torch stays off the GPU (gloo rendezvous only): see _lib.runtime_providers.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "V-cycle iters/sec + fine-SpMV HBM GB/s, 3D Poisson 128M dofs at 1/2/4/8 GPU"
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md:36 (spec)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grid", type=int, default=512, help="grid points per side")
    ap.add_argument("--kind", default="poisson3d",
                    choices=["poisson2d", "poisson3d", "aniso3d", "elastic3d"])
    ap.add_argument("--matrix", default=None,
                    help="Matrix Market file (e.g. SuiteSparse Flan_1565.mtx) instead of --kind")
    ap.add_argument("--partition", choices=["uniform", "nnz"], default="uniform",
                    help="row partition of a --matrix over N GPUs (SPEC §S7)")
    ap.add_argument("--max-coarse", type=int, default=1000)
    ap.add_argument("--agglomerate", type=int, default=32768,
                    help="levels >= 1 with <= this many rows are one part, replicated (0: off)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu-baseline", choices=["auto", "off"], default="auto")
    ap.add_argument("--cpu-cycles", type=int, default=10,
                    help="V-cycles of the CPU baseline sample (~1 s each at 512^3 on 16 threads)")
    ap.add_argument("--transport", choices=["rccl", "host"], default="rccl",
                    help="host = debug transport (ranks may share one GPU; not a perf mode)")
    ap.add_argument("--sweeps", default="1,1", help="nu1,nu2 of the V(nu1,nu2) cycle (SPEC S6)")
    ap.add_argument("--set", action="append", default=[], metavar="KEY=VALUE",
                    help="libpamg tuning option for an A/B run (pamg_set_option; INTEGRATION.md table)")
    ap.add_argument("--value-dict", action="store_true",
                    help="opt-in per-tile 4-bit value dictionaries where a tile has <= 16 distinct "
                         "values (exact; not the default layout)")
    ap.add_argument("--setup", choices=["gpu", "host"], default="gpu",
                    help="where the Galerkin products of the setup run (same bits either way)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    # libpamg first: it then binds to /opt/rocm's HIP 7.2 / RCCL 2.27.7 rather than the copies
    # the torch wheel bundles (HIP 7.0 / RCCL 2.26.6, same sonames; _lib.runtime_providers).
    # torch is only the process-group rendezvous here (gloo, CPU): it never touches the GPU,
    # so libpamg's runtime is the only one driving the device (device sync = ctx.sync()).
    import parallel_amg_amd as pa
    from parallel_amg_amd import _lib
    from parallel_amg_amd.partitioned import Context, PVector, mul
    from parallel_amg_amd.solver import OPS, AMGSolver

    _lib.lib()  # fail loudly if libpamg.so is missing
    import torch
    import torch.distributed as dist

    _lib.call("pamg_set_option", b"value_dict", int(args.value_dict))
    for kv in args.set:
        k, v = kv.split("=")
        _lib.call("pamg_set_option", k.encode(), int(v))
    nd = ctypes.c_int()
    _lib.call("pamg_device_count", ctypes.byref(nd))
    dev = local % max(nd.value, 1)
    if world > 1:
        dist.init_process_group("gloo")  # host messages; the device exchange is libpamg's RCCL
        be = pa.DistributedBackend()
    else:
        be = pa.SequentialBackend(1)
    log(f"runtime: {_lib.runtime_providers()}")

    def barrier():
        if world > 1:
            dist.barrier()

    ctx = Context(dev, be, transport=args.transport)
    t0 = time.time()
    if args.matrix:
        A, offs, xs = pa.load_problem(be, args.matrix, partition=args.partition)
        workload = f"{os.path.basename(args.matrix)} ({int(offs[-1])} rows) fp64"
    else:
        A, offs, xs = pa.generate_problem(be, args.kind, args.grid)
        workload = f"{args.kind} {args.grid}^{2 if args.kind == 'poisson2d' else 3} fp64"
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=args.max_coarse, agglomerate=args.agglomerate), log=log,
                           device=ctx if args.setup == "gpu" else None)
    t_setup = time.time() - t0
    log(f"setup {t_setup:.1f}s ({args.setup} products), {H.nlevels} levels")

    # hipGraph replay on one part; multi-part cycles run eagerly (RCCL + host-side exchange)
    use_graph = (not args.no_graph) and (world == 1 or args.transport == "rccl")
    S = AMGSolver(ctx, H, part=rank, graph=use_graph)
    nu1, nu2 = (int(v) for v in args.sweeps.split(","))
    S.set_sweeps(nu1, nu2)
    A0 = S.A[0]
    xst = PVector(ctx, A0.n_own_cols, A0.n_ghost, xs[rank])
    b = PVector(ctx, A0.nrows)
    mul(b, A0, xst)
    x = S.new_vector()
    del xst
    t_upload = time.time() - t0 - t_setup
    log(f"upload {t_upload:.1f}s")

    # ---- multi-part graph self-check: graph replay (RCCL captured) and eager launches must
    # give the same bits on every rank, else the timed run uses eager launches
    if use_graph and world > 1:
        xa, xb = S.new_vector(), S.new_vector()
        S.vcycle(xa, b, 2)
        S.set_graph(False)
        S.vcycle(xb, b, 2)
        same = bool(np.array_equal(xa.own_values().view(np.int64), xb.own_values().view(np.int64)))
        ok = be.allreduce_max({rank: 0.0 if same else 1.0}) == 0.0
        S.set_graph(ok)
        del xa, xb
        log(f"multi-part graph self-check: {'ok' if ok else 'MISMATCH -> eager'}")

    # ---- warmup + timed region -------------------------------------------------------
    if args.warmup:
        S.vcycle(x, b, args.warmup)
    def device_sync():  # the context's streams, then hipDeviceSynchronize (every stream)
        ctx.sync()
        _lib.call("pamg_device_sync", dev)

    device_sync()
    barrier()
    ts = time.perf_counter()
    S.vcycle_async(x, b, args.steps)
    device_sync()
    barrier()
    te = time.perf_counter()
    dt = te - ts
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    vps = args.steps / dt

    # ---- per-kernel timing (HIP events on the compute stream, eager) ------------------
    kprof = max(3, min(args.steps, 10))
    prof = S.profile(x, b, kprof) / kprof          # ms per V-cycle per (level, op)
    # roofline numerator: SURVEY §8(d)'s algorithmic bytes (plain CSR, 32-bit indices: 12 B
    # per nonzero + row pointers + x once + y [+ b]); the uploaded layout streams fewer
    # (24-bit / dictionary columns, 8-bit row lengths), reported beside it as format bytes
    obytes = S.op_bytes("csr")                      # algorithmic bytes per (level, op)
    fbytes = S.op_bytes("format")                   # bytes the uploaded layout streams
    post_ms = float(prof[0, 4]) / nu2 if S.L > 1 else float(prof[0, 5])  # one sweep
    post_bytes = float(obytes[0, 4]) if S.L > 1 else float(obytes[0, 5])
    post_fbytes = float(fbytes[0, 4]) if S.L > 1 else float(fbytes[0, 5])
    achieved = post_bytes / (post_ms * 1e-3) / 1e9
    spmv_ms = ctypes_bench_spmv(ctx, A0, x, S)
    spmv_bytes = S.csr_bytes(A0, 0)
    spmv_gbps = spmv_bytes / (spmv_ms * 1e-3) / 1e9
    hist = S.vcycle(x, b, 1, res_hist=True)

    levels = [{"rows": int(H.levels[l][rank].A.nrows), "nnz": int(H.levels[l][rank].A.nnz),
               "ms": {op: round(float(prof[l, k]), 4) for k, op in enumerate(OPS) if prof[l, k] > 0}}
              for l in range(S.L)]
    if rank == 0:
        log(json.dumps({"levels": levels}))

    # ---- CPU baseline: the oracle V-cycle on this same hierarchy (rank 0, N=1) --------
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        cpu = cpu_baseline(H, xs[0], args.cpu_cycles, log, (nu1, nu2))

    # HBM traffic of the dominant kernel from the committed rocprofv3 PMC passes of this exact
    # workload (tools/pmc_traffic.py; counters cannot be read from inside the process)
    # (only when the record was measured on the same column layout as this run)
    lay = _lib.layout_of(A0)
    c24, vd, rl8, cd, tm = lay["c24"], lay["vd"], lay["rl8"], lay["cd"], lay["tm"]
    tn = lay["tile_nnz"]
    kname = (f"k_rows_tm<2, {tn}, {cd}, false>" if tm
             else f"k_rows_tile2<2, {tn}, 256, false, false, 256, false, false, true, {cd}>" if cd
             else f"k_rows_tile2<2, {tn}, 256, false, false, 256, true, true>" if vd
             else f"k_rows_tile2<2, {tn}, 256, false, false, 256, true, false, true>" if rl8
             else f"k_rows_tile2<2, {tn}, 256, false, false, 256, true>" if c24
             else f"k_rows_tile2<2, {tn}, 256, false, false>")
    traffic, traffic_src = None, None
    pmc = os.path.join(ROOT, "profiles", "r01_pmc", "traffic_jacobi_512.json")
    if (not args.matrix and args.kind == "poisson3d" and args.grid == 512 and world == 1
            and os.path.exists(pmc)):
        rec = [r for r in json.load(open(pmc)) if r["kernel"] == kname]
        if rec:
            traffic, traffic_src = float(rec[0]["traffic_bytes"]), os.path.relpath(pmc, ROOT)
    # the fine SpMV's HBM rate from its committed PMC record (same workload and layout)
    spmv_traffic_gbps = None
    pmc_s = os.path.join(ROOT, "profiles", "r01_pmc", "traffic_spmv_512.json")
    if (not args.matrix and args.kind == "poisson3d" and args.grid == 512 and world == 1
            and os.path.exists(pmc_s)):
        sname = kname.replace("<2,", "<0,", 1)
        rec = [r for r in json.load(open(pmc_s)) if r["kernel"] == sname]
        if rec:
            spmv_traffic_gbps = round(float(rec[0]["traffic_bytes"]) / (spmv_ms * 1e-3) / 1e9, 1)

    # fine-level nonzeros of the whole problem (every rank holds only its own rows)
    nnz_fine = (sum(be.allgather({rank: int(H.levels[0][rank].A.nnz)})) if world > 1
                else int(sum(H.levels[0][p].A.nnz for p in H.levels[0])))
    if rank == 0:
        gl_rows = int(H.offsets(0)[-1])
        out = {
            "metric": METRIC,
            "value": round(vps, 4),
            "unit": "V-cycles/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SPEC.md §S2 grid operator, b = A x*, x0 = 0)",
            "config": {
                "workload": f"{workload}, SA-AMG V({nu1},{nu2}) weighted-Jacobi, "
                            f"{world} part(s)",
                "n": gl_rows, "nnz_fine": int(nnz_fine), "levels": S.L, "max_coarse": args.max_coarse,
                "parallelism": f"row-slab partition p{world}" + (
                    "" if world == 1 else " (RCCL ghost exchange)" if args.transport == "rccl"
                    else " (host debug transport)"),
                "graph": S.graph_state(),
                "transport": args.transport if world > 1 else None,
                # levels >= this one are held whole on every rank (SPEC §S7 agglomeration)
                "replicated_from_level": int(S.rep_level) if world > 1 else None,
                "value_dict": bool(args.value_dict),
                "options": list(args.set),
            },
            "fine_spmv_GBps": round(spmv_gbps, 1),
            "fine_spmv_frac": round(spmv_gbps / HBM_PEAK_GBPS, 4),
            # HBM bytes actually moved (PMC, profiles/r01_pmc) per second of the same launch
            "fine_spmv_traffic_GBps": spmv_traffic_gbps,
            "roofline": {
                "kernel": kname + " (level-0 post-smoothing Jacobi"
                          + (", tile-major slots" if tm else "")
                          + (f", {cd}-bit column dictionary" if cd else "")
                          + (", value dictionaries" if vd else "")
                          + (", 24-bit column stream" if c24 and not cd else "")
                          + (", 8-bit row lengths)" if rl8 else ")"),
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic, "traffic_source": traffic_src,
                "bytes_per_launch": int(post_bytes), "bytes_model": "SURVEY 8(d) CSR (12 B/nnz)",
                "format_bytes_per_launch": int(post_fbytes),
                "format_GBps": round(post_fbytes / (post_ms * 1e-3) / 1e9, 1),
                "ms_per_launch": round(post_ms, 4),
            },
            "cpu_baseline": cpu,
            "setup_s": round(t_setup, 1),
            "setup_products": args.setup,
            "final_residual": float(hist[0]),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def ctypes_bench_spmv(ctx, A0, x, S, reps=20) -> float:
    import ctypes as C

    from parallel_amg_amd._lib import call
    from parallel_amg_amd.partitioned import PVector
    y = PVector(ctx, A0.nrows)
    ms = C.c_double()
    call("pamg_bench_rowop", ctx.handle, A0.handle, 0, x.handle, None, y.handle, 0.0, reps,
         C.byref(ms))
    return ms.value


def cpu_baseline(H, xstar, ncycles, log, sweeps=(1, 1)):
    """Time the CPU oracle's V-cycle (oracle/pamg_oracle.c, OpenMP) on the same hierarchy."""
    from oracle import oracle as O
    lv = [H.levels[l][0] for l in range(H.nlevels)]
    Ho = O.hierarchy_from_levels([p.A for p in lv], [p.P for p in lv[:-1]], [p.R for p in lv[:-1]],
                                 [p.omega for p in lv], H.ainv)
    Ho.set_sweeps(*sweeps)
    A0 = lv[0].A
    x = np.zeros(A0.nrows)
    rhs = np.ascontiguousarray(xstar)  # any rhs: the cycle's work does not depend on values
    t = time.perf_counter()
    O.lib().orc_solve(Ho._h, x, rhs, ncycles, None)
    dt = time.perf_counter() - t
    cores = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    log(f"cpu baseline: {ncycles} V-cycle(s) in {dt:.2f}s on {cores} threads")
    return {"value": round(ncycles / dt, 5), "unit": "V-cycles/s", "cores": cores, "kind": "port",
            "sample": f"{ncycles} full V-cycle(s) of the same {A0.nrows}-row hierarchy by the C "
                      f"oracle (oracle/pamg_oracle.c, OpenMP, int64 indices); reference "
                      f"(Julia/PartitionedArrays) not runnable: no code in /root/reference"}


if __name__ == "__main__":
    main()
