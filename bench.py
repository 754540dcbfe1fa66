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
    ap.add_argument("--samples", type=int, default=5,
                    help="timed regions of exactly --steps V-cycles each; value = the median")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grid", type=int, default=512, help="grid points per side")
    ap.add_argument("--kind", default="poisson3d",
                    choices=["poisson2d", "poisson3d", "aniso3d", "elastic3d"])
    ap.add_argument("--matrix", default=None,
                    help="Matrix Market file (e.g. SuiteSparse Flan_1565.mtx) instead of --kind")
    ap.add_argument("--partition", choices=["uniform", "nnz", "rcm"], default="uniform",
                    help="row partition of a --matrix over N GPUs (SPEC §S7; rcm: graph partitioner = "
                         "reverse Cuthill-McKee renumbering + nnz-balanced blocks)")
    ap.add_argument("--rcm", action="store_true",
                    help="renumber a generated (and --permute'd) problem with the graph partitioner before "
                         "the nnz-balanced split")
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
    ap.add_argument("--value-dict", type=int, choices=[0, 1], default=1,
                    help="per-tile 4-bit value dictionaries where a tile has <= 16 distinct values (1, the "
                         "library default) or never (0)")
    ap.add_argument("--setup", choices=["gpu", "host"], default="gpu",
                    help="where the Galerkin products of the setup run (same bits either way)")
    ap.add_argument("--permute", type=int, default=None, metavar="SEED",
                    help="apply a seeded random symmetric permutation to the problem before setup "
                         "(destroys the grid numbering, as an FE mesh ordering would; 1 part only)")
    ap.add_argument("--reorder", choices=["auto", "off", "on", "agg"], default="auto",
                    help="locality permutation of the level operators inside the device layout "
                         "(AMGSolver reorder; one part; bits unchanged)")
    ap.add_argument("--pmc", choices=["auto", "committed", "off"], default="auto",
                    help="HBM traffic of the dominant kernel and the fine SpMV: auto = two rocprofv3 --pmc "
                         "passes (FETCH_SIZE, WRITE_SIZE) over tools/kbench.py's launches of the same "
                         "kernels on the same operator, run as child processes before this process touches "
                         "the GPU (N = 1, generated problems); committed = the records in profiles/pmc/ only")
    ap.add_argument("--pcg-rtol", type=float, default=1e-8,
                    help="time-to-solution leg: PCG with the V-cycle preconditioner to this "
                         "relative residual from x = 0 (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # counters first: the profiled child runs start before this process makes any HIP call
    live_pmc = None
    if args.pmc == "auto" and world == 1 and not args.matrix and args.permute is None and not args.rcm:
        live_pmc = pmc_live(args)

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
    if args.permute is not None or args.rcm:
        if args.matrix:
            raise SystemExit("--permute / --rcm: generated problems only (use --partition rcm for --matrix)")
        if world > 1:  # every rank builds the whole problem, reorders it identically, keeps its block
            A, offs, xs = pa.generate_problem(pa.SequentialBackend(1), args.kind, args.grid)
        if args.permute is not None:
            A, xs = pa.permute_problem(A, xs, args.permute)
            workload += f", randomly permuted (seed {args.permute})"
        if args.rcm:
            A, xs, _perm = pa.rcm_problem(A, xs)
            workload += ", RCM-renumbered"
        if world > 1 or args.rcm:
            A, offs, xs = pa.split_problem(be, A, xs, "nnz")
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=args.max_coarse, agglomerate=args.agglomerate), log=log,
                           device=ctx if args.setup == "gpu" else None)
    t_setup = time.time() - t0
    log(f"setup {t_setup:.1f}s ({args.setup} products), {H.nlevels} levels")

    # hipGraph replay on one part; multi-part cycles run eagerly (RCCL + host-side exchange)
    use_graph = (not args.no_graph) and (world == 1 or args.transport == "rccl")
    S = AMGSolver(ctx, H, part=rank, graph=use_graph, reorder=args.reorder if world == 1 else "off")
    if S.reordered:
        log(f"locality permutation on levels {S.reordered} (mean row span before/after: "
            f"{[S.span[l] for l in S.reordered]})")
    nu1, nu2 = (int(v) for v in args.sweeps.split(","))
    S.set_sweeps(nu1, nu2)
    A0 = S.A_dev[0]  # the hierarchy's own level-0 operator (device numbering where permuted)
    Af = S.fine_operator()  # the caller's numbering (b = A x* as the caller forms it)
    xst = PVector(ctx, Af.n_own_cols, Af.n_ghost, xs[rank])
    b = PVector(ctx, Af.nrows)
    mul(b, Af, xst)
    x = S.new_vector()
    del xst, Af
    t_upload = time.time() - t0 - t_setup
    log(f"upload {t_upload:.1f}s")

    # ---- multi-part graph self-check: graph replay (RCCL captured) and eager launches must
    # give the same bits on every rank. A mismatch would be a defect of the captured multi-rank
    # cycle: every rank then drops the graphs and the timed cycles run eagerly (the launches
    # the graphs would replay, issued one by one), and the line says so (graph_mismatch_ranks).
    graph_mismatch = None
    if use_graph and world > 1:
        xa, xb = S.new_vector(), S.new_vector()
        S.vcycle(xa, b, 2)
        S.set_graph(False)
        S.vcycle(xb, b, 2)
        same = bool(np.array_equal(xa.own_values().view(np.int64), xb.own_values().view(np.int64)))
        bad = [r for r, v in enumerate(be.allgather({rank: 0 if same else 1})) if v]
        del xa, xb
        log(f"multi-part graph self-check: {'ok' if not bad else f'MISMATCH on ranks {bad}: eager launches'}")
        if bad:
            graph_mismatch = bad
            use_graph = False
        else:
            S.set_graph(True)

    # ---- warmup + timed region -------------------------------------------------------
    if args.warmup:
        S.vcycle(x, b, args.warmup)
    def device_sync():  # the context's streams, then hipDeviceSynchronize (every stream)
        ctx.sync()
        _lib.call("pamg_device_sync", dev)

    times = []
    for _ in range(max(1, args.samples)):
        device_sync()
        barrier()
        ts = time.perf_counter()
        S.vcycle_async(x, b, args.steps)
        device_sync()
        barrier()
        dt = time.perf_counter() - ts
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        times.append(dt)
    dt = float(np.median(times))
    vps = args.steps / dt
    log(f"timed samples ({args.steps} V-cycles each, max over ranks): "
        + ", ".join(f"{t * 1e3:.1f} ms" for t in times))

    # ---- time to solution: PCG (V-cycle preconditioner) from x = 0 to --pcg-rtol ----------
    pcg = None
    if args.pcg_rtol > 0:
        xp = S.new_vector()
        device_sync()
        barrier()
        ts = time.perf_counter()
        its, phist = S.pcg(xp, b, rtol=args.pcg_rtol, maxit=200)
        device_sync()
        barrier()
        tp = time.perf_counter() - ts
        if world > 1:
            t = torch.tensor([tp], dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            tp = float(t.item())
        pcg = {"rtol": args.pcg_rtol, "iterations": int(its), "seconds": round(tp, 4),
               "final_rel_residual": float(phist[-1] / phist[0]) if phist[0] else 0.0,
               "converged": bool(phist[-1] <= args.pcg_rtol * phist[0])}
        log(f"pcg: {its} iterations, {tp:.3f} s to rtol {args.pcg_rtol:g}")
        del xp

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
    fused = fused_times(ctx, S, A0, x, b) if world == 1 and _lib.layout_of(A0).get("jr_fused") else None

    # per-(level, op) ms: this rank's, and the max over ranks (the critical path of a step)
    pmax = prof
    if world > 1:
        pmax = np.max(np.stack(be.allgather_array(prof.ravel())), axis=0).reshape(prof.shape)
    levels = [{"rows": int(H.levels[l][rank].A.nrows), "nnz": int(H.levels[l][rank].A.nnz),
               "ms": {op: round(float(prof[l, k]), 4) for k, op in enumerate(OPS) if prof[l, k] > 0},
               **({"ms_max_over_ranks": {op: round(float(pmax[l, k]), 4) for k, op in enumerate(OPS)
                                         if pmax[l, k] > 0}} if world > 1 else {})}
              for l in range(S.L)]
    exch = exchange_times(ctx, S, be, nu1, nu2) if world > 1 else None
    if rank == 0:
        log(json.dumps({"levels": levels, "exchange": exch}))

    # ---- CPU baseline: the oracle V-cycle on this same hierarchy (rank 0, N=1) --------
    # (+ parity at the benchmarked size: the oracle's x after --cpu-cycles cycles from x = 0 on the
    # real b against the GPU's x after the same cycles of the timed call, vcycle_async, bit for bit)
    cpu = parity = None
    if rank == 0 and world == 1 and args.cpu_baseline == "auto":
        xg = S.new_vector()
        S.vcycle_async(xg, b, args.cpu_cycles)
        device_sync()
        gx = xg.own_values()
        del xg
        cpu, xo = cpu_baseline(H, b.own_values(), args.cpu_cycles, log, (nu1, nu2))
        nd = int(np.count_nonzero(gx.view(np.int64) != xo.view(np.int64)))
        parity = {"cycles": args.cpu_cycles, "bit_exact": nd == 0, "differing_entries": nd,
                  "max_abs_diff": float(np.max(np.abs(gx - xo))) if nd else 0.0, "n": int(gx.size),
                  "gpu_path": "vcycle_async (the timed call: graph replay"
                              + (", cross-cycle pipeline)" if S.graph_state()["enabled"] else ")"),
                  "oracle": "oracle/pamg_oracle.c V-cycles on the same hierarchy (hierarchy_from_levels), x0 = 0, same b"}
        log(f"parity at the benchmarked size: {args.cpu_cycles} cycles, {nd} differing entries of {gx.size}")
        del gx, xo

    # HBM traffic of the dominant kernel from the committed rocprofv3 PMC passes of this exact
    # workload (tools/pmc_traffic.py; counters cannot be read from inside the process). A
    # record is used only when it was measured on the same kernel instance, the same tile
    # count (the uploaded layout) and the same kernels.hip source as this run.
    lay = _lib.layout_of(A0)
    cd, tm, tn = lay["cd"], lay["tm"], lay["tile_nnz"]
    # the timed cycles ran the cross-cycle pipeline: its k_sym_tb<3> launch (post-smoothing ->
    # next pre-smoothing -> residual, the matrix read once) is the dominant kernel
    pipelined = bool(fused and fused.get("chain3_ms"))
    # the instance name as rocprofv3 demangles it (every template argument, defaults included)
    tf = lambda v: "true" if v else "false"  # noqa: E731
    if pipelined:
        if lay.get("sym_vd"):  # the z-marching chain over the row-class dictionary (round 5)
            kname = "k_sym_zc<3, 1>"
        else:
            kname = "k_sym_tb<3>"
        post_ms = float(fused["chain3_ms"])
        # matrix once + in0 + b + the outputs the pipelined chain stores: the pre-smoothed iterate
        # and the residual (+ the post-smoothed iterate only with chain_store_x)
        nvec = 2 + _option("chain_store_x")
        post_bytes = float(S.csr_bytes(A0, nvec))
        post_fbytes = float(S.rowsum_bytes(A0, nvec))
        achieved = post_bytes / (post_ms * 1e-3) / 1e9
    elif lay.get("sym"):
        kname = _sym_kname(2, lay)
    elif tm:
        kname = (f"k_rows_tm<2, {tn}, {cd}, {tf(lay['anchored'])}, {tf(lay['x_stage'])}, "
                 f"{tf(lay['per_tile'])}>")
    elif cd:
        kname = f"k_rows_tile2<2, {tn}, false, false, true, {cd}, {tf(lay['per_tile'])}, {tf(lay['anchored'])}>"
    else:
        c24 = lay["c24"]
        kname = (f"k_rows_tile2<2, {tn}, {tf(c24)}, {tf(lay['vd'])}, {tf(lay['rl8'] and c24)}, "
                 f"0, false, false>")
    workload_key = f"{args.matrix or args.kind}:{args.grid}:p{world}:perm{args.permute}" + (":rcm" if args.rcm else "")
    src = kernel_source_sha()
    spmv_kname = _sym_kname(0, lay) if lay.get("sym") else kname.replace("<2,", "<0,", 1)
    traffic = spmv_traffic = None
    if live_pmc:  # this run's own counters (the child ran op 5 = the chain, op 2 = Jacobi, op 0 = SpMV)
        traffic = live_pmc.get(kname)
        spmv_traffic = live_pmc.get(spmv_kname)
    if args.pmc != "off":
        # (k_sym_tb's grid is its tile count, not the layout's: matched on name, workload and source)
        traffic = traffic or pmc_lookup("traffic_chain.json" if pipelined else "traffic_jacobi.json", kname,
                                        None if pipelined else lay["tiles"], workload_key, src)
        spmv_traffic = spmv_traffic or pmc_lookup("traffic_spmv.json", spmv_kname, lay["tiles"], workload_key, src)
    # Counter bytes (2 FETCH_SIZE + WRITE_SIZE) are what crossed the L2's memory side: exact bytes at
    # 128-B request granularity for 8- and 16-B loads (tools/fetch_calib.hip, profiles/r06_e/calib.json)
    # but Infinity-Cache hits included, so an UPPER bound on HBM bytes; the bytes the uploaded layout
    # must stream (format bytes) are the LOWER bound. A counter rate above the measured HBM read
    # ceiling (STREAM_CEILING) cannot all be HBM: the HBM figures then take the
    # format basis, and the counter rate is reported as bytes past L2 only.
    ceiling = STREAM_CEILING["read_GBps"]
    spmv_fbytes = float(S.rowsum_bytes(A0, 0))
    spmv_fmt_gbps = spmv_fbytes / (spmv_ms * 1e-3) / 1e9
    spmv_l2_gbps = (round(spmv_traffic["traffic_bytes"] / (spmv_ms * 1e-3) / 1e9, 1) if spmv_traffic else None)
    spmv_hbm_upper = min(spmv_l2_gbps, ceiling) if spmv_l2_gbps else None
    phys_bytes = float(traffic["traffic_bytes"]) if traffic else post_fbytes
    traffic_over_ceiling = bool(traffic and phys_bytes / (post_ms * 1e-3) / 1e9 > ceiling)
    if traffic_over_ceiling:
        phys_bytes = post_fbytes

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
                "graph_mismatch_ranks": graph_mismatch,
                "transport": args.transport if world > 1 else None,
                # levels >= this one are held whole on every rank (SPEC §S7 agglomeration)
                "replicated_from_level": int(S.rep_level) if world > 1 else None,
                "value_dict": bool(args.value_dict),
                # levels uploaded with a locality permutation (AMGSolver reorder)
                "reordered_levels": S.reordered,
                "options": list(args.set),
            },
            # level-0 fused passes (Options::jr_fuse) beside the separate sweeps they replace
            "fused_level0": fused,
            # fine SpMV (one launch = y = A0 x), the metric's "fine-SpMV HBM GB/s": the bytes its layout
            # must stream (matrix format + x once + y) over its launch time — the physical lower bound
            # of its HBM rate — and that over the 8 TB/s peak; the counter bytes past L2 ((2 FETCH_SIZE +
            # WRITE_SIZE) per launch, Infinity-Cache hits included) beside it, and the upper bound they
            # give the HBM rate (capped at the measured read ceiling)
            "fine_spmv_hbm_GBps": round(spmv_fmt_gbps, 1),
            "fine_spmv_hbm_frac": round(spmv_fmt_gbps / HBM_PEAK_GBPS, 4),
            "fine_spmv_hbm_basis": "format bytes (layout + x once + y) / launch time: the lower bound of the HBM rate",
            "fine_spmv_past_l2_GBps": spmv_l2_gbps,
            "fine_spmv_hbm_frac_upper": round(spmv_hbm_upper / HBM_PEAK_GBPS, 4) if spmv_hbm_upper else None,
            "fine_spmv_traffic_source": spmv_traffic["source"] if spmv_traffic else None,
            "fine_spmv_ms": round(spmv_ms, 4),
            # NOT HBM bytes: SURVEY 8(d)'s plain-CSR bytes (12 B/nnz) over the same time. The symmetric
            # layout streams about half of that, so this "CSR-equivalent" rate may exceed the peak
            "fine_spmv_csr_equiv_GBps": round(spmv_gbps, 1),
            "fine_spmv_csr_equiv_frac": round(spmv_gbps / HBM_PEAK_GBPS, 4),
            "samples_ms_per_step": [round(t / args.steps * 1e3, 4) for t in times],
            "roofline": {
                "kernel": kname + (" (level-0 chain of the pipelined cycles, one launch per cycle: post-smoothing "
                                   "Jacobi -> next pre-smoothing Jacobi -> residual, temporally blocked (z-marching, "
                                   "one barrier per plane) over the symmetric diagonal-class layout" + (" with its row-class dictionary" if lay.get("sym_vd")
                                                                        else "") +
                                   ", the matrix streamed once; stores the pre-smoothed iterate and the residual)"
                                   if pipelined else
                                   " (level-0 post-smoothing Jacobi, symmetric diagonal-class layout: "
                                   "diagonal + upper values per row, lower values from their mirrors)"
                                   if lay.get("sym") else " (level-0 post-smoothing Jacobi"
                          + (", tile-major slots" if tm else "")
                          + (f", {cd}-bit column dictionary" if cd else "")
                          + (", x staged in LDS" if lay.get("x_stage") else "")
                          + (", value dictionaries" if lay["vd"] else "")
                          + (", 24-bit column stream" if lay["c24"] and not cd else "")
                          + (", 8-bit row lengths)" if lay["rl8"] else ")")),
                # achieved / frac on a PHYSICAL basis: the HBM bytes the launch moved
                # (PMC counters) when they were collected, else the bytes its layout must stream
                # (format bytes), over the launch's HIP-event time; both are <= what HBM can move
                "bound": "hbm", "achieved": round(phys_bytes / (post_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBPS,
                "unit": "GB/s", "frac": round(phys_bytes / (post_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "frac_basis": ("PMC traffic per launch ((2 FETCH_SIZE + WRITE_SIZE) x 1 KiB, calibrated on known-byte "
                               "kernels: profiles/r06_e/calib.json) / launch time / peak"
                               if traffic and not traffic_over_ceiling else
                               "format bytes per launch (what the uploaded layout streams) / launch time / peak ("
                               + ("the counter rate exceeds the measured HBM read ceiling: Infinity-Cache hits)"
                                  if traffic_over_ceiling else "no PMC counters in this run)")),
                "traffic": traffic["traffic_bytes"] if traffic else None,
                "traffic_source": traffic["source"] if traffic else None,
                "hbm_frac": (round(traffic["traffic_bytes"] / (post_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
                             if traffic else None),
                # the layout's own algorithmic bytes (format) and their rate
                "format_bytes_per_launch": int(post_fbytes),
                "format_GBps": round(post_fbytes / (post_ms * 1e-3) / 1e9, 1),
                "format_frac": round(post_fbytes / (post_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
                "traffic_over_format": round(traffic["traffic_bytes"] / post_fbytes, 3) if traffic else None,
                # NOT a roofline fraction: SURVEY 8(d)'s plain-CSR bytes (12 B/nnz) over the same time; the
                # row-class dictionary streams ~1/30 of that matrix, so this rate exceeds the HBM peak
                "csr_equiv_bytes_per_launch": int(post_bytes), "csr_equiv_model": "SURVEY 8(d) CSR (12 B/nnz)",
                "csr_equiv_GBps": round(achieved, 1),
                "csr_equiv_frac": round(achieved / HBM_PEAK_GBPS, 4),
                "ms_per_launch": round(post_ms, 4),
                # the practical streaming ceiling beside the 8 TB/s spec: plain coalesced kernels
                # reading 11 streams per written one (the Jacobi's read:write mix) / reading only,
                # measured on an MI355X with tools/stream_ceiling.hip
                "stream_ceiling": STREAM_CEILING,
            },
            "cpu_baseline": cpu,
            # the timed path against the oracle at the benchmarked size (BASELINE.json:5 tolerance: bit-exact)
            f"parity_{args.grid}" if not args.matrix else "parity": parity,
            # per level: rows / nonzeros of rank 0's part and ms per V-cycle per op (HIP events,
            # eager launches; N > 1: + the max over ranks); exchange: ghost-exchange times
            "levels": levels,
            "exchange": exch,
            "time_to_solution": pcg,
            "setup_s": round(t_setup, 1),
            "setup_products": args.setup,
            "final_residual": float(hist[0]),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def exchange_times(ctx, S, be, nu1, nu2, reps=20) -> dict:
    """N > 1: time of one ghost exchange (consistent!, synchronous, this rank's view) of every
    level's A / R / P column plan, and the exchanges one V(nu1, nu2) cycle makes — A_l: nu1 (level
    0) or nu1 - 1 (zero-guess first sweep on l >= 1) + 1 residual + nu2 post sweeps; R_l and P_l:
    one each — as ms per cycle (an upper bound: each timed call syncs the stream; inside the
    graph-replayed cycle the A exchanges overlap the interior rows). Max over ranks."""
    from parallel_amg_amd.partitioned import PVector, consistent
    out, total = [], 0.0
    for l in range(S.L):
        rec = {}
        mats = [("A", S.A_dev[l])] + ([("R", S.R[l]), ("P", S.P[l])] if l < S.L - 1 else [])
        for name, M in mats:
            if M.plan is None:
                continue
            v = PVector(ctx, M.plan.n_own, M.plan.n_ghost)
            consistent(v, M.plan)
            t = time.perf_counter()
            for _ in range(reps):
                consistent(v, M.plan)
            rec[name] = (time.perf_counter() - t) / reps * 1e3
        out.append(rec)
    # max over ranks per (level, plan)
    keys = [(l, k) for l in range(S.L) for k in ("A", "R", "P")]
    mine = [out[l].get(k, 0.0) for l, k in keys]
    allv = np.max(np.stack(be.allgather_array(np.asarray(mine, np.float64))), axis=0)
    per = []
    for l in range(S.L):
        d = {k: round(float(allv[3 * l + j]), 4) for j, k in enumerate(("A", "R", "P")) if allv[3 * l + j] > 0}
        na = (nu1 if l == 0 else nu1 - 1) + 1 + nu2 if l < S.L - 1 else 0
        cyc = na * d.get("A", 0.0) + d.get("R", 0.0) + d.get("P", 0.0)
        total += cyc
        per.append({"ms_per_exchange": d, "exchanges_per_cycle": {"A": na, "R": 1 if "R" in d else 0,
                                                                   "P": 1 if "P" in d else 0},
                    "ms_per_cycle": round(cyc, 4)})
    return {"per_level": per, "ms_per_cycle_upper_bound": round(total, 4),
            "note": "synchronous consistent! per plan, max over ranks; the replicated tail's all-gather is "
                    "inside levels[rep-1].restrict"}


def _option(key: str) -> int:
    from parallel_amg_amd import _lib
    v = ctypes.c_int64()
    _lib.call("pamg_get_option", key.encode(), ctypes.byref(v))
    return int(v.value)


def _sym_kname(op: int, lay: dict) -> str:
    """The symmetric-layout row kernel's instance name as rocprofv3 demangles it: k_rows_symd<OP,
    NU, CH> (row-class dictionary; CH = symd_chunks for NU <= 3), k_rows_sym2 / k_rows_sym<OP, NU>."""
    nu = lay["cd_offsets"]
    if lay.get("sym_vd") and lay.get("jr_fused") and nu == 3 and _option("sym_zm"):
        return f"k_sym_zm<{op}>"  # the whole one-part grid operator's z-marching sweep
    if lay.get("sym_vd"):
        return f"k_rows_symd<{op}, {nu}, {_option('symd_chunks') if nu <= 3 else 1}>"
    return f"k_rows_sym{'2' if lay['sym_rows'] == 2 else ''}<{op}, {nu}>"


def kernel_source_sha() -> str:
    import hashlib
    with open(os.path.join(ROOT, "parallel_amg_amd", "csrc", "kernels.hip"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


STREAM_CEILING = {"mix11to1_GBps": 5104.0, "read_GBps": 6311.0,
                  "source": "profiles/r02_exp/stream_ceiling.jsonl (tools/stream_ceiling.hip, 8 GiB, best grid)"}


def fused_times(ctx, S, A0, x, b, reps=10):
    """ms of the level-0 fused passes: k_sym_jr (Jacobi -> residual, through pamg_jacobi_residual,
    synchronous calls) and the pipeline's k_sym_chain (post -> pre -> residual, HIP events), with
    the separate sweeps they replace measured the same way."""
    from parallel_amg_amd.partitioned import jacobi_residual, residual
    from parallel_amg_amd import _lib
    t, r, xx = S.new_vector(), S.new_vector(), S.new_vector()

    def per_call(fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        return (time.perf_counter() - t0) / reps * 1e3

    out = {"jacobi_residual_fused_ms": round(per_call(lambda: jacobi_residual(t, r, A0, x, b, 0.66)), 4)}
    with option("jr_fuse", 0):
        out["jacobi_then_residual_ms"] = round(per_call(lambda: (jacobi_residual(t, r, A0, x, b, 0.66))), 4)
    out["residual_ms"] = round(per_call(lambda: residual(r, A0, t, b)), 4)
    ch = S.bench_chain(xx, b, reps)
    out["chain3_ms"] = round(ch, 4) if ch is not None else None
    return out


def option(name, value):
    import contextlib

    from parallel_amg_amd import _lib

    @contextlib.contextmanager
    def cm():
        old = ctypes.c_int64()
        _lib.call("pamg_get_option", name.encode(), ctypes.byref(old))
        _lib.call("pamg_set_option", name.encode(), int(value))
        try:
            yield
        finally:
            _lib.call("pamg_set_option", name.encode(), old.value)
    return cm()


def pmc_live(args):
    """HBM bytes per launch of the pipelined cycles' chain kernel (k_sym_tb<3>) and the fine SpMV
    on this run's operator, from two rocprofv3 --pmc passes (FETCH_SIZE, then WRITE_SIZE: one
    counter per run, MI355X_MICROARCH.md §HBM) over tools/kbench.py, which uploads the same
    level-0 operator with the same options and launches exactly those kernels (ops 5 and 0).
    Called before this process makes any HIP call: the children are separate programs started
    from a process that has not initialised the GPU. Returns {kernel: {"traffic_bytes", ...}}
    (bytes = (2 FETCH_SIZE + WRITE_SIZE) KiB x 1024, the gfx950 correction for 16-B/lane
    streams), or None if a pass fails (the committed records are used then)."""
    import shutil
    import subprocess
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        log("pmc: rocprofv3 not found")
        return None
    tmp = tempfile.mkdtemp(prefix="pamg_pmc_")
    kb = [sys.executable, "-u", os.path.join(ROOT, "tools", "kbench.py"), "--n", str(args.grid), "--kind", args.kind,
          "--levels", "1", "--ops", "0,2,5", "--reps", "3", "--configs", f"1024:1:1:{int(args.value_dict)}",
          ]
    for kv in args.set:
        kb += ["--set", kv]
    agg = {}
    t0 = time.time()
    try:
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, counter)
            cmd = ["timeout", "-s", "KILL", "240", prof, "--pmc", counter, "-d", d, "-o", "p",
                   "--output-format", "csv", "--"] + kb
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
            if r.returncode != 0:
                log(f"pmc: {counter} pass failed (rc {r.returncode}): {r.stderr[-400:]}")
                return None
            for (name, blocks), vals in pmc_csv(d, counter).items():
                agg.setdefault(name, {}).setdefault(blocks, {})[counter] = sum(vals) / len(vals)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    out = {}
    for name, grids in agg.items():
        # one grid per counted kernel instance, or its counters could come from another launch
        if len(grids) != 1:
            log(f"pmc: {name} ran with {len(grids)} grids {sorted(grids)}: not used")
            continue
        (c,) = grids.values()
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            out[name] = {"traffic_bytes": (2.0 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0,
                         "fetch_kib": c["FETCH_SIZE"], "write_kib": c["WRITE_SIZE"],
                         "source": "live: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over tools/kbench.py "
                                   "(bench.py child runs), (2 FETCH + WRITE) x 1 KiB per launch"}
    log(f"pmc: live passes in {time.time() - t0:.0f}s: "
        + ", ".join(f"{k} {v['traffic_bytes'] / 1e9:.2f} GB" for k, v in out.items()))
    return out


def pmc_csv(path, counter):
    """{(kernel name, blocks): [values]} of one counter from a rocprofv3 -d directory's csv."""
    import collections
    import csv
    import glob
    import re
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True)):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].replace("pamg::(anonymous namespace)::", "").replace("void ", "")
            name = re.sub(r"\(.*", "", name)
            agg[(name, int(r["Grid_Size"]) // max(1, int(r["Workgroup_Size"])))].append(float(r["Counter_Value"]))
    return agg


def pmc_lookup(fname, kname, tiles, workload_key, src):
    """The committed PMC traffic record (profiles/pmc/<fname>, tools/pmc_traffic.py) of this
    kernel instance on this workload, tile count and kernels.hip source; None otherwise."""
    path = os.path.join(ROOT, "profiles", "pmc", fname)
    if not os.path.exists(path):
        return None
    for r in json.load(open(path)):
        if (r.get("kernel") == kname and (tiles is None or r.get("blocks") == tiles) and r.get("workload") == workload_key
                and r.get("kernels_hip_sha16") == src):
            return {"traffic_bytes": float(r["traffic_bytes"]), "source": os.path.relpath(path, ROOT)}
    return None


def ctypes_bench_spmv(ctx, A0, x, S, reps=20) -> float:
    import ctypes as C

    from parallel_amg_amd._lib import call
    from parallel_amg_amd.partitioned import PVector
    y = PVector(ctx, A0.nrows)
    ms = C.c_double()
    call("pamg_bench_rowop", ctx.handle, A0.handle, 0, x.handle, None, y.handle, 0.0, reps,
         C.byref(ms))
    return ms.value


def host_cpu_info() -> dict:
    """Cores this process may run on (affinity set), the machine's count, OMP_NUM_THREADS, the
    cgroup CPU quota (cpu.max, in cores) and the CPU model."""
    info = {"affinity": len(os.sched_getaffinity(0)), "nproc": os.cpu_count(),
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "cgroup_quota_cores": None, "cpu_model": "?"}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            info["cgroup_quota_cores"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    try:
        with open("/proc/cpuinfo") as f:
            info["cpu_model"] = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        pass
    return info


def cpu_baseline(H, b, ncycles, log, sweeps=(1, 1)):
    """Time the CPU oracle's V-cycle (oracle/pamg_oracle.c, OpenMP) on the same hierarchy, on
    every core of this process's affinity set (all host cores), plus the CPU
    fine-level SpMV rate on the same algorithmic bytes as the GPU's fine_spmv_csr_equiv_GBps
    (plain CSR, 12 B/nnz; the oracle's int64 columns stream more than that)."""
    from oracle import oracle as O
    info = host_cpu_info()
    # every core this process may use: the affinity set, capped by the cgroup CPU quota (a
    # 256-CPU affinity under a 16-core quota runs 256 threads time-sliced on 16 cores: measured
    # 4.5x slower than 16 threads, profiles/r03_sym/bench.log)
    cores = info["affinity"]
    if info["cgroup_quota_cores"]:
        cores = max(1, min(cores, int(info["cgroup_quota_cores"])))
    O.lib().orc_set_threads(cores)
    lv = [H.levels[l][0] for l in range(H.nlevels)]
    Ho = O.hierarchy_from_levels([p.A for p in lv], [p.P for p in lv[:-1]], [p.R for p in lv[:-1]],
                                 [p.omega for p in lv], H.ainv)
    Ho.set_sweeps(*sweeps)
    A0 = lv[0].A
    x = np.zeros(A0.nrows)
    rhs = np.ascontiguousarray(b, np.float64)  # the timed cycles' own b (x is compared with the GPU's)
    t = time.perf_counter()
    O.lib().orc_solve(Ho._h, x, rhs, ncycles, None)
    dt = time.perf_counter() - t
    del Ho
    # fine SpMV: the oracle's y = A0 x (int64 indices), reps timed; GB/s on SURVEY 8(d) bytes
    Ao = O.CSR(A0.rowptr, A0.col.astype(np.int64), A0.val, A0.ncols)
    y = np.empty(A0.nrows)
    O.lib().orc_spmv(Ao.nrows, Ao.rowptr, Ao.col, Ao.val, rhs, y)  # warm
    reps = 3
    t = time.perf_counter()
    for _ in range(reps):
        O.lib().orc_spmv(Ao.nrows, Ao.rowptr, Ao.col, Ao.val, rhs, y)
    ts = (time.perf_counter() - t) / reps
    spmv_bytes = 12 * A0.nnz + 4 * (A0.nrows + 1) + 8 * A0.ncols + 8 * A0.nrows
    threads = int(O.lib().orc_get_threads())
    log(f"cpu baseline: {ncycles} V-cycle(s) in {dt:.2f}s, fine SpMV {ts * 1e3:.1f} ms on {threads} threads "
        f"(affinity {cores}, nproc {info['nproc']}, quota {info['cgroup_quota_cores']}; {info['cpu_model']})")
    return {"value": round(ncycles / dt, 5), "unit": "V-cycles/s", "cores": threads, "kind": "port",
            "fine_spmv_csr_GBps": round(spmv_bytes / ts / 1e9, 2), "fine_spmv_ms": round(ts * 1e3, 2),
            "affinity_cores": cores, "nproc": info["nproc"], "omp_num_threads_env": info["omp_num_threads"],
            "cgroup_quota_cores": info["cgroup_quota_cores"], "cpu_model": info["cpu_model"],
            "sample": f"{ncycles} full V-cycle(s) of the same {A0.nrows}-row hierarchy by the C "
                      f"oracle (oracle/pamg_oracle.c, OpenMP on {cores} threads = the affinity set capped "
                      f"by the cgroup CPU quota, int64 "
                      f"indices) + {reps} fine SpMVs; reference (Julia/PartitionedArrays) not runnable: "
                      f"no code in /root/reference"}, x


if __name__ == "__main__":
    main()
