/*
 * pamg.h — C-ABI of the MI355X-native AMG V-cycle solve path (libpamg.so).
 *
 * Drop-in boundary. The reference (tirtho109/parallel_AMG) contains only
 * README.md:1-2 ("Apply AMG algorithm parallelly using PartitionedArrays.jl") — there is no
 * reference FFI to mirror line by line. Each entry point below replaces the PartitionedArrays
 * operation named in its comment (the surface an AMG solver written against
 * PartitionedArrays calls, README.md:2); INTEGRATION.md shows the Julia `ccall` binding and
 * the Python ctypes binding (parallel_amg_amd/_lib.py) a maintainer would use.
 *
 * Conventions
 *  - Every function returns int: PAMG_OK (0) or a negative PAMG_E_* code; the message of the
 *    last failure on the calling thread is pamg_last_error().
 *  - Handles are opaque and owned by the library; free them with the matching _destroy.
 *  - Host arrays are copied; the caller keeps ownership and may free them after the call.
 *  - Device calls are enqueued on the context's compute stream and are complete on return
 *    unless the name ends in _async (then pamg_ctx_sync() completes them).
 *  - One host thread per context; one context per GPU; one GPU per process (the
 *    PartitionedArrays "one part per MPI rank" shape; ranks exchange ghosts over RCCL).
 *  - Numerics: SPEC.md (fp64 values, int32 device indices, fixed summation order).
 */
#ifndef PAMG_H
#define PAMG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PAMG_OK 0
#define PAMG_E_ARG (-1)      /* bad argument / shape mismatch */
#define PAMG_E_HIP (-2)      /* HIP runtime error */
#define PAMG_E_RCCL (-3)     /* RCCL error */
#define PAMG_E_OVERFLOW (-4) /* index does not fit the device int32 layout */
#define PAMG_E_SETUP (-5)    /* setup failed (missing diagonal, non-SPD coarse matrix, ...) */
#define PAMG_E_STATE (-6)    /* call not valid in the current state (e.g. no communicator) */
#define PAMG_E_NOMEM (-7)    /* host or device allocation failed */

typedef struct pamg_ctx pamg_ctx;   /* one GPU, its streams and (optionally) an RCCL comm */
typedef struct pamg_plan pamg_plan; /* ghost layout + neighbour exchange lists (a PRange) */
typedef struct pamg_vec pamg_vec;   /* device PVector: own values then ghost slots */
typedef struct pamg_mat pamg_mat;   /* device PSparseMatrix part: own rows, local columns */
typedef struct pamg_hier pamg_hier; /* device AMG hierarchy (V-cycle) */
typedef struct pamg_hcsr pamg_hcsr; /* host CSR produced by the setup routines */

const char* pamg_version(void);
const char* pamg_last_error(void);

/* ------------------------------------------------------------------ context */
/* Replaces the PartitionedArrays backend objects (with_mpi / with_debug). */
int pamg_ctx_create(int device, pamg_ctx** out);
int pamg_ctx_destroy(pamg_ctx* ctx);
int pamg_ctx_sync(pamg_ctx* ctx);
/* References held on the context: the caller's handle (until pamg_ctx_destroy) plus one per
 * live plan, vector, matrix and hierarchy made on it; it is torn down when they reach 0
 * (diagnostics and tests: a failed create must leave the count unchanged). */
int pamg_ctx_refcount(const pamg_ctx* ctx, int* refs);
/* Number of visible GPUs, through libpamg's own HIP runtime (a driver that must not
 * initialise another runtime in the process asks here; see INTEGRATION.md, load order). */
int pamg_device_count(int* n);
/* hipDeviceSynchronize on `device`: waits for every stream of the process on that GPU (the
 * benchmark's sync brackets; pamg_ctx_sync waits only for the context's own streams). */
int pamg_device_sync(int device);
/* RCCL communicator for multi-part runs: rank 0 calls pamg_comm_unique_id, the 128 bytes are
 * broadcast by the host layer (MPI / torch.distributed), then every rank calls pamg_comm_init. */
int pamg_comm_unique_id(unsigned char id[128]);
/* Fails with PAMG_E_RCCL (message names the library file) when the RCCL the process bound
 * is older than the one libpamg was built against — e.g. a host that loaded the torch
 * wheel's bundled RCCL 2.26 before libpamg. */
int pamg_comm_init(pamg_ctx* ctx, int nranks, int rank, const unsigned char id[128]);
/* HIP runtime / RCCL versions this process resolved, beside the versions libpamg was built
 * against (HIP_VERSION, NCCL_VERSION_CODE). Any pointer may be NULL. */
int pamg_runtime_versions(int* hip_runtime, int* hip_built, int* rccl_runtime, int* rccl_built);
int pamg_comm_rank(const pamg_ctx* ctx, int* rank, int* nranks);
/* Debug transport (PartitionedArrays' debug-backend role): instead of RCCL, every exchange is
 * staged through host buffers and handed to `fn` (synchronously, no overlap). Lets several
 * ranks share ONE GPU (RCCL refuses that) so the multi-part data path can be tested on a
 * one-GPU machine. op 0: neighbour exchange — for k < n, send send_counts[k] doubles to
 * peer[k] and receive recv_counts[k] doubles from it (buffers concatenated in k order);
 * op 1: all-gather of send_counts[0] doubles per rank into recvbuf (rank order);
 * op 2: all-reduce (sum) of send_counts[0] doubles into recvbuf. Return 0 on success. */
typedef int (*pamg_host_comm_fn)(void* user, int op, int n, const int32_t* peer,
                                 const int64_t* send_counts, const double* sendbuf,
                                 const int64_t* recv_counts, double* recvbuf);
int pamg_comm_init_host(pamg_ctx* ctx, int nranks, int rank, pamg_host_comm_fn fn, void* user);
/* In-process transport (PartitionedArrays with_debug: all parts in one process): a world of
 * nparts sibling contexts, each registered under its rank and driven by its own host thread
 * (a context is not re-entrant). Ghost exchanges, the agglomeration all-gather and all-reduces
 * rendezvous in the world and move data by device-to-device copies along the plans' send/recv
 * lists — straight from the sibling's vector into the ghost slots (hipMemcpyAsync with peer
 * access across GPUs; siblings may share one GPU). Synchronous like the host transport: no
 * overlap, no graph capture. Ghost exchanges meet pairwise: a part waits only for the
 * neighbours its plan lists with a non-zero count, and each pair's exchanges are matched by
 * sequence number and plan tag (pamg_plan_set_tag) — parts whose schedules diverge fail with
 * PAMG_E_STATE instead of exchanging the wrong vectors. All-reduce / all-gather meet every rank.
 * A rank that does not arrive within 300 s, a failed collective, a failed part of a
 * pamg_world_* call or pamg_world_abort marks the world broken: every waiting and later
 * collective fails (PAMG_E_STATE) at once, so no sibling waits for a part that has given up.
 * pamg_world_reset clears that — call it only when no rank is inside a library call. The
 * pamg_world_* calls below (and the Python LocalWorld.run over all parts) reset the world
 * themselves once every part has returned, so one part's error (an argument error included)
 * fails that call only; a caller driving the ranks from its own threads calls
 * pamg_world_reset after a failure. Two parts whose tagged plans disagree on their counts
 * fail at once (PAMG_E_STATE), also when one of them lists the other with zero counts.
 * The world lives until it and all its contexts are destroyed. */
typedef struct pamg_world pamg_world;
int pamg_world_create(int nparts, pamg_world** out);
int pamg_world_destroy(pamg_world* w);
int pamg_world_abort(pamg_world* w);
int pamg_world_reset(pamg_world* w);
int pamg_world_state(pamg_world* w, int* broken);
int pamg_comm_init_local(pamg_ctx* ctx, pamg_world* w, int rank);
/* All parts of a world at once (one host thread per part inside, each on its own context; for
 * callers with one host thread, e.g. PartitionedArrays with_debug's map over the parts): the
 * per-part arrays are indexed by rank. The result of a failed part is returned with its message
 * ("part r: ..."). res_hist / iters receive rank 0's (every rank's are the same). */
int pamg_world_spmv(pamg_world* w, pamg_mat* const* A, pamg_vec* const* x, pamg_vec* const* y);
int pamg_world_exchange(pamg_world* w, pamg_plan* const* plan, pamg_vec* const* x);
int pamg_world_dot(pamg_world* w, pamg_vec* const* x, pamg_vec* const* y, double* out);
int pamg_world_vcycle(pamg_world* w, pamg_hier* const* H, pamg_vec* const* x, pamg_vec* const* b, int ncycles,
                      double* res_hist);
int pamg_world_pcg(pamg_world* w, pamg_hier* const* H, pamg_vec* const* x, pamg_vec* const* b, double rtol,
                   int maxit, int* iters, double* res_hist);

/* ------------------------------------------------------------------ exchange plan */
/* Replaces PRange / ExchangeGraph: ghosts [n_own, n_own+n_ghost) grouped by neighbour in
 * nbr order (recv_counts), and per neighbour the own indices sent to it (send_idx,
 * concatenated in nbr order, send_counts). A part may list its own rank (ghost copies of own
 * entries, served by an RCCL send/recv to self; refused under the host debug transport). */
int pamg_plan_create(pamg_ctx* ctx, int64_t n_own, int64_t n_ghost, int n_nbr,
                     const int32_t* nbr_rank, const int64_t* recv_counts,
                     const int64_t* send_counts, const int64_t* send_idx, pamg_plan** out);
/* Identity of the index space a plan describes (e.g. "level 2, the columns of R"), the same
 * number on every part; default 0. The in-process world refuses to pair two parts' exchanges
 * whose plans carry different tags, and fails at once when one part's plan lists the other with
 * zero counts while that one's plan of the same tag expects ghosts from it (RCCL and the host
 * transport ignore tags). A tag names one index space for the life of the world (or until
 * pamg_world_reset): plans of one tag must agree on their counts across parts. */
int pamg_plan_set_tag(pamg_plan* plan, int64_t tag);
int pamg_plan_destroy(pamg_plan* plan);

/* ------------------------------------------------------------------ vectors (PVector) */
int pamg_vec_create(pamg_ctx* ctx, int64_t n_own, int64_t n_ghost, pamg_vec** out);
int pamg_vec_destroy(pamg_vec* v);
int pamg_vec_size(const pamg_vec* v, int64_t* n_own, int64_t* n_ghost);
int pamg_vec_upload(pamg_ctx* ctx, pamg_vec* v, const double* own);     /* own_values(v) .= */
int pamg_vec_download(pamg_ctx* ctx, const pamg_vec* v, double* own);
/* ghost_values(x): the n_ghost ghost slots as last exchanged (debugging, tests). */
int pamg_vec_download_ghosts(pamg_ctx* ctx, const pamg_vec* v, double* ghost);
int pamg_vec_device_ptr(pamg_vec* v, double** dptr);                    /* zero-copy interop */
int pamg_vec_fill(pamg_ctx* ctx, pamg_vec* v, double value);            /* fill!(v, a) */
int pamg_vec_copy(pamg_ctx* ctx, const pamg_vec* src, pamg_vec* dst);   /* copy!(dst, src) */
int pamg_vec_axpby(pamg_ctx* ctx, double a, const pamg_vec* x, double b, pamg_vec* y); /* y=a x+b y */
int pamg_vec_dot(pamg_ctx* ctx, const pamg_vec* x, const pamg_vec* y, double* out);    /* dot */
int pamg_vec_nrm2(pamg_ctx* ctx, const pamg_vec* x, double* out);                      /* norm */
/* consistent!(x) |> wait : owners' values into the ghost slots described by plan. */
int pamg_exchange(pamg_ctx* ctx, const pamg_plan* plan, pamg_vec* x);
/* t = consistent!(x) ... wait(t), split: _begin enqueues the exchange on the context's comm
 * stream behind the work already enqueued and returns at once; _end joins it (later calls see
 * the ghosts) and waits. Work between the two overlaps the exchange; it must not read x's
 * ghost slots or write x's own entries. One exchange in flight per plan (PAMG_E_STATE
 * otherwise). The host debug transport completes the exchange inside _begin. */
int pamg_exchange_begin(pamg_ctx* ctx, pamg_plan* plan, pamg_vec* x);
int pamg_exchange_end(pamg_ctx* ctx, pamg_plan* plan, pamg_vec* x);

/* ------------------------------------------------------------------ matrices (PSparseMatrix) */
/* One part's own rows; columns already local (own 0..n_own-1 of the column space, then the
 * plan's ghosts), each row in ascending GLOBAL column order (SPEC §S1). col is int32 or int64
 * (col_is_64); index_base 0 or 1 (Julia). col_plan may be NULL for a single part. */
int pamg_mat_upload(pamg_ctx* ctx, int64_t nrows, int64_t ncols_local, const int64_t* rowptr,
                    const void* col, int col_is_64, const double* val, int index_base,
                    const pamg_plan* col_plan, pamg_mat** out);
/* The same upload with a locality permutation inside the device layout (replaces nothing in
 * PartitionedArrays: it is how a solver keeps a scattered numbering — an FE mesh, a random
 * renumbering — off the gather path). Device row i is caller row row_perm[i]; device own
 * column k is caller own column col_perm[k] (ghost columns are never permuted). NULL = the
 * identity. Each row keeps its entries in the caller's storage order, so every row sum
 * (SPEC §S3) has the caller's bits. Vectors applied to the matrix are in device numbering. */
int pamg_mat_upload_perm(pamg_ctx* ctx, int64_t nrows, int64_t ncols_local, const int64_t* rowptr,
                         const void* col, int col_is_64, const double* val, int index_base,
                         const pamg_plan* col_plan, const int64_t* row_perm,
                         const int64_t* col_perm, pamg_mat** out);
int pamg_mat_destroy(pamg_mat* A);
int pamg_mat_info(const pamg_mat* A, int64_t* nrows, int64_t* ncols_local, int64_t* nnz);
/* Bytes of matrix data one row operation streams in the layout chosen at upload: 8 B values +
 * 4 B (3 B in 24-bit column tiles, 0.5 / 1 B with a column dictionary) columns per nonzero,
 * 4 B row pointers (1 B with 8-bit row lengths), tile descriptors (+ 4-B column bases). */
int pamg_mat_stream_bytes(const pamg_mat* A, int64_t* bytes);
/* Layout the upload chose for the interior (set 0) or boundary (set 1) rows:
 * out[0] 24-bit columns, out[1] value dictionary, out[2] 8-bit row lengths,
 * out[3] column-dictionary index width (0, 4 or 8), out[4] column-dictionary offsets,
 * out[5] tile-major padded copy, out[6] its row-length slot per tile, out[7] the tile
 * budget (nonzeros per tile) the set was cut with, out[8] the number of short tiles (the
 * grid of the set's tile kernel), out[9] bit 0: the dictionary is anchored (offsets from each
 * row's first column) instead of row-relative; bit 1: every tile has its own table of out[4]
 * entries (per-tile dictionaries) instead of one table for the set; bit 2: the tile kernel
 * stages x in LDS (x_stage: the runs the set's offset clusters read, no x gathers); bit 3: the
 * set runs in the symmetric diagonal-class layout (sym_dia: diagonal + upper values per row,
 * lower values read from their mirrors; then out[4] = the upper offset classes and out[8] =
 * the kernel's grid); bit 4: that kernel takes two rows per lane (sym_rows 2); bit 5: the
 * matrix is a 7-point grid stencil the temporally blocked passes run on (k_sym_tb: the
 * level-0 Jacobi -> residual, and the pipelined cycles' post -> pre -> residual chain; jr_fuse);
 * bit 6: the tile-major set carries 8-bit per-tile value dictionaries (value_dict);
 * bit 7: the symmetric layout stores a 1-byte row class per row, its values in a table of
 * <= 64 (mask, diagonal, upper values) tuples (sym_vd); bit 8: retired (round 5; never set —
 * it named the per-tile x staging, deleted); bit 9: the set runs in
 * the sliced-ELL layout (ell: one row per lane, per-group 8-bit column-offset and value dictionaries;
 * then out[8] = the kernel's grid); bit 10: the set runs in the neighbour-coded prolongation layout
 * (pnc: a prolongation over a 7-point grid uploaded earlier on the same context, each column named
 * by the grid neighbour whose anchor it is; then out[3] = the value table's entries, out[4] = the
 * pattern table's, out[8] = the kernel's grid); bit 11: the set runs in the pattern-dictionary
 * layout (rpat: a restriction whose rows repeat <= 255 (offset, value) patterns from their first
 * column; then out[3] = the value table's entries, out[4] = the pattern count, out[8] = the kernel's
 * grid); bit 12: with bit 10, the rows hold 16-bit combination ids instead of 64-bit records
 * (pnc_compact; out[4] = the combinations); bit 13: with bit 9, one index byte per nonzero names an
 * (offset, value) pair of the group (ell_pair). */
int pamg_mat_layout(const pamg_mat* A, int set, int out[10]);

/* mul!(y, A, x): exchanges x's ghosts (overlapped with the interior rows), then y = A x. */
int pamg_spmv(pamg_ctx* ctx, const pamg_mat* A, pamg_vec* x, pamg_vec* y);
/* r = b - A x ; if nrm2 != NULL, *nrm2 = ||r|| over all parts. */
int pamg_residual(pamg_ctx* ctx, const pamg_mat* A, pamg_vec* x, const pamg_vec* b,
                  pamg_vec* r, double* nrm2);
/* nsweeps weighted-Jacobi sweeps on x (tmp is the ping-pong buffer; result in x). */
int pamg_jacobi(pamg_ctx* ctx, const pamg_mat* A, pamg_vec* x, const pamg_vec* b,
                pamg_vec* tmp, double omega, int nsweeps);
/* One weighted-Jacobi sweep and the residual of its result: t = x + omega D^-1 (b - A x),
 * r = b - A t (the level-0 pre-smoothing + residual of a V-cycle). On one part, for a 7-point
 * grid stencil in the symmetric layout (pamg_mat_layout bit 5) with jr_fuse on, both run in one
 * temporally blocked pass over the matrix (*fused = 1); otherwise two sweeps. The bits are the
 * same either way. fused may be NULL. */
int pamg_jacobi_residual(pamg_ctx* ctx, const pamg_mat* A, pamg_vec* x, const pamg_vec* b,
                         pamg_vec* t, pamg_vec* r, double omega, int* fused);

/* ------------------------------------------------------------------ hierarchy / V-cycle */
/* Levels 0..nlevels-1; P[l], R[l] for l < nlevels-1 (NULL entries otherwise). The coarsest
 * level is solved with Ainv (column-major, n_coarse x n_coarse, SPEC §S5).
 * Several ranks: levels >= rep_level (1 <= rep_level <= nlevels-1) are held whole on every
 * rank — the agglomerated tail of SPEC §S7, or just the coarsest level (rep_level =
 * nlevels-1). R[rep_level-1] yields this rank's rows [rep_offsets[rank], rep_offsets[rank+1])
 * of level rep_level, which are all-gathered; P[rep_level-1] and the tail's matrices read
 * whole vectors (no plan). A[rep_level] is whole unless rep_level = nlevels-1. One rank:
 * rep_level and rep_offsets are ignored (NULL allowed).
 * The hierarchy references (does not own) the matrices: keep them alive. */
int pamg_hier_create(pamg_ctx* ctx, int nlevels, pamg_mat* const* A, pamg_mat* const* P,
                     pamg_mat* const* R, const double* omega, int64_t n_coarse,
                     const double* ainv_colmajor, int rep_level, const int64_t* rep_offsets,
                     pamg_hier** out);
int pamg_hier_destroy(pamg_hier* H);
/* 1 = replay the V-cycle as a captured hipGraph (default 1 on one part and with RCCL; the
 * host debug transport cannot be captured), 0 = eager launches. A failed capture falls back
 * to eager launches (same RCCL sequence) and is reported on stderr. */
int pamg_hier_set_graph(pamg_hier* H, int enable);
/* V(nu1, nu2): Jacobi sweeps before / after the coarse correction (SPEC §S6; default 1, 1;
 * 1..64). The first pre-sweep on levels >= 1 is the zero-guess form. */
int pamg_hier_set_sweeps(pamg_hier* H, int nu1, int nu2);
/* Level-0 numbering of a hierarchy whose operators were uploaded with pamg_mat_upload_perm
 * (one part only): device row i of level 0 is caller row perm[i]. pamg_vcycle(_async) and
 * pamg_pcg then take x and b in the caller's numbering — gathered into the device numbering at
 * entry, x scattered back at exit. x after stationary V-cycles has the bits of the unpermuted
 * hierarchy's cycles (every row sum keeps its storage order). Reductions run in the device
 * order: pamg_vcycle's res_hist norms and pamg_pcg's dot products — hence its iterates — match
 * the unpermuted run to rounding only, not bit for bit. perm = NULL (or n = 0) removes it. */
int pamg_hier_set_perm(pamg_hier* H, int64_t n, const int64_t* perm);
/* enabled: graph replay currently on; captured: a graph exists; failed: a capture failed. */
int pamg_hier_graph_state(const pamg_hier* H, int* enabled, int* captured, int* failed);
/* x <- V(x) ncycles times (SPEC §S6); res_hist (ncycles, may be NULL) gets ||b - A x||. */
int pamg_vcycle(pamg_ctx* ctx, pamg_hier* H, pamg_vec* x, const pamg_vec* b, int ncycles,
                double* res_hist);
int pamg_vcycle_async(pamg_ctx* ctx, pamg_hier* H, pamg_vec* x, const pamg_vec* b, int ncycles);
/* Preconditioned CG on level 0 with one V-cycle (zero initial guess) as the preconditioner
 * (SPEC §S8; the Krylov caller of the path, e.g. IterativeSolvers.cg!(x, A, b; Pl = amg)).
 * Stops when ||r_k|| <= rtol ||r_0|| or after maxit iterations; *iters = iterations done;
 * res_hist (maxit + 1 entries, may be NULL) gets ||r_0||, ||r_1||, ... */
int pamg_pcg(pamg_ctx* ctx, pamg_hier* H, pamg_vec* x, const pamg_vec* b, double rtol,
             int maxit, int* iters, double* res_hist);
/* Kernel timing of the last pamg_vcycle/_async (events on the compute stream): per level,
 * milliseconds spent in [jacobi_pre, residual, restrict, prolong, jacobi_post, coarse]. */
int pamg_hier_profile(pamg_hier* H, int enable);
int pamg_hier_profile_read(pamg_hier* H, double* ms_per_level_op /* nlevels*6 */);

/* Micro-benchmark hook: `reps` back-to-back launches of one row operation of A (op 0 SpMV,
 * 1 residual, 2 Jacobi, 3 prolongate-add; no exchange; 4 / 5: the temporally blocked
 * Jacobi -> residual and Jacobi -> Jacobi -> residual passes, first output in y, where
 * pamg_mat_layout out[9] bit 5 is set), returning the average time per launch in ms measured
 * with HIP events on the launch stream. */
int pamg_bench_rowop(pamg_ctx* ctx, const pamg_mat* A, int op, pamg_vec* x, const pamg_vec* b,
                     pamg_vec* y, double omega, int reps, double* avg_ms);

/* Micro-benchmark hook of the cross-cycle pipeline: `reps` launches of its level-0 chain kernel
 * (post-smoothing -> next pre-smoothing -> residual, k_sym_zc<3>) on the hierarchy's own level-0
 * buffers and the given x / b (x is overwritten); average ms per launch (HIP events).
 * PAMG_E_STATE when the hierarchy does not qualify (one part, V(1,1), jr_fuse, level 0 with
 * pamg_mat_layout bit 5). */
int pamg_hier_bench_chain(pamg_hier* H, pamg_vec* x, const pamg_vec* b, int reps, double* avg_ms);

/* Process-wide knobs. Applied to later pamg_mat_upload calls: "tile_nnz" (1024 | 2048 | 4096,
 * nonzero budget of a 256-row tile), "tile_order" (0 natural | 1 banded XCD-blocked), "col24",
 * "long_tiles", "row_len8", "value_dict" (0 | 1 | 2), "col_dict", "col_dict_anchor", "col_dict_tile", "x_stage", "tm_tile_dicts" (0 | 1
 * layout features; "sym_dia": symmetric diagonal-class layout of a square operator's interior
 * rows where they qualify; "sym_rows" 1 | 2: rows per lane of its kernel; "jr_fuse": the
 * temporally blocked level-0 passes of the V-cycle and the cross-cycle pipeline, read at graph
 * capture), "long_tiles_min" (1..255 nonzeros per row from which sets of >= 32 x 4096
 * nonzeros per CU take 2048-nonzero tiles), "band_pct" / "band_pct_restrict" (percent scale of the banded
 * order's band; the second for operators with fewer rows than columns), "tile_major" (0 | 1 where measured faster | 2 every eligible set),
 * "sym_vd" (0 | 1: row-class dictionary of the symmetric layout), "ell" (0 | 1: sliced ELL for
 * large square operators with all own columns), "ell_restrict" (0 | 1: also restrictions, with
 * anchored offsets), "ell_min_rows" (rows from which ELL is taken), "ell_yblock" (0 | lines: the
 * blocked group order of a restriction over a grid), "pnc" (0 | 1: neighbour-coded
 * prolongations over a grid uploaded earlier on the context), "rpat" (0 | 1: pattern-dictionary
 * rows for restrictions whose rows repeat <= 255 patterns; tried before ELL), "pnc_compact" (0 | 1:
 * neighbour-coded rows as 16-bit ids of <= 1024 (pattern, values) combinations), "ell_pair" (0 | 1:
 * one ELL index byte per nonzero naming an (offset, value) pair where a group has <= 256). Read at launch:
 * "sym_zm" (0 | 1: z-marching single sweeps of the symmetric layout), "zm_chunks" (0 = auto |
 * z chunks per column of k_sym_zm), "tb_xfast" (0 | 1: x-fastest tile order of the chain),
 * "symd_chunks" (1 | 2 | 4), "chain_store_x" (0 | 1). Applied at every exchange:
 * "poison_ghosts" (0 | 1, debug: NaN-fill the ghost slots before each exchange). */
int pamg_set_option(const char* key, int64_t value);
int pamg_get_option(const char* key, int64_t* value);

/* ------------------------------------------------------------------ host setup (SPEC §S4) */
/* Host CSR: int64 rowptr, int32 columns (global ids), fp64 values. */
int pamg_hcsr_create(int64_t nrows, int64_t ncols, int64_t nnz, pamg_hcsr** out);
int pamg_hcsr_destroy(pamg_hcsr* M);
int pamg_hcsr_info(const pamg_hcsr* M, int64_t* nrows, int64_t* ncols, int64_t* nnz);
int pamg_hcsr_data(pamg_hcsr* M, int64_t** rowptr, int32_t** col, double** val);
/* Rows [r0, r1) of the SPEC §S2 grid operator; kind 0 poisson2d, 1 poisson3d, 2 aniso3d. */
int pamg_gen_grid(int kind, int64_t nx, int64_t ny, int64_t nz, double eps, int64_t r0,
                  int64_t r1, pamg_hcsr** out);
int pamg_gen_xstar(int64_t i0, int64_t n, uint64_t seed, double* out);
/* Rows [r0, r1) (r1 < 0: all) of a square Matrix Market coordinate file (real / integer /
 * pattern, general / symmetric), 1-based on disk, returned 0-based with ascending columns;
 * duplicates are summed in file order (BASELINE.json configs[4], SuiteSparse Flan_1565). */
int pamg_read_mtx(const char* path, int64_t r0, int64_t r1, int64_t* n_global, pamg_hcsr** out);
/* The file rows rows[0..nsel) (0-based, distinct) in that order — output row k is file row
 * rows[k]; columns keep the file numbering, ascending. A part's own rows under a renumbering
 * (e.g. its block of a reverse Cuthill-McKee order), without the whole matrix in memory. */
int pamg_read_mtx_rows(const char* path, int64_t nsel, const int64_t* rows, int64_t* n_global,
                       pamg_hcsr** out);
/* Entries per row of a Matrix Market file (symmetric mirrored): weights for the nnz-balanced
 * row partition (SPEC §S7). counts may be NULL to query *n_global only. */
int pamg_mtx_row_counts(const char* path, int64_t* n_global, int64_t* counts);
/* Reverse Cuthill-McKee order of a square matrix's (symmetrised) graph: order[k] = the old
 * row that becomes row k. The graph partitioner for irregularly numbered matrices (SURVEY
 * §8(f)-3): renumber with it, then cut contiguous nnz-balanced row blocks (SPEC §S7).
 * Deterministic (pseudo-peripheral start, neighbours by degree then index). */
int pamg_rcm_order(const pamg_hcsr* A, int64_t* order);
/* Locality order of a square level operator for pamg_mat_upload_perm: mode 0 identity,
 * 2 reverse Cuthill-McKee, 1 (auto) RCM only where the numbering is scattered — the mean row
 * span (largest - smallest column of a row) exceeds n/32 on a matrix of >= 4096 rows — and RCM
 * cuts that mean span at least 4x; else the identity. *applied = 1 when order is not the
 * identity; span_before / span_after (may be NULL) get the mean spans. */
int pamg_locality_order(const pamg_hcsr* A, int mode, int64_t* order, int* applied,
                        double* span_before, double* span_after);
/* Dense coarsest-level limit of pamg_setup_cholinv (rows); larger levels get PAMG_E_ARG. */
#define PAMG_MAX_DENSE_COARSE 16384
/* Gershgorin bound over own rows; A's rows are global rows row0.. (diagonal at col row0+i). */
int pamg_setup_gershgorin(const pamg_hcsr* A, int64_t row0, double* rho);
/* Decoupled standard aggregation (SPEC §S4.2-3): agg[i] local aggregate id or -1. */
int pamg_setup_aggregate(const pamg_hcsr* A, int64_t row0, double theta, int32_t* agg,
                         int64_t* n_agg);
/* Tentative prolongator rows: T[i, coarse0 + agg[i]] = 1/sqrt(|agg|). */
int pamg_setup_tentative(int64_t n, const int32_t* agg, int64_t n_agg, int64_t coarse0,
                         int64_t ncols_global, pamg_hcsr** out);
/* C = X * Y (SPEC §S4.5). Y's rows are the own rows [y0, y0+Yown.nrows) plus the ghost rows
 * Yghost whose global row ids are ghost_ids (ascending, n_ghost). Yghost may be NULL. */
int pamg_setup_spgemm(const pamg_hcsr* X, int64_t y0, const pamg_hcsr* Yown,
                      const int64_t* ghost_ids, int64_t n_ghost, const pamg_hcsr* Yghost,
                      pamg_hcsr** out);
/* In place: AT -> P = T - (omega / a_ii) * AT (SPEC §S4.6); A rows are global rows row0.. */
int pamg_setup_smooth(const pamg_hcsr* A, int64_t row0, const pamg_hcsr* T, pamg_hcsr* AT,
                      double omega);
/* Transpose of the local rows of P (global rows row0..) restricted to columns [c0, c1):
 * rows = coarse ids c0..c1-1, columns = global fine ids, ascending (SPEC §S4.7). */
int pamg_setup_transpose(const pamg_hcsr* P, int64_t row0, int64_t c0, int64_t c1,
                         pamg_hcsr** out);
/* GPU-side setup products: the contracts of pamg_setup_spgemm and
 * pamg_setup_transpose above, bit-identical results, computed on ctx's GPU (host CSR in and
 * out; device memory is released before returning). */
int pamg_dev_spgemm(pamg_ctx* ctx, const pamg_hcsr* X, int64_t y0, const pamg_hcsr* Yown,
                    const int64_t* ghost_ids, int64_t n_ghost, const pamg_hcsr* Yghost,
                    pamg_hcsr** out);
int pamg_dev_transpose(pamg_ctx* ctx, const pamg_hcsr* P, int64_t row0, int64_t c0, int64_t c1,
                       pamg_hcsr** out);
/* Row-wise concatenation of k CSR pieces with equal row counts (part order = column order). */
int pamg_setup_hstack_rows(int k, const pamg_hcsr* const* pieces, pamg_hcsr** out);
/* Dense Cholesky inverse of a full (single-piece) matrix, column-major out (SPEC §S5). */
int pamg_setup_cholinv(const pamg_hcsr* A, double* ainv_colmajor);

#ifdef __cplusplus
}
#endif
#endif /* PAMG_H */
