// pamg_device.h — device-side objects of libpamg (context, plans, vectors, matrices,
// hierarchy) and the kernel launchers of kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdint>
#include <array>
#include <mutex>
#include <vector>

#include "pamg_common.h"

namespace pamg {

// Row tiles of the LDS-staged CSR kernels (kernels.hip): each tile is a run of <= kTileRows
// consecutive rows (one per lane of the 256-thread workgroup) holding <= tile_nnz nonzeros;
// a row longer than the budget is a tile of its own in the "long" list.
constexpr int kBlock = 256;
constexpr int kTileRows = 256;

// x staging of row-relative dictionary tiles (TileSet::xs, k_rows_tm<..., XS>): the x values a
// tile reads are the runs [r0 + omin_c, r0 + nr - 1 + omin_c + wid_c] of its offset clusters c
// (offsets within kXsGap of each other share a run); they are loaded coalesced at kernel entry
// into LDS segments of `stride` doubles and the products read them there — no dependent x
// gathers. The dictionary table holds, at kXsIoff + index, each offset's LDS position
// c * stride + offset - omin_c.
constexpr int kXsMaxClusters = 12;
// tile-major sets of 2048-nonzero tiles: per-tile column / value tables of <= this many entries
constexpr int kTmSmallTab = 128;
constexpr int kXsCap = 1088;   // LDS doubles (8.5 KiB; 512^3 7-point: 5 runs x 210)
constexpr int kXsIoff = 128;   // table entries [128, 256): the LDS positions of offsets [0, 128)
constexpr int kXsGap = 48;
struct XStage {
    int ncl = 0, stride = 0, zix = -1, ncols = 0;
    int omin[kXsMaxClusters] = {}, wid[kXsMaxClusters] = {};
};
enum RowOp : int {
    OP_SPMV = 0,     // y = A x
    OP_RESID = 1,    // y = b - A x
    OP_JACOBI = 2,   // y = x + (omega (b - A x)) / a_ii
    OP_PROLONG = 3,  // y = y + A x      (x += P e)
};

struct TileSet {
    int4* d_short = nullptr;  // (row_begin, row_end, nnz_begin, nnz_end)
    int n_short = 0;
    int* d_long = nullptr;  // single rows
    int n_long = 0;
    int tile_nnz = 1024;  // nonzero budget the tiles were cut with
    // 24-bit column stream: every tile's columns lie in [base, base + 2^24), so a column is
    // stored as base (per tile) + 16-bit low part (pamg_mat::d_clo) + 8-bit high part (d_chi)
    int* d_base = nullptr;  // per short tile (same order as d_short), when c24
    bool c24 = false;
    // value dictionary (opt-in, Options::value_dict): every tile has <= 16 distinct values;
    // a value is a 4-bit index (pamg_mat::d_vidx) into the tile's 16-entry table
    double* d_vtab = nullptr;  // 16 per short tile
    bool vd = false;
    // 8-bit row lengths (pamg_mat::d_rlen) instead of row pointers: every row of a short tile
    // has <= 255 nonzeros (one row per lane, 24-bit columns, plain values)
    bool rl8 = false;
    // column dictionary (Options::col_dict; needs rl8): every nonzero of the short tiles has
    // column = row + d_ctab[i] for one of the set's <= 16 (cd = 4 bits) / <= 256 (cd = 8)
    // offsets; i is stored in pamg_mat::d_cidx (4 or 8 bits per nonzero)
    int cd = 0;
    int* d_ctab = nullptr;
    int ctab_n = 0;
    // anchored dictionary (Options::col_dict_anchor; tile-major sets only): column = the row's
    // first column + d_ctab[i]; the row anchors sit in the tile-major slots (d_tm_anc)
    bool anc = false;
    // per-tile dictionaries (Options::col_dict_tile; anchored: descriptor kernel, row-relative: tile-major slots): d_ctab holds
    // n_short tables of ctab_n entries; anchored ones take pamg_mat::d_anc16 + d_abase[tile]
    bool pt = false;
    int* d_abase = nullptr;
    // x staging (Options::x_stage): see XStage
    bool xs = false;
    XStage xst;
    // tile-major copies (Options::tile_major; kernels.hip k_rows_tm): tile t's values and
    // column stream at t * tile_nnz, its row lengths at t * tm_rs, zero-padded
    bool tm = false;
    int tm_rs = 0;                 // row-length slot per tile (>= its rows, multiple of 4)
    double* d_tm_val = nullptr;
    uint8_t* d_tm_cidx = nullptr;  // column dictionary indices (cd bits each)
    uint16_t* d_tm_clo = nullptr;  // or 24-bit columns: low 16 bits
    uint8_t* d_tm_chi = nullptr;   //   high 8 bits
    uint8_t* d_tm_rlen = nullptr;
    int* d_tm_anc = nullptr;       // anchored dictionary: each row's first column (tm_rs per tile)
    // 8-bit per-tile value dictionaries in tile-major slots (Options::value_dict, where every
    // tile of the set has <= 256 distinct values and the 4-bit ones do not fit): value = tile
    // t's table d_tm_vtab[t * tm_vt + index], index d_tm_vidx[t * tile_nnz + k]; d_tm_val unused
    int tm_vt = 0;                 // table entries per tile (0: plain values)
    uint8_t* d_tm_vidx = nullptr;
    double* d_tm_vtab = nullptr;
    // symmetric diagonal-class layout (Options::sym_dia; interior set of a square operator,
    // pamg_mat::sym): the set's rows run in k_rows_sym instead of tiles
    bool sym = false;
    // sliced-ELL layout (pamg_mat::ell; the whole interior set of a square operator): the set's rows run in
    // k_rows_ell instead of tiles
    bool ell = false;
    // neighbour-coded prolongation (pamg_mat::pnc; the whole set of a prolongation over a registered grid):
    // the rows run in k_rows_pnc instead of tiles
    bool pnc = false;
    // pattern-dictionary rows (pamg_mat::rpat; the whole interior set of a restriction): the rows run in
    // k_rows_rpat instead of tiles
    bool rpat = false;
    int max_short_len = 0;    // longest row in a short tile
    int64_t rows_short = 0;   // rows covered by the short tiles
    int64_t nnz_short = 0, nnz_long = 0;  // nonzeros covered by the tiles / the long rows
};

// Tuning knobs (pamg_set_option): kernel variant and tile budget used by later uploads.
struct Options {
    // defaults = fastest measured on MI355X at 512^3 (profiles/r01_kbench_*.jsonl):
    // 1024-nonzero / 256-row tiles
    int tile_nnz = 1024;       // 1024 / 2048 / 4096 (tiles always hold <= kTileRows rows)
    int tile_order = 1;        // 1: banded XCD-blocked tile order (see build_tiles)
    int col24 = 1;             // 1: 3-byte column stream where every tile's span fits 2^24
    int long_tiles = 1;        // 1: 4096-nonzero tiles for square operators with long rows (build_tiles)
    int long_tiles_min = 24;   // nonzeros per row from which sets of >= 32 x 4096 nonzeros per CU take 2048-nonzero tiles
    int row_len8 = 1;          // 1: 8-bit row lengths instead of 32-bit row pointers where they fit
    int value_dict = 1;        // 1: per-tile value dictionaries (4-bit for rectangular operators where a tile has
                               //    <= 16 distinct values, 8-bit in tile-major slots); 2: 8-bit ones only
    int col_dict = 1;          // 1: row-relative column dictionaries (4/8-bit) where they fit
    int tile_major = 1;        // tile-major padded copies (variant 4): 1 where measured faster, 2 all eligible
    int col_dict_tile = 1;     // 1: per-tile column dictionaries where no global table fits (and they beat 24-bit)
    int tm_tile_dicts = 1;     // 1: row-relative per-tile dictionary sets in tile-major slots (512^3 A1: -1..-3 %)
    int band_pct = 100;        // scale of the measured band of the XCD-blocked tile order (percent)
    int band_pct_restrict = 50;  // the same for operators with fewer rows than columns (restrictions)
    int x_stage = 1;           // 1: stage x runs in LDS for row-relative dictionary tile-major sets (no x gathers)
    int col_dict_anchor = 1;   // 1: anchored column dictionaries (col - row's first column) where row-relative ones do not fit
    int poison_ghosts = 0;     // 1 (debug): NaN-fill ghost slots before each exchange
    int sym_dia = 1;           // 1: symmetric diagonal-class layout for stencil-shaped symmetric operators
    int sym_rows = 2;          // rows per lane of its kernel (1 | 2)
    int jr_fuse = 1;           // 1: temporally blocked level-0 Jacobi -> residual / cross-cycle pipeline where the
                               //    operator is a grid stencil (k_sym_tb)
    int symd_chunks = 2;       // 512-row units per block of k_rows_symd (1, 2 or 4; 2: SpMV -2 %, residual and
                               // Jacobi -4..-5 %, 4: -1..-2 %; same-box A/B profiles/r04_g_c2/, r04_g_c4/)
    int chain_store_x = 0;     // 1: the pipelined chain also stores its post-smoothed iterate (never read)
    int tb_xfast = 1;          // blocked passes: tiles x-fastest (an XCD takes whole rows of tiles; chain -0.9 %,
                               // S = 2 pass -1.1 %, same-box A/B profiles/r05_l/) or y-fastest (0)
    int sym_zm = 1;            // 1: one-sweep ops of a whole one-part row-class grid operator march along z
                               //    (k_sym_zm); 0: k_rows_symd
    int zm_chunks = 0;         // z chunks per tile column of k_sym_zm (0: ~4 workgroups per CU)
    int ell = 1;               // 1: sliced ELL with per-group 8-bit dictionaries for square operators whose every row
                               //    is interior, where the tables fit (EllSet; the level-1 operator)
    int ell_min_rows = 65536;  // ... with at least this many rows
    int ell_restrict = 1;      // 1: also restrictions (fewer rows than columns), offsets from each row's first column
    int ell_yblock = 16;       // restrictions over a grid: groups processed in (y-block of this many lines, z, y)
                               //    order within each XCD's eighth (0: row order; 512^3 R0 0.81 -> 0.745 ms for any
                               //    block of 2..64 lines, profiles/r05_r/); read at upload
    int rpat = 1;              // 1: pattern-dictionary rows for restrictions whose rows repeat few patterns (RpatSet)
    int ell_pair = 1;          // 1: one index byte per ELL nonzero naming an (offset, value) pair where they fit
    int pnc_compact = 1;       // 1: 16-bit combination ids instead of 64-bit records where <= kPncCombMax fit
    int pnc = 1;               // 1: neighbour-coded prolongations over a grid registered on the context (PncSet)
    int sym_vd = 1;            // 1: row-class dictionary for the symmetric layout where the rows take <= kSymVdMax
                               //    distinct (mask, diagonal, upper values) tuples (SymDia::vd_n)
};

// Symmetric diagonal-class layout (k_rows_sym): a square operator whose interior rows use at
// most 2*kSymMaxU+1 row-relative offsets {-o_NU..-o_1, 0, o_1..o_NU} (a symmetric set), each
// row in ascending offset order, with bitwise-symmetric values a_ij == a_ji. Per own row i:
// the diagonal D[i], the upper values U_c[i] = a(i, i+o_c) (0 where absent), and a 16-bit
// mask (bit k: the k-th offset in ascending order is present; bit 15: the row belongs to the
// set). A lower value a(i, i-o_c) is read from its mirror U_c[i-o_c], so the matrix streams
// NU+1 values per row instead of 2*NU+1, with no column stream at all. (Where 2*NU+1 <= 7 the
// mask is one byte, the set flag in bit 7.)
constexpr int kSymMaxU = 7;
// Row-class dictionary of the symmetric layout (Options::sym_vd): at most this many distinct
// (mask, D, U_0 .. U_{nu-1}) bit tuples over the own rows; each row then stores its class id
// (1 byte) instead of mask + diagonal + nu upper values, the table sits in LDS
constexpr int kSymVdMax = 64;
// Temporal blocking of S dependent row sweeps (kernels.hip k_sym_tb): the operator is a 7-point
// grid stencil in natural order — classes {1, nx, nx*ny}, n = nx*ny*nz, and no row reaching
// across a grid line or plane (checked at upload) — so a workgroup owns a kTbX x kTbY column of
// the grid over a range of planes and streams it along z, computing the earlier sweeps on a
// halo it recomputes itself. No data passes between workgroups inside a launch.
struct TbGeom {
    int nx = 0, ny = 0, nz = 0;
    int tiles_x = 0, tiles_y = 0;   // kTbX x kTbY tiles of a plane
    int zchunks = 1, zlen = 0;      // planes per workgroup (the last chunk may be shorter)
    int zlo = 0, zhi = 0;           // output planes [zlo, zhi) of a launch (set by launch_sym_tb)
    int xfast = 0;                  // tile order: 0 y-fastest, 1 x-fastest (kernels.hip tb_ctx_init)
};
// Sliced ELL with per-group dictionaries (Options::ell; round 5, the level-1 operator and R0 of one
// part; on several parts the interior rows of a part's operator, its boundary rows carrying the length
// byte kEllSkip and running in tiles after the exchange): rows in
// slices of kEllW consecutive rows (one per lane of a wave), kEllGroup rows (a workgroup) sharing
// two tables of <= 256 entries — the rows' column offsets (col - row) and values (bit patterns).
// A slice stores its padded nonzeros k = 0 .. maxlen-1 as one column-index byte and one value-index
// byte per row, 4 consecutive k of a row packed in a dword, lanes interleaved: dword (k / 4, lane) at
// start + (k / 4) * kEllW + lane. Rows keep their storage order (the products are summed in it).
constexpr int kEllW = 64;
constexpr int kEllGroup = 256;
constexpr int kEllSkip = 255;  // length byte of a row outside the set (several parts: a boundary row)
struct EllSet {
    int64_t nslices = 0, ngroups = 0;
    int2* d_smeta = nullptr;     // per slice: (first dword of its index streams, maxlen)
    uint32_t* d_ci = nullptr;    // column-index stream
    uint32_t* d_vi = nullptr;    // value-index stream
    uint8_t* d_len = nullptr;    // per row: its length
    int4* d_gmeta = nullptr;     // per group: (offset-table start, entries, value-table start, entries)
    int* d_otab = nullptr;       // the groups' offset tables, concatenated
    double* d_vtab = nullptr;    // the groups' value tables, concatenated
    int* d_anc = nullptr;        // anchored (rectangular operators): per row the column its offsets start from
    // a restriction over a registered grid (its columns are the grid's points): the groups in a
    // processing order whose in-flight window is a compact (y, z) block of the grid instead of whole
    // planes (Options::ell_yblock; kernels.hip k_rows_ell), null otherwise
    int* d_gorder = nullptr;
    int64_t words = 0, otab_n = 0, vtab_n = 0;
    // paired dictionaries (Options::ell_pair): one index byte per nonzero names an (offset, value)
    // pair of the group (d_otab / d_vtab entries in parallel, gmeta .x == .z, .y == .w); d_vi null
    bool paired = false;
};

// Neighbour-coded prolongation (Options::pnc; round 5, the 512^3 P0): a prolongation (more rows than
// columns) whose rows are the points of a 7-point grid uploaded earlier on the same context — on one
// part all of them; on several parts a part's interior rows, its boundary rows (ghost columns) carrying
// the pattern id kPncSkip and running in tiles after the exchange (the grids: pamg_ctx::grids).
// Each column of row i is the anchor of one of the points i, i-1, i+1, i-nx, i+nx, i-M, i+M (codes 0..6) — the anchor of a row being the column of its largest
// value (in smoothed aggregation: the point's own aggregate; P = (I - w D^-1 A) P_tent reaches
// the aggregates of the point's stencil neighbours). Per row: the anchor (4 B) and a 64-bit record:
// bits 0-9 a pattern id (a global table of <= kPncPatMax words: bits 0-2 the row length, 3 + 3k
// the k-th entry's neighbour code), bits 10 + 7k the k-th entry's value index (a global table of
// <= kPncValMax bit patterns). 12 B per row against 3.5 B per nonzero + 1 B per row in tiles. Rows
// keep their storage order (SPEC S3 sums).
constexpr int kPncPatMax = 1024, kPncValMax = 128, kPncMaxLen = 7;
constexpr int kPncSkip = kPncPatMax - 1;  // pattern id of a row outside the set (several parts: a boundary row)
// Compact records (round 6): where the rows take at most kPncCombMax distinct (pattern word, value
// indices) combinations — 428 for the 512^3 P0, whose aggregates are nearly all alike — a row stores
// a 16-bit combination id (kPncCombSkip: outside the set) instead of the 64-bit record: 6 B per row
// with the anchor instead of 12. Then d_ptab holds the combinations' pattern words and d_pvals their
// value indices (7 bits per entry from bit 0), npat = the combinations, d_rec = null.
constexpr int kPncCombMax = 1024;
constexpr int kPncCombSkip = 0xffff;
struct PncSet {
    int nx = 0, ny = 0, nz = 0;
    int* d_anc = nullptr;       // nrows (+ pad)
    uint2* d_rec = nullptr;     // nrows (+ pad): the 64-bit records as (low, high) dwords
    uint16_t* d_cid = nullptr;  // compact records: nrows (+ pad) combination ids
    uint64_t* d_pvals = nullptr;
    uint32_t* d_ptab = nullptr;
    double* d_vtab = nullptr;
    int npat = 0, nval = 0;
    int grid = 0;               // workgroups of k_rows_pnc
};

// Pattern-dictionary rows (Options::rpat; round 6, the 512^3 R0): a restriction (fewer rows than columns)
// whose rows, read as (column - the row's first column, value bits) sequences in storage order, are
// copies of at most kRpatMax patterns of at most kRpatEnt entries in all. In smoothed aggregation a
// row of R = P^T is one aggregate's dilated shape, so the patterns are the aggregate shapes: 58 of
// them, 1,249 entries, for the 16.8M rows of the 512^3 R0 (the sliced ELL, 2 index bytes per padded
// nonzero, streamed 59 B per row). Per row: its first column (4 B) and pattern id (1 B; kRpatSkip: a
// row outside the set, several parts' boundary rows). Pattern p's entries at d_pent[start_p ..
// start_p + len_p): column offset in bits 0-23, value index (into d_vtab, <= 256 bit patterns) in
// bits 24-31. Rows keep their storage order (SPEC S3 sums); the groups of kEllGroup rows run in the
// ELL's blocked order over the registered grid of the columns (d_gorder) where there is one.
constexpr int kRpatMax = 255, kRpatEnt = 4096, kRpatMaxLen = 128;
constexpr int kRpatSkip = 255;
struct RpatSet {
    int64_t ngroups = 0;
    int* d_anc = nullptr;        // nrows (+ pad): the first column of each row
    uint8_t* d_pid = nullptr;    // nrows (+ pad): the pattern id of each row
    int2* d_pmeta = nullptr;     // per pattern: (first entry, entries)
    uint32_t* d_pent = nullptr;  // the patterns' entries, concatenated
    double* d_vtab = nullptr;    // the values' bit patterns
    int* d_gorder = nullptr;     // the groups' processing order (as EllSet::d_gorder), or null
    int npat = 0, nent = 0, nval = 0;
};

struct SymDia {
    int nu = 0;                     // upper offset classes
    int off[kSymMaxU] = {};         // ascending positive offsets
    int64_t ld = 0;                 // leading dimension of the U arrays
    int band = 0, band_blocks = 0, eighth = 0, nbands = 0;  // XCD-banded block order
    int rpl = 1;                    // rows per lane (k_rows_sym / k_rows_sym2)
    // temporally blocked sweeps (Options::jr_fuse; one part, every row in the set, nu = 3)
    bool tb_ok = false;
    // one part of several (z-slab of whole planes; a plane next to another part reads ghosts,
    // the set is the other planes): the blocked passes run on the planes whose halo stays inside
    // the set (S planes from a neighbour part) and the separate sweeps (with their exchanges) on
    // the rest (runtime.hip jr_part)
    bool tb_part = false;
    int part_lo = 0, part_hi = 0;   // the set's planes [part_lo, part_hi) (the others read ghosts)
    int plane0 = 0;                 // first plane of a plane-range launch of k_rows_sym / sym2
    int gap_at = 1 << 30, gap = 0;  // ... whose planes from gap_at on are shifted by gap (a second window)
    TbGeom tb;
    uint8_t* d_mask = nullptr;      // nrows (+ pad) masks of 1 byte (2 nu + 1 <= 7) or 2 bytes
    int mask_bytes = 2;
    double* d_diag = nullptr;       // nrows (+ pad)
    double* d_upper = nullptr;      // nu * ld
    // row-class dictionary (vd_n > 0; then d_mask / d_diag / d_upper are not allocated): row i's
    // class d_tid[i]; class e's values d_vtab[e * (nu + 1) + {0: D, 1 + c: U_c}], mask d_mtab[e]
    // (the in-set flag included); the lower value a(i, i - o_c) is U_c of class d_tid[i - o_c]
    int vd_n = 0;
    int vd_main = 0;                // the most frequent class (k_rows_symd's register fast path)
    uint8_t* d_tid = nullptr;       // nrows (+ pad)
    double* d_vtab = nullptr;
    uint32_t* d_mtab = nullptr;
};
Options& options();

}  // namespace pamg

struct pamg_ctx {
    int device = 0;
    // references: the caller's handle + one per plan / vector / matrix / hierarchy on it
    // (runtime.hip ctx_ref / ctx_unref); the context is torn down when the last one is dropped
    std::atomic<int> refs{1};
    hipStream_t s_comp = nullptr;  // compute stream
    hipStream_t s_comm = nullptr;  // ghost exchange stream
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    ncclComm_t comm = nullptr;
    int rank = 0, nranks = 1;
    pamg_host_comm_fn host_fn = nullptr;  // debug transport (pamg_comm_init_host)
    void* host_user = nullptr;
    pamg_world* world = nullptr;           // in-process transport (pamg_comm_init_local)
    hipEvent_t ev_ready = nullptr;         //   "the vector I posted is written" (on s_comp / s_comm)
    std::vector<double> h_send, h_recv;   // staging for the debug transport
    double* d_red = nullptr;  // reduction workspace (partials + result)
    int red_cap = 0;
    double* h_red = nullptr;  // pinned host scalar
    // upload staging (runtime.hip h2d): two pinned 64 MiB buffers and their DMA-done events,
    // created on first use on this context's device and owned by the context
    char* stage[2] = {nullptr, nullptr};
    hipEvent_t stage_done[2] = {nullptr, nullptr};
    // 7-point grids of the square operators uploaded on this context in the temporally blocked
    // layout (SymDia::tb_ok): (rows, nx, ny, nz) — a later prolongation with as many rows may take
    // the neighbour-coded layout over one of them (pamg::PncSet)
    std::vector<std::array<int64_t, 4>> grids;
    std::mutex grids_mu;  // (uploads on one context from several host threads)
};

void ctx_ref(pamg_ctx* ctx);
void ctx_unref(pamg_ctx* ctx);

struct pamg_plan {
    pamg_ctx* ctx = nullptr;
    int64_t n_own = 0, n_ghost = 0;
    std::vector<int> nbr;
    std::vector<int64_t> recv_off, send_off;  // n_nbr + 1
    int* d_send_idx = nullptr;
    double* d_sendbuf = nullptr;
    // per neighbour: first own index if its send list is one contiguous run (the boundary
    // planes of a slab partition), else -1; all_contig: no pack kernel is needed at all
    std::vector<int64_t> send_run;
    bool all_contig = false;
    // split exchange (pamg_exchange_begin / _end): completion event on the comm stream
    hipEvent_t ev_done = nullptr;
    const void* in_flight = nullptr;  // the vector of the exchange begun and not yet ended
    // identity of the index space the plan describes, the same on every part (pamg_plan_set_tag;
    // 0 = untagged): the in-process world refuses to pair two parts' exchanges whose tags differ
    int64_t tag = 0;
};

struct pamg_vec {
    pamg_ctx* ctx = nullptr;
    int64_t n_own = 0, n_ghost = 0;
    double* d = nullptr;  // n_own + n_ghost (+ padding)
};

struct pamg_mat {
    pamg_ctx* ctx = nullptr;
    int64_t nrows = 0, ncols = 0, nnz = 0;
    int* d_rowptr = nullptr;
    int* d_col = nullptr;
    uint16_t* d_clo = nullptr;  // 24-bit column stream (TileSet::c24): low 16 bits
    uint8_t* d_chi = nullptr;   //   and high 8 bits of (column - tile base)
    uint8_t* d_vidx = nullptr;  // value dictionary indices, two per byte (TileSet::vd)
    uint8_t* d_rlen = nullptr;  // row lengths, when a tile set uses them (TileSet::rl8)
    uint8_t* d_cidx = nullptr;  // column dictionary indices (TileSet::cd; 4 or 8 bits each)
    uint16_t* d_anc16 = nullptr;  // per-tile anchored dictionaries: row's first column - tile base
    double* d_val = nullptr;
    double* d_diag = nullptr;  // a_ii for square matrices (zero-guess Jacobi), else null
    const pamg_plan* plan = nullptr;
    pamg::SymDia sym;        // the interior set's symmetric diagonal-class layout (TileSet::sym)
    pamg::TileSet interior;  // rows with own columns only (overlap with the exchange)
    pamg::TileSet boundary;  // rows with >= 1 ghost column
    pamg::EllSet ell;        // the interior set's sliced-ELL layout (TileSet::ell)
    pamg::PncSet pnc;        // the neighbour-coded prolongation layout (TileSet::pnc)
    pamg::RpatSet rpat;      // the pattern-dictionary restriction layout (TileSet::rpat)
    int64_t stream_bytes = 0;  // matrix bytes one apply reads (values, columns, row pointers, tiles)
};

namespace pamg {

// kernels.hip launchers (all asynchronous on `s`).
void launch_rows(const pamg_mat& A, const TileSet& ts, int op, const double* x, const double* b,
                 const double* xold, double* y, double omega, hipStream_t s);
void launch_jacobi_zero(int64_t n, const double* b, const double* diag, double omega, double* y,
                        hipStream_t s);
void launch_dense_gemv(int64_t n_rows, int64_t n_cols, int64_t row0, const double* ainv_rm,
                       const double* b, double* y, hipStream_t s);
void launch_pack(int64_t n, const int* idx, const double* x, double* out, hipStream_t s);
void launch_fill(int64_t n, double v, double* y, hipStream_t s);
// S (2 | 3) dependent sweeps in one temporally blocked launch (k_sym_tb; A.sym.tb_ok): stage 0
// is a weighted-Jacobi sweep from in0 into out[0]; stage s > 0 reads stage s-1's result, a
// Jacobi sweep into out[s], the last one the residual b - A t when last_resid.
struct TbArgs {
    int nstages = 0;
    bool last_resid = false;
    const double* in0 = nullptr;
    double* out[3] = {nullptr, nullptr, nullptr};
    const double* b = nullptr;
    double omega = 0.0;
};
constexpr int kTbX = 64, kTbY = 16;  // output tile of a workgroup (grid points in x, y)
void launch_sym_tb(const pamg_mat& A, const TbArgs& ta, hipStream_t s);
// a row operation of the symmetric set on the grid planes [p0, p1) and [p2, p3) only (band = one
// plane; p1 <= p2), one launch
void launch_sym_planes(const pamg_mat& A, int op, int p0, int p1, const double* x, const double* b, double* y,
                       double omega, hipStream_t s, int p2 = 0, int p3 = 0);
// dst[i] = src[perm[i]] (gather), or dst[perm[i]] = src[i] (scatter)
void launch_permute(int64_t n, const int* perm, const double* src, double* dst, bool scatter, hipStream_t s);
void launch_axpby(int64_t n, double a, const double* x, double b, double* y, hipStream_t s);
// Deterministic two-pass dot: writes the local sum to *out (device).
void launch_dot(int64_t n, const double* x, const double* y, double* partials, int nparts,
                double* out, hipStream_t s);
int dot_partials(int64_t n);
// x += alpha p; r -= alpha q; out = r.r (bit-identical to two launch_axpby + launch_dot)
void launch_cg_update(int64_t n, double alpha, const double* p, const double* q, double* x, double* r,
                      double* partials, int np, double* out, hipStream_t s);

}  // namespace pamg
