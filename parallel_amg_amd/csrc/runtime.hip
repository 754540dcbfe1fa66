// runtime.hip — C-ABI implementation of the device side of libpamg (include/pamg.h):
// context and streams, RCCL communicator, exchange plans (PartitionedArrays' PRange ghost
// layout), device vectors and matrices, mul!/residual/Jacobi with the ghost exchange
// overlapped with the interior rows, and the V-cycle driver (SPEC.md §S6) replayed as a
// captured hipGraph.
#include <dlfcn.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <functional>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "pamg_device.h"

using pamg::fail;

pamg::Options& pamg::options() {
    static Options o;
    return o;
}

#define HIPC(expr)                                                                    \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(PAMG_E_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr,        \
                        hipGetErrorString(e_));                                       \
    } while (0)

#define NCCLC(expr)                                                                   \
    do {                                                                              \
        ncclResult_t r_ = (expr);                                                     \
        if (r_ != ncclSuccess)                                                        \
            return fail(PAMG_E_RCCL, "%s:%d %s: %s", __FILE__, __LINE__, #expr,       \
                        ncclGetErrorString(r_));                                      \
    } while (0)

#define CHECK(expr)                   \
    do {                              \
        int rc_ = (expr);             \
        if (rc_ != PAMG_OK) return rc_; \
    } while (0)

namespace {

constexpr int kVecPad = 8;  // trailing doubles so 16-byte vector loads never run off the end

template <class T>
int dalloc(T** p, int64_t n) {
    *p = nullptr;
    if (n <= 0) return PAMG_OK;
    HIPC(hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (size_t)n));
    return PAMG_OK;
}

template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree(p);
    p = nullptr;
}

int set_device(const pamg_ctx* ctx) {
    HIPC(hipSetDevice(ctx->device));
    return PAMG_OK;
}

// ---- host side of the upload: threads for the per-nonzero passes, pinned staging for copies
// Threads: OMP_NUM_THREADS if set (16 on the GPU box), else the hardware count, at most 64.
// Zero device memory in the context's stream order and wait for it: hipMemset runs on the
// null stream, which the context's non-blocking streams do not wait for, so a kernel enqueued
// right after it could run first (found in round 5: PCG's first initial residual raced with the
// zeroing of its freshly allocated vectors).
int dzero(pamg_ctx* ctx, void* p, size_t bytes) {
    HIPC(hipMemsetAsync(p, 0, bytes, ctx->s_comp));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int host_threads() {
    static const int n = [] {
        const char* e = std::getenv("OMP_NUM_THREADS");
        int v = e ? std::atoi(e) : 0;
        if (v <= 0) v = (int)std::thread::hardware_concurrency();
        return std::max(1, std::min(v, 64));
    }();
    return n;
}

// f(begin, end) over [0, n) in contiguous chunks, one per thread (each chunk's work is
// independent of the others; results are the same for any thread count)
template <class F>
void par_for(int64_t n, F&& f) {
    const int nt = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, n / 16384));
    if (nt <= 1) {
        if (n > 0) f((int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(nt);
    for (int t = 0; t < nt; ++t) {
        const int64_t a = n * t / nt, b = n * (t + 1) / nt;
        th.emplace_back([&f, a, b] { f(a, b); });
    }
    for (auto& x : th) x.join();
}

// Host-to-device copy of a large pageable buffer through two pinned 64 MiB staging buffers:
// threads copy chunk k into one while the DMA engine moves chunk k-1 out of the other.
int h2d(pamg_ctx* ctx, void* dst, const void* src, size_t bytes) {
    constexpr size_t kChunk = size_t(64) << 20;
    if (bytes == 0) return PAMG_OK;
    if (bytes < (size_t(4) << 20)) {
        HIPC(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
        return PAMG_OK;
    }
    // per context (one host thread per context, pamg.h): the events belong to ctx's device
    char** stage = ctx->stage;
    hipEvent_t* done = ctx->stage_done;
    for (int k = 0; k < 2; ++k) {
        if (!stage[k]) HIPC(hipHostMalloc(reinterpret_cast<void**>(&stage[k]), kChunk, hipHostMallocPortable));
        if (!done[k]) HIPC(hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
    }
    hipStream_t s = ctx->s_comp;
    size_t off = 0;
    for (int k = 0; off < bytes; k ^= 1) {
        const size_t m = std::min(kChunk, bytes - off);
        HIPC(hipEventSynchronize(done[k]));  // the DMA out of this buffer has finished
        const char* from = static_cast<const char*>(src) + off;
        char* to = stage[k];
        par_for((int64_t)((m + 4095) / 4096), [&](int64_t a, int64_t b) {
            const size_t lo = (size_t)a * 4096, hi = std::min(m, (size_t)b * 4096);
            std::memcpy(to + lo, from + lo, hi - lo);
        });
        HIPC(hipMemcpyAsync(static_cast<char*>(dst) + off, to, m, hipMemcpyHostToDevice, s));
        HIPC(hipEventRecord(done[k], s));
        off += m;
    }
    HIPC(hipStreamSynchronize(s));
    return PAMG_OK;
}

// PAMG_TRACE_UPLOAD=1: per-phase host times of each matrix upload on stderr
// std::vector storage whose sizing constructor leaves the elements uninitialised: the upload's
// column and row-pointer copies (up to 3.75 GB at 512^3) are filled by parallel loops, not zeroed
// first on one thread
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <class U, class... Args>
    void construct(U* p, Args&&... args) {
        if constexpr (sizeof...(Args) == 0)
            ::new ((void*)p) U;
        else
            ::new ((void*)p) U(std::forward<Args>(args)...);
    }
};
using IdxVec = std::vector<int, NoInitAlloc<int>>;
using PtrVec = std::vector<int64_t, NoInitAlloc<int64_t>>;


struct UploadTrace {
    bool on = std::getenv("PAMG_TRACE_UPLOAD") != nullptr;
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    int64_t nnz = 0;
    void mark(const char* what) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "[pamg upload nnz=%lld] %-14s %8.3f s\n", (long long)nnz, what,
                     std::chrono::duration<double>(now - t).count());
        t = now;
    }
};

// Compute units of the current device (256 on MI355X), for occupancy-keyed layout rules
int device_cus() {
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return 256;
    return cus;
}

// Greedy tiling of the rows listed in `rows` (ascending) into runs of consecutive rows with
// <= kTileRows rows and <= tile_nnz nonzeros; rows above the budget become "long" rows.
// tile_order 1 (banded XCD-blocked order) for a square matrix of half-bandwidth `band`:
// cut the rows into super-rows of `band` rows (one grid plane for the stencils), give XCD k
// the k-th eighth of every super-row, and interleave the 8 sequences so block b (XCD b % 8,
// as dispatch is observed to deal blocks) walks its eighth plane after plane. The x lines of
// rows z-1, z, z+1 of one eighth then stay in that XCD's L2. Speed only: any order is correct.
// (Cutting each eighth into sub-slabs walked one after another was measured slower on every
// operator and removed: DESIGN.md "Measured and rejected".)
static std::vector<int4> xcd_band_order(const std::vector<int4>& tiles, int64_t band) {
    std::vector<std::vector<int4>> bucket(8);
    for (const auto& t : tiles) bucket[((int64_t)(t.x % band) * 8) / band].push_back(t);
    size_t m = 0;
    for (auto& b : bucket) m = std::max(m, b.size());
    std::vector<int4> out;
    out.reserve(8 * m);
    for (size_t i = 0; i < m; ++i)
        for (int k = 0; k < 8; ++k) out.push_back(i < bucket[k].size() ? bucket[k][i] : make_int4(0, 0, 0, 0));
    return out;
}

// Value dictionaries of a 24-bit tile set: every tile holds <= 16 distinct values (bit
// patterns, so -0.0 / NaN payloads survive); indices go to vidx (4 bits per entry). Tiles are
// independent (tables in parallel); the indices go through a byte per nonzero and are packed by
// byte afterwards, since two tiles can share the byte of an odd boundary.
int build_value_dict(const std::vector<int4>& tiles, const double* val, pamg::TileSet* ts,
                     std::vector<uint8_t>* vidx, size_t nslots) {
    const int64_t nt = (int64_t)tiles.size();
    std::vector<double> tab(tiles.size() * 16, 0.0);
    std::atomic<bool> over{false};
    par_for(nt, [&](int64_t a, int64_t b) {
        for (int64_t t = a; t < b && !over; ++t) {
            uint64_t key[16];
            int nk = 0;
            for (int k = tiles[t].z; k < tiles[t].w; ++k) {
                uint64_t u;
                std::memcpy(&u, &val[k], 8);
                int j = 0;
                while (j < nk && key[j] != u) ++j;
                if (j == nk) {
                    if (nk == 16) {  // does not fit: plain values for this set
                        over = true;
                        return;
                    }
                    key[nk++] = u;
                    tab[t * 16 + j] = val[k];
                }
            }
        }
    });
    if (over) return PAMG_OK;
    std::vector<uint8_t> one(2 * nslots, 0);  // nonzeros outside every tile (long rows) keep 0
    par_for(nt, [&](int64_t a, int64_t b) {
        for (int64_t t = a; t < b; ++t) {
            const double* tt = &tab[t * 16];
            for (int k = tiles[t].z; k < tiles[t].w; ++k) {
                int j = 0;
                while (std::memcmp(&tt[j], &val[k], 8) != 0) ++j;
                one[k] = (uint8_t)j;
            }
        }
    });
    if (vidx->empty()) vidx->assign(nslots, 0);
    par_for((int64_t)nslots, [&](int64_t a, int64_t b) {
        for (int64_t q = a; q < b; ++q) (*vidx)[q] |= (uint8_t)(one[2 * q] | (one[2 * q + 1] << 4));
    });
    CHECK(dalloc(&ts->d_vtab, (int64_t)tab.size()));
    HIPC(hipMemcpy(ts->d_vtab, tab.data(), sizeof(double) * tab.size(), hipMemcpyHostToDevice));
    ts->vd = true;
    return PAMG_OK;
}

// Per own column: the largest gap between consecutive rows that read it (0 if fewer than two
// do). Row chunks in parallel, each over the column range its rows touch (first / last reader
// and the largest gap inside the chunk), then merged per column in chunk order: the values of
// one sequential pass. A matrix whose chunks together span more than ~2x the columns (no band
// structure) takes the sequential pass.
std::vector<int> column_reuse_gaps(const PtrVec& rp, const IdxVec& ci, int64_t nrows,
                                   int64_t ncols) {
    std::vector<int> gap(ncols, 0);
    const int nch = (int)std::min<int64_t>(host_threads(), std::max<int64_t>(1, nrows / 65536));
    std::vector<int64_t> r0(nch + 1);
    for (int t = 0; t <= nch; ++t) r0[t] = nrows * t / nch;
    // one thread per chunk (par_for would keep a handful of items on one thread)
    auto each_chunk = [nch](const std::function<void(int)>& f) {
        std::vector<std::thread> th;
        for (int t = 0; t < nch; ++t) th.emplace_back([&f, t] { f(t); });
        for (auto& x : th) x.join();
    };
    std::vector<int> lo(nch, INT32_MAX), hi(nch, -1);
    each_chunk([&](int t) {
        int a = INT32_MAX, b = -1;
        for (int64_t k = rp[r0[t]]; k < rp[r0[t + 1]]; ++k)
            if (ci[k] < ncols) {
                a = std::min(a, ci[k]);
                b = std::max(b, ci[k]);
            }
        lo[t] = a;
        hi[t] = b;
    });
    int64_t span = 0;
    for (int t = 0; t < nch; ++t) span += hi[t] >= lo[t] ? (int64_t)hi[t] - lo[t] + 1 : 0;
    if (nch == 1 || span > 2 * ncols + 65536) {
        std::vector<int> last(ncols, -1);
        for (int64_t i = 0; i < nrows; ++i)
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                const int c = ci[k];
                if (c < ncols) {
                    if (last[c] >= 0) gap[c] = std::max(gap[c], (int)i - last[c]);
                    last[c] = (int)i;
                }
            }
        return gap;
    }
    // per chunk, over [lo, hi]: first reader, last reader, largest gap inside the chunk
    std::vector<std::vector<int>> first(nch), last(nch), cgap(nch);
    each_chunk([&](int t) {
        if (hi[t] < lo[t]) return;
        const int64_t w = (int64_t)hi[t] - lo[t] + 1;
        first[t].assign(w, -1);
        last[t].assign(w, -1);
        cgap[t].assign(w, 0);
        int* f = first[t].data();
        int* l = last[t].data();
        int* g = cgap[t].data();
        for (int64_t i = r0[t]; i < r0[t + 1]; ++i)
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                const int c = ci[k];
                if (c >= ncols) continue;
                const int j = c - lo[t];
                if (l[j] >= 0) g[j] = std::max(g[j], (int)i - l[j]);
                else f[j] = (int)i;
                l[j] = (int)i;
            }
    });
    par_for(ncols, [&](int64_t a, int64_t b) {
        for (int64_t c = a; c < b; ++c) {
            int g = 0, prev = -1;
            for (int t = 0; t < nch; ++t) {
                if (c < lo[t] || c > hi[t]) continue;
                const int64_t j = c - lo[t];
                if (first[t][j] < 0) continue;
                if (prev >= 0) g = std::max(g, first[t][j] - prev);
                g = std::max(g, cgap[t][j]);
                prev = last[t][j];
            }
            gap[c] = g;
        }
    });
    return gap;
}

int build_tiles(const PtrVec& rp, const std::vector<int>& rows, bool square,
                pamg::TileSet* ts, int64_t band, const IdxVec& ci,
                std::vector<uint16_t>* lo, std::vector<uint8_t>* hi, const double* val,
                std::vector<uint8_t>* vidx, std::vector<int4>* tiles_out, bool tall = false) {
    const auto& opt = pamg::options();
    int tnnz = opt.tile_nnz;
    const int trows = pamg::kTileRows;
    // long_tiles: operators with long rows (coarse A_l, R_l: >= 48 nonzeros per row on
    // average) take 4096-nonzero tiles instead of the default 1024 — their time goes into the
    // in-order add chain of each row (SPEC §S3), and a tile of 4x the rows runs 4x the chains
    // side by side (512^3: A2 0.139 -> 0.110 ms, R1 0.458 -> 0.439 ms,
    // profiles/r01_kbench_512_tnnz.jsonl); the 7- and 27-point levels keep 1024. Square
    // operators only: the long-row restriction R1 (188 nonzeros per row, tile-major) is 9 %
    // faster with 1024 (profiles/r02_exp/kbench512_level12_tiles.jsonl), A2 13 % slower.
    if (opt.long_tiles && square && tnnz == 1024 && !rows.empty()) {
        int64_t nz = 0;
        for (int r : rows) nz += rp[r + 1] - rp[r];
        // >= 48 per row always; from long_tiles_min (24) per row when the set is large enough
        // to keep the chip full with 4096-nonzero tiles: >= 32 of them per CU (512^3 A1, 31 per
        // row, ~500 tiles per CU on one GPU and ~60 on each of 8: residual -3 %, Jacobi -2 %;
        // the 6 M-nonzero A1 of 128^3, 6 per CU, is 9 % slower with them,
        // profiles/r02_exp/bench_long_tiles_min_ab/). Keyed on the CU count, not on a fixed
        // nonzero count, so a part of an 8-GPU run takes the layout one GPU takes.
        // Round 3 (8-bit per-tile value dictionaries): the set under the second rule (512^3 A1)
        // takes 2048-nonzero tiles — residual + Jacobi 1.85 -> 1.80 ms on one box; 3072 1.83
        // (profiles/r03_jdiag/kb.jsonl) — A2 (>= 48 per row) stays at 4096 (2048: Jacobi +5 %).
        const int64_t nr = (int64_t)rows.size();
        if (nz >= 48 * nr)
            tnnz = 4096;
        else if (nz >= (int64_t)opt.long_tiles_min * nr && nz >= int64_t(32) * 4096 * device_cus())
            tnnz = 2048;
    } else if (opt.long_tiles && !square && !tall && tnnz == 1024 && !rows.empty()) {
        // Round 4: a restriction with 24 .. 47 nonzeros per row on a set large enough for the
        // rule above (512^3 R0: 32 per row, anchored dictionary in tile-major slots) takes
        // 2048-nonzero tiles: 1.09-1.10 -> 1.03 ms (4096: 1.03), profiles/r04_p/kbench_tn.jsonl;
        // the long-row R1 (~150 per row) stays at 1024 (2048 / 4096: +14-16 %, r03)
        int64_t nz = 0;
        for (int r : rows) nz += rp[r + 1] - rp[r];
        const int64_t nr = (int64_t)rows.size();
        if (nz >= (int64_t)opt.long_tiles_min * nr && nz < 48 * nr && nz >= int64_t(32) * 4096 * device_cus())
            tnnz = 2048;
    }
    ts->tile_nnz = tnnz;
    std::vector<int4> tiles;
    std::vector<int> longr;
    size_t i = 0;
    while (i < rows.size()) {
        const int r = rows[i];
        const int64_t len = rp[r + 1] - rp[r];
        // the kernel streams [rp[r] & ~3, end): the alignment head counts against the budget
        const int64_t head = rp[r] & 3;
        if (head + len > tnnz) {
            longr.push_back(r);
            ++i;
            continue;
        }
        int end = r + 1;
        int64_t nz = head + len;
        size_t j = i + 1;
        while (j < rows.size() && rows[j] == end && end - r < trows) {
            const int64_t l2 = rp[end + 1] - rp[end];
            if (nz + l2 > tnnz) break;
            nz += l2;
            ++end;
            ++j;
        }
        tiles.push_back(make_int4(r, end, (int)rp[r], (int)rp[end]));
        ts->nnz_short += rp[end] - rp[r];
        ts->rows_short += end - r;
        for (int q = r; q < end; ++q) ts->max_short_len = std::max(ts->max_short_len, (int)(rp[q + 1] - rp[q]));
        i = j;
    }
    for (int r : longr) ts->nnz_long += rp[r + 1] - rp[r];
    if (opt.tile_order == 1 && band >= 64 && tiles.size() >= 64) tiles = xcd_band_order(tiles, band);
    ts->n_short = (int)tiles.size();
    ts->n_long = (int)longr.size();
    CHECK(dalloc(&ts->d_short, ts->n_short));
    CHECK(dalloc(&ts->d_long, ts->n_long));
    // 24-bit column stream: usable when every tile's columns span < 2^24 (banded matrices;
    // not for tiles that reach the ghost columns of a large part)
    ts->c24 = false;
    if (opt.col24 && !tiles.empty()) {
        const int64_t nt = (int64_t)tiles.size();
        std::vector<int> base(nt, 0);
        std::vector<char> fit(nt, 1);
        par_for(nt, [&](int64_t a, int64_t b) {
            for (int64_t t = a; t < b; ++t) {
                const int4 d = tiles[t];
                int mn = INT32_MAX, mx = 0;
                for (int k = d.z; k < d.w; ++k) {
                    mn = std::min(mn, ci[k]);
                    mx = std::max(mx, ci[k]);
                }
                if (d.w == d.z) mn = mx = 0;
                base[t] = mn;
                fit[t] = (int64_t)mx - mn < (int64_t(1) << 24);
            }
        });
        if (std::all_of(fit.begin(), fit.end(), [](char f) { return f != 0; })) {
            if (lo->empty()) {
                lo->assign(ci.size(), 0);
                hi->assign(ci.size(), 0);
            }
            par_for(nt, [&](int64_t a, int64_t b) {
                for (int64_t t = a; t < b; ++t)
                    for (int k = tiles[t].z; k < tiles[t].w; ++k) {
                        const uint32_t dlt = (uint32_t)(ci[k] - base[t]);
                        (*lo)[k] = (uint16_t)(dlt & 0xffffu);
                        (*hi)[k] = (uint8_t)(dlt >> 16);
                    }
            });
            CHECK(dalloc(&ts->d_base, (int64_t)tiles.size()));
            HIPC(hipMemcpy(ts->d_base, base.data(), sizeof(int) * base.size(), hipMemcpyHostToDevice));
            ts->c24 = true;
        }
    }
    // 4-bit per-tile value dictionaries for the prolongations (more rows than columns: P0
    // 1.21 ms vs 1.40 with 8-bit column dictionaries, 512^3, profiles/r03_r0/); the other
    // operators keep their column dictionaries in tile-major slots with 8-bit value
    // dictionaries there (build_tile_major: R0 1.06 vs 1.12 ms, elastic3d 80^3 A0 0.206 vs
    // 0.237 ms, profiles/r03_r0/, profiles/r03_e80/)
    ts->vd = false;
    if (opt.value_dict == 1 && ts->c24 && val && tall)
        CHECK(build_value_dict(tiles, val, ts, vidx, (ci.size() + 1) / 2 + 8));
    ts->rl8 = opt.row_len8 && ts->c24 && ts->max_short_len <= 255 && ts->n_short > 0 &&
              ts->nnz_short <= 16 * ts->rows_short;
    // ^ short rows only: the 3 B/row saved are 3-8 % of a 4-7-nonzero row (A0 SpMV -2 %, P0
    //   -5..-8 %) but ~1 % of a 30-nonzero row, where the scan's latency costs more (R0, A1
    //   +2..3 %; profiles/r01_kbench_512_rl8.jsonl); with the value dictionaries too (P0)
    if (ts->n_short)
        HIPC(hipMemcpy(ts->d_short, tiles.data(), sizeof(int4) * tiles.size(), hipMemcpyHostToDevice));
    if (ts->n_long)
        HIPC(hipMemcpy(ts->d_long, longr.data(), sizeof(int) * longr.size(), hipMemcpyHostToDevice));
    tiles_out->swap(tiles);
    return PAMG_OK;
}

// Per-tile column dictionaries (Options::col_dict_tile) for tile sets no global table fits:
// every tile carries its own table of <= 256 offsets (capacity ctab_n = the largest tile's
// count rounded up to a power of two >= 16, so 4-bit indices where every tile has <= 16),
// row-relative (col - row: the coarse operators, 33 offsets per tile on average for A1 at
// 512^3 against ~10^4 in the whole matrix) or anchored (col - the row's middle column, stored
// as a 16-bit delta from a per-tile base: the prolongators, a few per tile). The form
// with fewer bytes is taken, and only if it streams less than the 24-bit columns; it runs in
// the descriptor kernel (k_rows_tile2), not in tile-major slots.
int build_tile_dicts(pamg_mat* A, const PtrVec& rp, const IdxVec& ci,
                     const std::vector<int4>& tiles, pamg::TileSet* ts, std::vector<uint8_t>* idx,
                     std::vector<int>* tab, std::vector<uint16_t>* anc16) {
    const int64_t nt = (int64_t)tiles.size();
    if (nt == 0) return PAMG_OK;
    // anchor of a row: its middle column (for a prolongator row, its own aggregate's
    // neighbourhood), so one tile's anchors stay within a 16-bit span
    auto mid_col = [&](int r) { return rp[r + 1] > rp[r] ? ci[rp[r] + (rp[r + 1] - rp[r] - 1) / 2] : 0; };
    int64_t nz = 0, rows = 0;
    for (const int4& t : tiles) {
        nz += t.w - t.z;
        rows += t.y - t.x;
    }
    // per tile: distinct offsets in first-occurrence order (count only), both forms
    std::vector<int> cnt_rel(nt), cnt_anc(nt), base(nt, 0);
    std::vector<char> span_ok(nt, 1);
    auto distinct = [&](const int4& t, bool anchored, int* out_tab, int cap) {
        constexpr int kCells = 2048;
        int key[kCells], slot[kCells];
        std::fill(slot, slot + kCells, -1);
        int n = 0;
        for (int r = t.x; r < t.y; ++r) {
            const int an = anchored ? mid_col(r) : r;
            for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
                const int o = ci[k] - an;
                uint32_t h = ((uint32_t)o * 0x9E3779B1u) >> 21;
                while (slot[h] >= 0 && key[h] != o) h = (h + 1) & (kCells - 1);
                if (slot[h] < 0) {
                    if (n == cap) return cap + 1;
                    key[h] = o;
                    slot[h] = n;
                    if (out_tab) out_tab[n] = o;
                    ++n;
                }
                if (idx && out_tab) (*idx)[k] = (uint8_t)slot[h];
            }
        }
        return n;
    };
    par_for(nt, [&](int64_t a, int64_t b) {
        for (int64_t t = a; t < b; ++t) {
            const int4 d = tiles[t];
            cnt_rel[t] = distinct(d, false, nullptr, 256);
            cnt_anc[t] = distinct(d, true, nullptr, 256);
            int mn = INT32_MAX, mx = INT32_MIN;
            for (int r = d.x; r < d.y; ++r)
                if (rp[r + 1] > rp[r]) {
                    mn = std::min(mn, mid_col(r));
                    mx = std::max(mx, mid_col(r));
                }
            base[t] = mn == INT32_MAX ? 0 : mn;
            span_ok[t] = mn == INT32_MAX || (int64_t)mx - mn < 65536;
        }
    });
    auto cap_of = [](int m) {
        int c = 16;
        while (c < m) c <<= 1;
        return c;
    };
    const int mrel = *std::max_element(cnt_rel.begin(), cnt_rel.end());
    const int manc = *std::max_element(cnt_anc.begin(), cnt_anc.end());
    const bool anc_ok = manc <= 256 && std::all_of(span_ok.begin(), span_ok.end(), [](char c) { return c != 0; });
    auto bytes = [&](int m, bool anchored) -> double {
        const int c = cap_of(m);
        return (c <= 16 ? 0.5 : 1.0) * (double)nz + 4.0 * c * nt + (anchored ? 2.0 * rows : 0.0);
    };
    const double b24 = 3.0 * (double)nz + 4.0 * nt;  // the 24-bit stream it would replace
    bool use_anc = false;
    double best = b24;
    if (mrel <= 256 && bytes(mrel, false) < best) best = bytes(mrel, false);
    if (anc_ok && bytes(manc, true) < best) {
        best = bytes(manc, true);
        use_anc = true;
    }
    if (std::getenv("PAMG_TRACE_UPLOAD"))
        std::fprintf(stderr, "[pamg upload] per-tile dictionaries: %lld tiles, max offsets/tile row-relative %d, "
                     "anchored %d (16-bit span %s) -> %s\n", (long long)nt, mrel, manc, anc_ok ? "ok" : "no",
                     best >= b24 ? "24-bit kept" : use_anc ? "anchored" : "row-relative");
    if (best >= b24) return PAMG_OK;
    const int cap = cap_of(use_anc ? manc : mrel);
    tab->assign((size_t)nt * cap, 0);
    if (use_anc && anc16->empty()) anc16->assign((size_t)A->nrows + kVecPad, 0);
    par_for(nt, [&](int64_t a, int64_t b) {
        for (int64_t t = a; t < b; ++t) {
            distinct(tiles[t], use_anc, tab->data() + (size_t)t * cap, cap);
            if (use_anc)
                for (int r = tiles[t].x; r < tiles[t].y; ++r)
                    (*anc16)[r] = rp[r + 1] > rp[r] ? (uint16_t)(mid_col(r) - base[t]) : 0;
        }
    });
    if (use_anc) {
        CHECK(dalloc(&ts->d_abase, nt));
        HIPC(hipMemcpy(ts->d_abase, base.data(), sizeof(int) * nt, hipMemcpyHostToDevice));
    }
    ts->pt = true;
    ts->anc = use_anc;
    ts->ctab_n = cap;
    return PAMG_OK;
}

// Column dictionaries (Options::col_dict). A tile set whose short-tile nonzeros have at most
// 256 distinct row-relative offsets col - row (the fine-grid stencils: 7 for the 7-point
// Poisson, 5 in 2D, 99 for elastic3d) stores each column as an index into the set's offset
// table: 4 bits where every such set of the matrix has <= 16 offsets, else 8 bits (one width
// per matrix, so the interior and boundary sets share d_cidx). The kernel rebuilds the
// column as row + table[index] (exact); its rows come from the 8-bit row lengths, so a
// dictionary set also turns rl8 on. Against the 24-bit stream this saves 2.5 B/nonzero
// (4-bit) or 2 B/nonzero (8-bit) of the 11-12 B a nonzero streams.
int build_col_dicts(pamg_mat* A, const PtrVec& rp, const IdxVec& ci,
                    const std::vector<int4>& t_in, const std::vector<int4>& t_bd,
                    std::vector<uint8_t>* idx8) {
    const auto& opt = pamg::options();
    pamg::TileSet* sets[2] = {&A->interior, &A->boundary};
    const std::vector<int4>* tl[2] = {&t_in, &t_bd};
    std::vector<uint8_t> idx;  // 8-bit index per nonzero (packed to 4 bits below if they fit)
    std::vector<int> tab[2];   // global table, or (per-tile sets) nt x ctab_n tables
    std::vector<uint16_t> anc16;  // per-tile anchored sets: each row's first column - tile base
    for (int q = 0; q < 2; ++q) {
        pamg::TileSet* ts = sets[q];
        if (!opt.col_dict || ts->n_short == 0 || ts->max_short_len > 255)
            continue;
        // a set with 4-bit value dictionaries (the prolongators) keeps its 24-bit columns
        // (per-tile column dictionaries there measured 8 % slower)
        if (ts->vd) continue;
        if (idx.empty()) idx.assign((size_t)A->nnz + kVecPad, 0);
        const std::vector<int4>& tiles = *tl[q];
        const int64_t nt = (int64_t)tiles.size();
        // Offset of a nonzero: col - row (row-relative: stencils), or col - the row's first
        // column (anchored: rows of a repeated shape whose columns do not follow the row
        // index, e.g. a restriction's 5x5x5 neighbourhoods of an aggregate root: 75 offsets).
        // Anchored sets are read only by the tile-major kernel (the row anchors live in its
        // slots), so they need tile_major on.
        auto try_dict = [&](bool anchored) -> bool {
            auto anchor = [&](int r) { return anchored ? (rp[r + 1] > rp[r] ? ci[rp[r]] : 0) : r; };
            // Distinct offsets in first-occurrence order (tile order, then storage order):
            // every chunk of tiles lists its own (<= 257) in parallel, the lists are merged in
            // chunk order — the same table a single sequential pass builds.
            const int nch = std::max(1, std::min<int>(host_threads(), (int)(nt / 64)));
            std::vector<std::vector<int>> firsts(nch);
            auto scan = [&](int64_t a, int64_t b, std::vector<int>& out) {
                constexpr int kCells = 1024;  // open addressing: offset -> seen
                int key[kCells];
                bool used[kCells] = {};
                for (int64_t t = a; t < b && out.size() <= 256; ++t)
                    for (int r = tiles[t].x; r < tiles[t].y; ++r) {
                        const int an = anchor(r);
                        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
                            const int o = ci[k] - an;
                            uint32_t h = ((uint32_t)o * 0x9E3779B1u) >> 22;
                            while (used[h] && key[h] != o) h = (h + 1) & (kCells - 1);
                            if (!used[h]) {
                                used[h] = true;
                                key[h] = o;
                                out.push_back(o);
                                if (out.size() > 256) return;
                            }
                        }
                    }
            };
            {
                std::vector<std::thread> th;
                for (int c = 0; c < nch; ++c)
                    th.emplace_back([&, c] { scan(nt * c / nch, nt * (c + 1) / nch, firsts[c]); });
                for (auto& x : th) x.join();
            }
            constexpr int kCells = 1024;
            int key[kCells], slot[kCells];
            std::fill(slot, slot + kCells, -1);
            auto find = [&](int o) {
                uint32_t h = ((uint32_t)o * 0x9E3779B1u) >> 22;
                while (slot[h] >= 0 && key[h] != o) h = (h + 1) & (kCells - 1);
                return h;
            };
            tab[q].clear();
            for (int c = 0; c < nch; ++c)
                for (int o : firsts[c]) {
                    const uint32_t h = find(o);
                    if (slot[h] >= 0) continue;
                    if (tab[q].size() == 256) {
                        tab[q].clear();
                        return false;
                    }
                    key[h] = o;
                    slot[h] = (int)tab[q].size();
                    tab[q].push_back(o);
                }
            par_for(nt, [&](int64_t a, int64_t b) {
                for (int64_t t = a; t < b; ++t)
                    for (int r = tiles[t].x; r < tiles[t].y; ++r) {
                        const int an = anchor(r);
                        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) idx[k] = (uint8_t)slot[find(ci[k] - an)];
                    }
            });
            return true;
        };
        ts->anc = false;
        ts->pt = false;
        if (try_dict(false)) continue;
        if (opt.col_dict_anchor && opt.tile_major && try_dict(true)) {
            ts->anc = true;
            continue;
        }
        if (opt.col_dict_tile) CHECK(build_tile_dicts(A, rp, ci, tiles, ts, &idx, &tab[q], &anc16));
    }
    int width = 0;
    for (int q = 0; q < 2; ++q) {
        if (tab[q].empty()) continue;
        const size_t entries = sets[q]->pt ? (size_t)sets[q]->ctab_n : tab[q].size();
        width = std::max(width, entries <= 16 ? 4 : 8);
    }
    if (width == 0) return PAMG_OK;
    for (int q = 0; q < 2; ++q) {
        if (tab[q].empty()) continue;
        pamg::TileSet* ts = sets[q];
        if (ts->pt) {  // nt x ctab_n per-tile tables (+ 256 so any index of the last tile stays inside)
            tab[q].resize(tab[q].size() + 256, 0);
            CHECK(dalloc(&ts->d_ctab, (int64_t)tab[q].size()));
            CHECK(h2d(A->ctx, ts->d_ctab, tab[q].data(), sizeof(int) * tab[q].size()));
        } else {
            std::vector<int> tab256(256, 0);  // any 8-bit index stays inside the allocation
            std::copy(tab[q].begin(), tab[q].end(), tab256.begin());
            CHECK(dalloc(&ts->d_ctab, (int64_t)tab256.size()));
            HIPC(hipMemcpy(ts->d_ctab, tab256.data(), sizeof(int) * tab256.size(), hipMemcpyHostToDevice));
            ts->ctab_n = (int)tab[q].size();
        }
        ts->cd = width;
        ts->rl8 = true;
    }
    if (!anc16.empty()) {
        CHECK(dalloc(&A->d_anc16, (int64_t)anc16.size()));
        CHECK(h2d(A->ctx, A->d_anc16, anc16.data(), sizeof(uint16_t) * anc16.size()));
    }
    if (width == 4) {
        std::vector<uint8_t> nib(((size_t)A->nnz + 1) / 2 + kVecPad, 0);
        const int64_t nb = (A->nnz + 1) / 2;
        par_for(nb, [&](int64_t a, int64_t b) {
            for (int64_t j = a; j < b; ++j) {
                const int64_t k = 2 * j;
                nib[j] = (uint8_t)((idx[k] & 15) | (k + 1 < A->nnz ? (idx[k + 1] & 15) << 4 : 0));
            }
        });
        CHECK(dalloc(&A->d_cidx, (int64_t)nib.size()));
        CHECK(h2d(A->ctx, A->d_cidx, nib.data(), nib.size()));
    } else {
        CHECK(dalloc(&A->d_cidx, (int64_t)idx.size()));
        CHECK(h2d(A->ctx, A->d_cidx, idx.data(), idx.size()));
    }
    idx8->swap(idx);
    return PAMG_OK;
}

// x staging (Options::x_stage; pamg::XStage) for a tile-major set with a set-wide row-relative
// dictionary: cluster the sorted offsets (a new run where the gap exceeds kXsGap), and when
// the runs of the widest tile fit (<= kXsMaxClusters runs, rows + run width <= 256 lanes,
// all runs in kXsCap doubles) write each offset's LDS position into the table at kXsIoff.
int build_x_stage(pamg_mat* A, pamg::TileSet* ts, int rs) {
    using pamg::kXsCap;
    using pamg::kXsGap;
    using pamg::kXsIoff;
    using pamg::kXsMaxClusters;
    ts->xs = false;
    if (!pamg::options().x_stage || !ts->cd || ts->anc || ts->pt || ts->ctab_n > kXsIoff || ts->ctab_n == 0)
        return PAMG_OK;
    std::vector<int> tab(256);
    HIPC(hipMemcpy(tab.data(), ts->d_ctab, sizeof(int) * 256, hipMemcpyDeviceToHost));
    std::vector<int> off(tab.begin(), tab.begin() + ts->ctab_n);
    std::vector<int> srt(off);
    std::sort(srt.begin(), srt.end());
    std::vector<int> cmin, cmax;
    for (int o : srt) {
        if (cmin.empty() || (int64_t)o - cmax.back() > kXsGap) {
            cmin.push_back(o);
            cmax.push_back(o);
        } else {
            cmax.back() = o;
        }
    }
    const int ncl = (int)cmin.size();
    int wmax = 0;
    for (int c = 0; c < ncl; ++c) wmax = std::max(wmax, cmax[c] - cmin[c]);
    const int stride = rs + wmax;
    if (ncl > kXsMaxClusters || stride > 256 || ncl * stride > kXsCap) return PAMG_OK;
    pamg::XStage& x = ts->xst;
    x = pamg::XStage{};
    x.ncl = ncl;
    x.stride = stride;
    x.ncols = (int)A->ncols;
    for (int c = 0; c < ncl; ++c) {
        x.omin[c] = cmin[c];
        x.wid[c] = cmax[c] - cmin[c];
    }
    for (int i = 0; i < ts->ctab_n; ++i) {
        int c = 0;
        while (off[i] > cmax[c]) ++c;
        tab[kXsIoff + i] = c * stride + (off[i] - cmin[c]);
        if (off[i] == 0) x.zix = i;
    }
    HIPC(hipMemcpy(ts->d_ctab, tab.data(), sizeof(int) * 256, hipMemcpyHostToDevice));
    ts->xs = true;
    return PAMG_OK;
}

// Tile-major copies (Options::tile_major, kernel variant 4 k_rows_tm): for a tile set with
// one row per lane (<= 256 rows per tile, rows <= 255 nonzeros) and 24-bit or dictionary
// columns, tile t's values, column stream and row lengths are copied to fixed, zero-padded
// slots (t * tile_nnz, t * tm_rs), so the kernel addresses every pre-gather load from its
// block index. The CSR arrays stay resident for the other variants and the long rows.
int build_tile_major(pamg_mat* A, int64_t n_own_cols, const PtrVec& rp,
                     const IdxVec& ci, const double* val,
                     const std::vector<int4>& t_in, const std::vector<int4>& t_bd,
                     const std::vector<uint16_t>& lo, const std::vector<uint8_t>& hi,
                     const std::vector<uint8_t>& idx8) {
    const auto& opt = pamg::options();
    pamg::TileSet* sets[2] = {&A->interior, &A->boundary};
    const std::vector<int4>* tl[2] = {&t_in, &t_bd};
    for (int q = 0; q < 2; ++q) {
        pamg::TileSet* ts = sets[q];
        ts->tm = false;
        // per-tile dictionaries run in the descriptor kernel, row-relative ones in tile-major
        // slots with tm_tile_dicts
        if (ts->pt && (ts->anc || !opt.tm_tile_dicts)) continue;
        if (!opt.tile_major || ts->vd || ts->n_short == 0 || ts->max_short_len > 255 ||
            !(ts->cd || (ts->c24 && !lo.empty())) || (ts->cd && idx8.empty()) || !val) {
            if (ts->anc) return fail(PAMG_E_STATE, "upload: anchored column dictionary without tile-major slots");
            continue;
        }
        // tile_major 1 (default): the sets where it measured faster at 512^3
        // (profiles/r01_kbench_512_tm_*.jsonl) — column-dictionary sets (A0: Jacobi -9 %,
        // residual -7 %, SpMV -5 %) and the non-square operators whose tiles fill >= 97 % of
        // their slots (R0 -5..-7 %, P1 -3 %); P0's row-limited tiles leave ~8 % of each slot as
        // padding (+5 %) and the square coarse A1 gains nothing (Jacobi +3 %): variant 1.
        // tile_major 2: every eligible set (A/B, tests).
        if (opt.tile_major == 1 && !ts->cd) {
            const double fill = (double)ts->nnz_short / ((double)ts->n_short * (double)ts->tile_nnz);
            if (n_own_cols == A->nrows || fill < 0.97) continue;
        }
        const std::vector<int4>& tiles = *tl[q];
        const int64_t nt = (int64_t)tiles.size(), tn = ts->tile_nnz;
        // k_rows_tm keeps per-tile tables of <= kTmSmallTab entries in LDS for 2048-nonzero tiles:
        // a set with longer per-tile column tables stays in the descriptor kernel
        if (ts->pt && tn == 2048 && ts->ctab_n > pamg::kTmSmallTab) {
            if (UploadTrace{}.on)
                std::fprintf(stderr, "[pamg upload nnz=%lld] set %d: per-tile column tables of %d > %d entries on "
                             "2048-nonzero tiles: descriptor kernel instead of tile-major slots\n",
                             (long long)A->nnz, q, ts->ctab_n, pamg::kTmSmallTab);
            continue;
        }
        int rs = 0;
        for (const int4& t : tiles) rs = std::max(rs, t.y - t.x);
        rs = (rs + 3) & ~3;
        // every slot is written whole (nonzeros, then zero padding) by the thread that owns its
        // tile, so the buffers need no serial zero fill
        const int cdw = ts->cd;
        // 8-bit per-tile value dictionaries (value_dict): every tile <= 256 distinct values
        // (bit patterns: +0.0 and -0.0 stay distinct)
        int vt = 0;
        if (opt.value_dict) {
            std::atomic<int> vmax{0};
            std::atomic<bool> over{false};
            par_for(nt, [&](int64_t a, int64_t b) {
                std::vector<uint64_t> u;
                for (int64_t i = a; i < b && !over; ++i) {
                    const int4 t = tiles[i];
                    u.assign(reinterpret_cast<const uint64_t*>(val) + t.z, reinterpret_cast<const uint64_t*>(val) + t.w);
                    std::sort(u.begin(), u.end());
                    const int d = (int)(std::unique(u.begin(), u.end()) - u.begin());
                    if (d > 256) over = true;
                    int m = vmax.load();
                    while (d > m && !vmax.compare_exchange_weak(m, d)) {
                    }
                }
            });
            if (!over) vt = std::max(4, (vmax.load() + 3) & ~3);
            if (tn == 2048 && vt > pamg::kTmSmallTab) {  // (the kernel's LDS table, see above)
                if (UploadTrace{}.on)
                    std::fprintf(stderr, "[pamg upload nnz=%lld] set %d: a 2048-nonzero tile has %d > %d distinct "
                                 "values: 8-B values instead of the 8-bit value dictionary\n",
                                 (long long)A->nnz, q, vmax.load(), pamg::kTmSmallTab);
                vt = 0;
            }
            if (over && UploadTrace{}.on)
                std::fprintf(stderr, "[pamg upload nnz=%lld] set %d: a tile has > 256 distinct values: 8-B values\n",
                             (long long)A->nnz, q);
        }
        std::unique_ptr<double[]> tv(vt ? nullptr : new double[nt * tn + kVecPad]);
        std::unique_ptr<uint8_t[]> tvi(vt ? new uint8_t[nt * tn + kVecPad] : nullptr);
        std::unique_ptr<double[]> tvt(vt ? new double[nt * vt + kVecPad] : nullptr);
        std::unique_ptr<uint8_t[]> trl(new uint8_t[nt * rs + kVecPad]);
        const int64_t ncb = cdw == 4 ? tn / 2 : tn;  // column-stream bytes per slot (cd / chi)
        std::unique_ptr<uint8_t[]> tci(new uint8_t[nt * ncb + kVecPad]);
        std::unique_ptr<uint16_t[]> tcl(cdw ? nullptr : new uint16_t[nt * tn + kVecPad]);
        std::unique_ptr<int[]> tan(ts->anc ? new int[nt * rs + kVecPad] : nullptr);
        par_for(nt, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) {
                const int4 t = tiles[i];
                const int cnt = t.w - t.z;
                uint8_t* rl = &trl[i * rs];
                for (int r = 0; r < rs; ++r) rl[r] = t.x + r < t.y ? (uint8_t)(rp[t.x + r + 1] - rp[t.x + r]) : 0;
                if (tan)  // row anchors: each row's first column (anchored column dictionary)
                    for (int r = 0; r < rs; ++r) {
                        const int row = t.x + r;
                        tan[i * rs + r] = row < t.y && rp[row + 1] > rp[row] ? ci[rp[row]] : 0;
                    }
                if (vt) {  // the tile's table in first-occurrence order, indices per nonzero
                    double* tab = &tvt[i * vt];
                    uint8_t* vi = &tvi[i * tn];
                    uint64_t hk[512];
                    int16_t hv[512];
                    std::fill(hv, hv + 512, (int16_t)-1);
                    int nd = 0;
                    for (int k = 0; k < cnt; ++k) {
                        uint64_t key;
                        std::memcpy(&key, &val[t.z + k], sizeof(key));
                        uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 55);  // 9 bits
                        while (hv[h] >= 0 && hk[h] != key) h = (h + 1) & 511;
                        if (hv[h] < 0) {
                            hk[h] = key;
                            hv[h] = (int16_t)nd;
                            std::memcpy(&tab[nd++], &key, sizeof(key));
                        }
                        vi[k] = (uint8_t)hv[h];
                    }
                    std::fill(tab + nd, tab + vt, 0.0);
                    std::fill(vi + cnt, vi + tn, (uint8_t)0);
                } else {
                    double* v = &tv[i * tn];
                    std::memcpy(v, val + t.z, sizeof(double) * cnt);
                    std::fill(v + cnt, v + tn, 0.0);
                }
                uint8_t* c = &tci[i * ncb];
                if (cdw == 4) {
                    std::fill(c, c + ncb, (uint8_t)0);
                    for (int k = 0; k < cnt; ++k) c[k >> 1] |= (uint8_t)((idx8[t.z + k] & 15) << (4 * (k & 1)));
                } else if (cdw == 8) {
                    std::memcpy(c, &idx8[t.z], cnt);
                    std::fill(c + cnt, c + tn, (uint8_t)0);
                } else {
                    uint16_t* l = &tcl[i * tn];
                    std::memcpy(l, &lo[t.z], sizeof(uint16_t) * cnt);
                    std::fill(l + cnt, l + tn, (uint16_t)0);
                    std::memcpy(c, &hi[t.z], cnt);
                    std::fill(c + cnt, c + tn, (uint8_t)0);
                }
            }
        });
        if (tv) std::fill(&tv[nt * tn], &tv[nt * tn] + kVecPad, 0.0);
        std::fill(&trl[nt * rs], &trl[nt * rs] + kVecPad, (uint8_t)0);
        std::fill(&tci[nt * ncb], &tci[nt * ncb] + kVecPad, (uint8_t)0);
        if (tcl) std::fill(&tcl[nt * tn], &tcl[nt * tn] + kVecPad, (uint16_t)0);
        if (tan) {
            std::fill(&tan[nt * rs], &tan[nt * rs] + kVecPad, 0);
            CHECK(dalloc(&ts->d_tm_anc, nt * rs + kVecPad));
            CHECK(h2d(A->ctx, ts->d_tm_anc, tan.get(), sizeof(int) * (nt * rs + kVecPad)));
        }
        if (vt) {
            std::fill(&tvi[nt * tn], &tvi[nt * tn] + kVecPad, (uint8_t)0);
            std::fill(&tvt[nt * vt], &tvt[nt * vt] + kVecPad, 0.0);
            CHECK(dalloc(&ts->d_tm_vidx, nt * tn + kVecPad));
            CHECK(h2d(A->ctx, ts->d_tm_vidx, tvi.get(), nt * tn + kVecPad));
            CHECK(dalloc(&ts->d_tm_vtab, nt * vt + kVecPad));
            CHECK(h2d(A->ctx, ts->d_tm_vtab, tvt.get(), sizeof(double) * (nt * vt + kVecPad)));
        } else {
            CHECK(dalloc(&ts->d_tm_val, nt * tn + kVecPad));
            CHECK(h2d(A->ctx, ts->d_tm_val, tv.get(), sizeof(double) * (nt * tn + kVecPad)));
        }
        ts->tm_vt = vt;
        CHECK(dalloc(&ts->d_tm_rlen, nt * rs + kVecPad));
        CHECK(h2d(A->ctx, ts->d_tm_rlen, trl.get(), nt * rs + kVecPad));
        if (cdw) {
            CHECK(dalloc(&ts->d_tm_cidx, nt * ncb + kVecPad));
            CHECK(h2d(A->ctx, ts->d_tm_cidx, tci.get(), nt * ncb + kVecPad));
        } else {
            CHECK(dalloc(&ts->d_tm_clo, nt * tn + kVecPad));
            CHECK(dalloc(&ts->d_tm_chi, nt * tn + kVecPad));
            CHECK(h2d(A->ctx, ts->d_tm_clo, tcl.get(), sizeof(uint16_t) * (nt * tn + kVecPad)));
            CHECK(h2d(A->ctx, ts->d_tm_chi, tci.get(), nt * tn + kVecPad));
        }
        ts->tm_rs = rs;
        ts->tm = true;
        CHECK(build_x_stage(A, ts, rs));
    }
    return PAMG_OK;
}

// Symmetric diagonal-class layout of the interior rows (pamg::SymDia, k_rows_sym), when they
// qualify: <= 2*kSymMaxU+1 distinct row-relative offsets forming a symmetric set with 0, every
// interior row's entries in strictly ascending offset order (so the kernel's ascending sum is
// the storage-order sum of SPEC §S3), and every lower entry bit-identical to its mirror
// a(i-o, i) in row i-o. Otherwise nothing is built and the rows keep their tiles.
// a copy of the context's registered grids (pamg_ctx::grids)
std::vector<std::array<int64_t, 4>> grids_of(pamg_ctx* ctx) {
    std::lock_guard<std::mutex> lk(ctx->grids_mu);
    return ctx->grids;
}

int build_sym_dia(pamg_mat* A, const PtrVec& rp, const IdxVec& ci, const double* val,
                  const std::vector<int>& inner, const std::function<int64_t()>& get_band) {
    using pamg::kSymMaxU;
    const int64_t n = A->nrows;
    constexpr int kMaxOff = 2 * kSymMaxU + 1;
    // distinct offsets of the interior rows (per thread, merged)
    std::mutex mu;
    std::vector<int> offs;
    std::atomic<bool> too_many{false};
    par_for((int64_t)inner.size(), [&](int64_t a, int64_t b) {
        std::vector<int> loc;
        for (int64_t q = a; q < b && !too_many; ++q) {
            const int i = inner[q];
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                const int o = ci[k] - i;
                if (std::find(loc.begin(), loc.end(), o) == loc.end()) {
                    loc.push_back(o);
                    if ((int)loc.size() > kMaxOff) {
                        too_many = true;
                        return;
                    }
                }
            }
        }
        std::lock_guard<std::mutex> g(mu);
        for (int o : loc)
            if (std::find(offs.begin(), offs.end(), o) == offs.end()) offs.push_back(o);
    });
    if (too_many || (int)offs.size() > kMaxOff) return PAMG_OK;
    std::sort(offs.begin(), offs.end());
    const int no = (int)offs.size();
    if (no % 2 == 0 || offs[no / 2] != 0) return PAMG_OK;
    for (int k = 0; k < no; ++k)
        if (offs[k] != -offs[no - 1 - k]) return PAMG_OK;
    const int nu = no / 2;
    if (nu < 1) return PAMG_OK;  // diagonal-only rows: the tile path (no class to mirror)
    pamg::SymDia sd;
    sd.nu = nu;
    for (int c = 0; c < nu; ++c) sd.off[c] = offs[nu + 1 + c];
    sd.ld = (n + 63) / 64 * 64 + 64;
    const int mb = 2 * nu + 1 <= 7 ? 1 : 2;  // mask bytes per row (kernels.hip SymMask)
    const uint32_t in_flag = mb == 1 ? 0x80u : 0x8000u;
    // (zeroed by parallel loops: 5 GB at 512^3)
    std::vector<uint16_t, NoInitAlloc<uint16_t>> mask(n + kVecPad);
    std::vector<double, NoInitAlloc<double>> dg(n + kVecPad), up((size_t)nu * sd.ld);
    std::vector<char, NoInitAlloc<char>> in_set(n);
    par_for(n + kVecPad, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            mask[i] = 0;
            dg[i] = 0.0;
            if (i < n) in_set[i] = 0;
        }
    });
    par_for((int64_t)up.size(), [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) up[i] = 0.0;
    });
    par_for((int64_t)inner.size(), [&](int64_t a, int64_t b) {
        for (int64_t q = a; q < b; ++q) in_set[inner[q]] = 1;
    });
    auto cls = [&](int o) { return (int)(std::lower_bound(offs.begin(), offs.end(), o) - offs.begin()); };
    std::atomic<bool> bad{false};
    par_for(n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b && !bad; ++i) {
            // every own row: diagonal and upper values (the mirrors interior rows read)
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                const int o = ci[k] - (int)i;
                if (ci[k] >= n) continue;  // ghost column (boundary rows)
                if (o == 0) dg[i] = val[k];
                else if (o > 0) {
                    const int c = cls(o);
                    if (c < no && offs[c] == o) up[(size_t)(c - nu - 1) * sd.ld + i] = val[k];
                }
            }
            if (!in_set[i]) continue;
            uint32_t m = in_flag;
            int last = -1;
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                const int o = ci[k] - (int)i;
                const int c = cls(o);
                if (c <= last) {  // not strictly ascending
                    bad = true;
                    break;
                }
                last = c;
                m |= 1u << c;
                if (o < 0) {  // the mirror a(i+o, i) must exist with the same bits
                    const int64_t j = i + o;
                    bool found = false;
                    for (int64_t kk = rp[j]; kk < rp[j + 1]; ++kk)
                        if (ci[kk] == (int)i) {
                            found = std::memcmp(&val[kk], &val[k], sizeof(double)) == 0;
                            break;
                        }
                    if (!found) {
                        bad = true;
                        break;
                    }
                }
            }
            mask[i] = (uint16_t)m;
        }
    });
    if (bad) return PAMG_OK;
    // A part of several (a z-slab of whole planes, SymDia::tb_part): the set must be exactly its
    // planes 1 .. nz-2 (the first and last plane read ghosts); its bands are whole planes, so
    // the separate sweeps can run on plane windows (launch_sym_planes)
    const int64_t Mp = nu == 3 ? sd.off[2] : 0;
    const bool whole = A->ncols == n && (int64_t)inner.size() == n;
    bool part = false;
    int plo = 0, phi = 0;
    if (!whole && nu == 3 && Mp > 0 && n % Mp == 0 && n / Mp >= 6 && !inner.empty() && inner.size() % Mp == 0 &&
        inner.front() % Mp == 0) {
        const int nzp = (int)(n / Mp);
        plo = (int)(inner.front() / Mp);
        phi = plo + (int)(inner.size() / Mp);
        part = (plo == 0 || plo == 1) && (phi == nzp || phi == nzp - 1) && phi - plo < nzp;
        for (size_t q = 0; q < inner.size() && part; ++q) part = inner[q] == inner.front() + (int64_t)q;
    }
    // XCD-banded block order (natural order: one band)
    // (a 7-point grid's column reuse gap is one plane less one line, M - nx: no need to measure it —
    // column_reuse_gaps over 938M nonzeros took 0.6 s of the 512^3 upload)
    const bool grid7 = nu == 3 && sd.off[0] == 1 && sd.off[2] % sd.off[1] == 0;
    const int64_t band = grid7 ? (int64_t)sd.off[2] - sd.off[1] : get_band();
    int64_t bd = (pamg::options().tile_order == 1 && band >= 8 * pamg::kBlock) ? band : n;
    if (part && Mp >= 8 * pamg::kBlock) bd = Mp;
    sd.band = (int)bd;
    sd.rpl = pamg::options().sym_rows;
    const int64_t rows_per_block = (int64_t)pamg::kBlock * sd.rpl;
    sd.band_blocks = (int)((bd + rows_per_block - 1) / rows_per_block);
    sd.eighth = (sd.band_blocks + 7) / 8;
    sd.nbands = (int)((n + bd - 1) / bd);
    sd.mask_bytes = mb;
    // Row-class dictionary (Options::sym_vd, two rows per lane): the distinct (mask, D, U_0 ..
    // U_{nu-1}) bit tuples of the own rows in first-occurrence order (chunks scanned in
    // parallel, merged in chunk order — the table one sequential pass builds); a constant-
    // coefficient stencil has one per boundary case (512^3 Poisson: 27)
    std::vector<uint8_t> tid;
    std::vector<double> vtab;
    std::vector<uint32_t> mtab;
    if (pamg::options().sym_vd && sd.rpl == 2) {
        using Key = std::array<uint64_t, 2 + kSymMaxU>;
        auto key_of = [&](int64_t i) {
            Key k{};
            k[0] = mask[i];
            std::memcpy(&k[1], &dg[i], 8);
            for (int c = 0; c < nu; ++c) std::memcpy(&k[2 + c], &up[(size_t)c * sd.ld + i], 8);
            return k;
        };
        const int nch = std::max(1, std::min<int>(host_threads(), (int)(n / 65536)));
        std::vector<std::vector<Key>> firsts(nch);
        std::atomic<bool> over{false};
        {
            std::vector<std::thread> th;
            for (int c = 0; c < nch; ++c)
                th.emplace_back([&, c] {
                    std::vector<Key>& f = firsts[c];
                    int last = -1;
                    for (int64_t i = n * c / nch, e = n * (c + 1) / nch; i < e && !over; ++i) {
                        const Key k = key_of(i);
                        if (last >= 0 && f[last] == k) continue;
                        last = -1;
                        for (int q = 0; q < (int)f.size() && last < 0; ++q)
                            if (f[q] == k) last = q;
                        if (last >= 0) continue;
                        if ((int)f.size() == pamg::kSymVdMax) {
                            over = true;
                            break;
                        }
                        f.push_back(k);
                        last = (int)f.size() - 1;
                    }
                });
            for (auto& x : th) x.join();
        }
        std::vector<Key> tab;
        for (int c = 0; c < nch && !over; ++c)
            for (const Key& k : firsts[c]) {
                if (std::find(tab.begin(), tab.end(), k) != tab.end()) continue;
                if ((int)tab.size() == pamg::kSymVdMax) {
                    over = true;
                    break;
                }
                tab.push_back(k);
            }
        if (!over && !tab.empty()) {
            tid.assign(n + kVecPad, 0);
            par_for(n, [&](int64_t a, int64_t b) {
                int last = 0;
                for (int64_t i = a; i < b; ++i) {
                    const Key k = key_of(i);
                    if (tab[last] != k) last = (int)(std::find(tab.begin(), tab.end(), k) - tab.begin());
                    tid[i] = (uint8_t)last;
                }
            });
            const int nv = (int)tab.size();
            vtab.assign((size_t)nv * (nu + 1) + kVecPad, 0.0);
            mtab.assign(nv + kVecPad, 0u);
            for (int e = 0; e < nv; ++e) {
                mtab[e] = (uint32_t)tab[e][0];
                for (int c = 0; c <= nu; ++c) std::memcpy(&vtab[(size_t)e * (nu + 1) + c], &tab[e][1 + c], 8);
            }
            sd.vd_n = nv;
            // the most frequent class (a grid's interior rows): k_rows_symd's register fast path
            std::vector<int64_t> cnt(nv, 0);
            {
                std::mutex mu;
                par_for(n, [&](int64_t a, int64_t b) {
                    std::vector<int64_t> c(nv, 0);
                    for (int64_t i = a; i < b; ++i) ++c[tid[i]];
                    std::lock_guard<std::mutex> lk(mu);
                    for (int e = 0; e < nv; ++e) cnt[e] += c[e];
                });
            }
            sd.vd_main = (int)(std::max_element(cnt.begin(), cnt.end()) - cnt.begin());
        }
    }
    if (sd.vd_n) {
        CHECK(dalloc(&sd.d_tid, (int64_t)tid.size()));
        CHECK(h2d(A->ctx, sd.d_tid, tid.data(), tid.size()));
        CHECK(dalloc(&sd.d_vtab, (int64_t)vtab.size()));
        CHECK(h2d(A->ctx, sd.d_vtab, vtab.data(), sizeof(double) * vtab.size()));
        CHECK(dalloc(&sd.d_mtab, (int64_t)mtab.size()));
        CHECK(h2d(A->ctx, sd.d_mtab, mtab.data(), sizeof(uint32_t) * mtab.size()));
    } else {
        CHECK(dalloc(&sd.d_mask, (n + kVecPad) * mb));
        CHECK(dalloc(&sd.d_diag, n + kVecPad));
        CHECK(dalloc(&sd.d_upper, (int64_t)nu * sd.ld));
        if (mb == 1) {
            std::vector<uint8_t> m8(mask.begin(), mask.end());
            CHECK(h2d(A->ctx, sd.d_mask, m8.data(), m8.size()));
        } else {
            CHECK(h2d(A->ctx, sd.d_mask, mask.data(), sizeof(uint16_t) * mask.size()));
        }
        CHECK(h2d(A->ctx, sd.d_diag, dg.data(), sizeof(double) * dg.size()));
        CHECK(h2d(A->ctx, sd.d_upper, up.data(), sizeof(double) * up.size()));
    }
    // temporally blocked sweeps (kernels.hip k_sym_tb): one part with every row in the set, a
    // 7-point grid stencil in natural order (classes 1, nx, nx*ny; n = nx*ny*nz) whose rows
    // never reach across a grid line (the -1 / +1 / -nx / +nx classes absent at x = 0 / nx-1 /
    // y = 0 / ny-1), tiles of kTbX x kTbY
    part = part && sd.band == Mp;
    if (nu == 3 && mb == 1 && (whole || part) && sd.off[0] == 1 && sd.off[2] % sd.off[1] == 0 && n % sd.off[2] == 0) {
        const int nx = sd.off[1], ny = sd.off[2] / sd.off[1];
        const int nz = (int)(n / sd.off[2]);
        bool ok = nx % pamg::kTbX == 0 && ny % pamg::kTbY == 0;
        std::atomic<bool> cross{false};
        if (ok)
            par_for(n, [&](int64_t a0, int64_t b0) {
                for (int64_t i = a0; i < b0 && !cross; ++i) {
                    const int x = (int)(i % nx), y = (int)((i / nx) % ny);
                    const uint32_t m = mask[i];  // ascending classes -M, -nx, -1, 0, 1, nx, M
                    if (((m & 4u) && x == 0) || ((m & 16u) && x == nx - 1) || ((m & 2u) && y == 0) ||
                        ((m & 32u) && y == ny - 1))
                        cross = true;
                }
            });
        if (ok && !cross) {
            pamg::TbGeom& g = sd.tb;
            g.nx = nx;
            g.ny = ny;
            g.nz = nz;
            g.tiles_x = nx / pamg::kTbX;
            g.tiles_y = ny / pamg::kTbY;
            // about one workgroup per CU (one fits: registers), planes split when a plane has
            // fewer tiles than the chip has CUs
            const int tiles = g.tiles_x * g.tiles_y;
            const int want = std::max(1, (device_cus() + tiles - 1) / tiles);
            g.zchunks = std::max(1, std::min(want, nz / 4 > 0 ? nz / 4 : 1));
            g.zlen = (nz + g.zchunks - 1) / g.zchunks;
            g.zchunks = (nz + g.zlen - 1) / g.zlen;
            g.zlo = 0;
            g.zhi = nz;
            sd.tb_ok = whole;
            sd.tb_part = part;
            if (whole || part) {  // (a later prolongation / restriction over this grid: pnc, ELL group order)
                const std::array<int64_t, 4> gk{n, nx, ny, nz};
                std::lock_guard<std::mutex> lk(A->ctx->grids_mu);
                auto& gs = A->ctx->grids;
                if (std::find(gs.begin(), gs.end(), gk) == gs.end()) gs.push_back(gk);
            }
            sd.part_lo = part ? plo : 0;
            sd.part_hi = part ? phi : nz;
        }
    }
    A->sym = sd;
    A->interior.sym = true;
    A->interior.rows_short = (int64_t)inner.size();
    return PAMG_OK;
}

// A restriction over a registered grid (Options::ell_yblock > 0; its columns are the grid's points):
// the groups of kEllGroup rows of each XCD's eighth (kernels.hip k_rows_ell / k_rows_rpat) in
// (y / yblock, z, y) order of their first row's anchor, so the window of groups in flight is a
// compact (y, z) block of the grid, not whole planes. *d_order stays null otherwise.
int blocked_group_order(pamg_ctx* ctx, const std::vector<int>& anc, int64_t ng, int64_t own_cols, int** d_order) {
    using pamg::kEllGroup;
    const int yb = pamg::options().ell_yblock;
    for (const auto& gr : grids_of(ctx))
        if (yb > 0 && gr[0] == own_cols) {
            const int64_t gnx = gr[1], gny = gr[2], gM = gr[1] * gr[2];
            std::vector<int64_t> key(ng);
            par_for(ng, [&](int64_t a, int64_t b) {
                for (int64_t g = a; g < b; ++g) {
                    const int64_t c = anc[g * kEllGroup];
                    const int64_t y = (c / gnx) % gny, z = c / gM;
                    key[g] = ((y / yb) << 40) | (z << 20) | y;
                }
            });
            const int64_t per = (ng + 7) / 8;
            std::vector<int> order(ng);
            for (int64_t g = 0; g < ng; ++g) order[g] = (int)g;
            for (int64_t e = 0; e < 8; ++e) {
                const int64_t lo = std::min(ng, e * per), hi = std::min(ng, (e + 1) * per);
                std::stable_sort(order.begin() + lo, order.begin() + hi, [&](int p, int q) { return key[p] < key[q]; });
            }
            CHECK(dalloc(d_order, ng));
            CHECK(h2d(ctx, *d_order, order.data(), sizeof(int) * ng));
            break;
        }
    return PAMG_OK;
}

// Sliced ELL with per-group dictionaries (Options::ell, pamg::EllSet): a square operator whose
// rows are all interior, in slices of kEllW rows padded to the slice's longest row, kEllGroup
// rows sharing one table of column offsets (col - row) and one of values (bit patterns), each of
// <= 256 entries. Declines (leaves the tile layouts to the caller) where a table would be larger or
// a row longer than 255. Rows keep their storage order, so the kernel sums every row's products in
// the SPEC §S3 order.
// Rectangular operators (anchored: a restriction) take their offsets from each row's first column
// (col - col_first(row)), the anchors stored per row.
// Several parts: the set is the interior rows only (`inner`, ascending); the slices still span every
// row index, the boundary rows marked skipped (length byte kEllSkip: no load, no store — the
// boundary tiles compute them after the exchange).
int build_ell(pamg_mat* A, const PtrVec& rp, const IdxVec& ci, const double* val,
              bool anchored, const std::vector<int>& inner) {
    using pamg::kEllGroup;
    using pamg::kEllSkip;
    using pamg::kEllW;
    const int64_t n = A->nrows;
    std::vector<char> in_set;
    if ((int64_t)inner.size() != n) {
        in_set.assign(n, 0);
        for (int i : inner) in_set[i] = 1;
    }
    auto member = [&](int64_t i) { return in_set.empty() || in_set[i]; };
    auto base_of = [&](int64_t i) -> int { return anchored ? (rp[i + 1] > rp[i] ? ci[rp[i]] : 0) : (int)i; };
    const int64_t ns = (n + kEllW - 1) / kEllW, ng = (n + kEllGroup - 1) / kEllGroup;
    std::vector<int> slen(ns, 0);
    std::atomic<bool> ok{true};
    par_for(ns, [&](int64_t a, int64_t b) {
        for (int64_t q = a; q < b; ++q) {
            int m = 0;
            for (int64_t i = q * kEllW; i < std::min(n, (q + 1) * kEllW); ++i)
                if (member(i)) m = std::max<int>(m, (int)(rp[i + 1] - rp[i]));
            if (m >= kEllSkip) ok = false;
            slen[q] = m;
        }
    });
    if (!ok) return PAMG_OK;
    std::vector<int2> smeta(ns);
    int64_t words = 0;
    for (int64_t q = 0; q < ns; ++q) {
        smeta[q] = make_int2((int)words, slen[q]);
        words += (int64_t)kEllW * ((slen[q] + 3) / 4);
        if (words >= INT32_MAX) return PAMG_OK;
    }
    // per group, one pass: an entry's offset and value take the index of their first appearance in
    // the group (open addressing over 512 slots, stamped per group instead of cleared), and the index
    // bytes go straight into the slice streams (a slice lies in one group: no two threads share a word)
    // Paired dictionaries (Options::ell_pair, round 6): where every group has <= 256 distinct (offset,
    // value) pairs — the 512^3 A1: a regular 27-point-like stencil over the aggregates — one index byte
    // per nonzero names the pair (the offset and value tables then run in parallel); otherwise one byte
    // each into separate offset and value tables.
    std::vector<std::vector<int>> goff(ng);
    std::vector<std::vector<uint64_t>> gval(ng);
    std::vector<uint32_t> cw(words + 1, 0u), vw;
    std::vector<uint8_t> len(n + kVecPad, 0);
    bool paired = pamg::options().ell_pair != 0;
    if (paired) {
        std::atomic<bool> fits{true};
        par_for(ng, [&](int64_t a, int64_t b) {
            constexpr int kSlots = 1024;
            std::vector<int> pid(kSlots), pstamp(kSlots, -1), pkey_o(kSlots);
            std::vector<uint64_t> pkey_v(kSlots);
            std::vector<int> o;
            std::vector<uint64_t> v;
            for (int64_t g = a; g < b && fits; ++g) {
                const int stamp = (int)(g - a);
                o.clear();
                v.clear();
                const int64_t r1 = std::min(n, (g + 1) * kEllGroup);
                for (int64_t i = g * kEllGroup; i < r1 && fits; ++i) {
                    if (!member(i)) {
                        len[i] = (uint8_t)kEllSkip;
                        continue;
                    }
                    len[i] = (uint8_t)(rp[i + 1] - rp[i]);
                    const int64_t q = i / kEllW, lane = i % kEllW;
                    const int base = base_of(i);
                    for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                        const int kk = (int)(k - rp[i]);
                        const int off = ci[k] - base;
                        uint64_t u;
                        std::memcpy(&u, &val[k], 8);
                        uint32_t h = (uint32_t)((((uint64_t)(uint32_t)off * 0x9E3779B1u) ^ u ^ (u >> 29)) *
                                                0x9E3779B97F4A7C15ull >> 54);
                        while (pstamp[h] == stamp && (pkey_o[h] != off || pkey_v[h] != u)) h = (h + 1) & (kSlots - 1);
                        if (pstamp[h] != stamp) {
                            pstamp[h] = stamp;
                            pkey_o[h] = off;
                            pkey_v[h] = u;
                            pid[h] = (int)o.size();
                            o.push_back(off);
                            v.push_back(u);
                            if (o.size() > 256) {
                                fits = false;
                                break;
                            }
                        }
                        const int64_t w = smeta[q].x + (int64_t)(kk / 4) * kEllW + lane;
                        cw[w] |= (uint32_t)pid[h] << (8 * (kk % 4));
                    }
                }
                goff[g] = o;
                gval[g] = v;
            }
        });
        if (!fits) {  // back to separate tables: start over
            paired = false;
            std::fill(cw.begin(), cw.end(), 0u);
        }
    }
    if (!paired) vw.assign(words + 1, 0u);
    if (!paired) par_for(ng, [&](int64_t a, int64_t b) {
        constexpr int kSlots = 512;
        std::vector<int> okey(kSlots), oid(kSlots), ostamp(kSlots, -1), vid(kSlots), vstamp(kSlots, -1);
        std::vector<uint64_t> vkey(kSlots);
        std::vector<int> o;
        std::vector<uint64_t> v;
        for (int64_t g = a; g < b && ok; ++g) {
            const int stamp = (int)(g - a);
            o.clear();
            v.clear();
            const int64_t r1 = std::min(n, (g + 1) * kEllGroup);
            for (int64_t i = g * kEllGroup; i < r1; ++i) {
                if (!member(i)) {
                    len[i] = (uint8_t)kEllSkip;
                    continue;
                }
                len[i] = (uint8_t)(rp[i + 1] - rp[i]);
                const int64_t q = i / kEllW, lane = i % kEllW;
                const int base = base_of(i);
                for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                    const int kk = (int)(k - rp[i]);
                    const int off = ci[k] - base;
                    uint32_t h = ((uint32_t)off * 0x9E3779B1u) >> 23;
                    while (ostamp[h] == stamp && okey[h] != off) h = (h + 1) & (kSlots - 1);
                    if (ostamp[h] != stamp) {
                        ostamp[h] = stamp;
                        okey[h] = off;
                        oid[h] = (int)o.size();
                        o.push_back(off);
                    }
                    uint64_t u;
                    std::memcpy(&u, &val[k], 8);
                    uint32_t hv = (uint32_t)((u ^ (u >> 29)) * 0x9E3779B97F4A7C15ull >> 55);
                    while (vstamp[hv] == stamp && vkey[hv] != u) hv = (hv + 1) & (kSlots - 1);
                    if (vstamp[hv] != stamp) {
                        vstamp[hv] = stamp;
                        vkey[hv] = u;
                        vid[hv] = (int)v.size();
                        v.push_back(u);
                    }
                    if (o.size() > 256 || v.size() > 256) {
                        ok = false;
                        return;
                    }
                    const int64_t w = smeta[q].x + (int64_t)(kk / 4) * kEllW + lane;
                    cw[w] |= (uint32_t)oid[h] << (8 * (kk % 4));
                    vw[w] |= (uint32_t)vid[hv] << (8 * (kk % 4));
                }
            }
            goff[g] = o;
            gval[g] = v;
        }
    });
    if (!ok) return PAMG_OK;
    std::vector<int4> gmeta(ng);
    int64_t on = 0, vn = 0;
    for (int64_t g = 0; g < ng; ++g) {
        gmeta[g] = make_int4((int)on, (int)goff[g].size(), (int)vn, (int)gval[g].size());
        on += (int64_t)goff[g].size();
        vn += (int64_t)gval[g].size();
    }
    std::vector<int> otab(on + 1, 0);
    std::vector<double> vtab(vn + 1, 0.0);
    par_for(ng, [&](int64_t a, int64_t b) {
        for (int64_t g = a; g < b; ++g) {
            std::copy(goff[g].begin(), goff[g].end(), otab.begin() + gmeta[g].x);
            for (size_t e = 0; e < gval[g].size(); ++e) std::memcpy(&vtab[gmeta[g].z + e], &gval[g][e], 8);
        }
    });
    pamg::EllSet& E = A->ell;
    pamg_ctx* ctx = A->ctx;
    E.nslices = ns;
    E.ngroups = ng;
    E.words = words;
    E.otab_n = on;
    E.vtab_n = vn;
    E.paired = paired;
    CHECK(dalloc(&E.d_smeta, ns));
    CHECK(dalloc(&E.d_ci, words + 1));
    if (!paired) CHECK(dalloc(&E.d_vi, words + 1));
    CHECK(dalloc(&E.d_len, n + kVecPad));
    CHECK(dalloc(&E.d_gmeta, ng));
    CHECK(dalloc(&E.d_otab, on + 1));
    CHECK(dalloc(&E.d_vtab, vn + 1));
    CHECK(h2d(ctx, E.d_smeta, smeta.data(), sizeof(int2) * ns));
    CHECK(h2d(ctx, E.d_ci, cw.data(), sizeof(uint32_t) * (words + 1)));
    if (!paired) CHECK(h2d(ctx, E.d_vi, vw.data(), sizeof(uint32_t) * (words + 1)));
    CHECK(h2d(ctx, E.d_len, len.data(), len.size()));
    CHECK(h2d(ctx, E.d_gmeta, gmeta.data(), sizeof(int4) * ng));
    CHECK(h2d(ctx, E.d_otab, otab.data(), sizeof(int) * (on + 1)));
    CHECK(h2d(ctx, E.d_vtab, vtab.data(), sizeof(double) * (vn + 1)));
    if (anchored) {
        std::vector<int> anc(n + kVecPad, 0);
        par_for(n, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) anc[i] = base_of(i);
        });
        CHECK(dalloc(&E.d_anc, n + kVecPad));
        CHECK(h2d(ctx, E.d_anc, anc.data(), sizeof(int) * anc.size()));
        CHECK(blocked_group_order(ctx, anc, ng, A->plan ? A->plan->n_own : A->ncols, &E.d_gorder));
    }
    A->interior.ell = true;
    return PAMG_OK;
}

// Neighbour-coded prolongation (Options::pnc, pamg::PncSet): every row's columns named by the
// grid neighbours whose anchors they are. Declines (leaves the tile layouts to the caller) where a
// row is longer than kPncMaxLen, a column is no neighbour's anchor, or a table would overflow.
int build_pnc(pamg_mat* A, const PtrVec& rp, const IdxVec& ci, const double* val,
              const std::array<int64_t, 4>& grid, const std::vector<int>& inner) {
    using pamg::kPncMaxLen;
    using pamg::kPncSkip;
    const int64_t n = A->nrows;
    // several parts: the interior rows only (the boundary rows — ghost columns — run in their tiles
    // after the exchange; their records carry the skip pattern id)
    std::vector<char> in_set;
    if ((int64_t)inner.size() != n) {
        in_set.assign(n, 0);
        for (int i : inner) in_set[i] = 1;
    }
    auto member = [&](int64_t i) { return in_set.empty() || in_set[i]; };
    const int64_t nx = grid[1], ny = grid[2], nz = grid[3], M = nx * ny;
    if (n != nx * ny * nz || n <= 0 || M % 256 != 0) return PAMG_OK;  // (k_rows_pnc: 256-point blocks of a plane)
    std::vector<int> anc(n + kVecPad, 0);
    std::atomic<bool> ok{true};
    par_for(n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b && ok; ++i) {
            if (member(i) && rp[i + 1] - rp[i] > kPncMaxLen) {
                ok = false;
                return;
            }
            int64_t best = rp[i];
            for (int64_t k = rp[i] + 1; k < rp[i + 1]; ++k)
                if (val[k] > val[best]) best = k;
            anc[i] = rp[i + 1] > rp[i] ? ci[best] : 0;
        }
    });
    if (!ok) return PAMG_OK;
    // pass 1: each row's pattern word (length, codes) and the distinct patterns and values
    std::vector<uint32_t> pw(n);
    std::mutex mu;
    std::vector<uint32_t> pats;
    std::vector<uint64_t> vals;
    const int64_t d[7] = {0, -1, 1, -nx, nx, -M, M};
    par_for(n, [&](int64_t a, int64_t b) {
        // this chunk's distinct patterns and values (open addressing; the tables' limits are far below
        // the slot counts, so a chunk past them stops)
        constexpr int kPS = 4096, kVS = 1024;
        std::vector<uint32_t> pkey(kPS, 0xffffffffu);
        std::vector<uint64_t> vkey(kVS);
        std::vector<char> vused(kVS, 0);
        std::vector<uint32_t> lp;
        std::vector<uint64_t> lv;
        for (int64_t i = a; i < b && ok; ++i) {
            if (!member(i)) continue;
            const int64_t x = i % nx, y = (i / nx) % ny, z = i / M;
            const bool in[7] = {true, x > 0, x < nx - 1, y > 0, y < ny - 1, z > 0, z < nz - 1};
            uint32_t w = (uint32_t)(rp[i + 1] - rp[i]);
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                int c = 0;
                while (c < 7 && !(in[c] && anc[i + d[c]] == ci[k])) ++c;
                if (c == 7) {
                    ok = false;
                    return;
                }
                w |= (uint32_t)c << (3 + 3 * (k - rp[i]));
                uint64_t u;
                std::memcpy(&u, &val[k], 8);
                uint32_t h = (uint32_t)((u ^ (u >> 29)) * 0x9E3779B97F4A7C15ull >> 54);
                while (vused[h] && vkey[h] != u) h = (h + 1) & (kVS - 1);
                if (!vused[h]) {
                    vused[h] = 1;
                    vkey[h] = u;
                    lv.push_back(u);
                    if (lv.size() > (size_t)pamg::kPncValMax) {
                        ok = false;
                        return;
                    }
                }
            }
            pw[i] = w;
            uint32_t h = (w * 0x9E3779B1u) >> 20;
            while (pkey[h] != 0xffffffffu && pkey[h] != w) h = (h + 1) & (kPS - 1);
            if (pkey[h] == 0xffffffffu) {
                pkey[h] = w;
                lp.push_back(w);
                if (lp.size() > (size_t)kPncSkip) {
                    ok = false;
                    return;
                }
            }
        }
        std::lock_guard<std::mutex> lk(mu);
        pats.insert(pats.end(), lp.begin(), lp.end());
        vals.insert(vals.end(), lv.begin(), lv.end());
        std::sort(pats.begin(), pats.end());
        pats.erase(std::unique(pats.begin(), pats.end()), pats.end());
        std::sort(vals.begin(), vals.end());
        vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
    });
    if (!ok || pats.size() > (size_t)kPncSkip || vals.size() > (size_t)pamg::kPncValMax) return PAMG_OK;
    // pass 2: the records (pattern id, value indices)
    std::vector<uint2> rec(n + kVecPad, make_uint2(0u, 0u));
    par_for(n, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            if (!member(i)) {
                rec[i] = make_uint2((uint32_t)kPncSkip, 0u);
                continue;
            }
            uint64_t r = (uint64_t)(std::lower_bound(pats.begin(), pats.end(), pw[i]) - pats.begin());
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                uint64_t u;
                std::memcpy(&u, &val[k], 8);
                const uint64_t vi = (uint64_t)(std::lower_bound(vals.begin(), vals.end(), u) - vals.begin());
                r |= vi << (10 + 7 * (k - rp[i]));
            }
            rec[i] = make_uint2((uint32_t)r, (uint32_t)(r >> 32));
        }
    });
    std::vector<double> vtab(vals.size());
    for (size_t e = 0; e < vals.size(); ++e) std::memcpy(&vtab[e], &vals[e], 8);
    // compact records: the distinct (pattern word, value indices) combinations, numbered in sorted order
    std::vector<std::pair<uint32_t, uint64_t>> combs;
    if (pamg::options().pnc_compact) {
        std::atomic<bool> fits{true};
        par_for(n, [&](int64_t a, int64_t b) {
            std::vector<std::pair<uint32_t, uint64_t>> lc;
            std::pair<uint32_t, uint64_t> last{0xffffffffu, 0};
            for (int64_t i = a; i < b && fits; ++i) {
                if (!member(i)) continue;
                const uint64_t r = ((uint64_t)rec[i].y << 32) | rec[i].x;
                const std::pair<uint32_t, uint64_t> c{pats[r & 1023u], r >> 10};
                if (c == last) continue;
                last = c;
                if (std::find(lc.begin(), lc.end(), c) == lc.end()) {
                    lc.push_back(c);
                    if (lc.size() > (size_t)pamg::kPncCombMax) fits = false;
                }
            }
            std::lock_guard<std::mutex> lk(mu);
            combs.insert(combs.end(), lc.begin(), lc.end());
            std::sort(combs.begin(), combs.end());
            combs.erase(std::unique(combs.begin(), combs.end()), combs.end());
            if (combs.size() > (size_t)pamg::kPncCombMax) fits = false;
        });
        if (!fits) combs.clear();
    }
    pamg::PncSet& P = A->pnc;
    pamg_ctx* ctx = A->ctx;
    P.nx = (int)nx;
    P.ny = (int)ny;
    P.nz = (int)nz;
    P.npat = (int)pats.size();
    P.nval = (int)vals.size();
    // k_rows_pnc's grid (pamg_mat_layout out[8]): one workgroup per 256-point plane block and 32-plane
    // chunk (kernels.hip launch_pnc)
    {
        const int64_t zlen = std::min<int64_t>(32, nz);
        P.grid = (int)((M / 256 * ((nz + zlen - 1) / zlen) + 7) / 8 * 8);
    }
    CHECK(dalloc(&P.d_anc, n + kVecPad));
    CHECK(dalloc(&P.d_vtab, (int64_t)vals.size()));
    CHECK(h2d(ctx, P.d_anc, anc.data(), sizeof(int) * anc.size()));
    CHECK(h2d(ctx, P.d_vtab, vtab.data(), sizeof(double) * vtab.size()));
    if (!combs.empty()) {
        std::vector<uint16_t> cid(n + kVecPad, (uint16_t)pamg::kPncCombSkip);
        par_for(n, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) {
                if (!member(i)) continue;
                const uint64_t r = ((uint64_t)rec[i].y << 32) | rec[i].x;
                const std::pair<uint32_t, uint64_t> c{pats[r & 1023u], r >> 10};
                cid[i] = (uint16_t)(std::lower_bound(combs.begin(), combs.end(), c) - combs.begin());
            }
        });
        std::vector<uint32_t> cw(combs.size());
        std::vector<uint64_t> cv(combs.size());
        for (size_t e = 0; e < combs.size(); ++e) {
            cw[e] = combs[e].first;
            cv[e] = combs[e].second;
        }
        P.npat = (int)combs.size();
        CHECK(dalloc(&P.d_cid, n + kVecPad));
        CHECK(dalloc(&P.d_ptab, (int64_t)cw.size()));
        CHECK(dalloc(&P.d_pvals, (int64_t)cv.size()));
        CHECK(h2d(ctx, P.d_cid, cid.data(), sizeof(uint16_t) * cid.size()));
        CHECK(h2d(ctx, P.d_ptab, cw.data(), sizeof(uint32_t) * cw.size()));
        CHECK(h2d(ctx, P.d_pvals, cv.data(), sizeof(uint64_t) * cv.size()));
    } else {
        CHECK(dalloc(&P.d_rec, n + kVecPad));
        CHECK(dalloc(&P.d_ptab, (int64_t)pats.size()));
        CHECK(h2d(ctx, P.d_rec, rec.data(), sizeof(uint2) * rec.size()));
        CHECK(h2d(ctx, P.d_ptab, pats.data(), sizeof(uint32_t) * pats.size()));
    }
    A->interior.pnc = true;
    return PAMG_OK;
}

// Pattern-dictionary rows (Options::rpat, pamg::RpatSet): a restriction whose rows, as (column - first
// column, value bits) sequences, repeat at most kRpatMax patterns (<= kRpatEnt entries, <= 256 values,
// offsets < 2^24, rows of 1 .. kRpatMaxLen entries). Declines (leaves ELL / tiles to the caller)
// otherwise. The patterns are numbered in first-appearance order (chunks scanned in parallel, merged
// in chunk order: the numbering one sequential pass gives).
int build_rpat(pamg_mat* A, const PtrVec& rp, const IdxVec& ci, const double* val, const std::vector<int>& inner) {
    using pamg::kRpatEnt;
    using pamg::kRpatMax;
    using pamg::kRpatMaxLen;
    using pamg::kRpatSkip;
    const int64_t n = A->nrows;
    if (n <= 0) return PAMG_OK;
    std::vector<char> in_set;
    if ((int64_t)inner.size() != n) {
        in_set.assign(n, 0);
        for (int i : inner) in_set[i] = 1;
    }
    auto member = [&](int64_t i) { return in_set.empty() || in_set[i]; };
    // a row's pattern key: length, offsets, value bits
    auto row_hash = [&](int64_t i) {
        uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)(rp[i + 1] - rp[i]);
        const int64_t c0 = ci[rp[i]];
        for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
            uint64_t u;
            std::memcpy(&u, &val[k], 8);
            h = (h ^ (uint64_t)(ci[k] - c0)) * 0x100000001B3ull;
            h = (h ^ u) * 0x9E3779B97F4A7C15ull;
            h ^= h >> 29;
        }
        return h;
    };
    auto same = [&](int64_t i, int64_t j) {
        const int64_t L = rp[i + 1] - rp[i];
        if (L != rp[j + 1] - rp[j]) return false;
        const int64_t ci0 = ci[rp[i]], cj0 = ci[rp[j]];
        for (int64_t k = 0; k < L; ++k) {
            if (ci[rp[i] + k] - ci0 != ci[rp[j] + k] - cj0) return false;
            if (std::memcmp(&val[rp[i] + k], &val[rp[j] + k], 8) != 0) return false;
        }
        return true;
    };
    // pass 1: each chunk's distinct patterns (hash, representative row) in first-appearance order
    const int nch = std::max(1, std::min<int>(host_threads() * 4, (int)(n / 65536)));
    std::vector<std::vector<std::pair<uint64_t, int64_t>>> firsts(nch);
    std::atomic<bool> ok{true};
    {
        std::vector<std::thread> th;
        const int nt = std::min(nch, host_threads());
        std::atomic<int> next{0};
        for (int t = 0; t < nt; ++t)
            th.emplace_back([&] {
                for (int c; ok && (c = next.fetch_add(1)) < nch;) {
                    auto& f = firsts[c];
                    int last = -1;
                    for (int64_t i = n * c / nch, e = n * (c + 1) / nch; i < e && ok; ++i) {
                        if (!member(i)) continue;
                        const int64_t L = rp[i + 1] - rp[i];
                        if (L < 1 || L > kRpatMaxLen) {
                            ok = false;
                            break;
                        }
                        for (int64_t k = rp[i] + 1; k < rp[i + 1]; ++k)
                            if (ci[k] <= ci[k - 1] || (int64_t)ci[k] - ci[rp[i]] >= (int64_t(1) << 24)) ok = false;
                        const uint64_t h = row_hash(i);
                        if (last >= 0 && f[last].first == h && same(f[last].second, i)) continue;
                        last = -1;
                        for (int q = 0; q < (int)f.size() && last < 0; ++q)
                            if (f[q].first == h && same(f[q].second, i)) last = q;
                        if (last >= 0) continue;
                        if ((int)f.size() == kRpatMax) {
                            ok = false;
                            break;
                        }
                        f.emplace_back(h, i);
                        last = (int)f.size() - 1;
                    }
                }
            });
        for (auto& x : th) x.join();
    }
    if (!ok) return PAMG_OK;
    std::vector<std::pair<uint64_t, int64_t>> pats;  // (hash, representative row)
    for (int c = 0; c < nch; ++c)
        for (const auto& e : firsts[c]) {
            bool seen = false;
            for (const auto& q : pats) seen = seen || (q.first == e.first && same(q.second, e.second));
            if (seen) continue;
            if ((int)pats.size() == kRpatMax) return PAMG_OK;
            pats.push_back(e);
        }
    if (pats.empty()) return PAMG_OK;
    // the entries and the value table
    std::vector<int2> pmeta(pats.size());
    std::vector<uint32_t> pent;
    std::vector<uint64_t> vals;
    for (size_t p = 0; p < pats.size(); ++p) {
        const int64_t r = pats[p].second;
        pmeta[p] = make_int2((int)pent.size(), (int)(rp[r + 1] - rp[r]));
        for (int64_t k = rp[r]; k < rp[r + 1]; ++k) {
            uint64_t u;
            std::memcpy(&u, &val[k], 8);
            size_t vi = std::find(vals.begin(), vals.end(), u) - vals.begin();
            if (vi == vals.size()) {
                if (vals.size() == 256) return PAMG_OK;
                vals.push_back(u);
            }
            pent.push_back((uint32_t)(ci[k] - ci[rp[r]]) | ((uint32_t)vi << 24));
        }
        if ((int)pent.size() > kRpatEnt) return PAMG_OK;
    }
    // pass 2: every row's pattern id (hash lookup, full compare) and first column
    std::vector<std::pair<uint64_t, int>> byhash(pats.size());
    for (size_t p = 0; p < pats.size(); ++p) byhash[p] = {pats[p].first, (int)p};
    std::sort(byhash.begin(), byhash.end());
    std::vector<uint8_t> pid(n + kVecPad, (uint8_t)kRpatSkip);
    std::vector<int> anc(n + kVecPad, 0);
    par_for(n, [&](int64_t a, int64_t b) {
        int last = -1;
        for (int64_t i = a; i < b; ++i) {
            anc[i] = rp[i + 1] > rp[i] ? ci[rp[i]] : 0;
            if (!member(i)) continue;
            if (last >= 0 && same(pats[last].second, i)) {
                pid[i] = (uint8_t)last;
                continue;
            }
            const uint64_t h = row_hash(i);
            last = -1;
            for (auto it = std::lower_bound(byhash.begin(), byhash.end(), std::make_pair(h, -1));
                 it != byhash.end() && it->first == h && last < 0; ++it)
                if (same(pats[it->second].second, i)) last = it->second;
            if (last < 0) {  // (cannot happen: every row's pattern was collected in pass 1)
                ok = false;
                return;
            }
            pid[i] = (uint8_t)last;
        }
    });
    if (!ok) return PAMG_OK;
    std::vector<double> vtab(vals.size());
    for (size_t e = 0; e < vals.size(); ++e) std::memcpy(&vtab[e], &vals[e], 8);
    pamg::RpatSet& R = A->rpat;
    pamg_ctx* ctx = A->ctx;
    R.ngroups = (n + pamg::kEllGroup - 1) / pamg::kEllGroup;
    R.npat = (int)pats.size();
    R.nent = (int)pent.size();
    R.nval = (int)vals.size();
    CHECK(dalloc(&R.d_anc, n + kVecPad));
    CHECK(dalloc(&R.d_pid, n + kVecPad));
    CHECK(dalloc(&R.d_pmeta, R.npat));
    CHECK(dalloc(&R.d_pent, R.nent));
    CHECK(dalloc(&R.d_vtab, R.nval));
    CHECK(h2d(ctx, R.d_anc, anc.data(), sizeof(int) * anc.size()));
    CHECK(h2d(ctx, R.d_pid, pid.data(), pid.size()));
    CHECK(h2d(ctx, R.d_pmeta, pmeta.data(), sizeof(int2) * pmeta.size()));
    CHECK(h2d(ctx, R.d_pent, pent.data(), sizeof(uint32_t) * pent.size()));
    CHECK(h2d(ctx, R.d_vtab, vtab.data(), sizeof(double) * vtab.size()));
    CHECK(blocked_group_order(ctx, anc, R.ngroups, A->plan ? A->plan->n_own : A->ncols, &R.d_gorder));
    A->interior.rpat = true;
    return PAMG_OK;
}

void free_rpat(pamg::RpatSet& R) {
    dfree(R.d_anc);
    dfree(R.d_pid);
    dfree(R.d_pmeta);
    dfree(R.d_pent);
    dfree(R.d_vtab);
    dfree(R.d_gorder);
    R = pamg::RpatSet{};
}

void free_pnc(pamg::PncSet& P) {
    dfree(P.d_anc);
    dfree(P.d_rec);
    dfree(P.d_cid);
    dfree(P.d_pvals);
    dfree(P.d_ptab);
    dfree(P.d_vtab);
    P = pamg::PncSet{};
}

void free_ell(pamg::EllSet& E) {
    dfree(E.d_gorder);
    dfree(E.d_smeta);
    dfree(E.d_ci);
    dfree(E.d_vi);
    dfree(E.d_len);
    dfree(E.d_gmeta);
    dfree(E.d_otab);
    dfree(E.d_vtab);
    dfree(E.d_anc);
    E = pamg::EllSet{};
}

void free_tiles(pamg::TileSet& ts) {
    dfree(ts.d_short);
    dfree(ts.d_long);
    dfree(ts.d_base);
    dfree(ts.d_vtab);
    dfree(ts.d_ctab);
    ts.cd = ts.ctab_n = 0;
    dfree(ts.d_tm_val);
    dfree(ts.d_tm_cidx);
    dfree(ts.d_tm_clo);
    dfree(ts.d_tm_chi);
    dfree(ts.d_tm_rlen);
    dfree(ts.d_tm_anc);
    dfree(ts.d_tm_vidx);
    dfree(ts.d_tm_vtab);
    ts.tm_vt = 0;
    dfree(ts.d_abase);
    ts.anc = ts.pt = ts.xs = false;
    ts.tm = false;
    ts.tm_rs = 0;
    ts.c24 = ts.vd = ts.rl8 = false;
    ts.max_short_len = 0;
    ts.rows_short = 0;
    ts.n_short = ts.n_long = 0;
}

}  // namespace

// In-process world of sibling contexts (pamg_comm_init_local).
// Ghost exchanges rendezvous PAIRWISE: a part meets only the neighbours its plan lists with a
// non-zero count (so a part with no neighbours, or a decoupled pair of parts, never waits for
// the others — ADVICE r4), and each directed pair carries a sequence number and the plan's tag,
// so two parts whose schedules diverge fail with PAMG_E_STATE instead of exchanging the wrong
// vectors. All-reduce and all-gather are world-wide collectives: every rank
// calls them, they meet at a generation barrier. A failed or abandoned collective marks the
// world broken (every waiting rank fails at once); pamg_world_reset clears that once every rank
// has returned.
struct pamg_world {
    int n = 0;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::string why;  // first reason the world broke
    int refs = 1;  // the creator's + one per registered context
    struct Slot {
        const double* x = nullptr;        // the posted vector / buffer
        hipEvent_t ready = nullptr;       // recorded after the work that wrote x
        double scalar = 0.0;              // all-reduce operand
    };
    std::vector<Slot> slot;
    // directed pair (q -> p) at index q * n + p: q's post for its exchanges with p
    struct Post {
        uint64_t seq = 0;                 // exchanges q has posted for p so far
        uint64_t read = 0;                // of those, the ones p has finished reading
        const double* x = nullptr;
        const pamg_plan* plan = nullptr;
        hipEvent_t ready = nullptr;
        int64_t tag = 0;
        // q is in (or has made) an exchange under plan tag zero_tag that lists p with zero counts,
        // after zero_at exchanges with p: a p waiting for q's post #zero_at + 1 under the same tag
        // expects a non-zero count — the two parts' plans disagree (fail at once, not
        // after the 300 s timeout)
        uint64_t zero_at = UINT64_MAX;
        int64_t zero_tag = 0;
    };
    std::vector<Post> post;
    std::vector<pamg_ctx*> ctx;
    static constexpr int kTimeoutS = 300;
    void abort_locked(const char* reason) {
        if (!broken) why = reason;
        broken = true;
        cv.notify_all();
    }
    void abort(const char* reason) {
        std::lock_guard<std::mutex> lk(mu);
        abort_locked(reason);
    }
    // wait (lock held) until pred() or the world breaks; false on a break or timeout
    template <class P>
    bool wait_locked(std::unique_lock<std::mutex>& lk, P pred, const char* what) {
        if (broken) return false;
        if (!cv.wait_for(lk, std::chrono::seconds(kTimeoutS), [&] { return pred() || broken; })) {
            abort_locked(what);
            return false;
        }
        return !broken;
    }
    // false when a rank does not come within 300 s (or the world broke): every waiting rank
    // then fails instead of hanging
    bool barrier() {
        std::unique_lock<std::mutex> lk(mu);
        if (broken) return false;
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        return wait_locked(lk, [&] { return gen != g; }, "a rank did not arrive at a collective within 300 s");
    }
    void release() {
        bool last;
        {
            std::lock_guard<std::mutex> lk(mu);
            last = --refs == 0;
        }
        if (last) delete this;
    }
};

namespace {

// a synchronous transport (host staging or the in-process world): exchanges complete inside
// the call, so nothing overlaps them and nothing can be graph-captured
bool sync_transport(const pamg_ctx* ctx) { return ctx->host_fn != nullptr || ctx->world != nullptr; }

// The in-process exchange. For every neighbour q with a non-zero count, part me posts (x, plan,
// tag, ready event) on the pair (me -> q) under the next sequence number, waits for q's post of
// the same number on (q -> me), checks that both posts carry the same tag and matching counts,
// copies the segment q's send list holds for it straight from q's vector into its ghost slots —
// a contiguous run by one copy, any other list by a gather kernel reading the sibling's vector —
// waits for its copies, marks q's post read, and before returning waits until each neighbour has
// read its own post (so x is not written while a sibling still reads it).
int exchange_local(const pamg_plan* plan, double* x, hipStream_t s) {
    pamg_ctx* ctx = plan->ctx;
    pamg_world* w = ctx->world;
    const int me = ctx->rank, nn = (int)plan->nbr.size(), n = w->n;
    std::vector<int> ks, zs;  // neighbours this exchange pairs with; neighbours listed with zero counts
    for (int k = 0; k < nn; ++k)
        (plan->recv_off[k + 1] > plan->recv_off[k] || plan->send_off[k + 1] > plan->send_off[k] ? ks : zs).push_back(k);
    if (!zs.empty() && plan->tag != 0) {
        std::lock_guard<std::mutex> lk(w->mu);
        for (int k : zs) {
            pamg_world::Post& p = w->post[(size_t)me * n + plan->nbr[k]];
            p.zero_at = p.seq;
            p.zero_tag = plan->tag;
        }
        w->cv.notify_all();
    }
    if (ks.empty()) return PAMG_OK;
    HIPC(hipEventRecord(ctx->ev_ready, s));
    std::vector<uint64_t> seq(ks.size());
    {
        std::lock_guard<std::mutex> lk(w->mu);
        if (w->broken) return fail(PAMG_E_STATE, "local exchange: the world is broken (%s)", w->why.c_str());
        for (size_t i = 0; i < ks.size(); ++i) {
            pamg_world::Post& p = w->post[(size_t)me * n + plan->nbr[ks[i]]];
            p.x = x;
            p.plan = plan;
            p.ready = ctx->ev_ready;
            p.tag = plan->tag;
            seq[i] = ++p.seq;
        }
        w->cv.notify_all();
    }
    int rc = PAMG_OK;
    for (size_t i = 0; i < ks.size() && rc == PAMG_OK; ++i) {
        const int k = ks[i], q = plan->nbr[k];
        pamg_world::Post sq;
        {
            std::unique_lock<std::mutex> lk(w->mu);
            const pamg_world::Post& pq = w->post[(size_t)q * n + me];
            auto zero_listed = [&] { return plan->tag != 0 && pq.zero_tag == plan->tag && pq.zero_at + 1 == seq[i]; };
            if (!w->wait_locked(lk, [&] { return pq.seq >= seq[i] || zero_listed(); },
                                "a neighbour part did not post its exchange within 300 s"))
                return fail(PAMG_E_STATE, "local exchange: part %d waited for part %d: the world is broken (%s)", me, q,
                            w->why.c_str());
            if (pq.seq < seq[i]) {
                w->abort_locked("exchange count mismatch");
                return fail(PAMG_E_STATE,
                            "local exchange: part %d expects %lld ghosts from part %d and sends it %lld, but part %d's plan "
                            "(tag %lld) lists part %d with zero counts", me,
                            (long long)(plan->recv_off[k + 1] - plan->recv_off[k]), q,
                            (long long)(plan->send_off[k + 1] - plan->send_off[k]), q, (long long)plan->tag, me);
            }
            sq = pq;
            if (sq.seq != seq[i] || sq.tag != plan->tag) {
                w->abort_locked("exchange pairing mismatch");
                return fail(PAMG_E_STATE,
                            "local exchange: part %d's exchange #%llu with part %d (plan tag %lld) met part %d's exchange "
                            "#%llu (plan tag %lld): the parts' schedules diverged", me, (unsigned long long)seq[i], q,
                            (long long)plan->tag, q, (unsigned long long)sq.seq, (long long)sq.tag);
            }
        }
        const pamg_plan* pq = sq.plan;
        int kq = -1;
        for (int j = 0; pq && j < (int)pq->nbr.size(); ++j)
            if (pq->nbr[j] == me) kq = j;
        const int64_t cnt = plan->recv_off[k + 1] - plan->recv_off[k];
        const int64_t scnt = plan->send_off[k + 1] - plan->send_off[k];
        if (kq < 0 || pq->send_off[kq + 1] - pq->send_off[kq] != cnt || pq->recv_off[kq + 1] - pq->recv_off[kq] != scnt) {
            w->abort("exchange count mismatch");
            return fail(PAMG_E_STATE, "local exchange: part %d expects %lld ghosts from part %d, which sends %lld", me,
                        (long long)cnt, q, kq < 0 ? 0LL : (long long)(pq->send_off[kq + 1] - pq->send_off[kq]));
        }
        if (cnt == 0) continue;
        double* dst = x + plan->n_own + plan->recv_off[k];
        if (hipStreamWaitEvent(s, sq.ready, 0) != hipSuccess) {
            rc = fail(PAMG_E_HIP, "local exchange: stream wait failed");
            break;
        }
        if (pq->send_run[kq] >= 0) {
            if (hipMemcpyAsync(dst, sq.x + pq->send_run[kq], sizeof(double) * cnt, hipMemcpyDefault, s) != hipSuccess)
                rc = fail(PAMG_E_HIP, "local exchange: copy from part %d failed", q);
        } else {
            pamg::launch_pack(cnt, pq->d_send_idx + pq->send_off[kq], sq.x, dst, s);
        }
    }
    if (rc == PAMG_OK && hipStreamSynchronize(s) != hipSuccess) rc = fail(PAMG_E_HIP, "local exchange: sync failed");
    std::unique_lock<std::mutex> lk(w->mu);
    if (rc != PAMG_OK) {
        w->abort_locked("a part's exchange failed");
        return rc;
    }
    for (size_t i = 0; i < ks.size(); ++i) w->post[(size_t)plan->nbr[ks[i]] * n + me].read = seq[i];
    w->cv.notify_all();
    for (size_t i = 0; i < ks.size(); ++i) {
        const int q = plan->nbr[ks[i]];
        const pamg_world::Post& mine = w->post[(size_t)me * n + q];
        if (!w->wait_locked(lk, [&] { return mine.read >= seq[i]; }, "a neighbour part did not read its exchange within 300 s"))
            return fail(PAMG_E_STATE, "local exchange: part %d waited for part %d to read: the world is broken (%s)", me,
                        q, w->why.c_str());
    }
    return PAMG_OK;
}

// sum of the ranks' *v in rank order, on every rank
int allreduce_local(pamg_ctx* ctx, double* v) {
    pamg_world* w = ctx->world;
    w->slot[ctx->rank].scalar = *v;
    if (!w->barrier()) return fail(PAMG_E_STATE, "local all-reduce: a sibling part did not arrive");
    double sum = 0.0;
    for (int q = 0; q < w->n; ++q) sum += w->slot[q].scalar;
    if (!w->barrier()) return fail(PAMG_E_STATE, "local all-reduce: a sibling part did not arrive");
    *v = sum;
    return PAMG_OK;
}

// every rank's cnt doubles at its src, in rank order, into dst (cnt per rank)
int allgather_local(pamg_ctx* ctx, const double* src, int64_t cnt, double* dst, hipStream_t s) {
    pamg_world* w = ctx->world;
    const int me = ctx->rank;
    w->slot[me].x = src;
    w->slot[me].ready = ctx->ev_ready;
    HIPC(hipEventRecord(ctx->ev_ready, s));
    if (!w->barrier()) return fail(PAMG_E_STATE, "local all-gather: a sibling part did not arrive");
    int rc = PAMG_OK;
    for (int q = 0; q < w->n && rc == PAMG_OK && cnt > 0; ++q) {
        if (hipStreamWaitEvent(s, w->slot[q].ready, 0) != hipSuccess ||
            hipMemcpyAsync(dst + (size_t)q * cnt, w->slot[q].x, sizeof(double) * cnt, hipMemcpyDefault, s) != hipSuccess)
            rc = fail(PAMG_E_HIP, "local all-gather: copy from part %d failed", q);
    }
    if (rc == PAMG_OK && hipStreamSynchronize(s) != hipSuccess) rc = fail(PAMG_E_HIP, "local all-gather: sync failed");
    if (!w->barrier() && rc == PAMG_OK) rc = fail(PAMG_E_STATE, "local all-gather: a sibling part did not arrive");
    return rc;
}

// Ghost exchange of plan on stream s: pack own values, grouped RCCL send/recv straight into
// the ghost slots [n_own + recv_off[k], ...).
int exchange_on(const pamg_plan* plan, double* x, hipStream_t s) {
    pamg_ctx* ctx = plan->ctx;
    const int nn = (int)plan->nbr.size();
    if (nn == 0) return PAMG_OK;
    if (!ctx->comm && !sync_transport(ctx))
        return fail(PAMG_E_STATE, "exchange: plan has neighbours but no communicator");
    // debug (SURVEY §5 race detection): NaN in the ghost slots before every exchange, so a
    // row that reads a ghost before the exchange has landed shows up as NaN
    if (pamg::options().poison_ghosts)
        pamg::launch_fill(plan->recv_off[nn], __builtin_nan(""), x + plan->n_own, s);
    if (ctx->world) return exchange_local(plan, x, s);
    // contiguous send lists go straight from x; the others are packed first
    if (!plan->all_contig)
        pamg::launch_pack(plan->send_off[nn], plan->d_send_idx, x, plan->d_sendbuf, s);
    auto send_ptr = [&](int k) -> const double* {
        return plan->send_run[k] >= 0 ? x + plan->send_run[k] : plan->d_sendbuf + plan->send_off[k];
    };
    if (ctx->host_fn) {  // debug transport: synchronous host staging
        const int64_t ns = plan->send_off[nn], nr = plan->recv_off[nn];
        ctx->h_send.resize(ns + 1);
        ctx->h_recv.resize(nr + 1);
        std::vector<int64_t> sc(nn), rc(nn);
        for (int k = 0; k < nn; ++k) {
            sc[k] = plan->send_off[k + 1] - plan->send_off[k];
            rc[k] = plan->recv_off[k + 1] - plan->recv_off[k];
            if (sc[k])
                HIPC(hipMemcpyAsync(ctx->h_send.data() + plan->send_off[k], send_ptr(k),
                                    sizeof(double) * sc[k], hipMemcpyDeviceToHost, s));
        }
        HIPC(hipStreamSynchronize(s));
        if (ctx->host_fn(ctx->host_user, 0, nn, plan->nbr.data(), sc.data(), ctx->h_send.data(), rc.data(),
                         ctx->h_recv.data()) != 0)
            return fail(PAMG_E_RCCL, "exchange: host transport failed");
        if (nr) HIPC(hipMemcpyAsync(x + plan->n_own, ctx->h_recv.data(), sizeof(double) * nr, hipMemcpyHostToDevice, s));
        HIPC(hipStreamSynchronize(s));
        return PAMG_OK;
    }
    NCCLC(ncclGroupStart());
    for (int k = 0; k < nn; ++k) {
        const size_t sc = (size_t)(plan->send_off[k + 1] - plan->send_off[k]);
        const size_t rc = (size_t)(plan->recv_off[k + 1] - plan->recv_off[k]);
        if (sc) NCCLC(ncclSend(send_ptr(k), sc, ncclDouble, plan->nbr[k], ctx->comm, s));
        if (rc) NCCLC(ncclRecv(x + plan->n_own + plan->recv_off[k], rc, ncclDouble, plan->nbr[k], ctx->comm, s));
    }
    NCCLC(ncclGroupEnd());
    return PAMG_OK;
}

// y = op(A, x[, b]) with x's ghosts exchanged first; interior rows overlap the exchange.
int apply(pamg_ctx* ctx, const pamg_mat* A, int op, double* x, const double* b, double* y,
          double omega) {
    hipStream_t s = ctx->s_comp;
    bool comm = A->plan && !A->plan->nbr.empty();
    if (comm && sync_transport(ctx)) {  // debug / in-process transport: exchange first, no overlap
        CHECK(exchange_on(A->plan, x, s));
        comm = false;
    }
    if (comm) {
        HIPC(hipEventRecord(ctx->ev_fork, s));
        HIPC(hipStreamWaitEvent(ctx->s_comm, ctx->ev_fork, 0));
        CHECK(exchange_on(A->plan, x, ctx->s_comm));
        HIPC(hipEventRecord(ctx->ev_join, ctx->s_comm));
    }
    pamg::launch_rows(*A, A->interior, op, x, b, x, y, omega, s);
    if (comm) HIPC(hipStreamWaitEvent(s, ctx->ev_join, 0));
    pamg::launch_rows(*A, A->boundary, op, x, b, x, y, omega, s);
    HIPC(hipGetLastError());
    return PAMG_OK;
}

// S dependent sweeps (S = 2: Jacobi -> residual; S = 3: Jacobi -> Jacobi -> residual, the
// pipeline's chain) on one part of several whose level is a z-slab in the symmetric layout
// (SymDia::tb_part): the blocked pass k_sym_tb<S> covers the output planes that need no ghost
// (S-1 planes in from a neighbour part) and runs while in0's ghosts travel; the set's planes
// next to them then take the separate sweep, the planes with ghost columns (the boundary
// tiles) theirs after the exchange; each later stage exchanges its input's ghosts while the
// set's planes take the separate sweep, then the boundary planes. Every row's value is the
// separate sweeps' (SPEC §S3 bits).
// exch = false (pamg_bench_rowop): the same launches without the exchanges, to time one part's
// kernels alone (the per-part figures of the multi-GPU model)
int sweeps_part(pamg_ctx* ctx, const pamg_mat* A, int S, const double* in0, double* const* out, const double* b,
                double omega, bool exch = true) {
    hipStream_t s = ctx->s_comp;
    const pamg::SymDia& sd = A->sym;
    const int nz = sd.tb.nz;
    const int zlo = sd.part_lo == 0 ? 0 : sd.part_lo + S - 1, zhi = sd.part_hi == nz ? nz : sd.part_hi - (S - 1);
    auto stage = [&](double* v, auto&& overlapped, auto&& after) -> int {
        bool comm = exch && A->plan && !A->plan->nbr.empty();
        if (comm && sync_transport(ctx)) {  // debug / in-process transport: exchange first, no overlap
            CHECK(exchange_on(A->plan, v, s));
            comm = false;
        }
        if (comm) {
            HIPC(hipEventRecord(ctx->ev_fork, s));
            HIPC(hipStreamWaitEvent(ctx->s_comm, ctx->ev_fork, 0));
            CHECK(exchange_on(A->plan, v, ctx->s_comm));
            HIPC(hipEventRecord(ctx->ev_join, ctx->s_comm));
        }
        overlapped();
        if (comm) HIPC(hipStreamWaitEvent(s, ctx->ev_join, 0));
        after();
        HIPC(hipGetLastError());
        return PAMG_OK;
    };
    pamg::TbArgs ta;
    ta.nstages = S;
    ta.last_resid = true;
    ta.in0 = in0;
    for (int q = 0; q < S; ++q) ta.out[q] = out[q];
    ta.b = b;
    ta.omega = omega;
    for (int q = 0; q < S; ++q) {
        const int op = q == S - 1 ? pamg::OP_RESID : pamg::OP_JACOBI;
        const double w = q == S - 1 ? 0.0 : omega;
        double* v = const_cast<double*>(q == 0 ? in0 : out[q - 1]);
        CHECK(stage(
            v,
            [&]() {
                if (q == 0) pamg::launch_sym_tb(*A, ta, s);
                // the set's planes next to the neighbour parts, both sides in one launch
                pamg::launch_sym_planes(*A, op, sd.part_lo, zlo, v, b, out[q], w, s, zhi, sd.part_hi);
            },
            [&]() { pamg::launch_rows(*A, A->boundary, op, v, b, v, out[q], w, s); }));
    }
    return PAMG_OK;
}

int jr_part(pamg_ctx* ctx, const pamg_mat* A, double* x, const double* b, double* t, double* r, double omega) {
    double* out[2] = {t, r};
    return sweeps_part(ctx, A, 2, x, out, b, omega);
}

// The deterministic dot x.y over the own rows of every rank (fixed-grid partials, then the
// cross-rank sum); `partial` enqueues the partials + final kernels (default: launch_dot).
template <class F>
int reduce_with(pamg_ctx* ctx, int64_t n, double* out, F partial) {
    hipStream_t s = ctx->s_comp;
    const int np = pamg::dot_partials(n);
    if (np + 1 > ctx->red_cap) return fail(PAMG_E_STATE, "reduction workspace too small");
    double* res = ctx->d_red + ctx->red_cap - 1;
    partial(np, ctx->d_red, res, s);
    if (ctx->comm && ctx->nranks > 1) NCCLC(ncclAllReduce(res, res, 1, ncclDouble, ncclSum, ctx->comm, s));
    HIPC(hipMemcpyAsync(ctx->h_red, res, sizeof(double), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    *out = *ctx->h_red;
    if (ctx->world && ctx->nranks > 1) CHECK(allreduce_local(ctx, out));
    if (ctx->host_fn && ctx->nranks > 1) {
        const int64_t one = 1;
        double sum = 0.0;
        if (ctx->host_fn(ctx->host_user, 2, 1, nullptr, &one, out, &one, &sum) != 0)
            return fail(PAMG_E_RCCL, "allreduce: host transport failed");
        *out = sum;
    }
    return PAMG_OK;
}

int reduce_scalar(pamg_ctx* ctx, int64_t n, const double* x, const double* y, double* out) {
    return reduce_with(ctx, n, out, [&](int np, double* parts, double* res, hipStream_t s) {
        pamg::launch_dot(n, x, y, parts, np, res, s);
    });
}

}  // namespace

// ------------------------------------------------------------------ hierarchy type

struct pamg_hier {
    pamg_ctx* ctx = nullptr;
    int L = 0;
    std::vector<const pamg_mat*> A, P, R;
    std::vector<double> omega;
    // per-level work vectors (level 0: t, r only; x and b belong to the caller)
    std::vector<double*> x, b, t, r;
    std::vector<int64_t> nown;
    // coarsest level
    int64_t nc = 0;
    double* d_ainv = nullptr;          // row-major nc x nc (the ABI hands it over column-major)
    // replicated tail (SPEC §S7 agglomeration): levels >= rep are held whole on every rank;
    // the restriction into level rep yields this rank's rows [coffs[me], coffs[me+1]), which
    // are all-gathered (in blocks of cmax) into the whole vector
    int rep = 0;
    std::vector<int64_t> coffs;        // nranks + 1
    int64_t cmax = 0;                  // max rows per rank of level rep
    double* d_bgather = nullptr;       // nranks * cmax (+ nc scratch for the one-level case)
    double* d_bsend = nullptr;         // cmax
    // graph replay
    bool use_graph = true;
    hipGraphExec_t gexec = nullptr;
    // cross-cycle pipeline (Options::jr_fuse, stationary cycles): head (first cycle without its
    // level-0 post-smoothing), two steady segments (the previous cycle's post-smoothing fused
    // with this cycle's pre-smoothing and residual, then the rest of the cycle; the level-0
    // iterate alternates between t[0] and u0), two tails (the last post-smoothing)
    hipGraphExec_t g_head = nullptr, g_steady[2] = {nullptr, nullptr}, g_tail[2] = {nullptr, nullptr};
    const double* gp_x = nullptr;
    const double* gp_b = nullptr;
    double* u0 = nullptr;
    const double* g_x = nullptr;
    const double* g_b = nullptr;
    bool g_zero0 = false;
    bool graph_failed = false;
    // PCG workspace (level-0 layout, allocated on first use)
    double *pcg_r = nullptr, *pcg_z = nullptr, *pcg_p = nullptr, *pcg_q = nullptr;
    // level-0 locality permutation (pamg_hier_set_perm): device row i = caller row perm[i];
    // the caller's x and b are gathered into px / pb at entry and x is scattered back at exit
    int* d_perm = nullptr;
    double *px = nullptr, *pb = nullptr;
    // profiling
    int nu1 = 1, nu2 = 1;  // V(nu1, nu2) Jacobi sweeps (SPEC §S6)
    bool prof = false;
    std::vector<hipEvent_t> ev;
    std::vector<std::pair<int, int>> ev_tag;  // (level, op) per event pair
    std::vector<double> prof_ms;              // L * 6
};

namespace {

// All-gather this rank's block of level H->rep (in d_bsend) into the rank blocks of
// d_bgather, then compact them into global order at dst.
int gather_rep(pamg_hier* H, double* dst, hipStream_t s) {
    pamg_ctx* ctx = H->ctx;
    const int nr = (int)H->coffs.size() - 1;
    if (ctx->host_fn) {
        ctx->h_send.resize(H->cmax + 1);
        ctx->h_recv.resize((size_t)nr * H->cmax + 1);
        HIPC(hipMemcpyAsync(ctx->h_send.data(), H->d_bsend, sizeof(double) * H->cmax, hipMemcpyDeviceToHost, s));
        HIPC(hipStreamSynchronize(s));
        const int64_t cnt = H->cmax, tot = (int64_t)nr * H->cmax;
        if (ctx->host_fn(ctx->host_user, 1, nr, nullptr, &cnt, ctx->h_send.data(), &tot, ctx->h_recv.data()) != 0)
            return fail(PAMG_E_RCCL, "allgather: host transport failed");
        HIPC(hipMemcpyAsync(H->d_bgather, ctx->h_recv.data(), sizeof(double) * tot, hipMemcpyHostToDevice, s));
    } else if (ctx->world) {
        CHECK(allgather_local(ctx, H->d_bsend, H->cmax, H->d_bgather, s));
    } else {
        NCCLC(ncclAllGather(H->d_bsend, H->d_bgather, (size_t)H->cmax, ncclDouble, ctx->comm, s));
    }
    for (int q = 0; q < nr; ++q) {
        const int64_t c = H->coffs[q + 1] - H->coffs[q];
        if (c)
            HIPC(hipMemcpyAsync(dst + H->coffs[q], H->d_bgather + (size_t)q * H->cmax,
                                sizeof(double) * c, hipMemcpyDeviceToDevice, s));
    }
    return PAMG_OK;
}

// x_L = Ainv b_L. b_L is whole on every rank, except for a one-level hierarchy on several
// ranks (level 0 is the caller's distributed vector): gather it, solve the own rows.
int coarse_solve(pamg_hier* H, const double* bL, double* xL, hipStream_t s) {
    pamg_ctx* ctx = H->ctx;
    const int nr = (int)H->coffs.size() - 1;
    if (H->L > 1 || nr == 1) {
        pamg::launch_dense_gemv(H->nc, H->nc, 0, H->d_ainv, bL, xL, s);
        return PAMG_OK;
    }
    const int me = ctx->rank;
    const int64_t own0 = H->coffs[me], nown = H->coffs[me + 1] - own0;
    HIPC(hipMemcpyAsync(H->d_bsend, bL, sizeof(double) * nown, hipMemcpyDeviceToDevice, s));
    double* full = H->d_bgather + (size_t)nr * H->cmax;
    CHECK(gather_rep(H, full, s));
    pamg::launch_dense_gemv(nown, H->nc, own0, H->d_ainv, full, xL, s);
    return PAMG_OK;
}

struct ProfScope {
    pamg_hier* H;
    int lev, op;
    hipStream_t s;
    ProfScope(pamg_hier* h, int l, int o, hipStream_t st) : H(h), lev(l), op(o), s(st) {
        if (!H->prof) return;
        hipEvent_t e;
        (void)hipEventCreate(&e);
        (void)hipEventRecord(e, s);
        H->ev.push_back(e);
    }
    ~ProfScope() {
        if (!H->prof) return;
        hipEvent_t e;
        (void)hipEventCreate(&e);
        (void)hipEventRecord(e, s);
        H->ev.push_back(e);
        H->ev_tag.emplace_back(lev, op);
    }
};

// One V-cycle (SPEC §S6), enqueued on the compute stream; result in x. zero0: the level-0
// initial guess is zero (preconditioner use), so the level-0 pre-smoothing takes the
// zero-guess form too (bit-identical to the full sweep from x = 0, SPEC §S3).
// Level-0 segments of the cross-cycle pipeline (vcycle_raw): l0_given — the level-0 pre-smoothed
// iterate and residual are already in t0 / r0 (a k_sym_chain launch made them); l0_post —
// whether this call ends with the level-0 post-smoothing (else the prolongated t0 is left for
// the next chain launch). Defaults: one whole cycle.
struct L0Seg {
    bool given = false;
    double* t0 = nullptr;
    double* r0 = nullptr;
    bool post = true;
};

int vcycle_enqueue(pamg_hier* H, double* x, const double* b, bool zero0 = false, L0Seg seg = L0Seg{}) {
    pamg_ctx* ctx = H->ctx;
    hipStream_t s = ctx->s_comp;
    const int L = H->L;
    if (L == 1) {
        ProfScope p(H, 0, 5, s);
        return coarse_solve(H, b, x, s);
    }
    H->x[0] = x;
    H->b[0] = const_cast<double*>(b);
    // V(nu1, nu2): the pre-smoothed iterate of level l ends in t[l] or r[l] (sweeps
    // ping-pong between them); the residual goes to the other one; the post-smoothing
    // sweeps ping-pong between x[l] and the spare so that the last one writes x[l]
    std::vector<double*> cur(L, nullptr), spare(L, nullptr);
    for (int l = 0; l < L - 1; ++l) {
        const pamg_mat* A = H->A[l];
        double *c = H->t[l], *o = H->r[l];
        if (l == 0 && seg.given) {  // made by the chain launch before this call
            cur[0] = seg.t0;
            spare[0] = seg.r0;
            ProfScope p(H, 0, 2, s);
            CHECK(apply(ctx, H->R[0], pamg::OP_SPMV, seg.r0, nullptr, H->b[1], 0.0));
            continue;
        }
        // level 0, V(1, nu2) from a given guess: the pre-smoothing sweep and the residual in one
        // temporally blocked pass (k_sym_tb, S = 2; both timed as jacobi_pre)
        const bool fuse = l == 0 && !zero0 && H->nu1 == 1 && pamg::options().jr_fuse && A->interior.sym &&
                          A->sym.tb_ok && !(A->plan && !A->plan->nbr.empty());
        // one part of several: the blocked pass on the slab's inner planes (jr_part)
        const bool fuse_part = !fuse && l == 0 && !zero0 && H->nu1 == 1 && pamg::options().jr_fuse &&
                               A->interior.sym && A->sym.tb_part;
        if (fuse_part) {
            ProfScope p(H, l, 0, s);
            CHECK(jr_part(ctx, A, H->x[0], H->b[0], c, o, H->omega[0]));
        } else if (fuse) {
            ProfScope p(H, l, 0, s);
            pamg::TbArgs ta;
            ta.nstages = 2;
            ta.last_resid = true;
            ta.in0 = H->x[0];
            ta.out[0] = c;
            ta.out[1] = o;
            ta.b = H->b[0];
            ta.omega = H->omega[0];
            pamg::launch_sym_tb(*A, ta, s);
            HIPC(hipGetLastError());
        } else {
            ProfScope p(H, l, 0, s);
            if (l == 0 && !zero0)
                CHECK(apply(ctx, A, pamg::OP_JACOBI, H->x[0], H->b[0], c, H->omega[0]));
            else
                pamg::launch_jacobi_zero(H->nown[l], H->b[l], A->d_diag, H->omega[l], c, s);
            for (int k = 1; k < H->nu1; ++k) {
                CHECK(apply(ctx, A, pamg::OP_JACOBI, c, H->b[l], o, H->omega[l]));
                std::swap(c, o);
            }
        }
        cur[l] = c;
        spare[l] = o;
        if (!fuse && !fuse_part) {
            ProfScope p(H, l, 1, s);
            CHECK(apply(ctx, A, pamg::OP_RESID, c, H->b[l], o, 0.0));
        }
        {
            ProfScope p(H, l, 2, s);
            if (l + 1 == H->rep && ctx->nranks > 1) {  // into the replicated tail
                CHECK(apply(ctx, H->R[l], pamg::OP_SPMV, o, nullptr, H->d_bsend, 0.0));
                CHECK(gather_rep(H, H->b[l + 1], s));
            } else {
                CHECK(apply(ctx, H->R[l], pamg::OP_SPMV, o, nullptr, H->b[l + 1], 0.0));
            }
        }
    }
    {
        ProfScope p(H, L - 1, 5, s);
        CHECK(coarse_solve(H, H->b[L - 1], H->x[L - 1], s));
    }
    for (int l = L - 2; l >= 0; --l) {
        {
            ProfScope p(H, l, 3, s);
            CHECK(apply(ctx, H->P[l], pamg::OP_PROLONG, H->x[l + 1], nullptr, cur[l], 0.0));
        }
        if (l == 0 && !seg.post) break;
        {
            ProfScope p(H, l, 4, s);
            double* in = cur[l];
            for (int k = 0; k < H->nu2; ++k) {
                double* out = ((H->nu2 - k) % 2 == 1) ? H->x[l] : spare[l];
                CHECK(apply(ctx, H->A[l], pamg::OP_JACOBI, in, H->b[l], out, H->omega[l]));
                if (out == spare[l]) spare[l] = in;
                in = out;
            }
        }
    }
    HIPC(hipGetLastError());
    return PAMG_OK;
}

}  // namespace

// ------------------------------------------------------------------ C-ABI

extern "C" {


int pamg_ctx_create(int device, pamg_ctx** out) {
    if (!out) return fail(PAMG_E_ARG, "ctx_create: out is NULL");
    int ndev = 0;
    HIPC(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(PAMG_E_ARG, "ctx_create: device %d of %d", device, ndev);
    auto c = std::make_unique<pamg_ctx>();
    c->device = device;
    HIPC(hipSetDevice(device));
    HIPC(hipStreamCreateWithFlags(&c->s_comp, hipStreamNonBlocking));
    HIPC(hipStreamCreateWithFlags(&c->s_comm, hipStreamNonBlocking));
    HIPC(hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming));
    HIPC(hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
    c->red_cap = 2048;
    CHECK(dalloc(&c->d_red, c->red_cap));
    HIPC(hipHostMalloc(reinterpret_cast<void**>(&c->h_red), sizeof(double)));
    *out = c.release();
    return PAMG_OK;
}

int pamg_ctx_destroy(pamg_ctx* ctx) {
    if (!ctx) return PAMG_OK;
    ctx_unref(ctx);
    return PAMG_OK;
}

}  // extern "C"

namespace {
// The context's teardown, when its last reference is dropped: the caller's handle
// (pamg_ctx_destroy) and one per plan / vector / matrix / hierarchy made on it. So the handles
// may be destroyed in any order — e.g. by a garbage collector that finalises a context before
// the vectors that referenced it.
void ctx_teardown(pamg_ctx* ctx) {
    (void)hipSetDevice(ctx->device);
    (void)hipStreamSynchronize(ctx->s_comp);
    (void)hipStreamSynchronize(ctx->s_comm);
    if (ctx->comm) ncclCommDestroy(ctx->comm);
    if (ctx->world) {
        {
            std::lock_guard<std::mutex> lk(ctx->world->mu);
            ctx->world->ctx[ctx->rank] = nullptr;
        }
        ctx->world->release();
    }
    if (ctx->ev_ready) (void)hipEventDestroy(ctx->ev_ready);
    dfree(ctx->d_red);
    if (ctx->h_red) (void)hipHostFree(ctx->h_red);
    for (int k = 0; k < 2; ++k) {
        if (ctx->stage[k]) (void)hipHostFree(ctx->stage[k]);
        if (ctx->stage_done[k]) (void)hipEventDestroy(ctx->stage_done[k]);
    }
    (void)hipEventDestroy(ctx->ev_fork);
    (void)hipEventDestroy(ctx->ev_join);
    (void)hipStreamDestroy(ctx->s_comp);
    (void)hipStreamDestroy(ctx->s_comm);
    delete ctx;
}
}  // namespace

void ctx_ref(pamg_ctx* ctx) { ctx->refs.fetch_add(1); }
void ctx_unref(pamg_ctx* ctx) {
    if (ctx->refs.fetch_sub(1) == 1) ctx_teardown(ctx);
}

extern "C" {

int pamg_device_count(int* n) {
    if (!n) return fail(PAMG_E_ARG, "device_count: NULL");
    HIPC(hipGetDeviceCount(n));
    return PAMG_OK;
}

int pamg_ctx_refcount(const pamg_ctx* ctx, int* refs) {
    if (!ctx || !refs) return fail(PAMG_E_ARG, "ctx_refcount: bad args");
    *refs = (int)ctx->refs.load();
    return PAMG_OK;
}

int pamg_ctx_sync(pamg_ctx* ctx) {
    if (!ctx) return fail(PAMG_E_ARG, "ctx_sync: NULL");
    HIPC(hipStreamSynchronize(ctx->s_comm));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_device_sync(int device) {
    HIPC(hipSetDevice(device));
    HIPC(hipDeviceSynchronize());
    return PAMG_OK;
}

int pamg_comm_unique_id(unsigned char id[128]) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId is 128 bytes");
    ncclUniqueId u;
    NCCLC(ncclGetUniqueId(&u));
    std::memcpy(id, &u, 128);
    return PAMG_OK;
}

int pamg_runtime_versions(int* hip_runtime, int* hip_built, int* rccl_runtime, int* rccl_built) {
    int hv = 0, rv = 0;
    HIPC(hipRuntimeGetVersion(&hv));
    NCCLC(ncclGetVersion(&rv));
    if (hip_runtime) *hip_runtime = hv;
    if (hip_built) *hip_built = HIP_VERSION;
    if (rccl_runtime) *rccl_runtime = rv;
    if (rccl_built) *rccl_built = NCCL_VERSION_CODE;
    return PAMG_OK;
}

int pamg_comm_init(pamg_ctx* ctx, int nranks, int rank, const unsigned char id[128]) {
    if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(PAMG_E_ARG, "comm_init: bad args");
    // The RCCL this process resolved librccl.so.1 to must be the one libpamg was compiled
    // against or newer. A host that loaded another ROCm copy first (the torch wheel bundles
    // HIP 7.0 + RCCL 2.26.6 under the same sonames) binds libpamg's RCCL calls to that older
    // library and its HIP runtime; round 1 saw that combination segfault inside the first
    // captured V-cycle ("Library load order"). Refuse it with an error instead.
    {
        int rv = 0;
        NCCLC(ncclGetVersion(&rv));
        if (rv < NCCL_VERSION_CODE) {
            Dl_info di{};
            const char* path = dladdr(reinterpret_cast<void*>(&ncclGetVersion), &di) && di.dli_fname
                                   ? di.dli_fname : "?";
            return fail(PAMG_E_RCCL,
                        "comm_init: RCCL %d loaded from %s is older than the RCCL %d libpamg was built "
                        "against; load libpamg before any other ROCm copy (e.g. before importing torch)",
                        rv, path, NCCL_VERSION_CODE);
        }
    }
    CHECK(set_device(ctx));
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    NCCLC(ncclCommInitRank(&ctx->comm, nranks, u, rank));
    ctx->rank = rank;
    ctx->nranks = nranks;
    return PAMG_OK;
}

int pamg_comm_init_host(pamg_ctx* ctx, int nranks, int rank, pamg_host_comm_fn fn, void* user) {
    if (!ctx || !fn || nranks < 1 || rank < 0 || rank >= nranks)
        return fail(PAMG_E_ARG, "comm_init_host: bad args");
    if (ctx->comm) return fail(PAMG_E_STATE, "comm_init_host: context already has an RCCL communicator");
    ctx->host_fn = fn;
    ctx->host_user = user;
    ctx->rank = rank;
    ctx->nranks = nranks;
    return PAMG_OK;
}

int pamg_world_create(int nparts, pamg_world** out) {
    if (!out || nparts < 1) return fail(PAMG_E_ARG, "world_create: bad args");
    auto w = new pamg_world();
    w->n = nparts;
    w->slot.resize(nparts);
    w->post.resize((size_t)nparts * nparts);
    w->ctx.assign(nparts, nullptr);
    *out = w;
    return PAMG_OK;
}

int pamg_world_destroy(pamg_world* w) {
    if (w) w->release();
    return PAMG_OK;
}

int pamg_world_abort(pamg_world* w) {
    if (!w) return fail(PAMG_E_ARG, "world_abort: NULL");
    w->abort("pamg_world_abort");
    return PAMG_OK;
}

int pamg_world_reset(pamg_world* w) {
    if (!w) return fail(PAMG_E_ARG, "world_reset: NULL");
    std::lock_guard<std::mutex> lk(w->mu);
    w->broken = false;
    w->why.clear();
    w->arrived = 0;
    for (auto& p : w->post) p = pamg_world::Post();
    return PAMG_OK;
}

int pamg_world_state(pamg_world* w, int* broken) {
    if (!w || !broken) return fail(PAMG_E_ARG, "world_state: bad args");
    std::lock_guard<std::mutex> lk(w->mu);
    *broken = w->broken ? 1 : 0;
    return PAMG_OK;
}

int pamg_comm_init_local(pamg_ctx* ctx, pamg_world* w, int rank) {
    if (!ctx || !w || rank < 0 || rank >= w->n) return fail(PAMG_E_ARG, "comm_init_local: bad args");
    if (ctx->comm || ctx->host_fn || ctx->world)
        return fail(PAMG_E_STATE, "comm_init_local: the context already has a transport");
    CHECK(set_device(ctx));
    {
        std::lock_guard<std::mutex> lk(w->mu);
        if (w->ctx[rank]) return fail(PAMG_E_STATE, "comm_init_local: rank %d is taken", rank);
        // siblings on other GPUs read this one's vectors and it reads theirs (peer access; an
        // already enabled pair is fine)
        for (pamg_ctx* o : w->ctx) {
            if (!o || o->device == ctx->device) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, ctx->device, o->device) != hipSuccess || !can)
                return fail(PAMG_E_HIP, "comm_init_local: devices %d and %d cannot access each other", ctx->device,
                            o->device);
            for (int d = 0; d < 2; ++d) {
                (void)hipSetDevice(d == 0 ? ctx->device : o->device);
                const hipError_t e = hipDeviceEnablePeerAccess(d == 0 ? o->device : ctx->device, 0);
                if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
                    return fail(PAMG_E_HIP, "comm_init_local: peer access %d <-> %d: %s", ctx->device, o->device,
                                hipGetErrorString(e));
                (void)hipGetLastError();
            }
            CHECK(set_device(ctx));
        }
        w->ctx[rank] = ctx;
        ++w->refs;
    }
    if (!ctx->ev_ready) HIPC(hipEventCreateWithFlags(&ctx->ev_ready, hipEventDisableTiming));
    ctx->world = w;
    ctx->rank = rank;
    ctx->nranks = w->n;
    return PAMG_OK;
}

}  // extern "C"

namespace {
// f(r) for every rank r of w, each on its own host thread (the world's contexts meet inside);
// the first failure's code, with the failing part's message in this thread's error state
template <class F>
int world_each(pamg_world* w, F&& f) {
    if (!w) return fail(PAMG_E_ARG, "world: NULL");
    for (int r = 0; r < w->n; ++r)
        if (!w->ctx[r]) return fail(PAMG_E_STATE, "world: rank %d has no context", r);
    std::vector<int> rc(w->n, PAMG_OK), order(w->n, INT32_MAX);
    std::vector<std::string> msg(w->n);
    std::vector<std::thread> th;
    std::atomic<int> nfail{0};
    for (int r = 0; r < w->n; ++r)
        th.emplace_back([&, r] {
            rc[r] = f(r);
            if (rc[r] != PAMG_OK) {
                msg[r] = pamg::last_error();
                order[r] = nfail.fetch_add(1);
                w->abort("a part's call failed");  // its siblings stop waiting for it now
            }
        });
    for (auto& t : th) t.join();
    if (nfail.load() == 0) return PAMG_OK;
    // the part that failed first (the cause; the others failed because the world broke)
    const int r = (int)(std::min_element(order.begin(), order.end()) - order.begin());
    // every part has returned (the library owns all the world's threads here), so the break
    // that released the siblings is cleared: one part's argument error leaves the world usable
    // for the next call
    (void)pamg_world_reset(w);
    return fail(rc[r], "part %d: %s", r, msg[r].c_str());
}
}  // namespace

extern "C" {

int pamg_world_spmv(pamg_world* w, pamg_mat* const* A, pamg_vec* const* x, pamg_vec* const* y) {
    if (!A || !x || !y) return fail(PAMG_E_ARG, "world_spmv: bad args");
    return world_each(w, [&](int r) { return pamg_spmv(w->ctx[r], A[r], x[r], y[r]); });
}

int pamg_world_exchange(pamg_world* w, pamg_plan* const* plan, pamg_vec* const* x) {
    if (!plan || !x) return fail(PAMG_E_ARG, "world_exchange: bad args");
    return world_each(w, [&](int r) { return pamg_exchange(w->ctx[r], plan[r], x[r]); });
}

int pamg_world_dot(pamg_world* w, pamg_vec* const* x, pamg_vec* const* y, double* out) {
    if (!x || !y || !out || !w) return fail(PAMG_E_ARG, "world_dot: bad args");
    std::vector<double> v(w->n, 0.0);
    CHECK(world_each(w, [&](int r) { return pamg_vec_dot(w->ctx[r], x[r], y[r], &v[r]); }));
    *out = v[0];  // (every rank holds the same sum)
    return PAMG_OK;
}

int pamg_world_vcycle(pamg_world* w, pamg_hier* const* H, pamg_vec* const* x, pamg_vec* const* b, int ncycles,
                      double* res_hist) {
    if (!H || !x || !b || !w) return fail(PAMG_E_ARG, "world_vcycle: bad args");
    // every rank takes the same schedule: with a history each computes the norms (an all-reduce
    // per cycle), so each gets a buffer of its own and rank 0's is returned
    if (ncycles < 0) return fail(PAMG_E_ARG, "world_vcycle: ncycles < 0");
    std::vector<std::vector<double>> hist(w->n, std::vector<double>(res_hist ? (size_t)ncycles : 0));
    CHECK(world_each(w, [&](int r) {
        return pamg_vcycle(w->ctx[r], H[r], x[r], b[r], ncycles, res_hist ? hist[r].data() : nullptr);
    }));
    if (res_hist) std::copy(hist[0].begin(), hist[0].end(), res_hist);
    return PAMG_OK;
}

int pamg_world_pcg(pamg_world* w, pamg_hier* const* H, pamg_vec* const* x, pamg_vec* const* b, double rtol,
                   int maxit, int* iters, double* res_hist) {
    if (!H || !x || !b || !w) return fail(PAMG_E_ARG, "world_pcg: bad args");
    if (maxit < 0) return fail(PAMG_E_ARG, "world_pcg: maxit < 0");
    std::vector<std::vector<double>> hist(w->n, std::vector<double>(res_hist ? (size_t)maxit + 1 : 0));
    std::vector<int> it(w->n, 0);
    CHECK(world_each(w, [&](int r) {
        return pamg_pcg(w->ctx[r], H[r], x[r], b[r], rtol, maxit, &it[r], res_hist ? hist[r].data() : nullptr);
    }));
    if (iters) *iters = it[0];
    if (res_hist) std::copy(hist[0].begin(), hist[0].end(), res_hist);
    return PAMG_OK;
}

int pamg_comm_rank(const pamg_ctx* ctx, int* rank, int* nranks) {
    if (!ctx) return fail(PAMG_E_ARG, "comm_rank: NULL");
    if (rank) *rank = ctx->rank;
    if (nranks) *nranks = ctx->nranks;
    return PAMG_OK;
}

int pamg_plan_create(pamg_ctx* ctx, int64_t n_own, int64_t n_ghost, int n_nbr,
                     const int32_t* nbr_rank, const int64_t* recv_counts,
                     const int64_t* send_counts, const int64_t* send_idx, pamg_plan** out) {
    if (!ctx || !out || n_own < 0 || n_ghost < 0 || n_nbr < 0)
        return fail(PAMG_E_ARG, "plan_create: bad args");
    if (n_nbr > 0 && (!nbr_rank || !recv_counts || !send_counts))
        return fail(PAMG_E_ARG, "plan_create: neighbour arrays missing");
    if (n_own >= INT32_MAX || n_own + n_ghost >= INT32_MAX)
        return fail(PAMG_E_OVERFLOW, "plan_create: sizes exceed int32");
    CHECK(set_device(ctx));
    // released through pamg_plan_destroy on every error path
    std::unique_ptr<pamg_plan, int (*)(pamg_plan*)> p(new pamg_plan, pamg_plan_destroy);
    p->ctx = ctx;
    ctx_ref(ctx);
    p->n_own = n_own;
    p->n_ghost = n_ghost;
    p->nbr.assign(nbr_rank, nbr_rank + n_nbr);
    p->recv_off.assign(n_nbr + 1, 0);
    p->send_off.assign(n_nbr + 1, 0);
    for (int k = 0; k < n_nbr; ++k) {
        // a part may be its own neighbour (ghost copies of own entries, e.g. a periodic wrap
        // on one part): RCCL serves that as a send/recv to self; the host transport does not
        if (nbr_rank[k] < 0 || nbr_rank[k] >= ctx->nranks || (nbr_rank[k] == ctx->rank && ctx->host_fn))
            return fail(PAMG_E_ARG, "plan_create: bad neighbour rank %d", nbr_rank[k]);
        p->recv_off[k + 1] = p->recv_off[k] + recv_counts[k];
        p->send_off[k + 1] = p->send_off[k] + send_counts[k];
    }
    if (p->recv_off[n_nbr] != n_ghost)
        return fail(PAMG_E_ARG, "plan_create: recv counts sum %lld != n_ghost %lld",
                    (long long)p->recv_off[n_nbr], (long long)n_ghost);
    const int64_t ns = p->send_off[n_nbr];
    std::vector<int> idx(ns);
    for (int64_t k = 0; k < ns; ++k) {
        if (send_idx[k] < 0 || send_idx[k] >= n_own)
            return fail(PAMG_E_ARG, "plan_create: send index %lld out of range", (long long)send_idx[k]);
        idx[k] = (int)send_idx[k];
    }
    p->send_run.assign(n_nbr, -1);
    p->all_contig = true;
    for (int k = 0; k < n_nbr; ++k) {
        const int64_t a = p->send_off[k], e = p->send_off[k + 1];
        bool run = e > a;
        for (int64_t j = a + 1; run && j < e; ++j) run = idx[j] == idx[j - 1] + 1;
        if (run) p->send_run[k] = idx[a];
        else if (e > a) p->all_contig = false;
    }
    CHECK(dalloc(&p->d_send_idx, ns));
    CHECK(dalloc(&p->d_sendbuf, ns));
    if (ns) HIPC(hipMemcpy(p->d_send_idx, idx.data(), sizeof(int) * ns, hipMemcpyHostToDevice));
    *out = p.release();
    return PAMG_OK;
}

int pamg_plan_set_tag(pamg_plan* p, int64_t tag) {
    if (!p) return fail(PAMG_E_ARG, "plan_set_tag: NULL");
    p->tag = tag;
    return PAMG_OK;
}

int pamg_plan_destroy(pamg_plan* p) {
    if (!p) return PAMG_OK;
    (void)hipSetDevice(p->ctx->device);
    if (p->in_flight) (void)hipStreamSynchronize(p->ctx->s_comm);
    if (p->ev_done) (void)hipEventDestroy(p->ev_done);
    dfree(p->d_send_idx);
    dfree(p->d_sendbuf);
    pamg_ctx* owner = p->ctx;
    delete p;
    ctx_unref(owner);
    return PAMG_OK;
}

int pamg_vec_create(pamg_ctx* ctx, int64_t n_own, int64_t n_ghost, pamg_vec** out) {
    if (!ctx || !out || n_own < 0 || n_ghost < 0) return fail(PAMG_E_ARG, "vec_create: bad args");
    CHECK(set_device(ctx));
    std::unique_ptr<pamg_vec, int (*)(pamg_vec*)> v(new pamg_vec, pamg_vec_destroy);
    v->ctx = ctx;
    ctx_ref(ctx);
    v->n_own = n_own;
    v->n_ghost = n_ghost;
    CHECK(dalloc(&v->d, n_own + n_ghost + kVecPad));
    HIPC(hipMemsetAsync(v->d, 0, sizeof(double) * (n_own + n_ghost + kVecPad), ctx->s_comp));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    *out = v.release();
    return PAMG_OK;
}

int pamg_vec_destroy(pamg_vec* v) {
    if (!v) return PAMG_OK;
    (void)hipSetDevice(v->ctx->device);
    (void)hipStreamSynchronize(v->ctx->s_comp);
    dfree(v->d);
    pamg_ctx* owner = v->ctx;
    delete v;
    ctx_unref(owner);
    return PAMG_OK;
}

int pamg_vec_size(const pamg_vec* v, int64_t* n_own, int64_t* n_ghost) {
    if (!v) return fail(PAMG_E_ARG, "vec_size: NULL");
    if (n_own) *n_own = v->n_own;
    if (n_ghost) *n_ghost = v->n_ghost;
    return PAMG_OK;
}

int pamg_vec_upload(pamg_ctx* ctx, pamg_vec* v, const double* own) {
    if (!ctx || !v || (!own && v->n_own)) return fail(PAMG_E_ARG, "vec_upload: bad args");
    CHECK(set_device(ctx));
    if (v->n_own) HIPC(hipMemcpyAsync(v->d, own, sizeof(double) * v->n_own, hipMemcpyHostToDevice, ctx->s_comp));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_vec_download(pamg_ctx* ctx, const pamg_vec* v, double* own) {
    if (!ctx || !v || (!own && v->n_own)) return fail(PAMG_E_ARG, "vec_download: bad args");
    CHECK(set_device(ctx));
    if (v->n_own) HIPC(hipMemcpyAsync(own, v->d, sizeof(double) * v->n_own, hipMemcpyDeviceToHost, ctx->s_comp));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_vec_download_ghosts(pamg_ctx* ctx, const pamg_vec* v, double* ghost) {
    if (!ctx || !v || (!ghost && v->n_ghost)) return fail(PAMG_E_ARG, "vec_download_ghosts: bad args");
    CHECK(set_device(ctx));
    if (v->n_ghost)
        HIPC(hipMemcpyAsync(ghost, v->d + v->n_own, sizeof(double) * v->n_ghost, hipMemcpyDeviceToHost,
                            ctx->s_comp));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_vec_device_ptr(pamg_vec* v, double** dptr) {
    if (!v || !dptr) return fail(PAMG_E_ARG, "vec_device_ptr: bad args");
    *dptr = v->d;
    return PAMG_OK;
}

int pamg_vec_fill(pamg_ctx* ctx, pamg_vec* v, double value) {
    if (!ctx || !v) return fail(PAMG_E_ARG, "vec_fill: bad args");
    CHECK(set_device(ctx));
    pamg::launch_fill(v->n_own, value, v->d, ctx->s_comp);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_vec_copy(pamg_ctx* ctx, const pamg_vec* src, pamg_vec* dst) {
    if (!ctx || !src || !dst || src->n_own != dst->n_own) return fail(PAMG_E_ARG, "vec_copy: shape mismatch");
    CHECK(set_device(ctx));
    if (src->n_own)
        HIPC(hipMemcpyAsync(dst->d, src->d, sizeof(double) * src->n_own, hipMemcpyDeviceToDevice, ctx->s_comp));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_vec_axpby(pamg_ctx* ctx, double a, const pamg_vec* x, double b, pamg_vec* y) {
    if (!ctx || !x || !y || x->n_own != y->n_own) return fail(PAMG_E_ARG, "vec_axpby: shape mismatch");
    CHECK(set_device(ctx));
    pamg::launch_axpby(x->n_own, a, x->d, b, y->d, ctx->s_comp);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_vec_dot(pamg_ctx* ctx, const pamg_vec* x, const pamg_vec* y, double* out) {
    if (!ctx || !x || !y || !out || x->n_own != y->n_own) return fail(PAMG_E_ARG, "vec_dot: shape mismatch");
    CHECK(set_device(ctx));
    return reduce_scalar(ctx, x->n_own, x->d, y->d, out);
}

int pamg_vec_nrm2(pamg_ctx* ctx, const pamg_vec* x, double* out) {
    if (!ctx || !x || !out) return fail(PAMG_E_ARG, "vec_nrm2: bad args");
    CHECK(set_device(ctx));
    double s = 0.0;
    CHECK(reduce_scalar(ctx, x->n_own, x->d, x->d, &s));
    *out = std::sqrt(s);
    return PAMG_OK;
}

int pamg_exchange(pamg_ctx* ctx, const pamg_plan* plan, pamg_vec* x) {
    if (!ctx || !plan || !x) return fail(PAMG_E_ARG, "exchange: bad args");
    if (x->n_own != plan->n_own || x->n_ghost < plan->n_ghost)
        return fail(PAMG_E_ARG, "exchange: vector does not fit the plan");
    CHECK(set_device(ctx));
    CHECK(exchange_on(plan, x->d, ctx->s_comp));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

// consistent!(x) split in two (PartitionedArrays returns a task to wait on): begin forks the
// exchange onto the comm stream behind everything already enqueued on the compute stream and
// returns; end joins it back (later compute-stream work sees the ghosts) and waits for it.
// Between the two the caller may run anything that does not touch x's ghost slots or write
// its send entries. The host debug transport has nothing to overlap: begin does it all.
int pamg_exchange_begin(pamg_ctx* ctx, pamg_plan* plan, pamg_vec* x) {
    if (!ctx || !plan || !x) return fail(PAMG_E_ARG, "exchange_begin: bad args");
    if (x->n_own != plan->n_own || x->n_ghost < plan->n_ghost)
        return fail(PAMG_E_ARG, "exchange_begin: vector does not fit the plan");
    if (plan->in_flight) return fail(PAMG_E_STATE, "exchange_begin: the plan has an exchange in flight");
    CHECK(set_device(ctx));
    if (sync_transport(ctx)) {
        CHECK(exchange_on(plan, x->d, ctx->s_comp));
        plan->in_flight = x;
        return PAMG_OK;
    }
    if (!plan->ev_done) HIPC(hipEventCreateWithFlags(&plan->ev_done, hipEventDisableTiming));
    HIPC(hipEventRecord(ctx->ev_fork, ctx->s_comp));
    HIPC(hipStreamWaitEvent(ctx->s_comm, ctx->ev_fork, 0));
    CHECK(exchange_on(plan, x->d, ctx->s_comm));
    HIPC(hipEventRecord(plan->ev_done, ctx->s_comm));
    plan->in_flight = x;
    return PAMG_OK;
}

int pamg_exchange_end(pamg_ctx* ctx, pamg_plan* plan, pamg_vec* x) {
    if (!ctx || !plan || !x) return fail(PAMG_E_ARG, "exchange_end: bad args");
    if (plan->in_flight != x) return fail(PAMG_E_STATE, "exchange_end: no exchange of this vector in flight");
    CHECK(set_device(ctx));
    plan->in_flight = nullptr;
    if (!sync_transport(ctx)) {
        HIPC(hipStreamWaitEvent(ctx->s_comp, plan->ev_done, 0));
        HIPC(hipEventSynchronize(plan->ev_done));
    }
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_mat_upload(pamg_ctx* ctx, int64_t nrows, int64_t ncols, const int64_t* rowptr,
                    const void* col, int col_is_64, const double* val, int index_base,
                    const pamg_plan* plan, pamg_mat** out) {
    if (!ctx || !out || nrows < 0 || ncols < 0 || !rowptr || (index_base != 0 && index_base != 1))
        return fail(PAMG_E_ARG, "mat_upload: bad args");
    const int64_t nnz = rowptr[nrows] - index_base;
    if (nnz < 0 || (nnz > 0 && (!col || !val))) return fail(PAMG_E_ARG, "mat_upload: bad arrays");
    if (nnz >= INT32_MAX - 16 || nrows >= INT32_MAX || ncols >= INT32_MAX)
        return fail(PAMG_E_OVERFLOW, "mat_upload: nnz/rows/cols exceed the int32 device layout");
    const int64_t n_own_cols = plan ? plan->n_own : ncols;
    if (plan && plan->n_own + plan->n_ghost != ncols)
        return fail(PAMG_E_ARG, "mat_upload: ncols %lld != plan own+ghost %lld", (long long)ncols,
                    (long long)(plan->n_own + plan->n_ghost));
    CHECK(set_device(ctx));
    UploadTrace tr;
    tr.nnz = nnz;
    PtrVec rp(nrows + 1);
    IdxVec ci(nnz + kVecPad);
    {
        std::atomic<int64_t> bad_row{INT64_MAX};
        par_for(nrows + 1, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) {
                rp[i] = rowptr[i] - index_base;
                if (i > 0 && rowptr[i] < rowptr[i - 1]) {
                    int64_t cur = bad_row.load();
                    while (i - 1 < cur && !bad_row.compare_exchange_weak(cur, i - 1)) {
                    }
                }
            }
        });
        if (bad_row.load() != INT64_MAX)
            return fail(PAMG_E_ARG, "mat_upload: rowptr not monotone at %lld", (long long)bad_row.load());
    }
    if (rp[0] != 0) return fail(PAMG_E_ARG, "mat_upload: rowptr[0] != index_base");
    for (int k = 0; k < kVecPad; ++k) ci[nnz + k] = 0;
    {
        std::atomic<int64_t> bad_at{INT64_MAX};
        par_for(nnz, [&](int64_t a, int64_t b) {
            for (int64_t k = a; k < b; ++k) {
                const int64_t c = (col_is_64 ? static_cast<const int64_t*>(col)[k]
                                             : (int64_t) static_cast<const int32_t*>(col)[k]) - index_base;
                if (c < 0 || c >= ncols) {
                    int64_t cur = bad_at.load();
                    while (k < cur && !bad_at.compare_exchange_weak(cur, k)) {
                    }
                    return;
                }
                ci[k] = (int)c;
            }
        });
        if (bad_at.load() != INT64_MAX) {
            const int64_t k = bad_at.load();
            const int64_t c = (col_is_64 ? static_cast<const int64_t*>(col)[k]
                                         : (int64_t) static_cast<const int32_t*>(col)[k]) - index_base;
            return fail(PAMG_E_ARG, "mat_upload: column %lld out of range", (long long)c);
        }
    }
    tr.mark("columns");
    // released through pamg_mat_destroy on every error path (no device memory leaks)
    std::unique_ptr<pamg_mat, int (*)(pamg_mat*)> A(new pamg_mat, pamg_mat_destroy);
    A->ctx = ctx;
    ctx_ref(ctx);  // (before the first failure point: the deleter drops it)
    A->nrows = nrows;
    A->ncols = ncols;
    A->nnz = nnz;
    A->plan = plan;
    // classify rows: interior (own columns only) or boundary (>= 1 ghost column), and find
    // the diagonal (threads over row ranges)
    std::vector<int> inner, bnd;
    std::vector<double> diag(n_own_cols == nrows ? nrows : 0, 0.0);  // (square operators only)
    std::vector<char> ghost_row(nrows, 0);
    std::atomic<bool> has_all_diag{n_own_cols == nrows};
    // (no ghost columns and no diagonal to find — a one-part prolongation or restriction: nothing
    // to scan)
    const bool scan = n_own_cols == nrows || ncols != n_own_cols;
    if (scan) par_for(nrows, [&](int64_t a, int64_t b) {
        bool all = true;
        for (int64_t i = a; i < b; ++i) {
            bool g = false, d = false;
            for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
                const int c = ci[k];
                g |= c >= n_own_cols;
                if (c == i && n_own_cols == nrows) {
                    diag[i] = val[k];
                    d = true;
                }
            }
            if (!d || diag[i] == 0.0) all = false;
            ghost_row[i] = g;
        }
        if (!all) has_all_diag = false;
    });
    std::atomic<int64_t> n_ghost_rows{0};
    par_for(nrows, [&](int64_t a, int64_t b) {
        int64_t c = 0;
        for (int64_t i = a; i < b; ++i) c += ghost_row[i];
        n_ghost_rows += c;
    });
    if (n_ghost_rows.load() == 0) {  // (one part: every row interior, listed in parallel)
        inner.resize(nrows);
        par_for(nrows, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) inner[i] = (int)i;
        });
    } else {
        for (int64_t i = 0; i < nrows; ++i) (ghost_row[i] ? bnd : inner).push_back((int)i);
    }
    std::vector<char>().swap(ghost_row);
    tr.mark("classify");
    // The row distance at which rows share x entries, for the banded tile order: per own
    // column the largest gap between consecutive rows that read it (one grid plane for a
    // stencil, one aggregate layer for a restriction); band = its 90th percentile over the
    // columns. (Sequential: the gaps depend on the row order.) Computed when a layout that
    // uses it is tried (the symmetric layout, tiles): not for rows that all go to ELL / pnc.
    int64_t band = -1;
    auto get_band = [&]() -> int64_t {
        if (band >= 0) return band;
        band = 0;
        std::vector<int> max_gap = column_reuse_gaps(rp, ci, nrows, n_own_cols);
        auto end = std::remove(max_gap.begin(), max_gap.end(), 0);
        const size_t m = (size_t)(end - max_gap.begin());
        if (m > 0) {
            auto q = max_gap.begin() + (ptrdiff_t)((m * 9) / 10);
            std::nth_element(max_gap.begin(), q, end);
            band = *q;
            // restriction-shaped operators (fewer rows than columns: R0 reads the fine vector
            // through 5x5x5 root neighbourhoods) walk half-layer bands: each XCD's window
            // of fine lines between reuses halves (512^3 R0 -3 % in kbench,
            // profiles/r02_exp/kbench512_band_pct_r0_p0.jsonl; in the bench R0 -1 %, R1 -2.5 %,
            // the cycle within noise: bench_band_pct_restrict_ab/)
            const int pct = nrows < n_own_cols ? pamg::options().band_pct_restrict : pamg::options().band_pct;
            if (pct != 100) band = std::max<int64_t>(1, band * pct / 100);
        }
        tr.mark("band");
        return band;
    };
    if (pamg::options().sym_dia && n_own_cols == nrows && has_all_diag && !inner.empty())
        CHECK(build_sym_dia(A.get(), rp, ci, val, inner, get_band));
    if (A->interior.sym) inner.clear();  // the interior rows run in k_rows_sym, not in tiles
    tr.mark("sym dia");
    // square operators (offsets from the row) and restrictions (fewer rows than columns; offsets from
    // each row's first column)
    // (several parts: the interior rows, when they are >= 3/4 of the operator — a 512^3 z-slab part's level 1)
    // restrictions whose rows repeat few patterns (an aggregate shape each): pattern-dictionary rows
    if (pamg::options().rpat && !A->interior.sym && n_own_cols > nrows && nrows > 0 &&
        (int64_t)inner.size() * 4 >= (int64_t)nrows * 3) {
        CHECK(build_rpat(A.get(), rp, ci, val, inner));
        if (A->interior.rpat) inner.clear();  // the rows run in k_rows_rpat, not in tiles
        tr.mark("rpat");
    }
    if (pamg::options().ell && !A->interior.sym && !A->interior.rpat && n_own_cols >= nrows && nrows > 0 &&
        (int64_t)inner.size() * 4 >= (int64_t)nrows * 3 && nrows >= pamg::options().ell_min_rows &&
        (n_own_cols == nrows || pamg::options().ell_restrict)) {
        CHECK(build_ell(A.get(), rp, ci, val, n_own_cols != nrows, inner));
        if (A->interior.ell) inner.clear();  // the rows run in k_rows_ell, not in tiles
        tr.mark("ell");
    }
    // a prolongation over a 7-point grid uploaded earlier on this context: neighbour-coded rows
    if (pamg::options().pnc && n_own_cols < nrows && (int64_t)inner.size() * 4 >= (int64_t)nrows * 3) {
        // (every registered grid of this row count, the latest first: grids of one size but other
        // shapes may be registered too, and the neighbour check decides)
        const auto grids = grids_of(ctx);
        for (auto g = grids.rbegin(); g != grids.rend() && !A->interior.pnc; ++g)
            if ((*g)[0] == nrows) CHECK(build_pnc(A.get(), rp, ci, val, *g, inner));
        if (A->interior.pnc) inner.clear();  // the rows run in k_rows_pnc, not in tiles
        tr.mark("pnc");
    }
    // the CSR copies: read by the tile and long-row kernels only, so not uploaded when every row
    // runs in the symmetric, ELL or neighbour-coded layout (the 512^3 A0, A1, R0, P0: 29 GB less)
    if (!inner.empty() || !bnd.empty()) {
        std::vector<int> rp32(nrows + 1);
        par_for(nrows + 1, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) rp32[i] = (int)rp[i];
        });
        CHECK(dalloc(&A->d_rowptr, nrows + 1));
        CHECK(dalloc(&A->d_col, nnz + kVecPad));
        CHECK(dalloc(&A->d_val, nnz + kVecPad));
        CHECK(h2d(ctx, A->d_rowptr, rp32.data(), sizeof(int) * (nrows + 1)));
        CHECK(h2d(ctx, A->d_col, ci.data(), sizeof(int) * (nnz + kVecPad)));
        CHECK(dzero(ctx, A->d_val, sizeof(double) * (nnz + kVecPad)));
        if (nnz) CHECK(h2d(ctx, A->d_val, val, sizeof(double) * nnz));
    }
    if (has_all_diag && nrows > 0) {
        CHECK(dalloc(&A->d_diag, nrows));
        CHECK(h2d(ctx, A->d_diag, diag.data(), sizeof(double) * nrows));
    }
    tr.mark("csr copies");
    std::vector<uint16_t> lo;
    std::vector<uint8_t> hi, vidx;
    {
        std::vector<int4> t_in, t_bd;
        const bool square = n_own_cols == nrows;
        const bool tall = n_own_cols < nrows;  // a prolongation's shape
        const int64_t tb = inner.empty() && bnd.empty() ? 0 : get_band();
        CHECK(build_tiles(rp, inner, square, &A->interior, tb, ci, &lo, &hi, val, &vidx, &t_in, tall));
        CHECK(build_tiles(rp, bnd, square, &A->boundary, tb, ci, &lo, &hi, val, &vidx, &t_bd, tall));
        tr.mark("tiles");
        std::vector<uint8_t> idx8;
        CHECK(build_col_dicts(A.get(), rp, ci, t_in, t_bd, &idx8));
        tr.mark("col dicts");
        CHECK(build_tile_major(A.get(), n_own_cols, rp, ci, val, t_in, t_bd, lo, hi, idx8));
        tr.mark("tile-major");
    }
    if (A->interior.rl8 || A->boundary.rl8) {
        std::vector<uint8_t> rl(nrows + kVecPad, 0);
        par_for(nrows, [&](int64_t a, int64_t b) {
            for (int64_t i = a; i < b; ++i) rl[i] = (uint8_t)std::min<int64_t>(255, rp[i + 1] - rp[i]);
        });
        CHECK(dalloc(&A->d_rlen, nrows + kVecPad));
        CHECK(h2d(ctx, A->d_rlen, rl.data(), rl.size()));
    }
    if (!vidx.empty()) {
        CHECK(dalloc(&A->d_vidx, (int64_t)vidx.size()));
        CHECK(h2d(ctx, A->d_vidx, vidx.data(), vidx.size()));
    }
    // the bytes one apply streams, per tile set: long rows (row pointer, 12 B/nonzero, list
    // entry) + short tiles in their layout — row bounds (1 B/row with 8-bit lengths, else 4-B
    // row pointers), columns (4 B; 3 B 24-bit; cd/8 B with a dictionary + its 4-B offsets),
    // values (8 B; or a 4-bit index + the tile's 128-B table), 16-B descriptors (+ a 4-B
    // column base with 24-bit columns); a tile-major set streams whole padded slots
    // (tile_nnz values and column entries, tm_rs row lengths per tile). + the closing pointer.
    A->stream_bytes = 4;
    // symmetric diagonal-class layout: 8/16-bit mask, diagonal and nu upper values per row (the
    // mirrored lower values are the same lines, re-read from cache)
    if (A->interior.sym)
        A->stream_bytes += A->sym.vd_n ? nrows + (int64_t)A->sym.vd_n * (8 * (A->sym.nu + 1) + 4)
                                       : nrows * (A->sym.mask_bytes + 8 + 8 * (int64_t)A->sym.nu);
    // sliced ELL: two index bytes per padded nonzero, a length byte per row, the slice and group
    // descriptors and the group tables
    if (A->interior.ell)
        A->stream_bytes += (A->ell.paired ? 4 : 8) * A->ell.words + nrows + 8 * A->ell.nslices + 16 * A->ell.ngroups + 4 * A->ell.otab_n +
                           8 * A->ell.vtab_n + (A->ell.d_anc ? 4 * nrows : 0);
    // neighbour-coded prolongation: the anchor and the record per row, the two tables
    if (A->interior.pnc)
        A->stream_bytes += (A->pnc.d_cid ? 6 : 12) * nrows + (A->pnc.d_cid ? 12 : 4) * A->pnc.npat + 8 * A->pnc.nval;
    // pattern-dictionary rows: the first column and the pattern id per row, the tables
    if (A->interior.rpat) A->stream_bytes += 5 * nrows + 8 * A->rpat.npat + 4 * A->rpat.nent + 8 * A->rpat.nval;
    for (const pamg::TileSet* t : {&A->interior, &A->boundary}) {
        if (t->sym || t->ell || t->pnc || t->rpat) continue;  // counted above
        const int64_t ns = t->n_short, nz = t->nnz_short;
        int64_t b = 8 * (int64_t)t->n_long + 12 * t->nnz_long;
        const bool base = t->c24 && !t->cd;
        if (t->tm) {  // whole padded slots: tile_nnz values + column entries + tm_rs lengths
            const int64_t tn = t->tile_nnz;
            const int64_t rowb = t->tm_rs;
            const int64_t valb = t->tm_vt ? tn + 8 * (int64_t)t->tm_vt : 8 * tn;  // 8-bit indices + table
            b += ns * (rowb * (t->anc ? 5 : 1) + valb + (t->cd ? t->cd * tn / 8 : 3 * tn) + 16 + (base ? 4 : 0)) +
                 (t->cd ? 4 * t->ctab_n * (t->pt ? ns : 1) : 0);
        } else {
            b += (t->rl8 ? 1 : 4) * t->rows_short;
            b += t->cd ? (t->cd * nz + 7) / 8 + 4 * t->ctab_n * (t->pt ? ns : 1) : (t->c24 ? 3 : 4) * nz;
            if (t->pt && t->anc) b += 2 * t->rows_short + 4 * ns;  // 16-bit anchors + tile bases
            b += t->vd ? nz / 2 + 128 * ns : 8 * nz;
            b += (16 + (base ? 4 : 0)) * ns;
        }
        A->stream_bytes += b;
    }
    if (!lo.empty()) {  // padded like d_col
        lo.resize(nnz + kVecPad, 0);
        hi.resize(nnz + kVecPad, 0);
        CHECK(dalloc(&A->d_clo, nnz + kVecPad));
        CHECK(dalloc(&A->d_chi, nnz + kVecPad));
        CHECK(h2d(ctx, A->d_clo, lo.data(), sizeof(uint16_t) * lo.size()));
        CHECK(h2d(ctx, A->d_chi, hi.data(), sizeof(uint8_t) * hi.size()));
    }
    tr.mark("rest");
    *out = A.release();
    return PAMG_OK;
}

// Locality permutation inside the device layout: device row i = caller row row_perm[i], own
// column c of the caller = device column inv(col_perm)[c] (ghost columns stay). Each row keeps
// its entries in the caller's storage order, so every row sum (SPEC §S3) keeps its bits; only
// the rows' places and the x entries they gather move.
static int check_perm(const int64_t* p, int64_t n, const char* what) {
    std::vector<char> seen(n, 0);
    for (int64_t i = 0; i < n; ++i) {
        if (p[i] < 0 || p[i] >= n || seen[p[i]])
            return fail(PAMG_E_ARG, "mat_upload_perm: %s is not a permutation of 0..%lld", what, (long long)(n - 1));
        seen[p[i]] = 1;
    }
    return PAMG_OK;
}

int pamg_mat_upload_perm(pamg_ctx* ctx, int64_t nrows, int64_t ncols, const int64_t* rowptr,
                         const void* col, int col_is_64, const double* val, int index_base,
                         const pamg_plan* plan, const int64_t* row_perm, const int64_t* col_perm,
                         pamg_mat** out) {
    if (!ctx || !out || nrows < 0 || ncols < 0 || !rowptr || (index_base != 0 && index_base != 1))
        return fail(PAMG_E_ARG, "mat_upload_perm: bad args");
    const int64_t nnz = rowptr[nrows] - index_base;
    if (nnz < 0 || rowptr[0] != index_base || (nnz > 0 && (!col || !val)))
        return fail(PAMG_E_ARG, "mat_upload_perm: bad arrays");
    if (nnz >= INT32_MAX - 16 || nrows >= INT32_MAX || ncols >= INT32_MAX)
        return fail(PAMG_E_OVERFLOW, "mat_upload_perm: nnz/rows/cols exceed the int32 device layout");
    const int64_t n_own_cols = plan ? plan->n_own : ncols;
    if (n_own_cols > ncols) return fail(PAMG_E_ARG, "mat_upload_perm: plan has more own columns than the matrix");
    if (row_perm) CHECK(check_perm(row_perm, nrows, "row_perm"));
    std::vector<int> cinv;
    if (col_perm) {
        CHECK(check_perm(col_perm, n_own_cols, "col_perm"));
        cinv.resize(n_own_cols);
        for (int64_t k = 0; k < n_own_cols; ++k) cinv[col_perm[k]] = (int)k;
    }
    std::vector<int64_t> rp(nrows + 1, 0);
    for (int64_t i = 0; i < nrows; ++i) {
        const int64_t r = row_perm ? row_perm[i] : i;
        const int64_t len = rowptr[r + 1] - rowptr[r];
        if (len < 0) return fail(PAMG_E_ARG, "mat_upload_perm: rowptr not monotone at %lld", (long long)r);
        rp[i + 1] = rp[i] + len;
    }
    std::vector<int> ci(nnz);
    std::vector<double> va(nnz);
    std::atomic<bool> bad{false};
    par_for(nrows, [&](int64_t a, int64_t b) {
        for (int64_t i = a; i < b; ++i) {
            const int64_t r = row_perm ? row_perm[i] : i;
            const int64_t s = rowptr[r] - index_base;
            for (int64_t k = 0; k < rp[i + 1] - rp[i]; ++k) {
                const int64_t c = (col_is_64 ? static_cast<const int64_t*>(col)[s + k]
                                             : (int64_t) static_cast<const int32_t*>(col)[s + k]) - index_base;
                if (c < 0 || c >= ncols) {
                    bad = true;
                    return;
                }
                ci[rp[i] + k] = (c < n_own_cols && col_perm) ? cinv[c] : (int)c;
                va[rp[i] + k] = val[s + k];
            }
        }
    });
    if (bad) return fail(PAMG_E_ARG, "mat_upload_perm: column out of range");
    return pamg_mat_upload(ctx, nrows, ncols, rp.data(), ci.data(), 0, va.data(), 0, plan, out);
}

int pamg_mat_destroy(pamg_mat* A) {
    if (!A) return PAMG_OK;
    (void)hipSetDevice(A->ctx->device);
    (void)hipStreamSynchronize(A->ctx->s_comp);
    dfree(A->d_rowptr);
    dfree(A->d_col);
    dfree(A->d_clo);
    dfree(A->d_rlen);
    dfree(A->d_chi);
    dfree(A->d_vidx);
    dfree(A->d_cidx);
    dfree(A->d_anc16);
    dfree(A->d_val);
    dfree(A->d_diag);
    dfree(A->sym.d_mask);
    dfree(A->sym.d_diag);
    dfree(A->sym.d_upper);
    dfree(A->sym.d_tid);
    dfree(A->sym.d_vtab);
    dfree(A->sym.d_mtab);
    free_tiles(A->interior);
    free_tiles(A->boundary);
    free_ell(A->ell);
    free_pnc(A->pnc);
    free_rpat(A->rpat);
    pamg_ctx* owner = A->ctx;
    delete A;
    ctx_unref(owner);
    return PAMG_OK;
}

int pamg_mat_info(const pamg_mat* A, int64_t* nrows, int64_t* ncols, int64_t* nnz) {
    if (!A) return fail(PAMG_E_ARG, "mat_info: NULL");
    if (nrows) *nrows = A->nrows;
    if (ncols) *ncols = A->ncols;
    if (nnz) *nnz = A->nnz;
    return PAMG_OK;
}

int pamg_mat_stream_bytes(const pamg_mat* A, int64_t* bytes) {
    if (!A || !bytes) return fail(PAMG_E_ARG, "mat_stream_bytes: bad args");
    *bytes = A->stream_bytes;
    return PAMG_OK;
}

int pamg_mat_layout(const pamg_mat* A, int set, int out[10]) {
    if (!A || !out || set < 0 || set > 1) return fail(PAMG_E_ARG, "mat_layout: bad args");
    const pamg::TileSet& t = set == 0 ? A->interior : A->boundary;
    out[0] = t.c24;
    out[1] = t.vd;
    out[2] = t.rl8;
    out[3] = t.cd;
    out[4] = t.ctab_n;
    out[5] = t.tm;
    out[6] = t.tm_rs;
    out[7] = t.tile_nnz;
    out[8] = t.n_short;
    out[9] = (t.anc ? 1 : 0) | (t.pt ? 2 : 0) | (t.xs ? 4 : 0) | (t.sym ? 8 : 0) | (t.sym && A->sym.rpl == 2 ? 16 : 0) |
             (t.sym && (A->sym.tb_ok || A->sym.tb_part) ? 32 : 0) | (t.tm && t.tm_vt ? 64 : 0) |
             (t.sym && A->sym.vd_n ? 128 : 0) | (t.ell ? 512 : 0) | (t.pnc ? 1024 : 0) | (t.rpat ? 2048 : 0) |
             (t.pnc && A->pnc.d_cid ? 4096 : 0) | (t.ell && A->ell.paired ? 8192 : 0);
    if (t.ell) out[8] = (int)A->ell.ngroups;  // k_rows_ell's grid
    if (t.rpat) {  // the pattern and value tables, k_rows_rpat's grid
        out[3] = A->rpat.nval;
        out[4] = A->rpat.npat;
        out[8] = (int)A->rpat.ngroups;
    }
    if (t.pnc) {  // the pattern and value tables, k_rows_pnc's grid
        out[3] = A->pnc.nval;
        out[4] = A->pnc.npat;
        out[8] = A->pnc.grid;
    }
    if (t.sym) {  // the symmetric diagonal-class layout: upper classes, k_rows_sym's grid
        out[4] = A->sym.nu;
        out[8] = A->sym.nbands * 8 * A->sym.eighth;
    }
    return PAMG_OK;
}

static int check_vec_for(const pamg_mat* A, const pamg_vec* x, const char* who) {
    const int64_t need_ghost = A->plan ? A->plan->n_ghost : 0;
    const int64_t own = A->plan ? A->plan->n_own : A->ncols;
    if (x->n_own != own || x->n_ghost < need_ghost)
        return fail(PAMG_E_ARG, "%s: input vector (%lld own, %lld ghost) does not fit the matrix columns (%lld own, %lld ghost)",
                    who, (long long)x->n_own, (long long)x->n_ghost, (long long)own, (long long)need_ghost);
    return PAMG_OK;
}

int pamg_spmv(pamg_ctx* ctx, const pamg_mat* A, pamg_vec* x, pamg_vec* y) {
    if (!ctx || !A || !x || !y) return fail(PAMG_E_ARG, "spmv: NULL");
    CHECK(check_vec_for(A, x, "spmv"));
    if (y->n_own != A->nrows) return fail(PAMG_E_ARG, "spmv: output size mismatch");
    if (x == y) return fail(PAMG_E_ARG, "spmv: x and y must differ");
    CHECK(set_device(ctx));
    CHECK(apply(ctx, A, pamg::OP_SPMV, x->d, nullptr, y->d, 0.0));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_residual(pamg_ctx* ctx, const pamg_mat* A, pamg_vec* x, const pamg_vec* b, pamg_vec* r,
                  double* nrm2) {
    if (!ctx || !A || !x || !b || !r) return fail(PAMG_E_ARG, "residual: NULL");
    CHECK(check_vec_for(A, x, "residual"));
    if (b->n_own != A->nrows || r->n_own != A->nrows || r == x)
        return fail(PAMG_E_ARG, "residual: size mismatch or aliasing");
    CHECK(set_device(ctx));
    CHECK(apply(ctx, A, pamg::OP_RESID, x->d, b->d, r->d, 0.0));
    if (nrm2) {
        double s = 0.0;
        CHECK(reduce_scalar(ctx, r->n_own, r->d, r->d, &s));
        *nrm2 = std::sqrt(s);
    }
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_jacobi(pamg_ctx* ctx, const pamg_mat* A, pamg_vec* x, const pamg_vec* b, pamg_vec* tmp,
                double omega, int nsweeps) {
    if (!ctx || !A || !x || !b || !tmp || nsweeps < 0) return fail(PAMG_E_ARG, "jacobi: bad args");
    CHECK(check_vec_for(A, x, "jacobi"));
    CHECK(check_vec_for(A, tmp, "jacobi"));
    if (!A->d_diag) return fail(PAMG_E_SETUP, "jacobi: matrix is not square or lacks a nonzero diagonal");
    if (b->n_own != A->nrows || tmp == x) return fail(PAMG_E_ARG, "jacobi: size mismatch or aliasing");
    CHECK(set_device(ctx));
    double* cur = x->d;
    double* nxt = tmp->d;
    for (int k = 0; k < nsweeps; ++k) {
        CHECK(apply(ctx, A, pamg::OP_JACOBI, cur, b->d, nxt, omega));
        std::swap(cur, nxt);
    }
    if (cur != x->d)
        HIPC(hipMemcpyAsync(x->d, cur, sizeof(double) * x->n_own, hipMemcpyDeviceToDevice, ctx->s_comp));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_jacobi_residual(pamg_ctx* ctx, const pamg_mat* A, pamg_vec* x, const pamg_vec* b, pamg_vec* t,
                         pamg_vec* r, double omega, int* fused) {
    if (!ctx || !A || !x || !b || !t || !r) return fail(PAMG_E_ARG, "jacobi_residual: NULL");
    CHECK(check_vec_for(A, x, "jacobi_residual"));
    CHECK(check_vec_for(A, t, "jacobi_residual"));
    if (!A->d_diag) return fail(PAMG_E_SETUP, "jacobi_residual: matrix is not square or lacks a nonzero diagonal");
    if (b->n_own != A->nrows || r->n_own != A->nrows || t == x || r == x || r == t || b == t || b == r)
        return fail(PAMG_E_ARG, "jacobi_residual: size mismatch or aliasing");
    CHECK(set_device(ctx));
    const bool fuse = pamg::options().jr_fuse && A->interior.sym && A->sym.tb_ok && !(A->plan && !A->plan->nbr.empty());
    const bool fuse_part = !fuse && pamg::options().jr_fuse && A->interior.sym && A->sym.tb_part;
    if (fuse_part) {
        CHECK(jr_part(ctx, A, x->d, b->d, t->d, r->d, omega));
    } else if (fuse) {
        pamg::TbArgs ta;
        ta.nstages = 2;
        ta.last_resid = true;
        ta.in0 = x->d;
        ta.out[0] = t->d;
        ta.out[1] = r->d;
        ta.b = b->d;
        ta.omega = omega;
        pamg::launch_sym_tb(*A, ta, ctx->s_comp);
        HIPC(hipGetLastError());
    } else {
        CHECK(apply(ctx, A, pamg::OP_JACOBI, x->d, b->d, t->d, omega));
        CHECK(apply(ctx, A, pamg::OP_RESID, t->d, b->d, r->d, 0.0));
    }
    if (fused) *fused = (fuse || fuse_part) ? 1 : 0;
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

int pamg_hier_create(pamg_ctx* ctx, int nlevels, pamg_mat* const* A, pamg_mat* const* P,
                     pamg_mat* const* R, const double* omega, int64_t n_coarse,
                     const double* ainv, int rep_level, const int64_t* rep_offsets,
                     pamg_hier** out) {
    if (!ctx || !out || nlevels < 1 || !A || !omega || !ainv || n_coarse < 1)
        return fail(PAMG_E_ARG, "hier_create: bad args");
    if (nlevels > 1 && (!P || !R)) return fail(PAMG_E_ARG, "hier_create: P/R missing");
    for (int l = 0; l < nlevels; ++l) {  // (before anything below dereferences them)
        if (!A[l]) return fail(PAMG_E_ARG, "hier_create: A[%d] is NULL", l);
        if (l < nlevels - 1 && (!P[l] || !R[l])) return fail(PAMG_E_ARG, "hier_create: P/R[%d] is NULL", l);
    }
    const int L = nlevels, nr = ctx->nranks, me = ctx->rank;
    if (nr == 1 || L == 1) rep_level = L - 1;
    if (rep_level < (L > 1 ? 1 : 0) || rep_level > L - 1)
        return fail(PAMG_E_ARG, "hier_create: rep_level %d outside [1, %d]", rep_level, L - 1);
    if (nr > 1 && !rep_offsets)
        return fail(PAMG_E_ARG, "hier_create: rep_offsets required with %d ranks", nr);
    CHECK(set_device(ctx));
    std::unique_ptr<pamg_hier, int (*)(pamg_hier*)> H(new pamg_hier, pamg_hier_destroy);
    H->ctx = ctx;
    ctx_ref(ctx);  // (before the first failure point: the deleter drops it)
    H->L = nlevels;
    H->rep = rep_level;
    // graph replay on one part and on RCCL multi-part runs (RCCL captures its p2p and
    // collectives); never with the host debug transport (host callbacks)
    H->use_graph = nr == 1 || (ctx->comm != nullptr && !ctx->host_fn);
    H->coffs.assign(nr + 1, 0);
    if (rep_offsets) {
        for (int q = 0; q <= nr; ++q) H->coffs[q] = rep_offsets[q];
    } else {
        H->coffs[1] = A[rep_level]->nrows;
    }
    for (int q = 0; q < nr; ++q) {
        if (H->coffs[q + 1] < H->coffs[q]) return fail(PAMG_E_ARG, "hier_create: rep_offsets not monotone");
        H->cmax = std::max(H->cmax, H->coffs[q + 1] - H->coffs[q]);
    }
    const int64_t n_rep = H->coffs[nr], rep_own = H->coffs[me + 1] - H->coffs[me];
    H->A.assign(A, A + L);
    H->P.assign(L, nullptr);
    H->R.assign(L, nullptr);
    H->omega.assign(omega, omega + L);
    H->x.assign(L, nullptr);
    H->b.assign(L, nullptr);
    H->t.assign(L, nullptr);
    H->r.assign(L, nullptr);
    H->nown.assign(L, 0);
    for (int l = 0; l < L; ++l) {
        if (!A[l]) return fail(PAMG_E_ARG, "hier_create: A[%d] is NULL", l);
        // levels >= rep are whole on every rank (the coarsest may be passed distributed: only
        // its inverse is used)
        H->nown[l] = (l == rep_level && L > 1) ? n_rep : A[l]->nrows;
    }
    if (L > 1 && nr > 1 && rep_level < L - 1 && A[rep_level]->nrows != n_rep)
        return fail(PAMG_E_ARG, "hier_create: A[%d] must be whole (%lld rows) on every rank",
                    rep_level, (long long)n_rep);
    for (int l = 0; l < L - 1; ++l) {
        if (!P[l] || !R[l]) return fail(PAMG_E_ARG, "hier_create: P/R[%d] is NULL", l);
        H->P[l] = P[l];
        H->R[l] = R[l];
        if (!A[l]->d_diag && A[l]->nrows > 0)  // (a part may own no row of a coarse level)
            return fail(PAMG_E_SETUP, "hier_create: A[%d] lacks a nonzero diagonal", l);
        const int64_t r_rows = (l + 1 == rep_level) ? rep_own : H->nown[l + 1];
        if (P[l]->nrows != A[l]->nrows || R[l]->nrows != r_rows)
            return fail(PAMG_E_ARG, "hier_create: level %d operator shapes inconsistent", l);
        if (l + 1 >= rep_level && (P[l]->plan || P[l]->ncols != H->nown[l + 1]))
            return fail(PAMG_E_ARG, "hier_create: P[%d] must read the whole level-%d vector (no plan, %lld columns)",
                        l, l + 1, (long long)H->nown[l + 1]);
    }
    // ghost capacity of each level's vectors = max over the plans that read them
    for (int l = 0; l < L; ++l) {
        int64_t g = 0;
        if (A[l]->plan) g = std::max(g, A[l]->plan->n_ghost);
        if (l < L - 1 && R[l]->plan) g = std::max(g, R[l]->plan->n_ghost);
        if (l > 0 && P[l - 1]->plan) g = std::max(g, P[l - 1]->plan->n_ghost);
        const int64_t n = H->nown[l] + g + kVecPad;
        if (l > 0) {
            CHECK(dalloc(&H->x[l], n));
            CHECK(dalloc(&H->b[l], n));
            CHECK(dzero(ctx, H->x[l], sizeof(double) * n));
            CHECK(dzero(ctx, H->b[l], sizeof(double) * n));
        }
        if (l < L - 1) {
            CHECK(dalloc(&H->t[l], n));
            CHECK(dalloc(&H->r[l], n));
            CHECK(dzero(ctx, H->t[l], sizeof(double) * n));
            CHECK(dzero(ctx, H->r[l], sizeof(double) * n));
        }
    }
    // coarsest level
    H->nc = n_coarse;
    if (H->nown[L - 1] != n_coarse && !(L == 1 && nr > 1))
        return fail(PAMG_E_ARG, "hier_create: coarsest level has %lld rows, n_coarse = %lld",
                    (long long)H->nown[L - 1], (long long)n_coarse);
    if (L == 1 && (n_rep != n_coarse || rep_own != A[0]->nrows))
        return fail(PAMG_E_ARG, "hier_create: rep_offsets inconsistent with the one-level hierarchy");
    {
        // row-major on the device: one wave reads a row of A^-1 coalesced (k_dense_gemv)
        std::vector<double> rm((size_t)n_coarse * n_coarse);
        for (int64_t j = 0; j < n_coarse; ++j)
            for (int64_t i = 0; i < n_coarse; ++i) rm[(size_t)i * n_coarse + j] = ainv[(size_t)j * n_coarse + i];
        CHECK(dalloc(&H->d_ainv, n_coarse * n_coarse));
        HIPC(hipMemcpy(H->d_ainv, rm.data(), sizeof(double) * rm.size(), hipMemcpyHostToDevice));
    }
    if (nr > 1) {
        CHECK(dalloc(&H->d_bgather, (int64_t)nr * H->cmax + n_rep + kVecPad));
        CHECK(dalloc(&H->d_bsend, H->cmax + kVecPad));
        CHECK(dzero(ctx, H->d_bsend, sizeof(double) * (H->cmax + kVecPad)));
    }
    H->prof_ms.assign((size_t)L * 6, 0.0);
    *out = H.release();
    return PAMG_OK;
}

static void drop_cycle_graph(pamg_hier* H) {
    if (H->gexec) (void)hipGraphExecDestroy(H->gexec);
    H->gexec = nullptr;
    H->g_x = H->g_b = nullptr;
}

static void drop_pipe_graphs(pamg_hier* H) {
    for (hipGraphExec_t* g : {&H->g_head, &H->g_steady[0], &H->g_steady[1], &H->g_tail[0], &H->g_tail[1]}) {
        if (*g) (void)hipGraphExecDestroy(*g);
        *g = nullptr;
    }
    H->gp_x = H->gp_b = nullptr;
}

static void drop_graph(pamg_hier* H) {
    drop_cycle_graph(H);
    drop_pipe_graphs(H);
}

int pamg_hier_destroy(pamg_hier* H) {
    if (!H) return PAMG_OK;
    (void)hipSetDevice(H->ctx->device);
    (void)hipStreamSynchronize(H->ctx->s_comp);
    drop_graph(H);
    for (size_t l = 0; l < H->t.size(); ++l) {
        if (l > 0) {
            dfree(H->x[l]);
            dfree(H->b[l]);
        }
        dfree(H->t[l]);
        dfree(H->r[l]);
    }
    dfree(H->d_ainv);
    dfree(H->d_bgather);
    dfree(H->d_bsend);
    dfree(H->pcg_r);
    dfree(H->pcg_z);
    dfree(H->pcg_p);
    dfree(H->pcg_q);
    dfree(H->u0);
    dfree(H->d_perm);
    dfree(H->px);
    dfree(H->pb);
    for (auto e : H->ev) (void)hipEventDestroy(e);
    pamg_ctx* owner = H->ctx;
    delete H;
    ctx_unref(owner);
    return PAMG_OK;
}

int pamg_hier_set_graph(pamg_hier* H, int enable) {
    if (!H) return fail(PAMG_E_ARG, "hier_set_graph: NULL");
    if (enable && sync_transport(H->ctx))
        return fail(PAMG_E_STATE, "hier_set_graph: the host debug / in-process transports cannot be graph-captured");
    H->use_graph = enable != 0;
    if (!H->use_graph) drop_graph(H);
    return PAMG_OK;
}

int pamg_hier_set_sweeps(pamg_hier* H, int nu1, int nu2) {
    if (!H || nu1 < 1 || nu2 < 1 || nu1 > 64 || nu2 > 64)
        return fail(PAMG_E_ARG, "hier_set_sweeps: need 1 <= nu1, nu2 <= 64");
    if (H->nu1 != nu1 || H->nu2 != nu2) {
        (void)hipSetDevice(H->ctx->device);
        (void)hipStreamSynchronize(H->ctx->s_comp);
        drop_graph(H);  // the captured cycle has the old sweep counts
    }
    H->nu1 = nu1;
    H->nu2 = nu2;
    return PAMG_OK;
}

int pamg_hier_set_perm(pamg_hier* H, int64_t n, const int64_t* perm) {
    if (!H) return fail(PAMG_E_ARG, "hier_set_perm: NULL");
    pamg_ctx* ctx = H->ctx;
    CHECK(set_device(ctx));
    HIPC(hipStreamSynchronize(ctx->s_comp));
    dfree(H->d_perm);
    dfree(H->px);
    dfree(H->pb);
    if (!perm || n == 0) return PAMG_OK;
    if (ctx->nranks > 1) return fail(PAMG_E_STATE, "hier_set_perm: one part only (permute a partition's rows before setup)");
    const pamg_mat* A0 = H->A[0];
    if (n != H->nown[0] || n != A0->ncols)
        return fail(PAMG_E_ARG, "hier_set_perm: %lld entries for a %lld-row level 0", (long long)n, (long long)H->nown[0]);
    std::vector<int> p(n);
    std::vector<char> seen(n, 0);
    for (int64_t i = 0; i < n; ++i) {
        if (perm[i] < 0 || perm[i] >= n || seen[perm[i]]) return fail(PAMG_E_ARG, "hier_set_perm: not a permutation");
        seen[perm[i]] = 1;
        p[i] = (int)perm[i];
    }
    CHECK(dalloc(&H->d_perm, n));
    CHECK(dalloc(&H->px, n + kVecPad));
    CHECK(dalloc(&H->pb, n + kVecPad));
    HIPC(hipMemcpy(H->d_perm, p.data(), sizeof(int) * n, hipMemcpyHostToDevice));
    CHECK(dzero(H->ctx, H->px, sizeof(double) * (n + kVecPad)));
    CHECK(dzero(H->ctx, H->pb, sizeof(double) * (n + kVecPad)));
    return PAMG_OK;
}

int pamg_hier_graph_state(const pamg_hier* H, int* enabled, int* captured, int* failed) {
    if (!H) return fail(PAMG_E_ARG, "hier_graph_state: NULL");
    if (enabled) *enabled = H->use_graph ? 1 : 0;
    if (captured) *captured = (H->gexec || H->g_head) ? 1 : 0;
    if (failed) *failed = H->graph_failed ? 1 : 0;
    return PAMG_OK;
}

int pamg_hier_profile(pamg_hier* H, int enable) {
    if (!H) return fail(PAMG_E_ARG, "hier_profile: NULL");
    H->prof = enable != 0;
    return PAMG_OK;
}

int pamg_hier_profile_read(pamg_hier* H, double* out) {
    if (!H || !out) return fail(PAMG_E_ARG, "hier_profile_read: bad args");
    CHECK(set_device(H->ctx));
    HIPC(hipStreamSynchronize(H->ctx->s_comp));
    for (size_t k = 0; k < H->ev_tag.size(); ++k) {
        float ms = 0.f;
        HIPC(hipEventElapsedTime(&ms, H->ev[2 * k], H->ev[2 * k + 1]));
        H->prof_ms[(size_t)H->ev_tag[k].first * 6 + H->ev_tag[k].second] += ms;
    }
    for (auto e : H->ev) (void)hipEventDestroy(e);
    H->ev.clear();
    H->ev_tag.clear();
    std::copy(H->prof_ms.begin(), H->prof_ms.end(), out);
    std::fill(H->prof_ms.begin(), H->prof_ms.end(), 0.0);
    return PAMG_OK;
}

// ncycles V-cycles on raw device vectors (graph replay when enabled; the captured graph is
// keyed on the vector addresses and the zero-guess flag).
// The k_sym_chain launch of a steady segment: the previous cycle's level-0 post-smoothing
// (t_prev -> x), this cycle's pre-smoothing (x -> t_next) and residual (t_next -> r[0]).
static int launch_chain3(pamg_hier* H, double* x, const double* b, const double* t_prev, double* t_next) {
    const pamg_mat* A = H->A[0];
    if (A->sym.tb_part) {  // one part of several: the blocked pass on the slab's inner planes
        double* out[3] = {x, t_next, H->r[0]};
        return sweeps_part(H->ctx, A, 3, t_prev, out, b, H->omega[0]);
    }
    pamg::TbArgs ta;
    ta.nstages = 3;
    ta.last_resid = true;
    ta.in0 = t_prev;
    // the post-smoothed iterate of cycle k is read only by this launch's next stage (from LDS):
    // the V-cycle's x is written by the tail's post-smoothing, so a steady chain stores it only
    // when asked (Options::chain_store_x; same bits either way)
    ta.out[0] = pamg::options().chain_store_x ? x : nullptr;
    ta.out[1] = t_next;
    ta.out[2] = H->r[0];
    ta.b = b;
    ta.omega = H->omega[0];
    pamg::launch_sym_tb(*A, ta, H->ctx->s_comp);
    HIPC(hipGetLastError());
    return PAMG_OK;
}

// Segments of the cross-cycle pipeline. seg 0: head (first cycle, no level-0 post-smoothing,
// iterate in t[0]); 1 / 2: steady, the iterate moving t[0] -> u0 / u0 -> t[0]; 3 / 4: tail (the
// last post-smoothing from t[0] / u0).
static int pipe_enqueue(pamg_hier* H, double* x, const double* b, int seg) {
    L0Seg sg;
    sg.post = false;
    if (seg == 0) return vcycle_enqueue(H, x, b, false, sg);
    double* t0 = H->t[0];
    double* u0 = H->u0;
    if (seg == 1 || seg == 2) {
        double* prev = seg == 1 ? t0 : u0;
        double* next = seg == 1 ? u0 : t0;
        {
            ProfScope p(H, 0, 0, H->ctx->s_comp);
            CHECK(launch_chain3(H, x, b, prev, next));
        }
        sg.given = true;
        sg.t0 = next;
        sg.r0 = H->r[0];
        return vcycle_enqueue(H, x, b, false, sg);
    }
    ProfScope p(H, 0, 4, H->ctx->s_comp);
    return apply(H->ctx, H->A[0], pamg::OP_JACOBI, seg == 3 ? t0 : u0, b, x, H->omega[0]);
}

// Eligible for the cross-cycle pipeline: one part, V(1, 1), level 0 in the symmetric layout with
// chain schedules, fusion on, a stationary run of >= 2 cycles from a given guess.
// Invariant across ranks: the decision is per rank (A->sym.tb_part depends on the
// part's shape), so ranks may disagree — one pipelining, its neighbour running separate cycles.
// That is correct only because both schedules issue the same exchanges in the same order on
// every level: pre-smoothing (A), residual (A), restriction (R), [tail all-gather], prolongation
// (P), post-smoothing (A) — the pipeline's chain does post-smoothing(k) (A), pre-smoothing(k+1)
// (A), residual(k+1) (A) through sweeps_part, one exchange per stage, in cycle order. Any change
// to either schedule must keep that sequence (tests/test_gpu_multipart.py: mixed ranks).
static bool pipe_ok(const pamg_hier* H, int ncycles, bool zero0) {
    if (zero0 || ncycles < 2 || H->L < 2 || H->prof || !pamg::options().jr_fuse || H->nu1 != 1 || H->nu2 != 1)
        return false;
    const pamg_mat* A = H->A[0];
    if (!A->interior.sym) return false;
    return (H->ctx->nranks == 1 && A->sym.tb_ok && !(A->plan && !A->plan->nbr.empty())) || A->sym.tb_part;
}

static int vcycle_pipe(pamg_hier* H, double* x, const double* b, int ncycles) {
    pamg_ctx* ctx = H->ctx;
    if (!H->u0) {
        const int64_t n = H->nown[0] + (H->A[0]->plan ? H->A[0]->plan->n_ghost : 0) + kVecPad;
        CHECK(dalloc(&H->u0, n));
        CHECK(dzero(H->ctx, H->u0, sizeof(double) * n));
    }
    const int K = ncycles;
    auto seg_of = [K](int k) { return k == 0 ? 0 : k < K ? (k % 2 == 1 ? 1 : 2) : ((K - 1) % 2 == 1 ? 4 : 3); };
    if (H->use_graph && (!H->g_head || H->gp_x != x || H->gp_b != b)) {
        drop_pipe_graphs(H);
        bool ok = true;
        hipGraphExec_t* slot[5] = {&H->g_head, &H->g_steady[0], &H->g_steady[1], &H->g_tail[0], &H->g_tail[1]};
        for (int sgi = 0; sgi < 5 && ok; ++sgi) {
            hipGraph_t g = nullptr;
            if (hipStreamBeginCapture(ctx->s_comp, hipStreamCaptureModeThreadLocal) != hipSuccess) {
                ok = false;
                break;
            }
            const int rc = pipe_enqueue(H, x, b, sgi);
            const hipError_t e2 = hipStreamEndCapture(ctx->s_comp, &g);
            ok = rc == PAMG_OK && e2 == hipSuccess && g && hipGraphInstantiate(slot[sgi], g, nullptr, nullptr, 0) == hipSuccess;
            if (g) (void)hipGraphDestroy(g);
        }
        if (ok) {
            H->gp_x = x;
            H->gp_b = b;
        } else {
            (void)hipGetLastError();
            drop_pipe_graphs(H);
            H->use_graph = false;
            H->graph_failed = true;
            fprintf(stderr, "[pamg] pipelined V-cycle graph capture failed (%s); using eager launches\n",
                    pamg::last_error().c_str());
        }
    }
    for (int k = 0; k <= K; ++k) {
        const int sg = seg_of(k);
        if (H->use_graph && H->g_head) {
            hipGraphExec_t ge = sg == 0 ? H->g_head : sg <= 2 ? H->g_steady[sg - 1] : H->g_tail[sg - 3];
            HIPC(hipGraphLaunch(ge, ctx->s_comp));
        } else {
            CHECK(pipe_enqueue(H, x, b, sg));
        }
    }
    return PAMG_OK;
}

static int vcycle_raw(pamg_hier* H, double* x, const double* b, int ncycles, bool zero0) {
    pamg_ctx* ctx = H->ctx;
    if (zero0 && ncycles != 1) return fail(PAMG_E_ARG, "vcycle: zero initial guess applies to one cycle");
    // stationary runs of >= 2 cycles: the cross-cycle pipeline (same operations, same bits)
    if (pipe_ok(H, ncycles, zero0)) return vcycle_pipe(H, x, b, ncycles);
    if (H->use_graph && !H->prof && (!H->gexec || H->g_x != x || H->g_b != b || H->g_zero0 != zero0)) {
        // Capture one cycle (RCCL exchanges included on several parts: RCCL records its
        // send/recv/all-gather as graph nodes). If capture fails, fall back to eager launches
        // for this hierarchy: both paths issue the same RCCL sequence, so ranks that did
        // capture and ranks that did not still match.
        drop_cycle_graph(H);
        hipGraph_t g = nullptr;
        int rc = PAMG_OK;
        hipError_t e1 = hipStreamBeginCapture(ctx->s_comp, hipStreamCaptureModeThreadLocal);
        if (e1 == hipSuccess) {
            rc = vcycle_enqueue(H, x, b, zero0);
            hipError_t e2 = hipStreamEndCapture(ctx->s_comp, &g);
            if (rc == PAMG_OK && e2 == hipSuccess && g &&
                hipGraphInstantiate(&H->gexec, g, nullptr, nullptr, 0) == hipSuccess) {
                H->g_x = x;
                H->g_b = b;
                H->g_zero0 = zero0;
            } else {
                H->gexec = nullptr;
            }
            if (g) (void)hipGraphDestroy(g);
        }
        if (!H->gexec) {
            (void)hipGetLastError();
            H->use_graph = false;
            H->graph_failed = true;
            fprintf(stderr, "[pamg] V-cycle graph capture failed (%s); using eager launches\n",
                    pamg::last_error().c_str());
        }
    }
    if (H->use_graph && !H->prof && H->gexec) {
        for (int k = 0; k < ncycles; ++k) HIPC(hipGraphLaunch(H->gexec, ctx->s_comp));
    } else {
        for (int k = 0; k < ncycles; ++k) CHECK(vcycle_enqueue(H, x, b, zero0 && k == 0));
    }
    return PAMG_OK;
}

// The caller's level-0 vectors in the device numbering: with a level-0 permutation, b is
// gathered into pb and (unless the guess is zero) x into px; without one they are used as is.
struct DeviceSpace {
    pamg_hier* H;
    double* x;
    const double* b;
    DeviceSpace(pamg_hier* h, pamg_vec* xv, const pamg_vec* bv, bool gather_x) : H(h), x(xv->d), b(bv->d) {
        if (!H->d_perm) return;
        const int64_t n = H->nown[0];
        hipStream_t s = H->ctx->s_comp;
        pamg::launch_permute(n, H->d_perm, bv->d, H->pb, false, s);
        if (gather_x) pamg::launch_permute(n, H->d_perm, xv->d, H->px, false, s);
        x = H->px;
        b = H->pb;
    }
    // x back to the caller's numbering
    void finish(pamg_vec* xv) {
        if (H->d_perm) pamg::launch_permute(H->nown[0], H->d_perm, H->px, xv->d, true, H->ctx->s_comp);
    }
};

static int vcycle_common(pamg_ctx* ctx, pamg_hier* H, pamg_vec* x, const pamg_vec* b, int ncycles) {
    if (!ctx || !H || !x || !b || ncycles < 0 || H->ctx != ctx) return fail(PAMG_E_ARG, "vcycle: bad args");
    const pamg_mat* A0 = H->A[0];
    CHECK(check_vec_for(A0, x, "vcycle"));
    if (b->n_own != A0->nrows) return fail(PAMG_E_ARG, "vcycle: b size mismatch");
    CHECK(set_device(ctx));
    DeviceSpace d(H, x, b, true);
    CHECK(vcycle_raw(H, d.x, d.b, ncycles, false));
    d.finish(x);
    HIPC(hipGetLastError());
    return PAMG_OK;
}

int pamg_vcycle_async(pamg_ctx* ctx, pamg_hier* H, pamg_vec* x, const pamg_vec* b, int ncycles) {
    return vcycle_common(ctx, H, x, b, ncycles);
}

int pamg_vcycle(pamg_ctx* ctx, pamg_hier* H, pamg_vec* x, const pamg_vec* b, int ncycles,
                double* res_hist) {
    if (!res_hist) {
        CHECK(vcycle_common(ctx, H, x, b, ncycles));
        HIPC(hipStreamSynchronize(ctx->s_comp));
        return PAMG_OK;
    }
    if (!ctx || !H || !x || !b || ncycles < 0 || H->ctx != ctx) return fail(PAMG_E_ARG, "vcycle: bad args");
    if (H->L < 1 || (!H->t[0] && H->L > 1)) return fail(PAMG_E_ARG, "vcycle: bad hierarchy");
    CHECK(check_vec_for(H->A[0], x, "vcycle"));
    if (b->n_own != H->A[0]->nrows) return fail(PAMG_E_ARG, "vcycle: b size mismatch");
    CHECK(set_device(ctx));
    DeviceSpace d(H, x, b, true);
    for (int k = 0; k < ncycles; ++k) {
        CHECK(vcycle_raw(H, d.x, d.b, 1, false));
        // r = b - A x into the level-0 residual buffer (1-level hierarchies use a temporary)
        double* r = H->L > 1 ? H->r[0] : nullptr;
        double* tmp = nullptr;
        if (!r) {
            CHECK(dalloc(&tmp, H->nown[0] + kVecPad));
            r = tmp;
        }
        int rc = apply(ctx, H->A[0], pamg::OP_RESID, d.x, d.b, r, 0.0);
        double s = 0.0;
        if (rc == PAMG_OK) rc = reduce_scalar(ctx, H->nown[0], r, r, &s);
        dfree(tmp);
        CHECK(rc);
        res_hist[k] = std::sqrt(s);
    }
    d.finish(x);
    HIPC(hipStreamSynchronize(ctx->s_comp));
    return PAMG_OK;
}

// Preconditioned CG with one V-cycle from a zero guess as M^-1 (SPEC §S8). The V(1,1) cycle
// with R = P^T and the same weighted Jacobi before and after is symmetric, so CG applies.
int pamg_pcg(pamg_ctx* ctx, pamg_hier* H, pamg_vec* x, const pamg_vec* b, double rtol,
             int maxit, int* iters, double* res_hist) {
    if (!ctx || !H || !x || !b || maxit < 0 || !(rtol >= 0.0) || H->ctx != ctx)
        return fail(PAMG_E_ARG, "pcg: bad args");
    const pamg_mat* A = H->A[0];
    CHECK(check_vec_for(A, x, "pcg"));
    if (b->n_own != A->nrows) return fail(PAMG_E_ARG, "pcg: b size mismatch");
    CHECK(set_device(ctx));
    const int64_t n = A->nrows;
    int64_t g = A->plan ? A->plan->n_ghost : 0;
    if (H->L > 1 && H->R[0]->plan) g = std::max(g, H->R[0]->plan->n_ghost);
    const int64_t cap = n + g + kVecPad;
    if (!H->pcg_r) {
        CHECK(dalloc(&H->pcg_r, cap));
        CHECK(dalloc(&H->pcg_z, cap));
        CHECK(dalloc(&H->pcg_p, cap));
        CHECK(dalloc(&H->pcg_q, cap));
        for (double* p : {H->pcg_r, H->pcg_z, H->pcg_p, H->pcg_q})
            CHECK(dzero(ctx, p, sizeof(double) * cap));
    }
    hipStream_t s = ctx->s_comp;
    double *r = H->pcg_r, *z = H->pcg_z, *p = H->pcg_p, *q = H->pcg_q;
    // with a level-0 permutation the whole iteration runs in the device numbering
    DeviceSpace d(H, x, b, true);
    double* xd = d.x;
    CHECK(apply(ctx, A, pamg::OP_RESID, xd, d.b, r, 0.0));
    double rr = 0.0;
    CHECK(reduce_scalar(ctx, n, r, r, &rr));
    const double nr0 = std::sqrt(rr);
    if (res_hist) res_hist[0] = nr0;
    int k = 0;
    if (nr0 > 0.0 && maxit > 0) {
        CHECK(vcycle_raw(H, z, r, 1, true));
        HIPC(hipMemcpyAsync(p, z, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
        double rz = 0.0;
        CHECK(reduce_scalar(ctx, n, r, z, &rz));
        while (k < maxit) {
            ++k;
            CHECK(apply(ctx, A, pamg::OP_SPMV, p, nullptr, q, 0.0));
            double pq = 0.0;
            CHECK(reduce_scalar(ctx, n, p, q, &pq));
            const double alpha = rz / pq;
            // x += alpha p; r -= alpha q; rr = r.r in one pass (bits of the unfused sequence)
            CHECK(reduce_with(ctx, n, &rr, [&](int np, double* parts, double* res, hipStream_t st) {
                pamg::launch_cg_update(n, alpha, p, q, xd, r, parts, np, res, st);
            }));
            const double nr = std::sqrt(rr);
            if (res_hist) res_hist[k] = nr;
            if (nr <= rtol * nr0) break;
            CHECK(vcycle_raw(H, z, r, 1, true));
            double rz_new = 0.0;
            CHECK(reduce_scalar(ctx, n, r, z, &rz_new));
            const double beta = rz_new / rz;
            rz = rz_new;
            pamg::launch_axpby(n, 1.0, z, beta, p, s);
        }
    }
    d.finish(x);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(s));
    if (iters) *iters = k;
    return PAMG_OK;
}

int pamg_set_option(const char* key, int64_t value) {
    if (!key) return fail(PAMG_E_ARG, "set_option: NULL key");
    auto& o = pamg::options();
    const std::string k(key);
    if (k == "tile_nnz" && (value == 1024 || value == 2048 || value == 4096)) o.tile_nnz = (int)value;
    else if (k == "tile_order" && (value == 0 || value == 1)) o.tile_order = (int)value;  // 0 natural, 1 banded XCD-blocked
    else if (k == "poison_ghosts" && (value == 0 || value == 1)) o.poison_ghosts = (int)value;
    else if (k == "col24" && (value == 0 || value == 1)) o.col24 = (int)value;
    else if (k == "long_tiles" && (value == 0 || value == 1)) o.long_tiles = (int)value;
    else if (k == "row_len8" && (value == 0 || value == 1)) o.row_len8 = (int)value;
    else if (k == "value_dict" && value >= 0 && value <= 2) o.value_dict = (int)value;
    else if (k == "col_dict" && (value == 0 || value == 1)) o.col_dict = (int)value;
    else if (k == "tile_major" && value >= 0 && value <= 2) o.tile_major = (int)value;
    else if (k == "col_dict_anchor" && (value == 0 || value == 1)) o.col_dict_anchor = (int)value;
    else if (k == "col_dict_tile" && (value == 0 || value == 1)) o.col_dict_tile = (int)value;
    else if (k == "x_stage" && (value == 0 || value == 1)) o.x_stage = (int)value;
    else if (k == "band_pct" && value >= 1 && value <= 10000) o.band_pct = (int)value;
    else if (k == "band_pct_restrict" && value >= 1 && value <= 10000) o.band_pct_restrict = (int)value;
    else if (k == "long_tiles_min" && value >= 1 && value <= 255) o.long_tiles_min = (int)value;
    else if (k == "tm_tile_dicts" && (value == 0 || value == 1)) o.tm_tile_dicts = (int)value;
    else if (k == "sym_dia" && (value == 0 || value == 1)) o.sym_dia = (int)value;
    else if (k == "sym_rows" && (value == 1 || value == 2)) o.sym_rows = (int)value;
    else if (k == "jr_fuse" && (value == 0 || value == 1)) o.jr_fuse = (int)value;
    else if (k == "sym_vd" && (value == 0 || value == 1)) o.sym_vd = (int)value;
    else if (k == "symd_chunks" && (value == 1 || value == 2 || value == 4)) o.symd_chunks = (int)value;
    else if (k == "sym_zm" && (value == 0 || value == 1)) o.sym_zm = (int)value;
    else if (k == "tb_xfast" && (value == 0 || value == 1)) o.tb_xfast = (int)value;
    else if (k == "ell" && (value == 0 || value == 1)) o.ell = (int)value;
    else if (k == "ell_restrict" && (value == 0 || value == 1)) o.ell_restrict = (int)value;
    else if (k == "pnc" && (value == 0 || value == 1)) o.pnc = (int)value;
    else if (k == "rpat" && (value == 0 || value == 1)) o.rpat = (int)value;
    else if (k == "pnc_compact" && (value == 0 || value == 1)) o.pnc_compact = (int)value;
    else if (k == "ell_pair" && (value == 0 || value == 1)) o.ell_pair = (int)value;
    else if (k == "ell_yblock" && value >= 0 && value <= 65536) o.ell_yblock = (int)value;
    else if (k == "ell_min_rows" && value >= 0 && value <= INT32_MAX) o.ell_min_rows = (int)value;
    else if (k == "zm_chunks" && value >= 0 && value <= 4096) o.zm_chunks = (int)value;
    else if (k == "chain_store_x" && (value == 0 || value == 1)) o.chain_store_x = (int)value;
    else return fail(PAMG_E_ARG, "set_option: unknown key or bad value: %s=%lld", key, (long long)value);
    return PAMG_OK;
}

int pamg_get_option(const char* key, int64_t* value) {
    if (!key || !value) return fail(PAMG_E_ARG, "get_option: bad args");
    const auto& o = pamg::options();
    const std::string k(key);
    if (k == "tile_nnz") *value = o.tile_nnz;
    else if (k == "tile_order") *value = o.tile_order;
    else if (k == "long_tiles") *value = o.long_tiles;
    else if (k == "row_len8") *value = o.row_len8;
    else if (k == "poison_ghosts") *value = o.poison_ghosts;
    else if (k == "col24") *value = o.col24;
    else if (k == "value_dict") *value = o.value_dict;
    else if (k == "col_dict") *value = o.col_dict;
    else if (k == "tile_major") *value = o.tile_major;
    else if (k == "col_dict_anchor") *value = o.col_dict_anchor;
    else if (k == "col_dict_tile") *value = o.col_dict_tile;
    else if (k == "x_stage") *value = o.x_stage;
    else if (k == "band_pct") *value = o.band_pct;
    else if (k == "band_pct_restrict") *value = o.band_pct_restrict;
    else if (k == "long_tiles_min") *value = o.long_tiles_min;
    else if (k == "tm_tile_dicts") *value = o.tm_tile_dicts;
    else if (k == "sym_dia") *value = o.sym_dia;
    else if (k == "sym_rows") *value = o.sym_rows;
    else if (k == "jr_fuse") *value = o.jr_fuse;
    else if (k == "sym_vd") *value = o.sym_vd;
    else if (k == "symd_chunks") *value = o.symd_chunks;
    else if (k == "sym_zm") *value = o.sym_zm;
    else if (k == "tb_xfast") *value = o.tb_xfast;
    else if (k == "ell") *value = o.ell;
    else if (k == "ell_restrict") *value = o.ell_restrict;
    else if (k == "pnc") *value = o.pnc;
    else if (k == "rpat") *value = o.rpat;
    else if (k == "pnc_compact") *value = o.pnc_compact;
    else if (k == "ell_pair") *value = o.ell_pair;
    else if (k == "ell_yblock") *value = o.ell_yblock;
    else if (k == "ell_min_rows") *value = o.ell_min_rows;
    else if (k == "zm_chunks") *value = o.zm_chunks;
    else if (k == "chain_store_x") *value = o.chain_store_x;
    else return fail(PAMG_E_ARG, "get_option: unknown key %s", key);
    return PAMG_OK;
}

int pamg_hier_bench_chain(pamg_hier* H, pamg_vec* x, const pamg_vec* b, int reps, double* avg_ms) {
    if (!H || !x || !b || reps < 1 || !avg_ms) return fail(PAMG_E_ARG, "hier_bench_chain: bad args");
    if (!pipe_ok(H, 2, false)) return fail(PAMG_E_STATE, "hier_bench_chain: the hierarchy does not run the cross-cycle pipeline");
    pamg_ctx* ctx = H->ctx;
    CHECK(check_vec_for(H->A[0], x, "hier_bench_chain"));
    CHECK(set_device(ctx));
    if (!H->u0) {
        const int64_t n = H->nown[0] + (H->A[0]->plan ? H->A[0]->plan->n_ghost : 0) + kVecPad;
        CHECK(dalloc(&H->u0, n));
        CHECK(dzero(H->ctx, H->u0, sizeof(double) * n));
    }
    hipEvent_t e0, e1;
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    hipStream_t s = ctx->s_comp;
    CHECK(launch_chain3(H, x->d, b->d, H->t[0], H->u0));
    HIPC(hipEventRecord(e0, s));
    for (int k = 0; k < reps; ++k) CHECK(launch_chain3(H, x->d, b->d, (k & 1) ? H->u0 : H->t[0], (k & 1) ? H->t[0] : H->u0));
    HIPC(hipEventRecord(e1, s));
    HIPC(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, e0, e1));
    *avg_ms = ms / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return PAMG_OK;
}

int pamg_bench_rowop(pamg_ctx* ctx, const pamg_mat* A, int op, pamg_vec* x, const pamg_vec* b,
                     pamg_vec* y, double omega, int reps, double* avg_ms) {
    if (!ctx || !A || !x || !y || reps < 1 || !avg_ms || op < 0 || op > 5)
        return fail(PAMG_E_ARG, "bench_rowop: bad args");
    if ((op == pamg::OP_RESID || op == pamg::OP_JACOBI || op >= 4) && !b) return fail(PAMG_E_ARG, "bench_rowop: b needed");
    if ((op == pamg::OP_JACOBI || op >= 4) && !A->d_diag)
        return fail(PAMG_E_SETUP, "bench_rowop: jacobi needs a square matrix");
    if (op >= 4 && !(A->interior.sym && (A->sym.tb_ok || A->sym.tb_part)))
        return fail(PAMG_E_STATE, "bench_rowop: op %d needs the temporally blocked layout (pamg_mat_layout bit 5)", op);
    if (x == y) return fail(PAMG_E_ARG, "bench_rowop: x and y must differ");
    CHECK(check_vec_for(A, x, "bench_rowop"));
    // a part's blocked passes (sweeps_part) feed each stage's output to the next stage's boundary
    // rows, which read its ghost slots: y and the scratch stages need the column length
    const bool part_tb = op >= 4 && A->sym.tb_part;
    if (part_tb) CHECK(check_vec_for(A, y, "bench_rowop (y: input of the next stage)"));
    CHECK(set_device(ctx));
    // ops 4 / 5: the temporally blocked passes k_sym_tb<2> (Jacobi -> residual) and <3>
    // (Jacobi -> Jacobi -> residual), the first output into y, the others into scratch
    double* scratch[2] = {nullptr, nullptr};
    if (op >= 4) {
        const int64_t len = part_tb ? (A->plan ? A->plan->n_own + A->plan->n_ghost : A->ncols) : A->nrows;
        for (double*& p : scratch) {
            CHECK(dalloc(&p, std::max<int64_t>(len, A->nrows) + kVecPad));
            CHECK(dzero(ctx, p, sizeof(double) * (size_t)(std::max<int64_t>(len, A->nrows) + kVecPad)));
        }
    }
    pamg::TbArgs ta;
    ta.nstages = op - 2;
    ta.last_resid = true;
    ta.in0 = x->d;
    // op 5 on one part mirrors the pipeline's chain (launch_chain3): its stage-0 output is stored
    // only with chain_store_x (a part's passes feed it to the edge planes: always stored there)
    ta.out[0] = op == 5 && !part_tb && !pamg::options().chain_store_x ? nullptr : y->d;
    ta.out[1] = scratch[0];
    ta.out[2] = scratch[1];
    ta.b = b ? b->d : nullptr;
    ta.omega = omega;
    hipEvent_t e0, e1;
    HIPC(hipEventCreate(&e0));
    HIPC(hipEventCreate(&e1));
    hipStream_t s = ctx->s_comp;
    const double* bd = b ? b->d : nullptr;
    auto once = [&]() {
        if (op >= 4 && A->sym.tb_part) {  // one part of several: its blocked pass + edge planes + boundary rows
            (void)sweeps_part(ctx, A, op - 2, x->d, ta.out, ta.b, omega, false);
        } else if (op >= 4) {
            pamg::launch_sym_tb(*A, ta, s);
        } else {
            pamg::launch_rows(*A, A->interior, op, x->d, bd, x->d, y->d, omega, s);
            pamg::launch_rows(*A, A->boundary, op, x->d, bd, x->d, y->d, omega, s);
        }
    };
    once();
    HIPC(hipEventRecord(e0, s));
    for (int k = 0; k < reps; ++k) once();
    HIPC(hipEventRecord(e1, s));
    HIPC(hipEventSynchronize(e1));
    float ms = 0.f;
    HIPC(hipEventElapsedTime(&ms, e0, e1));
    *avg_ms = ms / reps;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    for (double* p : scratch) dfree(p);
    return PAMG_OK;
}

}  // extern "C"
