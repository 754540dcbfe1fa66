// spgemm.hip — GPU-side Galerkin setup products: C = X*Y (SPEC §S4.5) and the
// restricted transpose R = P^T (SPEC §S4.7), bit-identical to setup.cpp's host routines of the
// same contract (pamg_setup_spgemm / pamg_setup_transpose) but computed on the context's GPU.
//
// SpGEMM (row-merge with per-row hash tables):
//   * every row i of C is owned by a group of G lanes inside one wavefront;
//   * the group walks X's row i in storage order (one X entry = one "step"); within a step the
//     lanes cover Y's row in parallel. A step's columns are distinct (Y rows have unique
//     columns), so no two lanes touch one accumulator in a step, and the wavefront's in-order
//     LDS (plus a fence per step) makes step a+1 see step a: each column's products are folded
//     in encounter order, the first one initialising the sum — exactly §S4.5;
//   * symbolic pass: count the distinct columns u_i (hash of keys only); scan -> rowptr;
//   * numeric pass: accumulate, compact the table, rank the keys (ascending column order) and
//     write the row at rowptr[i].
//   Tables live in LDS, sized T = nextpow2(2 min(m_i, ncols)) from the row's product count m_i
//   (8 bins, 32..4096 slots); a row whose distinct columns do not fit its table (only possible
//   in the capped 4096 bin) is redone by one wavefront with a table in global memory.
// Transpose: stable radix sort of P's entries by column (hipCUB), so each R row keeps P's row
// order — the order the host routine produces.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <memory>
#include <vector>

#include "pamg_device.h"

using pamg::fail;

#define HIPC(expr)                                                                    \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(PAMG_E_HIP, "%s:%d %s: %s", __FILE__, __LINE__, #expr,        \
                        hipGetErrorString(e_));                                       \
    } while (0)

#define CHECK(expr)                     \
    do {                                \
        int rc_ = (expr);               \
        if (rc_ != PAMG_OK) return rc_; \
    } while (0)

namespace {

constexpr int32_t kEmpty = -1;
constexpr int kBins = 8;        // LDS tables of 32 << b slots
constexpr int kMaxLdsT = 4096;

template <class T>
struct DBuf {  // device buffer released on every exit path
    T* p = nullptr;
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
    int alloc(int64_t n) {
        if (p) (void)hipFree(p);
        p = nullptr;
        if (n <= 0) return PAMG_OK;
        if (hipMalloc(reinterpret_cast<void**>(&p), sizeof(T) * (size_t)n) != hipSuccess)
            return fail(PAMG_E_NOMEM, "device setup: cannot allocate %lld x %zu bytes",
                        (long long)n, sizeof(T));
        return PAMG_OK;
    }
};

template <class T>
int h2d(DBuf<T>& d, const T* h, int64_t n, hipStream_t s) {
    CHECK(d.alloc(n));
    if (n > 0) HIPC(hipMemcpyAsync(d.p, h, sizeof(T) * (size_t)n, hipMemcpyHostToDevice, s));
    return PAMG_OK;
}

struct SgArgs {
    const int64_t* xrp;
    const int32_t* xr;    // Y row of each X entry (own rows, then ghost rows)
    const double* xv;
    const int64_t* yrp;
    const int32_t* ycol;
    const double* yv;
    int32_t* cnt;         // symbolic: distinct columns per row, -1 = did not fit
    const int64_t* crp;   // numeric: C row pointers
    int32_t* ccol;
    double* cval;
};

// table accessors: LDS tables use plain accesses; global tables go through L2 (the CAS on the
// keys is performed there, so plain loads could hit a stale L1 line)
template <bool GL, class T>
__device__ inline T tld(const T* p) {
    if constexpr (GL) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool GL, class T>
__device__ inline void tst(T* p, T v) {
    if constexpr (GL) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}
template <bool GL>
__device__ inline void step_fence() {
    if constexpr (GL) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    else __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ inline uint32_t hslot(int32_t j) { return (uint32_t)j * 2654435761u; }

template <int G>
__device__ inline int group_sum(int v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, G);
    return v;
}

// One row of C by a group of G lanes (lane in [0, G)); wshift = the group's first lane in
// its wavefront. key/acc: the row's table of T slots (T a power of two), keys preset to kEmpty.
template <int G, bool NUMERIC, bool GL>
__device__ inline void sg_row(const SgArgs& A, int32_t i, int32_t* key, double* acc, uint32_t T,
                              int lane, int wshift) {
    const uint32_t mask = T - 1;
    int ins = 0, full = 0;
    const int64_t a1 = A.xrp[i + 1];
    for (int64_t a = A.xrp[i]; a < a1; ++a) {
        const int32_t r = A.xr[a];
        const double x = NUMERIC ? A.xv[a] : 0.0;
        const int64_t b1 = A.yrp[r + 1];
        for (int64_t b = A.yrp[r] + lane; b < b1; b += G) {
            const int32_t j = A.ycol[b];
            uint32_t h = hslot(j) & mask;
            for (uint32_t probe = 0;; ++probe) {
                if (probe > mask) {
                    full = 1;
                    break;
                }
                const int32_t old = atomicCAS(&key[h], kEmpty, j);
                if (old == kEmpty) {
                    ++ins;
                    if (NUMERIC) tst<GL>(&acc[h], x * A.yv[b]);
                    break;
                }
                if (old == j) {
                    if (NUMERIC) tst<GL>(&acc[h], tld<GL>(&acc[h]) + x * A.yv[b]);
                    break;
                }
                h = (h + 1) & mask;
            }
        }
        step_fence<GL>();
    }
    if constexpr (!NUMERIC) {
        const int u = group_sum<G>(ins), f = group_sum<G>(full);
        if (lane == 0) A.cnt[i] = (f || (uint32_t)u > (3 * T) / 4) ? -1 : u;
        return;
    } else {
        // compact the occupied slots to [0, u) in slot order, then rank by column
        const uint64_t gmask = (G == 64) ? ~0ull : ((1ull << (G & 63)) - 1);
        uint32_t u = 0;
        for (uint32_t s0 = 0; s0 < T; s0 += G) {
            const uint32_t s = s0 + lane;
            const int32_t k = tld<GL>(&key[s]);
            const double v = tld<GL>(&acc[s]);
            const bool occ = k != kEmpty;
            const uint64_t gb = (__ballot(occ) >> wshift) & gmask;
            step_fence<GL>();
            if (occ) {
                const uint32_t p = u + (uint32_t)__popcll(gb & ((1ull << lane) - 1));
                tst<GL>(&key[p], k);
                tst<GL>(&acc[p], v);
            }
            u += (uint32_t)__popcll(gb);
            step_fence<GL>();
        }
        const int64_t c0 = A.crp[i];
        for (uint32_t e = lane; e < u; e += G) {
            const int32_t k = tld<GL>(&key[e]);
            uint32_t rank = 0;
            for (uint32_t t = 0; t < u; ++t) rank += (tld<GL>(&key[t]) < k) ? 1u : 0u;
            A.ccol[c0 + rank] = k;
            A.cval[c0 + rank] = tld<GL>(&acc[e]);
        }
    }
}

template <int T>
struct BinCfg {  // lanes per row and rows per block: <= 48 KB of LDS per block
    static constexpr int G = T <= 64 ? 4 : T <= 256 ? 8 : T <= 512 ? 16 : T <= 1024 ? 32 : 64;
    static constexpr int RPB = std::min(256 / G, (48 * 1024) / (12 * T));
};

template <int T, bool NUMERIC>
__global__ __launch_bounds__(BinCfg<T>::G* BinCfg<T>::RPB) void k_sg_lds(SgArgs A,
                                                                        const int32_t* rows,
                                                                        int64_t nrows) {
    constexpr int G = BinCfg<T>::G, RPB = BinCfg<T>::RPB;
    __shared__ int32_t skey[RPB * T];
    __shared__ double sacc[NUMERIC ? RPB * T : 1];
    for (int s = threadIdx.x; s < RPB * T; s += G * RPB) skey[s] = kEmpty;
    __syncthreads();
    const int g = threadIdx.x / G, lane = threadIdx.x % G;
    const int64_t ri = (int64_t)blockIdx.x * RPB + g;
    if (ri >= nrows) return;
    sg_row<G, NUMERIC, false>(A, rows[ri], skey + g * T, sacc + (NUMERIC ? g * T : 0), T, lane,
                              (int)(threadIdx.x & 63) - lane);
}

// rows that did not fit an LDS table: one wavefront per row, table in global memory
template <bool NUMERIC>
__global__ __launch_bounds__(64) void k_sg_glob(SgArgs A, const int32_t* rows,
                                                const int64_t* woff, int32_t* wkey,
                                                double* wacc) {
    const int64_t ri = blockIdx.x;
    const int64_t o = woff[ri];
    const uint32_t T = (uint32_t)(woff[ri + 1] - o);
    int32_t* key = wkey + o;
    for (uint32_t s = threadIdx.x; s < T; s += 64) tst<true>(&key[s], kEmpty);
    step_fence<true>();
    sg_row<64, NUMERIC, true>(A, rows[ri], key, wacc + o, T, threadIdx.x, 0);
}

__global__ void k_map_rows(const int32_t* xcol, int64_t nnz, int64_t y0, int64_t ny,
                           const int64_t* gids, int64_t ng, int32_t* xr, int* missing) {
    for (int64_t a = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; a < nnz;
         a += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = xcol[a];
        int64_t r = k - y0;
        if (r < 0 || r >= ny) {
            int64_t lo = 0, hi = ng;
            while (lo < hi) {
                const int64_t mid = (lo + hi) >> 1;
                if (gids[mid] < k) lo = mid + 1;
                else hi = mid;
            }
            if (lo < ng && gids[lo] == k) r = ny + lo;
            else {
                atomicAdd(missing, 1);
                r = 0;
            }
        }
        xr[a] = (int32_t)r;
    }
}

__device__ inline int bin_of(int64_t m, int64_t nc) {
    const int64_t t = 2 * std::min(m, nc);
    int b = 0;
    while (b < kBins - 1 && (int64_t(32) << b) < t) ++b;
    return b;
}

// product count m_i, bin (kBins = empty row) and bin population. The bin counters are hit by
// every row, so each block histograms its rows in LDS and adds once per bin (a global atomic
// per row serialised on a handful of addresses: 0.24 s at 134M rows).
__global__ __launch_bounds__(256) void k_row_products(const int64_t* xrp, const int32_t* xr,
                                                      const int64_t* yrp, int64_t n, int64_t nc,
                                                      int64_t* m, uint8_t* bin, int* bincnt) {
    __shared__ int hist[kBins + 1];
    if (threadIdx.x <= kBins) hist[threadIdx.x] = 0;
    __syncthreads();
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t s = 0;
        for (int64_t a = xrp[i]; a < xrp[i + 1]; ++a) s += yrp[xr[a] + 1] - yrp[xr[a]];
        m[i] = s;
        const int b = s == 0 ? kBins : bin_of(s, nc);
        bin[i] = (uint8_t)b;
        atomicAdd(&hist[b], 1);
    }
    __syncthreads();
    if (threadIdx.x <= kBins && hist[threadIdx.x]) atomicAdd(&bincnt[threadIdx.x], hist[threadIdx.x]);
}

// rows -> per-bin lists: each block reserves one range per bin, then places its rows in it
// (order inside a bin is irrelevant: every row's output position comes from the row pointers)
__global__ __launch_bounds__(256) void k_scatter_bins(const uint8_t* bin, int64_t n,
                                                      const int64_t* binoff, int* cursor,
                                                      int32_t* lists) {
    __shared__ int cnt[kBins + 1], base[kBins + 1];
    if (threadIdx.x <= kBins) cnt[threadIdx.x] = 0;
    __syncthreads();
    const int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    const int64_t step = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = i0; i < n; i += step) atomicAdd(&cnt[bin[i]], 1);
    __syncthreads();
    if (threadIdx.x < kBins) {
        base[threadIdx.x] = cnt[threadIdx.x] ? atomicAdd(&cursor[threadIdx.x], cnt[threadIdx.x]) : 0;
        cnt[threadIdx.x] = 0;
    }
    __syncthreads();
    for (int64_t i = i0; i < n; i += step) {
        const int b = bin[i];
        if (b >= kBins) continue;
        lists[binoff[b] + base[b] + atomicAdd(&cnt[b], 1)] = (int32_t)i;
    }
}

__global__ void k_counts_i64(const int32_t* cnt, const uint8_t* bin, int64_t n, int64_t* out,
                             int32_t* ovf_rows, int* n_ovf) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        int64_t c = bin[i] >= kBins ? 0 : cnt[i];
        if (c < 0) {
            if (ovf_rows) ovf_rows[atomicAdd(n_ovf, 1)] = (int32_t)i;
            c = 0;
        }
        out[i] = c;
    }
}

// ---- transpose ----
__global__ void k_tr_keys(const int64_t* rp, const int32_t* col, int64_t nr, int64_t c0,
                          int64_t c1, uint32_t* keys, int32_t* idx, int32_t* rid,
                          unsigned long long* cnt) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nr;
         i += (int64_t)gridDim.x * blockDim.x) {
        for (int64_t a = rp[i]; a < rp[i + 1]; ++a) {
            const int64_t c = col[a];
            const bool in = c >= c0 && c < c1;
            keys[a] = in ? (uint32_t)(c - c0) : (uint32_t)(c1 - c0);
            idx[a] = (int32_t)a;
            rid[a] = (int32_t)i;
            if (in) atomicAdd(&cnt[c - c0], 1ull);
        }
    }
}

__global__ void k_tr_fill(const int32_t* sidx, const int32_t* rid, const double* val,
                          int64_t nnz_out, int64_t row0, int32_t* rcol, double* rval) {
    for (int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; k < nnz_out;
         k += (int64_t)gridDim.x * blockDim.x) {
        const int32_t a = sidx[k];
        rcol[k] = (int32_t)(row0 + rid[a]);
        rval[k] = val[a];
    }
}

inline int grid_for(int64_t n, int block = 256) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + block - 1) / block, 65536));
}

int inclusive_scan_i64(const int64_t* in, int64_t* out, int64_t n, hipStream_t s) {
    if (n <= 0) return PAMG_OK;
    size_t bytes = 0;
    HIPC(hipcub::DeviceScan::InclusiveSum(nullptr, bytes, in, out, (int)n, s));
    DBuf<char> tmp;
    CHECK(tmp.alloc((int64_t)bytes + 1));
    HIPC(hipcub::DeviceScan::InclusiveSum(tmp.p, bytes, in, out, (int)n, s));
    HIPC(hipStreamSynchronize(s));
    return PAMG_OK;
}

template <int T>
int launch_bin(bool numeric, const SgArgs& A, const int32_t* rows, int64_t n, hipStream_t s) {
    if (n <= 0) return PAMG_OK;
    constexpr int RPB = BinCfg<T>::RPB, NT = BinCfg<T>::G * BinCfg<T>::RPB;
    const int64_t blocks = (n + RPB - 1) / RPB;
    if (numeric) hipLaunchKernelGGL((k_sg_lds<T, true>), dim3((unsigned)blocks), dim3(NT), 0, s, A, rows, n);
    else hipLaunchKernelGGL((k_sg_lds<T, false>), dim3((unsigned)blocks), dim3(NT), 0, s, A, rows, n);
    HIPC(hipGetLastError());
    return PAMG_OK;
}

int launch_bins(bool numeric, const SgArgs& A, const int32_t* lists,
                const std::vector<int64_t>& off, hipStream_t s) {
    const int32_t* L = lists;
    CHECK(launch_bin<32>(numeric, A, L + off[0], off[1] - off[0], s));
    CHECK(launch_bin<64>(numeric, A, L + off[1], off[2] - off[1], s));
    CHECK(launch_bin<128>(numeric, A, L + off[2], off[3] - off[2], s));
    CHECK(launch_bin<256>(numeric, A, L + off[3], off[4] - off[3], s));
    CHECK(launch_bin<512>(numeric, A, L + off[4], off[5] - off[4], s));
    CHECK(launch_bin<1024>(numeric, A, L + off[5], off[6] - off[5], s));
    CHECK(launch_bin<2048>(numeric, A, L + off[6], off[7] - off[6], s));
    CHECK(launch_bin<kMaxLdsT>(numeric, A, L + off[7], off[8] - off[7], s));
    return PAMG_OK;
}

uint64_t next_pow2(uint64_t v) {
    uint64_t t = 1;
    while (t < v) t <<= 1;
    return t;
}

bool valid(const pamg_hcsr* M) { return M && (int64_t)M->rp.size() == M->nr + 1; }

int dev_spgemm(pamg_ctx* ctx, const pamg_hcsr* X, int64_t y0, const pamg_hcsr* Yown,
               const int64_t* ghost_ids, int64_t n_ghost, const pamg_hcsr* Yghost,
               pamg_hcsr** out) {
    const hipStream_t s = ctx->s_comp;
    const int64_t n = X->nr, nnzx = X->nnz(), ny = Yown->nr, ng = n_ghost;
    const int64_t nnzo = Yown->nnz(), nnzg = ng > 0 ? Yghost->nnz() : 0;
    const int64_t nc = Yown->nc;
    if (nc >= (int64_t)INT32_MAX || ny + ng >= (int64_t)INT32_MAX || n >= (int64_t)INT32_MAX)
        return fail(PAMG_E_OVERFLOW, "dev_spgemm: sizes >= 2^31");
    HIPC(hipSetDevice(ctx->device));

    DBuf<int64_t> xrp, yrp, gids, m, binoff, crp, woff;
    DBuf<int32_t> xcol, xr, ycol, cnt, lists, ccol, ovf, wkey;
    DBuf<double> xv, yv, cval, wacc;
    DBuf<uint8_t> bin;
    DBuf<int> flags;  // [0] missing, [1..kBins+1] bin counts, [kBins+2..] cursors, last: n_ovf
    constexpr int kF = 2 * (kBins + 1) + 2;

    CHECK(h2d(xrp, X->rp.data(), n + 1, s));
    CHECK(h2d(xcol, X->col.data(), nnzx, s));
    CHECK(h2d(xv, X->val.data(), nnzx, s));
    // Y = own rows followed by ghost rows, one CSR
    std::vector<int64_t> grp;
    if (ng > 0) {
        grp.resize(ng);
        for (int64_t r = 0; r < ng; ++r) grp[r] = Yghost->rp[r + 1] + nnzo;
    }
    CHECK(yrp.alloc(ny + ng + 1));
    HIPC(hipMemcpyAsync(yrp.p, Yown->rp.data(), sizeof(int64_t) * (ny + 1), hipMemcpyHostToDevice, s));
    if (ng > 0)
        HIPC(hipMemcpyAsync(yrp.p + ny + 1, grp.data(), sizeof(int64_t) * ng, hipMemcpyHostToDevice, s));
    CHECK(ycol.alloc(nnzo + nnzg));
    CHECK(yv.alloc(nnzo + nnzg));
    if (nnzo > 0) {
        HIPC(hipMemcpyAsync(ycol.p, Yown->col.data(), 4 * nnzo, hipMemcpyHostToDevice, s));
        HIPC(hipMemcpyAsync(yv.p, Yown->val.data(), 8 * nnzo, hipMemcpyHostToDevice, s));
    }
    if (nnzg > 0) {
        HIPC(hipMemcpyAsync(ycol.p + nnzo, Yghost->col.data(), 4 * nnzg, hipMemcpyHostToDevice, s));
        HIPC(hipMemcpyAsync(yv.p + nnzo, Yghost->val.data(), 8 * nnzg, hipMemcpyHostToDevice, s));
    }
    CHECK(h2d(gids, ghost_ids, ng, s));
    CHECK(flags.alloc(kF));
    HIPC(hipMemsetAsync(flags.p, 0, sizeof(int) * kF, s));

    CHECK(xr.alloc(nnzx));
    if (nnzx > 0)
        hipLaunchKernelGGL(k_map_rows, dim3(grid_for(nnzx)), dim3(256), 0, s, xcol.p, nnzx, y0,
                           ny, gids.p, ng, xr.p, flags.p);
    CHECK(m.alloc(n));
    CHECK(bin.alloc(n));
    if (n > 0)
        hipLaunchKernelGGL(k_row_products, dim3(grid_for(n)), dim3(256), 0, s, xrp.p, xr.p,
                           yrp.p, n, nc, m.p, bin.p, flags.p + 1);
    HIPC(hipGetLastError());
    std::vector<int> hf(kF);
    HIPC(hipMemcpyAsync(hf.data(), flags.p, sizeof(int) * kF, hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    if (hf[0] > 0)
        return fail(PAMG_E_ARG,
                    "spgemm: %d column ids of X reference rows that are neither own nor ghost",
                    hf[0]);
    std::vector<int64_t> off(kBins + 2, 0);
    for (int b = 0; b <= kBins; ++b) off[b + 1] = off[b] + hf[1 + b];
    CHECK(h2d(binoff, off.data(), kBins + 2, s));
    CHECK(lists.alloc(off[kBins]));
    if (n > 0)
        hipLaunchKernelGGL(k_scatter_bins, dim3(grid_for(n)), dim3(256), 0, s, bin.p, n,
                           binoff.p, flags.p + 2 + kBins, lists.p);

    SgArgs A{xrp.p, xr.p, xv.p, yrp.p, ycol.p, yv.p, nullptr, nullptr, nullptr, nullptr};
    CHECK(cnt.alloc(n));
    A.cnt = cnt.p;
    CHECK(launch_bins(false, A, lists.p, off, s));

    // rows whose distinct columns overflowed an LDS table
    CHECK(crp.alloc(n + 1));
    CHECK(ovf.alloc(std::max<int64_t>(off[kBins] - off[kBins - 1], 1)));
    int* d_novf = flags.p + kF - 1;
    if (n > 0)
        hipLaunchKernelGGL(k_counts_i64, dim3(grid_for(n)), dim3(256), 0, s, cnt.p, bin.p, n,
                           crp.p + 1, ovf.p, d_novf);
    int novf = 0;
    HIPC(hipMemcpyAsync(&novf, d_novf, sizeof(int), hipMemcpyDeviceToHost, s));
    HIPC(hipStreamSynchronize(s));
    std::vector<int32_t> hovf(novf);
    // The global tables' offsets go to the device by an asynchronous copy that k_sg_glob reads on
    // the stream, so their host copy must outlive the copy: it lives until the final stream
    // synchronisation below. (It was a local of this if-block once: freed while the copy from
    // pageable memory could still be pending, which under contention — 8 ranks sharing one GPU —
    // gave k_sg_glob garbage table bounds and a tail level without its diagonal; DESIGN.md.)
    std::vector<int64_t> wo;
    if (novf > 0) {
        HIPC(hipMemcpy(hovf.data(), ovf.p, 4 * (size_t)novf, hipMemcpyDeviceToHost));
        std::vector<int64_t> hm(n);
        HIPC(hipMemcpy(hm.data(), m.p, 8 * (size_t)n, hipMemcpyDeviceToHost));
        wo.assign(novf + 1, 0);
        for (int r = 0; r < novf; ++r)
            wo[r + 1] = wo[r] + (int64_t)next_pow2(2 * (uint64_t)std::min(hm[hovf[r]], nc));
        CHECK(h2d(woff, wo.data(), novf + 1, s));
        CHECK(wkey.alloc(wo[novf]));
        CHECK(wacc.alloc(wo[novf]));
        hipLaunchKernelGGL(k_sg_glob<false>, dim3(novf), dim3(64), 0, s, A, ovf.p, woff.p,
                           wkey.p, wacc.p);
        HIPC(hipGetLastError());
        // the global pass always fits (T >= 2 min(m, ncols)); fold its counts in
        hipLaunchKernelGGL(k_counts_i64, dim3(grid_for(n)), dim3(256), 0, s, cnt.p, bin.p, n,
                           crp.p + 1, nullptr, nullptr);
    }
    HIPC(hipMemsetAsync(crp.p, 0, sizeof(int64_t), s));
    CHECK(inclusive_scan_i64(crp.p + 1, crp.p + 1, n, s));
    int64_t nnzc = 0;
    HIPC(hipMemcpy(&nnzc, crp.p + n, sizeof(int64_t), hipMemcpyDeviceToHost));

    CHECK(ccol.alloc(nnzc));
    CHECK(cval.alloc(nnzc));
    A.crp = crp.p;
    A.ccol = ccol.p;
    A.cval = cval.p;
    CHECK(launch_bins(true, A, lists.p, off, s));
    if (novf > 0) {
        hipLaunchKernelGGL(k_sg_glob<true>, dim3(novf), dim3(64), 0, s, A, ovf.p, woff.p,
                           wkey.p, wacc.p);
        HIPC(hipGetLastError());
    }
    auto C = std::make_unique<pamg_hcsr>();
    C->nr = n;
    C->nc = nc;
    C->rp.resize(n + 1);
    C->col.resize(nnzc);
    C->val.resize(nnzc);
    HIPC(hipMemcpyAsync(C->rp.data(), crp.p, 8 * (size_t)(n + 1), hipMemcpyDeviceToHost, s));
    if (nnzc > 0) {
        HIPC(hipMemcpyAsync(C->col.data(), ccol.p, 4 * (size_t)nnzc, hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(C->val.data(), cval.p, 8 * (size_t)nnzc, hipMemcpyDeviceToHost, s));
    }
    HIPC(hipStreamSynchronize(s));
    *out = C.release();
    return PAMG_OK;
}

int dev_transpose(pamg_ctx* ctx, const pamg_hcsr* P, int64_t row0, int64_t c0, int64_t c1,
                  pamg_hcsr** out) {
    const hipStream_t s = ctx->s_comp;
    const int64_t nr = P->nr, nnz = P->nnz(), m = c1 - c0;
    if (nnz >= (int64_t)INT32_MAX || m >= (int64_t)UINT32_MAX - 1 || row0 + nr >= (int64_t)INT32_MAX)
        return fail(PAMG_E_OVERFLOW, "dev_transpose: sizes >= 2^31");
    HIPC(hipSetDevice(ctx->device));
    DBuf<int64_t> rp;
    DBuf<int32_t> col, idx, sidx, rid, rcol;
    DBuf<uint32_t> keys, skeys;
    DBuf<double> val, rval;
    DBuf<unsigned long long> cnt;
    DBuf<int64_t> rrp;
    CHECK(h2d(rp, P->rp.data(), nr + 1, s));
    CHECK(h2d(col, P->col.data(), nnz, s));
    CHECK(h2d(val, P->val.data(), nnz, s));
    CHECK(keys.alloc(nnz));
    CHECK(skeys.alloc(nnz));
    CHECK(idx.alloc(nnz));
    CHECK(sidx.alloc(nnz));
    CHECK(rid.alloc(nnz));
    CHECK(cnt.alloc(m + 1));
    CHECK(rrp.alloc(m + 1));
    HIPC(hipMemsetAsync(cnt.p, 0, 8 * (size_t)(m + 1), s));
    if (nr > 0)
        hipLaunchKernelGGL(k_tr_keys, dim3(grid_for(nr)), dim3(256), 0, s, rp.p, col.p, nr, c0,
                           c1, keys.p, idx.p, rid.p, cnt.p);
    HIPC(hipGetLastError());
    if (nnz > 0) {
        int bits = 1;
        while (bits < 32 && (uint64_t(1) << bits) <= (uint64_t)m) ++bits;
        size_t bytes = 0;
        HIPC(hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, keys.p, skeys.p, idx.p, sidx.p,
                                                (int)nnz, 0, bits, s));
        DBuf<char> tmp;
        CHECK(tmp.alloc((int64_t)bytes + 1));
        HIPC(hipcub::DeviceRadixSort::SortPairs(tmp.p, bytes, keys.p, skeys.p, idx.p, sidx.p,
                                                (int)nnz, 0, bits, s));
        HIPC(hipStreamSynchronize(s));
    }
    HIPC(hipMemsetAsync(rrp.p, 0, sizeof(int64_t), s));
    CHECK(inclusive_scan_i64(reinterpret_cast<const int64_t*>(cnt.p), rrp.p + 1, m, s));
    int64_t nnzr = 0;
    HIPC(hipMemcpy(&nnzr, rrp.p + m, sizeof(int64_t), hipMemcpyDeviceToHost));
    CHECK(rcol.alloc(nnzr));
    CHECK(rval.alloc(nnzr));
    if (nnzr > 0)
        hipLaunchKernelGGL(k_tr_fill, dim3(grid_for(nnzr)), dim3(256), 0, s, sidx.p, rid.p,
                           val.p, nnzr, row0, rcol.p, rval.p);
    HIPC(hipGetLastError());
    auto R = std::make_unique<pamg_hcsr>();
    R->nr = m;
    R->nc = row0 + nr;
    R->rp.resize(m + 1);
    R->col.resize(nnzr);
    R->val.resize(nnzr);
    HIPC(hipMemcpyAsync(R->rp.data(), rrp.p, 8 * (size_t)(m + 1), hipMemcpyDeviceToHost, s));
    if (nnzr > 0) {
        HIPC(hipMemcpyAsync(R->col.data(), rcol.p, 4 * (size_t)nnzr, hipMemcpyDeviceToHost, s));
        HIPC(hipMemcpyAsync(R->val.data(), rval.p, 8 * (size_t)nnzr, hipMemcpyDeviceToHost, s));
    }
    HIPC(hipStreamSynchronize(s));
    *out = R.release();
    return PAMG_OK;
}

}  // namespace

extern "C" {

int pamg_dev_spgemm(pamg_ctx* ctx, const pamg_hcsr* X, int64_t y0, const pamg_hcsr* Yown,
                    const int64_t* ghost_ids, int64_t n_ghost, const pamg_hcsr* Yghost,
                    pamg_hcsr** out) {
    if (!ctx || !valid(X) || !valid(Yown) || !out) return fail(PAMG_E_ARG, "dev_spgemm: bad args");
    if (n_ghost > 0 && (!ghost_ids || !valid(Yghost) || Yghost->nr != n_ghost))
        return fail(PAMG_E_ARG, "dev_spgemm: ghost rows missing");
    try {
        return dev_spgemm(ctx, X, y0, Yown, ghost_ids, n_ghost, Yghost, out);
    } catch (...) {
        return fail(PAMG_E_NOMEM, "dev_spgemm: out of host memory");
    }
}

int pamg_dev_transpose(pamg_ctx* ctx, const pamg_hcsr* P, int64_t row0, int64_t c0, int64_t c1,
                       pamg_hcsr** out) {
    if (!ctx || !valid(P) || !out || c1 < c0) return fail(PAMG_E_ARG, "dev_transpose: bad args");
    try {
        return dev_transpose(ctx, P, row0, c0, c1, out);
    } catch (...) {
        return fail(PAMG_E_NOMEM, "dev_transpose: out of host memory");
    }
}

}  // extern "C"
