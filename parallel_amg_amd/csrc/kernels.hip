// kernels.hip — gfx950 (CDNA4) kernels of the AMG V-cycle solve path.
//
// Every row-sum kernel implements SPEC.md §S3 exactly: products p = a*x rounded, summed
// left to right in storage order from +0.0, never fused (built with -ffp-contract=off), so
// results are bit-identical to the CPU oracle and run-to-run deterministic.
//
// CSR row kernel (k_rows_tile): the path is HBM-bound sparse work (12 B/nnz of matrix
// stream + vectors, ~0.17 flop/B), so there is no MFMA here. One 256-thread workgroup takes
// a tile of <= 256 consecutive rows / <= 2048 nonzeros:
//   phase 0  the tile's row pointers -> LDS;
//   phase 1  the tile's columns/values are streamed with 16-byte loads (int4 / 2x double2
//            per lane, fully coalesced, 1 KiB per wave-instruction), each lane gathers its
//            four x[col] and writes the four products to LDS (the "LDS-staged partial
//            sums"); for Jacobi the lane that holds a row's diagonal stores it in LDS;
//   phase 2  one lane per row adds its products from LDS in storage order and applies the
//            epilogue (SpMV / residual / Jacobi / prolongate-add), coalesced stores.
// Rows longer than the tile budget go to k_rows_long (one workgroup per row, chunked).
//
// Variants of that tile body (pamg_set_option; the upload fixes the layout per tile set,
// launch_tile2 picks the kernel; every variant is bit-identical, tests/test_gpu_parity.py):
//   0  k_rows_tile    row pointers first, then the stream (first version)
//   1  k_rows_tile2   descriptor-driven: the stream is issued at entry from the tile's nonzero
//                     range; 24-bit columns, 8-bit row lengths, column / value dictionaries
//   4  k_rows_tm      tile-major slots: every pre-gather load addressed by tile index alone
//                     (default for dictionary sets and slot-filling non-square operators)
//   2, 3, 4p, 4f      wave tiles, persistent grids, one-barrier row flags: measured slower,
//                     kept for A/B ("Measured and rejected")
#include <type_traits>

#include "pamg_device.h"

namespace pamg {
namespace {

template <int OP>
__device__ __forceinline__ void epilogue(int r, double s, const double* __restrict__ x,
                                         const double* __restrict__ b, double* __restrict__ y,
                                         double omega, double d) {
    if constexpr (OP == OP_SPMV) {
        y[r] = s;
    } else if constexpr (OP == OP_RESID) {
        y[r] = b[r] - s;
    } else if constexpr (OP == OP_JACOBI) {
        const double u = b[r] - s;
        const double v = omega * u;
        const double w = v / d;
        y[r] = x[r] + w;
    } else {
        y[r] = y[r] + s;
    }
}

// Sum of lp[kb..ke) left to right from +0.0 (SPEC §S3). The chain of dependent fp64 adds is
// what bounds the long rows of the coarse operators, so nothing else may sit on it: full
// batches of 8 are read unconditionally (no exec-masked branches) and software-pipelined —
// batch m+1's LDS reads are in flight while batch m is added. The last, partial batch reads
// 8 slots (callers pad lp by 8) and selects +0.0 past the row end, which leaves the sum's
// bits unchanged: a sum started at +0.0 is never -0.0, and s + (+0.0) == s for every other s.
__device__ __forceinline__ void lds_batch8(const double* __restrict__ lp, int k, double (&p)[8]) {
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = lp[k + j];
}

__device__ __forceinline__ double row_sum_lds(const double* __restrict__ lp, int kb, int ke,
                                              double s = 0.0) {
    int k = kb;
    if (k + 8 <= ke) {
        // two register batches in alternation (no copies): p is added while q is read
        double p[8], q[8];
        lds_batch8(lp, k, p);
        k += 8;
        while (true) {
            if (k + 8 > ke) {
#pragma unroll
                for (int j = 0; j < 8; ++j) s = s + p[j];
                break;
            }
            lds_batch8(lp, k, q);
            k += 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) s = s + p[j];
            if (k + 8 > ke) {
#pragma unroll
                for (int j = 0; j < 8; ++j) s = s + q[j];
                break;
            }
            lds_batch8(lp, k, p);
            k += 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) s = s + q[j];
        }
    }
    if (k < ke) {
        double p[8];
        lds_batch8(lp, k, p);
#pragma unroll
        for (int j = 0; j < 8; ++j) s = s + ((k + j < ke) ? p[j] : 0.0);
    }
    return s;
}

// Variant 0 (first version, kept for A/B): row pointers first, then the column stream.
template <int OP>
__global__ __launch_bounds__(kBlock) void k_rows_tile(
    const int4* __restrict__ tiles, const int* __restrict__ rowptr, const int* __restrict__ col,
    const double* __restrict__ val, const double* __restrict__ x, const double* __restrict__ b,
    double* __restrict__ y, double omega) {
    __shared__ __attribute__((aligned(16))) double lprod[kTileNnz + 8];
    __shared__ int lrp[kTileRows + 1];
    __shared__ double ldiag[OP == OP_JACOBI ? kTileRows : 1];

    const int tid = threadIdx.x;
    const int4 t = tiles[blockIdx.x];
    const int r0 = t.x, nr = t.y - t.x;
    for (int i = tid; i <= nr; i += kBlock) lrp[i] = rowptr[r0 + i];
    __syncthreads();
    const int z0 = lrp[0], z1 = lrp[nr];
    const int za = z0 & ~3;  // 16-byte aligned start of the column stream

    for (int g = za + 4 * tid; g < z1; g += 4 * kBlock) {
        const int4 c4 = *reinterpret_cast<const int4*>(col + g);
        const double2 va = *reinterpret_cast<const double2*>(val + g);
        const double2 vb = *reinterpret_cast<const double2*>(val + g + 2);
        const int cc[4] = {c4.x, c4.y, c4.z, c4.w};
        const double vv[4] = {va.x, va.y, vb.x, vb.y};
        double p[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int k = g + e;
            const bool ok = (k >= z0) & (k < z1);
            p[e] = ok ? vv[e] * x[cc[e]] : 0.0;
            if constexpr (OP == OP_JACOBI) {
                const int rl = cc[e] - r0;  // own column id == local row id of its diagonal
                if (ok && rl >= 0 && rl < nr && k >= lrp[rl] && k < lrp[rl + 1]) ldiag[rl] = vv[e];
            }
        }
        *reinterpret_cast<double2*>(&lprod[g - za]) = make_double2(p[0], p[1]);
        *reinterpret_cast<double2*>(&lprod[g - za + 2]) = make_double2(p[2], p[3]);
    }
    __syncthreads();
    if (tid < nr) {
        const int r = r0 + tid;
        const int kb = lrp[tid] - za, ke = lrp[tid + 1] - za;
        const double s = row_sum_lds(lprod, kb, ke);
        epilogue<OP>(r, s, x, b, y, omega, OP == OP_JACOBI ? ldiag[tid] : 0.0);
    }
}

// Variant 1: the tile descriptor carries its nonzero range, so the column/value stream of
// every lane (TNNZ / 1024 groups of 4 nonzeros: one int4 + two double2 loads each) is issued
// at kernel entry together with the row-pointer slice; all x gathers of a lane are then
// issued back to back (branch-free: invalid lanes gather x[0] and discard it) before the
// products go to LDS. XCD=true maps contiguous tile chunks to each XCD (blocks b and b+8
// share an XCD) so neighbouring tiles' x lines stay in one L2.
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ int4 stream_load(const int4* p, std::true_type /*nt*/) {
    const i32x4 v = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(p));
    return make_int4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ double2 stream_load(const double2* p, std::true_type /*nt*/) {
    const f64x2 v = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p));
    return make_double2(v.x, v.y);
}
template <class T>
__device__ __forceinline__ T stream_load(const T* p, std::false_type) {
    return *p;
}

template <int OP, int TNNZ, int TROWS, bool XCD, bool NT = false, int BS = kBlock, bool C24 = false,
          bool VD = false, bool RL8 = false, int CD = 0>
__global__ __launch_bounds__(BS) void k_rows_tile2(
    const int4* __restrict__ tiles, int ntiles, const int* __restrict__ rowptr,
    const int* __restrict__ col, const double* __restrict__ val, const double* __restrict__ x,
    const double* __restrict__ b, double* __restrict__ y, double omega,
    const double* __restrict__ diag, const uint16_t* __restrict__ clo = nullptr,
    const uint8_t* __restrict__ chi = nullptr, const int* __restrict__ tbase = nullptr,
    const uint8_t* __restrict__ vidx = nullptr, const double* __restrict__ vtab = nullptr,
    const uint8_t* __restrict__ rlen = nullptr, const uint8_t* __restrict__ cidx = nullptr,
    const int* __restrict__ ctab = nullptr, int ctab_n = 0) {
    // C24: the column stream is 3 B/nonzero — per-tile base + 16-bit low part (8 B per lane)
    // + 8-bit high part (4 B per lane) instead of the 16-B int4 of 32-bit ids.
    // VD (opt-in): values are 4-bit indices (2 B per lane) into the tile's 16-value table,
    // read through L1 (the same 128 B for every lane of the tile) — exact fp64 values.
    // diag != nullptr (Jacobi only): a_ii from the stored diagonal instead of the in-tile
    // detection (same value, SPEC §S3; trades 8 B/row of reads for one barrier).
    constexpr int G = TNNZ / (4 * BS);
    static_assert(G >= 1 && TNNZ % (4 * BS) == 0, "tile budget must be a multiple of 4 x block");
    __shared__ __attribute__((aligned(16))) double lprod[TNNZ + 8];
    __shared__ int lrp[TROWS + 1];
    __shared__ double ldiag[OP == OP_JACOBI ? TROWS : 1];
    // RL8: row lengths are 8-bit (1 B/row instead of a 4-B row pointer); the row starts are
    // rebuilt from the tile's first nonzero by a wave-level scan + the wave totals (lwt)
    static_assert(!RL8 || TROWS <= BS, "8-bit row lengths: one row per lane");
    __shared__ int lwt[RL8 ? BS / 64 : 1];
    // CD (column dictionary, 4 or 8 bits per nonzero): column = row + ctab[index], with the
    // tile set's <= 16 / <= 256 distinct offsets (a stencil's 7 for A0) in LDS; every
    // position's row (lrow, tile-local) is marked by the lane that owns the row (RL8 scan)
    static_assert(CD == 0 || (RL8 && !C24 && !VD), "column dictionary: 8-bit rows, plain values");
    __shared__ int ltab[CD == 8 ? 256 : 16];
    __shared__ __attribute__((aligned(4))) uint8_t lrow[CD ? TNNZ + 8 : 4];

    int bid = blockIdx.x;
    if constexpr (XCD) {
        const int per = (ntiles + 7) >> 3;
        bid = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
        if (bid >= ntiles) return;
    }
    const int tid = threadIdx.x;
    const int4 t = tiles[bid];
    const int r0 = t.x, nr = t.y - t.x, z0 = t.z, z1 = t.w;
    const int za = z0 & ~3;

    int4 c4[G];
    double2 va[G], vb[G];
    uint16_t vn[G];  // VD: four 4-bit value indices per lane group
    uint32_t cn[G];  // CD: four 4- or 8-bit column dictionary indices per lane group
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int g = za + 4 * (tid + j * BS);
        const int gs = g < z1 ? g : za;  // clamp: never read past the (padded) arrays
        // NT: the once-read matrix stream goes non-temporal so the x lines (reused by the
        // z+-1 / y+-1 neighbour rows) keep their place in the XCD's L2
        using nt = std::integral_constant<bool, NT>;
        if constexpr (CD == 4) {
            cn[j] = *reinterpret_cast<const uint16_t*>(cidx + (gs >> 1));
        } else if constexpr (CD == 8) {
            cn[j] = *reinterpret_cast<const uint32_t*>(cidx + gs);
        } else if constexpr (C24) {
            const ushort4 lo = *reinterpret_cast<const ushort4*>(clo + gs);
            const uchar4 hi = *reinterpret_cast<const uchar4*>(chi + gs);
            const int cb = tbase[bid];
            c4[j] = make_int4(cb + (int)((uint32_t)lo.x | ((uint32_t)hi.x << 16)),
                              cb + (int)((uint32_t)lo.y | ((uint32_t)hi.y << 16)),
                              cb + (int)((uint32_t)lo.z | ((uint32_t)hi.z << 16)),
                              cb + (int)((uint32_t)lo.w | ((uint32_t)hi.w << 16)));
        } else {
            c4[j] = stream_load(reinterpret_cast<const int4*>(col + gs), nt{});
        }
        if constexpr (VD) {
            vn[j] = *reinterpret_cast<const uint16_t*>(vidx + (gs >> 1));
        } else {
            va[j] = stream_load(reinterpret_cast<const double2*>(val + gs), nt{});
            vb[j] = stream_load(reinterpret_cast<const double2*>(val + gs + 2), nt{});
        }
    }
    int rl_len = 0, rl_inc = 0;  // RL8: this lane's row length and wave-inclusive length sum
    if constexpr (RL8) {
        const int lane = tid & 63;
        rl_len = tid < nr ? (int)rlen[r0 + tid] : 0;
        rl_inc = rl_len;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int u = __shfl_up(rl_inc, off, 64);
            if (lane >= off) rl_inc += u;
        }
        if (lane == 63) lwt[tid >> 6] = rl_inc;
    } else {
        for (int i = tid; i <= nr; i += BS) lrp[i] = rowptr[r0 + i];
    }
    // row start of this lane's row (RL8, after a barrier has published lwt)
    auto rl_base = [&]() {
        int pre = z0;
#pragma unroll
        for (int q = 0; q < BS / 64; ++q) pre += q < (tid >> 6) ? lwt[q] : 0;
        return pre;
    };
    // one row per lane: fetch the epilogue's own-row operands (b, old x, y, a_ii) now, so
    // their latency hides under the column stream instead of trailing the LDS phase
    constexpr bool ONE_ROW = TROWS <= BS;
    double pb = 0.0, px = 0.0, py = 0.0, pd = 0.0;
    if constexpr (ONE_ROW) {
        if (tid < nr) {
            const int r = r0 + tid;
            if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[r];
            if constexpr (OP == OP_JACOBI) {
                px = x[r];
                if (diag) pd = diag[r];
            }
            if constexpr (OP == OP_PROLONG) py = y[r];
        }
    }
    if constexpr (CD != 0) {
        if (tid < ctab_n) ltab[tid] = ctab[tid];
        __syncthreads();  // lwt, ltab
        if (tid < nr) {
            const int e = rl_base() + rl_inc - za;
            for (int p = e - rl_len; p < e; ++p) lrow[p] = (uint8_t)tid;
        }
        __syncthreads();  // lrow
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int q = 4 * (tid + j * BS);
            const uint32_t rw = za + q < z1 ? *reinterpret_cast<const uint32_t*>(&lrow[q]) : 0u;
            int cc[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int ix = CD == 4 ? (int)((cn[j] >> (4 * e)) & 15u) : (int)((cn[j] >> (8 * e)) & 255u);
                cc[e] = r0 + (int)((rw >> (8 * e)) & 255u) + ltab[ix];
            }
            c4[j] = make_int4(cc[0], cc[1], cc[2], cc[3]);
        }
    } else if constexpr (OP == OP_JACOBI) {
        if (!diag) {
            __syncthreads();
            if constexpr (RL8) {  // the in-tile diagonal search needs every row's bounds
                const int base = rl_base();
                if (tid == 0) lrp[0] = z0;
                if (tid < TROWS) lrp[tid + 1] = base + rl_inc;
                __syncthreads();
            }
        }
    }

    double xv[G][4];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int g = za + 4 * (tid + j * BS);
        const int cc[4] = {c4[j].x, c4[j].y, c4[j].z, c4[j].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool ok = (g + e >= z0) & (g + e < z1);
            xv[j][e] = x[ok ? cc[e] : 0];
        }
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int g = za + 4 * (tid + j * BS);
        const int cc[4] = {c4[j].x, c4[j].y, c4[j].z, c4[j].w};
        double vv[4];
        if constexpr (VD) {
            const double* tt = vtab + 16 * (size_t)bid;
#pragma unroll
            for (int e = 0; e < 4; ++e) vv[e] = tt[(vn[j] >> (4 * e)) & 15];
        } else {
            vv[0] = va[j].x;
            vv[1] = va[j].y;
            vv[2] = vb[j].x;
            vv[3] = vb[j].y;
        }
        double p[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int k = g + e;
            const bool ok = (k >= z0) & (k < z1);
            p[e] = ok ? vv[e] * xv[j][e] : 0.0;
            if constexpr (OP == OP_JACOBI) {
                const int rl = cc[e] - r0;
                if constexpr (CD != 0) {
                    // the diagonal is the entry whose column is its own row
                    if (!diag && ok && rl == (int)lrow[k - za]) ldiag[rl] = vv[e];
                } else {
                    if (!diag && ok && rl >= 0 && rl < nr && k >= lrp[rl] && k < lrp[rl + 1])
                        ldiag[rl] = vv[e];
                }
            }
        }
        *reinterpret_cast<double2*>(&lprod[g - za]) = make_double2(p[0], p[1]);
        *reinterpret_cast<double2*>(&lprod[g - za + 2]) = make_double2(p[2], p[3]);
    }
    __syncthreads();
    if constexpr (ONE_ROW) {
        if (tid < nr) {
            int kb, ke;
            if constexpr (RL8) {
                const int base = rl_base();
                kb = base + rl_inc - rl_len - za;
                ke = base + rl_inc - za;
            } else {
                kb = lrp[tid] - za;
                ke = lrp[tid + 1] - za;
            }
            const double s = row_sum_lds(lprod, kb, ke);
            const int r = r0 + tid;
            if constexpr (OP == OP_SPMV) {
                y[r] = s;
            } else if constexpr (OP == OP_RESID) {
                y[r] = pb - s;
            } else if constexpr (OP == OP_JACOBI) {
                const double d = diag ? pd : ldiag[tid];
                const double u = pb - s;
                const double v = omega * u;
                const double w = v / d;
                y[r] = px + w;
            } else {
                y[r] = py + s;
            }
        }
    } else {
        for (int rr = tid; rr < nr; rr += BS) {
            const int kb = lrp[rr] - za, ke = lrp[rr + 1] - za;
            const double s = row_sum_lds(lprod, kb, ke);
            double d = 0.0;
            if constexpr (OP == OP_JACOBI) d = diag ? diag[r0 + rr] : ldiag[rr];
            epilogue<OP>(r0 + rr, s, x, b, y, omega, d);
        }
    }
}

// Variant 4, tile-major (TileSet::tm): tile t's values, column stream and row lengths live at
// fixed slots of padded per-set arrays — values/columns at t*TNNZ, row lengths at t*rs — so
// every load a block needs before its x gathers is addressed from blockIdx alone and issued
// at entry beside the descriptor load. Variant 1 has to wait for the descriptor (its nonzero
// range) before it can issue the stream, one dependent memory round trip more per tile.
// Columns: CD = 4 / 8, row + table[index] (column dictionary); CD = 0, tile base + 24-bit
// (16-bit low + 8-bit high) offset. Rows: one per lane, starts by a wave scan of the lengths;
// positions are tile-relative (no alignment head: a tile's slot starts at its first nonzero).
// Summation order, epilogues and Jacobi's in-tile diagonal are variant 1's (SPEC §S3).
// x prefetch (dictionary sets, pf_lo/pf_hi != 0): the tile's rows read x at row + offset for
// the set's offsets, so the lines of its farthest neighbours — [r0 + pf_lo, r0 + pf_lo + nr)
// and [r0 + pf_hi, ...), the grid planes below and above — are known from the descriptor.
// A few lanes load one word per 128-B line of both ranges at entry, beside the stream: the
// first touch of the plane above (a compulsory HBM miss) and the re-read of the plane below
// (evicted from L2 two plane slices ago) then overlap the stream instead of following it in
// the gather phase. The loaded words feed a never-taken store (poison is NaN) so the loads
// are kept; any index is clamped into [0, xlen).
template <int OP, int TNNZ, int CD, bool TR = false>
__global__ __launch_bounds__(kBlock) void k_rows_tm(
    const int4* __restrict__ tiles, const double* __restrict__ tval,
    const uint8_t* __restrict__ tcidx, const uint16_t* __restrict__ tclo,
    const uint8_t* __restrict__ tchi, const int* __restrict__ tbase,
    const uint8_t* __restrict__ trlen, int rs, const int* __restrict__ ctab, int ctab_n,
    const double* __restrict__ x, const double* __restrict__ b, double* __restrict__ y,
    double omega, const double* __restrict__ diag, int pf_lo = 0, int pf_hi = 0, int xlen = 0,
    double poison = __builtin_nan("")) {
    constexpr int BS = kBlock;
    constexpr int G = TNNZ / (4 * BS);
    static_assert(G >= 1 && TNNZ % (4 * BS) == 0, "tile budget must be a multiple of 4 x block");
    __shared__ __attribute__((aligned(16))) double lprod[TNNZ + 8];
    __shared__ double ldiag[OP == OP_JACOBI ? BS : 1];
    __shared__ int lwt[BS / 64];
    __shared__ int ltab[CD == 8 ? 256 : 16];
    __shared__ __attribute__((aligned(4))) uint8_t lrow[TNNZ + 8];

    const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    // slot position of this lane's e-th nonzero in group j: four consecutive positions per
    // lane (16-B loads), or TR: lane-consecutive positions per gather instruction (8-B loads;
    // an instruction's 64 gathers then come from ~9 rows instead of ~36: fewer x lines)
    auto pos = [&](int j, int e) {
        return TR ? 4 * (j * BS + 64 * (tid >> 6)) + 64 * e + lane : 4 * (tid + j * BS) + e;
    };
    const int4 d = tiles[t];
    const size_t sb = (size_t)t * TNNZ;
    double2 va[G], vb[G];
    uint32_t cn[G];
    ushort4 clo4[G];
    int cb = 0;
    if constexpr (CD == 0) cb = tbase[t];
    // the whole slot is loaded at entry (padding included: a load that waits for the
    // descriptor's nonzero count brings its round trip back — measured 2-15 % slower)
    auto load = [&](int j) {
        if constexpr (TR) {
            double v[4];
            uint32_t c = 0;
            uint16_t l[4] = {0, 0, 0, 0};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const size_t g = sb + pos(j, e);
                v[e] = tval[g];
                if constexpr (CD == 4) {
                    c |= (uint32_t)((tcidx[g >> 1] >> (4 * (g & 1))) & 15u) << (4 * e);
                } else if constexpr (CD == 8) {
                    c |= (uint32_t)tcidx[g] << (8 * e);
                } else {
                    l[e] = tclo[g];
                    c |= (uint32_t)tchi[g] << (8 * e);
                }
            }
            va[j] = make_double2(v[0], v[1]);
            vb[j] = make_double2(v[2], v[3]);
            cn[j] = c;
            clo4[j] = make_ushort4(l[0], l[1], l[2], l[3]);
            return;
        }
        const size_t q = sb + 4 * (tid + j * BS);
        va[j] = *reinterpret_cast<const double2*>(tval + q);
        vb[j] = *reinterpret_cast<const double2*>(tval + q + 2);
        if constexpr (CD == 4) {
            cn[j] = *reinterpret_cast<const uint16_t*>(tcidx + (q >> 1));
        } else if constexpr (CD == 8) {
            cn[j] = *reinterpret_cast<const uint32_t*>(tcidx + q);
        } else {  // 24-bit: low 16 bits per nonzero + the four high bytes packed in cn
            clo4[j] = *reinterpret_cast<const ushort4*>(tclo + q);
            cn[j] = *reinterpret_cast<const uint32_t*>(tchi + q);
        }
    };
#pragma unroll
    for (int j = 0; j < G; ++j) load(j);
    int rl_len = tid < rs ? (int)trlen[(size_t)t * rs + tid] : 0;
    if constexpr (CD != 0) {
        if (tid < ctab_n) ltab[tid] = ctab[tid];
    }
    int rl_inc = rl_len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(rl_inc, off, 64);
        if (lane >= off) rl_inc += u;
    }
    if (lane == 63) lwt[tid >> 6] = rl_inc;
    const int r0 = d.x, nr = d.y - d.x, cnt = d.w - d.z;
    double touch = 0.0;
    if constexpr (CD != 0) {
        if (pf_hi != 0) {
            const int nl = (nr + 15) / 16 + 1;  // 128-B lines of one nr-row range
            if (tid < 2 * nl) {
                const int base = r0 + (tid < nl ? pf_lo : pf_hi);
                int i = base + 16 * (tid < nl ? tid : tid - nl);
                i = i < 0 ? 0 : (i >= xlen ? xlen - 1 : i);
                touch = x[i];
            }
        }
    }
    double pb = 0.0, px = 0.0, py = 0.0, pd = 0.0;
    if (tid < nr) {
        const int r = r0 + tid;
        if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[r];
        if constexpr (OP == OP_JACOBI) {
            px = x[r];
            if (diag) pd = diag[r];
        }
        if constexpr (OP == OP_PROLONG) py = y[r];
    }
    // end of this lane's row (tile-relative): the wave's inclusive sum + the earlier waves'
    // totals, readable after the next barrier
    auto row_end = [&]() {
        int pre = 0;
#pragma unroll
        for (int q = 0; q < BS / 64; ++q) pre += q < (tid >> 6) ? lwt[q] : 0;
        return pre + rl_inc;
    };
    // Per-position row ids are needed for dictionary columns (row + offset) and for Jacobi's
    // in-tile diagonal; 24-bit SpMV / residual / prolongate-add skip them, so their gathers
    // follow the stream loads with no barrier in between.
    constexpr bool NEED_ROWS = CD != 0 || OP == OP_JACOBI;
    int re = 0;
    if constexpr (NEED_ROWS) {
        __syncthreads();  // lwt, ltab
        re = row_end();
        if (tid < nr)
            for (int p = re - rl_len; p < re; ++p) lrow[p] = (uint8_t)tid;
        __syncthreads();  // lrow
    }

    double xv[G][4];
    int cc[G][4];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int q = 4 * (tid + j * BS);
        uint32_t rw = 0u;
        if constexpr (NEED_ROWS) {
            if constexpr (TR) {
#pragma unroll
                for (int e = 0; e < 4; ++e) rw |= (uint32_t)lrow[pos(j, e)] << (8 * e);
            } else {
                rw = q < cnt ? *reinterpret_cast<const uint32_t*>(&lrow[q]) : 0u;
            }
        }
        if constexpr (CD == 0) {
            const uint16_t l4[4] = {clo4[j].x, clo4[j].y, clo4[j].z, clo4[j].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                cc[j][e] = cb + (int)((uint32_t)l4[e] | (((cn[j] >> (8 * e)) & 255u) << 16));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int ix = CD == 4 ? (int)((cn[j] >> (4 * e)) & 15u) : (int)((cn[j] >> (8 * e)) & 255u);
                cc[j][e] = r0 + (int)((rw >> (8 * e)) & 255u) + ltab[ix];
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[j][e] = x[pos(j, e) < cnt ? cc[j][e] : 0];
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int q = 4 * (tid + j * BS);
        uint32_t rw = 0u;
        if constexpr (NEED_ROWS) {
            if constexpr (TR) {
#pragma unroll
                for (int e = 0; e < 4; ++e) rw |= (uint32_t)lrow[pos(j, e)] << (8 * e);
            } else {
                rw = q < cnt ? *reinterpret_cast<const uint32_t*>(&lrow[q]) : 0u;
            }
        }
        const double vv[4] = {va[j].x, va[j].y, vb[j].x, vb[j].y};
        double p[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool ok = pos(j, e) < cnt;
            p[e] = ok ? vv[e] * xv[j][e] : 0.0;
            if constexpr (OP == OP_JACOBI) {
                const int rl = (int)((rw >> (8 * e)) & 255u);
                if (!diag && ok && cc[j][e] - r0 == rl) ldiag[rl] = vv[e];
            }
        }
        if constexpr (TR) {
#pragma unroll
            for (int e = 0; e < 4; ++e) lprod[pos(j, e)] = p[e];
        } else {
            *reinterpret_cast<double2*>(&lprod[q]) = make_double2(p[0], p[1]);
            *reinterpret_cast<double2*>(&lprod[q + 2]) = make_double2(p[2], p[3]);
        }
    }
    __syncthreads();
    if constexpr (!NEED_ROWS) re = row_end();
    if (tid < nr) {
        const double s = row_sum_lds(lprod, re - rl_len, re);
        const int r = r0 + tid;
        if constexpr (OP == OP_SPMV) {
            y[r] = s;
        } else if constexpr (OP == OP_RESID) {
            y[r] = pb - s;
        } else if constexpr (OP == OP_JACOBI) {
            const double dd = diag ? pd : ldiag[tid];
            const double u = pb - s;
            const double v = omega * u;
            const double w = v / dd;
            y[r] = px + w;
        } else {
            y[r] = py + s;
        }
    }
    if constexpr (CD != 0) {
        if (touch == poison) y[0] = touch;  // never: poison is NaN (keeps the prefetch loads)
    }
}

// Variant 4f (TileSet::tm_flags): variant 4 with row-start flags instead of row lengths, so a
// tile has ONE barrier. Every nonzero of the slot carries a "first of its row" bit (tflag, 4
// bits per lane) and every wave chunk of the slot the number of rows begun before it (twb, 16
// bits per wave and lane group: a tile may hold 256 rows). A lane finds the row of each of its four nonzeros inside its
// wave — ballots of the four flag bits, counts below the lane, plus the chunk's base — so
// columns (row + table[index], the table read through L1) and x gathers follow the stream
// loads with no barrier, no scan and no LDS row map. The lane holding a row's first nonzero
// publishes the row's start in LDS with the products; after the one barrier each row's lane
// sums [start, next start) in order (SPEC §S3). Needs every row of the set non-empty.
template <int OP, int TNNZ, int CD>
__global__ __launch_bounds__(kBlock) void k_rows_tmf(
    const int4* __restrict__ tiles, const double* __restrict__ tval,
    const uint8_t* __restrict__ tcidx, const uint16_t* __restrict__ tclo,
    const uint8_t* __restrict__ tchi, const int* __restrict__ tbase,
    const uint8_t* __restrict__ tflag, const uint16_t* __restrict__ twb,
    const int* __restrict__ ctab, const double* __restrict__ x, const double* __restrict__ b,
    double* __restrict__ y, double omega, const double* __restrict__ diag) {
    constexpr int BS = kBlock;
    constexpr int G = TNNZ / (4 * BS);
    static_assert(G >= 1 && TNNZ % (4 * BS) == 0, "tile budget must be a multiple of 4 x block");
    __shared__ __attribute__((aligned(16))) double lprod[TNNZ + 8];
    __shared__ double ldiag[OP == OP_JACOBI ? BS : 1];
    __shared__ int lstart[BS + 1];

    const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int4 d = tiles[t];
    const size_t sb = (size_t)t * TNNZ;
    double2 va[G], vb[G];
    uint32_t cn[G], fl[G];
    ushort4 clo4[G];
    int wb[G];
    int cb = 0;
    if constexpr (CD == 0) cb = tbase[t];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int q = 4 * (tid + j * BS);
        const size_t g = sb + q;
        va[j] = *reinterpret_cast<const double2*>(tval + g);
        vb[j] = *reinterpret_cast<const double2*>(tval + g + 2);
        if constexpr (CD == 4) {
            cn[j] = *reinterpret_cast<const uint16_t*>(tcidx + (g >> 1));
        } else if constexpr (CD == 8) {
            cn[j] = *reinterpret_cast<const uint32_t*>(tcidx + g);
        } else {
            clo4[j] = *reinterpret_cast<const ushort4*>(tclo + g);
            cn[j] = *reinterpret_cast<const uint32_t*>(tchi + g);
        }
        fl[j] = (uint32_t)(tflag[g >> 3] >> (4 * ((q >> 2) & 1))) & 15u;
        wb[j] = twb[(size_t)t * (4 * G) + j * 4 + w];
    }
    const int r0 = d.x, nr = d.y - d.x, cnt = d.w - d.z;
    double pb = 0.0, px = 0.0, py = 0.0, pd = 0.0;
    if (tid < nr) {
        const int r = r0 + tid;
        if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[r];
        if constexpr (OP == OP_JACOBI) {
            px = x[r];
            if (diag) pd = diag[r];
        }
        if constexpr (OP == OP_PROLONG) py = y[r];
    }
    const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    double xv[G][4];
    int cc[G][4], rw[G][4];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        // rows begun before this lane's first nonzero inside the wave chunk
        int excl = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) excl += __popcll(__ballot((fl[j] >> e) & 1u) & below);
#pragma unroll
        for (int e = 0; e < 4; ++e)
            rw[j][e] = wb[j] + excl + __popc(fl[j] & ((2u << e) - 1u)) - 1;
        if constexpr (CD == 0) {
            const uint16_t l4[4] = {clo4[j].x, clo4[j].y, clo4[j].z, clo4[j].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                cc[j][e] = cb + (int)((uint32_t)l4[e] | (((cn[j] >> (8 * e)) & 255u) << 16));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int ix = CD == 4 ? (int)((cn[j] >> (4 * e)) & 15u) : (int)((cn[j] >> (8 * e)) & 255u);
                cc[j][e] = r0 + rw[j][e] + ctab[ix];
            }
        }
        const int q = 4 * (tid + j * BS);
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[j][e] = x[q + e < cnt ? cc[j][e] : 0];
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int q = 4 * (tid + j * BS);
        const double vv[4] = {va[j].x, va[j].y, vb[j].x, vb[j].y};
        double p[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool ok = q + e < cnt;
            p[e] = ok ? vv[e] * xv[j][e] : 0.0;
            if (ok && ((fl[j] >> e) & 1u)) lstart[rw[j][e]] = q + e;
            if constexpr (OP == OP_JACOBI) {
                if (!diag && ok && cc[j][e] - r0 == rw[j][e]) ldiag[rw[j][e]] = vv[e];
            }
        }
        *reinterpret_cast<double2*>(&lprod[q]) = make_double2(p[0], p[1]);
        *reinterpret_cast<double2*>(&lprod[q + 2]) = make_double2(p[2], p[3]);
    }
    if (tid == 0) lstart[nr] = cnt;
    __syncthreads();
    if (tid < nr) {
        const double s = row_sum_lds(lprod, lstart[tid], lstart[tid + 1]);
        const int r = r0 + tid;
        if constexpr (OP == OP_SPMV) {
            y[r] = s;
        } else if constexpr (OP == OP_RESID) {
            y[r] = pb - s;
        } else if constexpr (OP == OP_JACOBI) {
            const double dd = diag ? pd : ldiag[tid];
            const double u = pb - s;
            const double v = omega * u;
            const double ww = v / dd;
            y[r] = px + ww;
        } else {
            y[r] = py + s;
        }
    }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops (lgkmcnt), NOT for
// its outstanding global loads (no vmcnt), so a prefetch issued before it stays in flight.
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Variant 4p (Options::tm_persist): variant 4's tile body in a persistent grid. Block b walks
// tiles b, b+G, b+2G, ... (G a multiple of 8: the block stays on its XCD's slice of the banded
// order). Tile-major slots are addressed by tile index alone, so the NEXT tile's values,
// column stream and row lengths are issued right after the current tile's x gathers into a
// second register set (two sets in alternation, no copies: a copy would wait for the loads)
// and stay in flight through the current tile's LDS sums, epilogue and stores. Barriers are
// LDS-only (lds_barrier), so no __syncthreads() drains the prefetch.
template <int OP, int TNNZ, int CD>
struct TmSlot {
    static constexpr int G = TNNZ / (4 * kBlock);
    double2 va[G], vb[G];
    uint32_t cn[G];
    ushort4 clo4[G];
    int rl;
};

template <int OP, int TNNZ, int CD>
__device__ __forceinline__ void tm_load(int t, TmSlot<OP, TNNZ, CD>& S, int tid,
                                        const double* __restrict__ tval,
                                        const uint8_t* __restrict__ tcidx,
                                        const uint16_t* __restrict__ tclo,
                                        const uint8_t* __restrict__ tchi,
                                        const uint8_t* __restrict__ trlen, int rs) {
    constexpr int G = TmSlot<OP, TNNZ, CD>::G;
    const size_t sb = (size_t)t * TNNZ;
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const size_t q = sb + 4 * (tid + j * kBlock);
        S.va[j] = *reinterpret_cast<const double2*>(tval + q);
        S.vb[j] = *reinterpret_cast<const double2*>(tval + q + 2);
        if constexpr (CD == 4) {
            S.cn[j] = *reinterpret_cast<const uint16_t*>(tcidx + (q >> 1));
        } else if constexpr (CD == 8) {
            S.cn[j] = *reinterpret_cast<const uint32_t*>(tcidx + q);
        } else {
            S.clo4[j] = *reinterpret_cast<const ushort4*>(tclo + q);
            S.cn[j] = *reinterpret_cast<const uint32_t*>(tchi + q);
        }
    }
    S.rl = tid < rs ? (int)trlen[(size_t)t * rs + tid] : 0;
}

struct TmArgs {
    const int4* tiles;
    const double* tval;
    const uint8_t* tcidx;
    const uint16_t* tclo;
    const uint8_t* tchi;
    const int* tbase;
    const uint8_t* trlen;
    int rs;
    const double* x;
    const double* b;
    double* y;
    double omega;
    const double* diag;
};

// One tile of variant 4p from slot C; prefetches tile tn into N behind the x gathers.
template <int OP, int TNNZ, int CD>
__device__ __forceinline__ void tm_tile(const TmArgs& a, int t, TmSlot<OP, TNNZ, CD>& C, int tn,
                                        TmSlot<OP, TNNZ, CD>& N, double* lprod, double* ldiag,
                                        int* lwt, const int* ltab, uint8_t* lrow) {
    constexpr int BS = kBlock;
    constexpr int G = TmSlot<OP, TNNZ, CD>::G;
    constexpr bool NEED_ROWS = CD != 0 || OP == OP_JACOBI;
    const int tid = threadIdx.x, lane = tid & 63;
    const int4 d = a.tiles[t];
    int cb = 0;
    if constexpr (CD == 0) cb = a.tbase[t];
    const int rl_len = C.rl;
    int rl_inc = rl_len;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int u = __shfl_up(rl_inc, off, 64);
        if (lane >= off) rl_inc += u;
    }
    if (lane == 63) lwt[tid >> 6] = rl_inc;
    const int r0 = d.x, nr = d.y - d.x, cnt = d.w - d.z;
    double pb = 0.0, px = 0.0, py = 0.0, pd = 0.0;
    if (tid < nr) {
        const int r = r0 + tid;
        if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = a.b[r];
        if constexpr (OP == OP_JACOBI) {
            px = a.x[r];
            if (a.diag) pd = a.diag[r];
        }
        if constexpr (OP == OP_PROLONG) py = a.y[r];
    }
    auto row_end = [&]() {
        int pre = 0;
#pragma unroll
        for (int q = 0; q < BS / 64; ++q) pre += q < (tid >> 6) ? lwt[q] : 0;
        return pre + rl_inc;
    };
    int re = 0;
    if constexpr (NEED_ROWS) {
        lds_barrier();  // lwt (and ltab on the first tile)
        re = row_end();
        if (tid < nr)
            for (int p = re - rl_len; p < re; ++p) lrow[p] = (uint8_t)tid;
        lds_barrier();  // lrow
    }
    double xv[G][4];
    int cc[G][4];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int q = 4 * (tid + j * BS);
        const uint32_t rw = NEED_ROWS && q < cnt ? *reinterpret_cast<const uint32_t*>(&lrow[q]) : 0u;
        if constexpr (CD == 0) {
            const uint16_t l4[4] = {C.clo4[j].x, C.clo4[j].y, C.clo4[j].z, C.clo4[j].w};
#pragma unroll
            for (int e = 0; e < 4; ++e)
                cc[j][e] = cb + (int)((uint32_t)l4[e] | (((C.cn[j] >> (8 * e)) & 255u) << 16));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int ix = CD == 4 ? (int)((C.cn[j] >> (4 * e)) & 15u) : (int)((C.cn[j] >> (8 * e)) & 255u);
                cc[j][e] = r0 + (int)((rw >> (8 * e)) & 255u) + ltab[ix];
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[j][e] = a.x[q + e < cnt ? cc[j][e] : 0];
    }
    tm_load<OP, TNNZ, CD>(tn, N, tid, a.tval, a.tcidx, a.tclo, a.tchi, a.trlen, a.rs);
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int q = 4 * (tid + j * BS);
        const uint32_t rw = NEED_ROWS && q < cnt ? *reinterpret_cast<const uint32_t*>(&lrow[q]) : 0u;
        const double vv[4] = {C.va[j].x, C.va[j].y, C.vb[j].x, C.vb[j].y};
        double p[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool ok = q + e < cnt;
            p[e] = ok ? vv[e] * xv[j][e] : 0.0;
            if constexpr (OP == OP_JACOBI) {
                const int rl = (int)((rw >> (8 * e)) & 255u);
                if (!a.diag && ok && cc[j][e] - r0 == rl) ldiag[rl] = vv[e];
            }
        }
        *reinterpret_cast<double2*>(&lprod[q]) = make_double2(p[0], p[1]);
        *reinterpret_cast<double2*>(&lprod[q + 2]) = make_double2(p[2], p[3]);
    }
    lds_barrier();  // lprod, ldiag (and lwt for the 24-bit ops)
    if constexpr (!NEED_ROWS) re = row_end();
    if (tid < nr) {
        const double s = row_sum_lds(lprod, re - rl_len, re);
        const int r = r0 + tid;
        if constexpr (OP == OP_SPMV) {
            a.y[r] = s;
        } else if constexpr (OP == OP_RESID) {
            a.y[r] = pb - s;
        } else if constexpr (OP == OP_JACOBI) {
            const double dd = a.diag ? pd : ldiag[tid];
            const double u = pb - s;
            const double v = a.omega * u;
            const double w = v / dd;
            a.y[r] = px + w;
        } else {
            a.y[r] = py + s;
        }
    }
    lds_barrier();  // every lane is done with this tile's lwt / lrow / lprod / ldiag
}

template <int OP, int TNNZ, int CD>
__global__ __launch_bounds__(kBlock) void k_rows_tmp(TmArgs a, int ntiles, const int* __restrict__ ctab,
                                                     int ctab_n) {
    __shared__ __attribute__((aligned(16))) double lprod[TNNZ + 8];
    __shared__ double ldiag[OP == OP_JACOBI ? kBlock : 1];
    __shared__ int lwt[kBlock / 64];
    __shared__ int ltab[CD == 8 ? 256 : 16];
    __shared__ __attribute__((aligned(4))) uint8_t lrow[TNNZ + 8];
    const int tid = threadIdx.x;
    int t = blockIdx.x;
    if (t >= ntiles) return;
    if constexpr (CD != 0) {
        if (tid < ctab_n) ltab[tid] = ctab[tid];
        lds_barrier();
    }
    TmSlot<OP, TNNZ, CD> A, B;
    tm_load<OP, TNNZ, CD>(t, A, tid, a.tval, a.tcidx, a.tclo, a.tchi, a.trlen, a.rs);
    const int step = gridDim.x;
    while (true) {  // two slots in alternation: A holds tile t, B receives the next one
        int tn = t + step;
        tm_tile<OP, TNNZ, CD>(a, t, A, tn < ntiles ? tn : t, B, lprod, ldiag, lwt, ltab, lrow);
        if (tn >= ntiles) break;
        t = tn;
        tn = t + step;
        tm_tile<OP, TNNZ, CD>(a, t, B, tn < ntiles ? tn : t, A, lprod, ldiag, lwt, ltab, lrow);
        if (tn >= ntiles) break;
        t = tn;
    }
}

// Variant 3: variant 1's tile body in a persistent grid. Block b walks tiles b, b+G, b+2G, ...
// (G = grid, a multiple of 8, so a block stays on one XCD's slice of the banded tile order)
// and issues the NEXT tile's descriptor-driven column/value stream right after the current
// tile's x gathers, so the HBM stream of tile t+1 overlaps the LDS sum / epilogue of tile t.
// Barriers are LDS-only (lds_barrier) so the prefetch is never drained by a __syncthreads().
template <int OP, int TNNZ, int TROWS>
__global__ __launch_bounds__(kBlock) void k_rows_pers(
    const int4* __restrict__ tiles, int ntiles, const int* __restrict__ rowptr,
    const int* __restrict__ col, const double* __restrict__ val, const double* __restrict__ x,
    const double* __restrict__ b, double* __restrict__ y, double omega) {
    constexpr int G = TNNZ / (4 * kBlock);
    static_assert(G >= 1 && TROWS <= kBlock, "one row per lane");
    __shared__ __attribute__((aligned(16))) double lprod[TNNZ + 8];
    __shared__ int lrp[TROWS + 1];
    __shared__ double ldiag[OP == OP_JACOBI ? TROWS : 1];
    const int tid = threadIdx.x;
    int t = blockIdx.x;
    if (t >= ntiles) return;
    int4 d = tiles[t];
    int4 c4[G];
    double2 va[G], vb[G];
    auto load = [&](const int4& dd) {
        const int za = dd.z & ~3;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int g = za + 4 * (tid + j * kBlock);
            const int gs = g < dd.w ? g : za;
            c4[j] = *reinterpret_cast<const int4*>(col + gs);
            va[j] = *reinterpret_cast<const double2*>(val + gs);
            vb[j] = *reinterpret_cast<const double2*>(val + gs + 2);
        }
    };
    load(d);
    for (; t < ntiles; t += gridDim.x) {
        const int r0 = d.x, nr = d.y - d.x, z0 = d.z, z1 = d.w, za = z0 & ~3;
        int4 cc4[G];
        double2 ca[G], cb[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            cc4[j] = c4[j];
            ca[j] = va[j];
            cb[j] = vb[j];
        }
        for (int i = tid; i <= nr; i += kBlock) lrp[i] = rowptr[r0 + i];
        double pb = 0.0, px = 0.0, py = 0.0;
        if (tid < nr) {
            const int r = r0 + tid;
            if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[r];
            if constexpr (OP == OP_JACOBI) px = x[r];
            if constexpr (OP == OP_PROLONG) py = y[r];
        }
        double xv[G][4];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int g = za + 4 * (tid + j * kBlock);
            const int cc[4] = {cc4[j].x, cc4[j].y, cc4[j].z, cc4[j].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool ok = (g + e >= z0) & (g + e < z1);
                xv[j][e] = x[ok ? cc[e] : 0];
            }
        }
        // prefetch the next tile's stream behind the gathers (counted vmcnt keeps it in flight)
        const int tn = t + gridDim.x;
        if (tn < ntiles) {
            d = tiles[tn];
            load(d);
        }
        lds_barrier();  // lrp visible (and the previous tile's phase 2 is done with lprod)
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int g = za + 4 * (tid + j * kBlock);
            const int cc[4] = {cc4[j].x, cc4[j].y, cc4[j].z, cc4[j].w};
            const double vv[4] = {ca[j].x, ca[j].y, cb[j].x, cb[j].y};
            double p[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = g + e;
                const bool ok = (k >= z0) & (k < z1);
                p[e] = ok ? vv[e] * xv[j][e] : 0.0;
                if constexpr (OP == OP_JACOBI) {
                    const int rl = cc[e] - r0;
                    if (ok && rl >= 0 && rl < nr && k >= lrp[rl] && k < lrp[rl + 1]) ldiag[rl] = vv[e];
                }
            }
            *reinterpret_cast<double2*>(&lprod[g - za]) = make_double2(p[0], p[1]);
            *reinterpret_cast<double2*>(&lprod[g - za + 2]) = make_double2(p[2], p[3]);
        }
        lds_barrier();
        if (tid < nr) {
            const int kb = lrp[tid] - za, ke = lrp[tid + 1] - za;
            const double s = row_sum_lds(lprod, kb, ke);
            const int r = r0 + tid;
            if constexpr (OP == OP_SPMV) {
                y[r] = s;
            } else if constexpr (OP == OP_RESID) {
                y[r] = pb - s;
            } else if constexpr (OP == OP_JACOBI) {
                const double u = pb - s;
                const double v = omega * u;
                const double w = v / ldiag[tid];
                y[r] = px + w;
            } else {
                y[r] = py + s;
            }
        }
        lds_barrier();  // phase 2 done before the next tile rewrites lrp / lprod / ldiag
    }
}

// Variant 2: wave tiles (<= 64 rows, <= WNNZ nonzeros) walked by a persistent grid, each wave
// keeping the NEXT tile's column/value stream in flight (registers) while it gathers, sums and
// stores the current one. No workgroup barrier anywhere: every wave owns an LDS slice; the
// tile descriptors come 64 at a time (one per lane) and are broadcast with readlane; the row
// bounds live in the lanes of their rows (phase 2 is one lane per row, as in variant 1).
template <int OP, int WNNZ>
__global__ __launch_bounds__(kBlock) void k_rows_wave(
    const int4* __restrict__ tiles, int ntiles, const int* __restrict__ rowptr,
    const int* __restrict__ col, const double* __restrict__ val, const double* __restrict__ x,
    const double* __restrict__ b, double* __restrict__ y, double omega,
    const double* __restrict__ diag) {
    constexpr int G = WNNZ / 256;
    constexpr int W = kBlock / 64;
    static_assert(G >= 1 && WNNZ % 256 == 0, "wave tile budget must be a multiple of 256");
    __shared__ __attribute__((aligned(16))) double lprod_all[W][WNNZ + 8];
    __shared__ double ldiag_all[OP == OP_JACOBI ? W : 1][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double* lprod = lprod_all[w];
    double* ldiag = ldiag_all[OP == OP_JACOBI ? w : 0];
    const int stride = gridDim.x * W;
    const int t0 = blockIdx.x * W + w;
    if (t0 >= ntiles) return;
    const int nit = (ntiles - t0 + stride - 1) / stride;
    const int4 z4 = make_int4(0, 0, 0, 0);

    auto bcast = [](const int4& v, int l) {
        return make_int4(__builtin_amdgcn_readlane(v.x, l), __builtin_amdgcn_readlane(v.y, l),
                         __builtin_amdgcn_readlane(v.z, l), __builtin_amdgcn_readlane(v.w, l));
    };
    int4 db = z4, dnb = z4;
    if (lane < nit) db = tiles[t0 + lane * stride];
    if (64 + lane < nit) dnb = tiles[t0 + (64 + lane) * stride];

    int4 c4[G];
    double2 va[G], vb[G];
    auto load = [&](const int4& d) {
        const int za = d.z & ~3;
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int g = za + 4 * (lane + 64 * j);
            const int gs = g < d.w ? g : za;
            c4[j] = *reinterpret_cast<const int4*>(col + gs);
            va[j] = *reinterpret_cast<const double2*>(val + gs);
            vb[j] = *reinterpret_cast<const double2*>(val + gs + 2);
        }
    };
    int4 dcur = bcast(db, 0);
    load(dcur);
    for (int i = 0; i < nit; ++i) {
        const int4 d = dcur;
        int4 cc4[G];
        double2 ca[G], cb[G];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            cc4[j] = c4[j];
            ca[j] = va[j];
            cb[j] = vb[j];
        }
        // prefetch: next tile's stream (and, every 64 tiles, the descriptor batch after next)
        const int in = i + 1;
        if (in < nit) {
            if ((in & 63) == 0) {
                db = dnb;
                if (in + 64 + lane < nit) dnb = tiles[t0 + (in + 64 + lane) * stride];
            }
            dcur = bcast(db, in & 63);
            load(dcur);
        }
        const int r0 = d.x, nr = d.y - d.x, z0 = d.z, z1 = d.w, za = z0 & ~3;
        int rs = 0, re = 0;
        if (lane < nr) {
            rs = rowptr[r0 + lane];
            re = rowptr[r0 + lane + 1];
        }
        double xv[G][4];
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int g = za + 4 * (lane + 64 * j);
            const int cc[4] = {cc4[j].x, cc4[j].y, cc4[j].z, cc4[j].w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const bool ok = (g + e >= z0) & (g + e < z1);
                xv[j][e] = x[ok ? cc[e] : 0];
            }
        }
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int g = za + 4 * (lane + 64 * j);
            const int cc[4] = {cc4[j].x, cc4[j].y, cc4[j].z, cc4[j].w};
            const double vv[4] = {ca[j].x, ca[j].y, cb[j].x, cb[j].y};
            double p[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int k = g + e;
                const bool ok = (k >= z0) & (k < z1);
                p[e] = ok ? vv[e] * xv[j][e] : 0.0;
                if constexpr (OP == OP_JACOBI) {
                    if (!diag) {
                        const int rl = cc[e] - r0;
                        const int rlc = (rl >= 0 && rl < nr) ? rl : 0;
                        const int lo = __shfl(rs, rlc, 64), hi = __shfl(re, rlc, 64);
                        if (ok && rl >= 0 && rl < nr && k >= lo && k < hi) ldiag[rl] = vv[e];
                    }
                }
            }
            *reinterpret_cast<double2*>(&lprod[g - za]) = make_double2(p[0], p[1]);
            *reinterpret_cast<double2*>(&lprod[g - za + 2]) = make_double2(p[2], p[3]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < nr) {
            double s = 0.0;
            for (int k = rs - za; k < re - za; ++k) s = s + lprod[k];
            double dd = 0.0;
            if constexpr (OP == OP_JACOBI) dd = diag ? diag[r0 + lane] : ldiag[lane];
            epilogue<OP>(r0 + lane, s, x, b, y, omega, dd);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

template <int OP>
__global__ __launch_bounds__(kBlock) void k_rows_long(
    const int* __restrict__ rows, const int* __restrict__ rowptr, const int* __restrict__ col,
    const double* __restrict__ val, const double* __restrict__ x, const double* __restrict__ b,
    double* __restrict__ y, double omega) {
    __shared__ double lprod[kBlock + 8];  // + 8: row_sum_lds reads (and discards) up to 7 past the end
    __shared__ double ldiag;
    const int tid = threadIdx.x;
    const int r = rows[blockIdx.x];
    const int z0 = rowptr[r], z1 = rowptr[r + 1];
    double s = 0.0;
    for (int base = z0; base < z1; base += kBlock) {
        const int k = base + tid;
        double p = 0.0;
        if (k < z1) {
            const int c = col[k];
            const double v = val[k];
            p = v * x[c];
            if constexpr (OP == OP_JACOBI) {
                if (c == r) ldiag = v;
            }
        }
        lprod[tid] = p;
        __syncthreads();
        if (tid == 0) s = row_sum_lds(lprod, 0, min(kBlock, z1 - base), s);
        __syncthreads();
    }
    if (tid == 0) epilogue<OP>(r, s, x, b, y, omega, OP == OP_JACOBI ? ldiag : 0.0);
}

__global__ void k_jacobi_zero(int64_t n, const double* __restrict__ b,
                              const double* __restrict__ diag, double omega,
                              double* __restrict__ y) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double u = b[i] - 0.0;
        const double v = omega * u;
        const double w = v / diag[i];
        y[i] = 0.0 + w;
    }
}

// x[row0 + i] for the caller's rows: s = sum_j ainv[(row0+i)*n + j] * b[j], j left to right
// (SPEC §S5, §S3). ainv is row-major on the device (transposed at upload), so one wave owns a
// row: its lanes read the row in coalesced 64-wide strips (16 loads in flight per lane), the
// products go to the wave's LDS slice, and lane 0 adds them in column order. The in-order add
// chain (~n dependent fp64 adds) is the floor; the first version (one lane per row walking a
// column-major A^-1, 4 loads in flight) was bound by n/4 serial L2 round trips (30 us at n=225).
constexpr int kGemvChunk = 1024;
__global__ __launch_bounds__(kBlock) void k_dense_gemv(int64_t n_rows, int64_t n,
                                                       int64_t row0,
                                                       const double* __restrict__ ainv,
                                                       const double* __restrict__ b,
                                                       double* __restrict__ y) {
    __shared__ __attribute__((aligned(16))) double lp_all[kBlock / 64][kGemvChunk + 8];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t i = (int64_t)blockIdx.x * (kBlock / 64) + w;
    if (i >= n_rows) return;  // whole waves only: the hand-offs below are wave-local
    const double* a = ainv + (row0 + i) * n;
    double* lp = lp_all[w];
    double s = 0.0;
    for (int64_t c = 0; c < n; c += kGemvChunk) {
        const int m = (int)((n - c) < kGemvChunk ? (n - c) : kGemvChunk);
#pragma unroll
        for (int q = 0; q < kGemvChunk / 64; ++q) {
            const int j = lane + 64 * q;
            if (j < m) {
                const double p = a[c + j] * b[c + j];
                lp[j] = p;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane == 0) s = row_sum_lds(lp, 0, m, s);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    if (lane == 0) y[i] = s;
}

__global__ void k_pack(int64_t n, const int* __restrict__ idx, const double* __restrict__ x,
                       double* __restrict__ out) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        out[i] = x[idx[i]];
}

__global__ void k_fill(int64_t n, double v, double* __restrict__ y) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        y[i] = v;
}

__global__ void k_axpby(int64_t n, double a, const double* __restrict__ x, double bb,
                        double* __restrict__ y) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double u = a * x[i];
        const double v = bb * y[i];
        y[i] = u + v;
    }
}

__device__ __forceinline__ double block_sum(double v, double* lds) {
    // wave64 shuffle tree, then the 4 wave sums in fixed order
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) lds[w] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0)
        for (int k = 0; k < (int)(blockDim.x >> 6); ++k) s += lds[k];
    return s;
}

__global__ __launch_bounds__(kBlock) void k_dot_partial(int64_t n, const double* __restrict__ x,
                                                        const double* __restrict__ y,
                                                        double* __restrict__ partials) {
    __shared__ double lds[kBlock / 64];
    double v = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock)
        v += x[i] * y[i];
    const double s = block_sum(v, lds);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

__global__ __launch_bounds__(kBlock) void k_dot_final(int np, const double* __restrict__ partials,
                                                      double* __restrict__ out) {
    __shared__ double lds[kBlock / 64];
    double v = 0.0;
    for (int i = threadIdx.x; i < np; i += kBlock) v += partials[i];
    const double s = block_sum(v, lds);
    if (threadIdx.x == 0) *out = s;
}

inline int grid_for(int64_t n, int cap = 8192) {
    int64_t g = (n + kBlock - 1) / kBlock;
    if (g < 1) g = 1;
    return (int)(g < cap ? g : cap);
}

// Variant 4p launch: a persistent grid of the resident blocks (a multiple of 8, the XCDs).
template <int OP, int TNNZ, int CD>
void launch_tmp(const TileSet& ts, const double* x, const double* b, double* y, double omega,
                const double* dg, hipStream_t s) {
    static int grid_cap = 0;
    if (grid_cap == 0) {
        int nb = 0, dev = 0, ncu = 256;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_rows_tmp<OP, TNNZ, CD>, kBlock, 0);
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        grid_cap = ((nb > 0 ? nb : 1) * ncu) & ~7;
        if (grid_cap < 8) grid_cap = 8;
    }
    const int grid = ts.n_short < grid_cap ? ts.n_short : grid_cap;
    TmArgs a{ts.d_short, ts.d_tm_val, ts.d_tm_cidx, ts.d_tm_clo, ts.d_tm_chi, ts.d_base,
             ts.d_tm_rlen, ts.tm_rs, x, b, y, omega, dg};
    k_rows_tmp<OP, TNNZ, CD><<<grid, kBlock, 0, s>>>(a, ts.n_short, ts.d_ctab, ts.ctab_n);
}

template <int OP, int TNNZ, int TROWS>
void launch_tile2(const pamg_mat& A, const TileSet& ts, const double* x, const double* b,
                  double* y, double omega, hipStream_t s) {
    const double* dg = (OP == OP_JACOBI && A.jacobi_diag) ? A.d_diag : nullptr;
    if (ts.tm && A.tm_persist) {
        if constexpr (TROWS <= kBlock) {
            if (ts.cd == 4) launch_tmp<OP, TNNZ, 4>(ts, x, b, y, omega, dg, s);
            else if (ts.cd == 8) launch_tmp<OP, TNNZ, 8>(ts, x, b, y, omega, dg, s);
            else launch_tmp<OP, TNNZ, 0>(ts, x, b, y, omega, dg, s);
        }
    } else if (ts.tm && ts.tm_flags) {
        if constexpr (TROWS <= kBlock) {
            if (ts.cd == 4)
                k_rows_tmf<OP, TNNZ, 4><<<ts.n_short, kBlock, 0, s>>>(
                    ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr, nullptr, ts.d_tm_flag,
                    ts.d_tm_wb, ts.d_ctab, x, b, y, omega, dg);
            else if (ts.cd == 8)
                k_rows_tmf<OP, TNNZ, 8><<<ts.n_short, kBlock, 0, s>>>(
                    ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr, nullptr, ts.d_tm_flag,
                    ts.d_tm_wb, ts.d_ctab, x, b, y, omega, dg);
            else
                k_rows_tmf<OP, TNNZ, 0><<<ts.n_short, kBlock, 0, s>>>(
                    ts.d_short, ts.d_tm_val, nullptr, ts.d_tm_clo, ts.d_tm_chi, ts.d_base, ts.d_tm_flag,
                    ts.d_tm_wb, nullptr, x, b, y, omega, dg);
        }
    } else if (ts.tm) {
        if constexpr (TROWS <= kBlock) {
            const int plo = A.x_prefetch ? ts.cd_min : 0, phi = A.x_prefetch ? ts.cd_max : 0;
            const int xl = (int)A.ncols;
            const double nan = __builtin_nan("");
            if (A.tm_transpose) {
                if (ts.cd == 4)
                    k_rows_tm<OP, TNNZ, 4, true><<<ts.n_short, kBlock, 0, s>>>(
                        ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr, nullptr, ts.d_tm_rlen,
                        ts.tm_rs, ts.d_ctab, ts.ctab_n, x, b, y, omega, dg, plo, phi, xl, nan);
                else if (ts.cd == 8)
                    k_rows_tm<OP, TNNZ, 8, true><<<ts.n_short, kBlock, 0, s>>>(
                        ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr, nullptr, ts.d_tm_rlen,
                        ts.tm_rs, ts.d_ctab, ts.ctab_n, x, b, y, omega, dg, plo, phi, xl, nan);
                else
                    k_rows_tm<OP, TNNZ, 0, true><<<ts.n_short, kBlock, 0, s>>>(
                        ts.d_short, ts.d_tm_val, nullptr, ts.d_tm_clo, ts.d_tm_chi, ts.d_base, ts.d_tm_rlen,
                        ts.tm_rs, nullptr, 0, x, b, y, omega, dg);
            } else if (ts.cd == 4)
                k_rows_tm<OP, TNNZ, 4><<<ts.n_short, kBlock, 0, s>>>(
                    ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr, nullptr, ts.d_tm_rlen,
                    ts.tm_rs, ts.d_ctab, ts.ctab_n, x, b, y, omega, dg, plo, phi, xl, nan);
            else if (ts.cd == 8)
                k_rows_tm<OP, TNNZ, 8><<<ts.n_short, kBlock, 0, s>>>(
                    ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr, nullptr, ts.d_tm_rlen,
                    ts.tm_rs, ts.d_ctab, ts.ctab_n, x, b, y, omega, dg, plo, phi, xl, nan);
            else
                k_rows_tm<OP, TNNZ, 0><<<ts.n_short, kBlock, 0, s>>>(
                    ts.d_short, ts.d_tm_val, nullptr, ts.d_tm_clo, ts.d_tm_chi, ts.d_base, ts.d_tm_rlen,
                    ts.tm_rs, nullptr, 0, x, b, y, omega, dg);
        }
    } else if (A.xcd_remap) {
        const int grid = ((ts.n_short + 7) / 8) * 8;
        k_rows_tile2<OP, TNNZ, TROWS, true><<<grid, kBlock, 0, s>>>(
            ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg);
    } else if (A.stream_nt) {
        k_rows_tile2<OP, TNNZ, TROWS, false, true><<<ts.n_short, kBlock, 0, s>>>(
            ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg);
    } else if (ts.cd && A.d_cidx && ts.rl8 && A.d_rlen) {
        if constexpr (TROWS <= kBlock) {
            if (ts.cd == 4)
                k_rows_tile2<OP, TNNZ, TROWS, false, false, kBlock, false, false, true, 4><<<ts.n_short, kBlock, 0, s>>>(
                    ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg, nullptr,
                    nullptr, nullptr, nullptr, nullptr, A.d_rlen, A.d_cidx, ts.d_ctab, ts.ctab_n);
            else
                k_rows_tile2<OP, TNNZ, TROWS, false, false, kBlock, false, false, true, 8><<<ts.n_short, kBlock, 0, s>>>(
                    ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg, nullptr,
                    nullptr, nullptr, nullptr, nullptr, A.d_rlen, A.d_cidx, ts.d_ctab, ts.ctab_n);
        }
    } else if (ts.c24 && A.d_clo && ts.vd && A.d_vidx) {
        k_rows_tile2<OP, TNNZ, TROWS, false, false, kBlock, true, true><<<ts.n_short, kBlock, 0, s>>>(
            ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg, A.d_clo,
            A.d_chi, ts.d_base, A.d_vidx, ts.d_vtab);
    } else if (ts.c24 && A.d_clo && ts.rl8 && A.d_rlen) {
        if constexpr (TROWS <= kBlock) {
            k_rows_tile2<OP, TNNZ, TROWS, false, false, kBlock, true, false, true><<<ts.n_short, kBlock, 0, s>>>(
                ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg, A.d_clo,
                A.d_chi, ts.d_base, nullptr, nullptr, A.d_rlen);
        }
    } else if (ts.c24 && A.d_clo) {
        k_rows_tile2<OP, TNNZ, TROWS, false, false, kBlock, true><<<ts.n_short, kBlock, 0, s>>>(
            ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg, A.d_clo,
            A.d_chi, ts.d_base);
    } else {
        k_rows_tile2<OP, TNNZ, TROWS, false><<<ts.n_short, kBlock, 0, s>>>(
            ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg);
    }
}

template <int OP, int WNNZ>
void launch_wave(const pamg_mat& A, const TileSet& ts, const double* x, const double* b,
                 double* y, double omega, hipStream_t s) {
    static int grid_cap = 0;  // resident blocks on the whole chip (persistent grid)
    if (grid_cap == 0) {
        int nb = 0, dev = 0, ncu = 256;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_rows_wave<OP, WNNZ>, kBlock, 0);
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        grid_cap = (nb > 0 ? nb : 1) * ncu;
    }
    const int need = (ts.n_short + kBlock / 64 - 1) / (kBlock / 64);
    const int grid = need < grid_cap ? need : grid_cap;
    const double* dg = (OP == OP_JACOBI && A.jacobi_diag) ? A.d_diag : nullptr;
    k_rows_wave<OP, WNNZ><<<grid, kBlock, 0, s>>>(ts.d_short, ts.n_short, A.d_rowptr, A.d_col,
                                                  A.d_val, x, b, y, omega, dg);
}

template <int OP, int TNNZ, int TROWS>
void launch_pers(const pamg_mat& A, const TileSet& ts, const double* x, const double* b,
                 double* y, double omega, hipStream_t s) {
    static int grid_cap = 0;  // resident blocks on the chip, a multiple of 8 (XCDs)
    if (grid_cap == 0) {
        int nb = 0, dev = 0, ncu = 256;
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_rows_pers<OP, TNNZ, TROWS>, kBlock, 0);
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        grid_cap = ((nb > 0 ? nb : 1) * ncu) & ~7;
        if (grid_cap < 8) grid_cap = 8;
    }
    const int grid = ts.n_short < grid_cap ? ts.n_short : grid_cap;
    k_rows_pers<OP, TNNZ, TROWS><<<grid, kBlock, 0, s>>>(ts.d_short, ts.n_short, A.d_rowptr,
                                                        A.d_col, A.d_val, x, b, y, omega);
}

template <int OP>
void launch_rows_op(const pamg_mat& A, const TileSet& ts, const double* x, const double* b,
                    double* y, double omega, hipStream_t s) {
    if (ts.n_short > 0) {
        if (A.rows_kernel == 3) {
            if (ts.tile_nnz == 2048) launch_pers<OP, 2048, 256>(A, ts, x, b, y, omega, s);
            else launch_pers<OP, 1024, 256>(A, ts, x, b, y, omega, s);
        } else if (A.rows_kernel == 2) {
            if (ts.tile_nnz == 256) launch_wave<OP, 256>(A, ts, x, b, y, omega, s);
            else if (ts.tile_nnz == 1024) launch_wave<OP, 1024>(A, ts, x, b, y, omega, s);
            else launch_wave<OP, 512>(A, ts, x, b, y, omega, s);
        } else if (A.rows_kernel == 0 && ts.tile_nnz == kTileNnz && ts.tile_rows == kTileRows) {
            k_rows_tile<OP><<<ts.n_short, kBlock, 0, s>>>(ts.d_short, A.d_rowptr, A.d_col,
                                                          A.d_val, x, b, y, omega);
        } else if (ts.tile_nnz == 512 && ts.tile_rows == 128) {
            const double* dg = (OP == OP_JACOBI && A.jacobi_diag) ? A.d_diag : nullptr;
            k_rows_tile2<OP, 512, 128, false, false, 128><<<ts.n_short, 128, 0, s>>>(
                ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg);
        } else if (ts.tile_nnz == 2048 && ts.tile_rows == 512) {
            const double* dg = (OP == OP_JACOBI && A.jacobi_diag) ? A.d_diag : nullptr;
            k_rows_tile2<OP, 2048, 512, false, false, 512><<<ts.n_short, 512, 0, s>>>(
                ts.d_short, ts.n_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, dg);
        } else if (ts.tile_nnz == 1024) {
            launch_tile2<OP, 1024, 256>(A, ts, x, b, y, omega, s);
        } else if (ts.tile_nnz == 4096 && ts.tile_rows == 512) {
            launch_tile2<OP, 4096, 512>(A, ts, x, b, y, omega, s);
        } else if (ts.tile_nnz == 4096) {
            launch_tile2<OP, 4096, 256>(A, ts, x, b, y, omega, s);
        } else {
            launch_tile2<OP, 2048, 256>(A, ts, x, b, y, omega, s);
        }
    }
    if (ts.n_long > 0)
        k_rows_long<OP><<<ts.n_long, kBlock, 0, s>>>(ts.d_long, A.d_rowptr, A.d_col, A.d_val, x,
                                                     b, y, omega);
}

}  // namespace

void launch_rows(const pamg_mat& A, const TileSet& ts, int op, const double* x, const double* b,
                 const double* /*xold*/, double* y, double omega, hipStream_t s) {
    switch (op) {
        case OP_SPMV: launch_rows_op<OP_SPMV>(A, ts, x, b, y, omega, s); break;
        case OP_RESID: launch_rows_op<OP_RESID>(A, ts, x, b, y, omega, s); break;
        case OP_JACOBI: launch_rows_op<OP_JACOBI>(A, ts, x, b, y, omega, s); break;
        default: launch_rows_op<OP_PROLONG>(A, ts, x, b, y, omega, s); break;
    }
}

void launch_jacobi_zero(int64_t n, const double* b, const double* diag, double omega, double* y,
                        hipStream_t s) {
    if (n > 0) k_jacobi_zero<<<grid_for(n), kBlock, 0, s>>>(n, b, diag, omega, y);
}

void launch_dense_gemv(int64_t n_rows, int64_t n_cols, int64_t row0, const double* ainv_rm,
                       const double* b, double* y, hipStream_t s) {
    constexpr int kRowsPerBlock = kBlock / 64;
    if (n_rows > 0)
        k_dense_gemv<<<(int)((n_rows + kRowsPerBlock - 1) / kRowsPerBlock), kBlock, 0, s>>>(n_rows, n_cols,
                                                                             row0, ainv_rm, b, y);
}

void launch_pack(int64_t n, const int* idx, const double* x, double* out, hipStream_t s) {
    if (n > 0) k_pack<<<grid_for(n), kBlock, 0, s>>>(n, idx, x, out);
}

void launch_fill(int64_t n, double v, double* y, hipStream_t s) {
    if (n > 0) k_fill<<<grid_for(n), kBlock, 0, s>>>(n, v, y);
}

void launch_axpby(int64_t n, double a, const double* x, double b, double* y, hipStream_t s) {
    if (n > 0) k_axpby<<<grid_for(n), kBlock, 0, s>>>(n, a, x, b, y);
}

int dot_partials(int64_t n) { return grid_for(n, 1024); }

void launch_dot(int64_t n, const double* x, const double* y, double* partials, int np,
                double* out, hipStream_t s) {
    k_dot_partial<<<np, kBlock, 0, s>>>(n, x, y, partials);
    k_dot_final<<<1, kBlock, 0, s>>>(np, partials, out);
}

}  // namespace pamg
