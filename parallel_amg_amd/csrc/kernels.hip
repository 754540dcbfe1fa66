// kernels.hip — gfx950 (CDNA4) kernels of the AMG V-cycle solve path.
//
// Every row-sum kernel implements SPEC.md §S3 exactly: products p = a*x rounded, summed
// left to right in storage order from +0.0, never fused (built with -ffp-contract=off), so
// results are bit-identical to the CPU oracle and run-to-run deterministic.
//
// CSR row kernels: the path is HBM-bound sparse work (12 B/nnz of matrix stream + vectors,
// ~0.17 flop/B), so there is no MFMA here. One 256-thread workgroup takes a tile of <= 256
// consecutive rows / <= TNNZ nonzeros (1024 by default, 4096 for long-row operators):
//   stream   the tile's columns/values are loaded with 16-byte loads per lane (1 KiB per
//            wave-instruction), each lane gathers its four x[col] and writes the four
//            products to LDS (the "LDS-staged partial sums"); for Jacobi the lane holding a
//            row's diagonal stores a_ii in LDS;
//   sum      one lane per row adds its products from LDS in storage order and applies the
//            epilogue (SpMV / residual / Jacobi / prolongate-add), coalesced stores.
// Rows longer than the tile budget go to k_rows_long (one workgroup per row, chunked).
//
// Two tile bodies (the upload fixes the layout per tile set, launch_tile picks the kernel;
// both are bit-identical, tests/test_gpu_parity.py):
//   k_rows_tile2  descriptor-driven: the stream is issued at entry from the tile's nonzero
//                 range; 32-bit or 24-bit columns, 8-bit row lengths, column / value
//                 dictionaries
//   k_rows_tm     tile-major slots: every pre-gather load addressed by tile index alone
//                 (default for column-dictionary sets and slot-filling non-square operators)
// Variants measured slower in round 1 (row-pointer-first tiles, wave tiles, persistent grids,
// row-start flags, x-line prefetch, transposed lane mapping, non-temporal streams, XCD
// chunk remap, stored-diagonal Jacobi) were removed; DESIGN.md "Measured and rejected" keeps
// their numbers.

#include "pamg_device.h"

namespace pamg {
namespace {

// Inclusive prefix sum over the 64 lanes of a wave with DPP lane moves (row_shr 1/2/4/8 inside
// each 16-lane row, then row_bcast 15 / 31 across rows): VALU-side, where __shfl_up's
// ds_bpermute costs an LDS round trip per step. The explicit lane predicates make the result
// independent of what DPP reads for out-of-row sources.
__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = threadIdx.x & 63, rl = lane & 15;
    int t;
    t = __builtin_amdgcn_mov_dpp(v, 0x111, 0xf, 0xf, false);  // row_shr:1
    if (rl >= 1) v += t;
    t = __builtin_amdgcn_mov_dpp(v, 0x112, 0xf, 0xf, false);  // row_shr:2
    if (rl >= 2) v += t;
    t = __builtin_amdgcn_mov_dpp(v, 0x114, 0xf, 0xf, false);  // row_shr:4
    if (rl >= 4) v += t;
    t = __builtin_amdgcn_mov_dpp(v, 0x118, 0xf, 0xf, false);  // row_shr:8
    if (rl >= 8) v += t;
    t = __builtin_amdgcn_mov_dpp(v, 0x142, 0xf, 0xf, false);  // row_bcast:15
    if (lane & 16) v += t;
    t = __builtin_amdgcn_mov_dpp(v, 0x143, 0xf, 0xf, false);  // row_bcast:31
    if (lane >= 32) v += t;
    return v;
}

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

// k_rows_tile2: the tile descriptor carries its nonzero range, so the column/value stream of
// every lane (TNNZ / 1024 groups of 4 nonzeros: one int4 + two double2 loads each) is issued
// at kernel entry together with the row-pointer slice; all x gathers of a lane are then
// issued back to back (branch-free: invalid lanes gather x[0] and discard it) before the
// products go to LDS.
template <int OP, int TNNZ, bool C24 = false, bool VD = false, bool RL8 = false, int CD = 0, bool PT = false,
          bool ANC = false>
__global__ __launch_bounds__(kBlock) void k_rows_tile2(
    const int4* __restrict__ tiles, const int* __restrict__ rowptr,
    const int* __restrict__ col, const double* __restrict__ val, const double* __restrict__ x,
    const double* __restrict__ b, double* __restrict__ y, double omega,
    const uint16_t* __restrict__ clo = nullptr, const uint8_t* __restrict__ chi = nullptr,
    const int* __restrict__ tbase = nullptr, const uint8_t* __restrict__ vidx = nullptr,
    const double* __restrict__ vtab = nullptr, const uint8_t* __restrict__ rlen = nullptr,
    const uint8_t* __restrict__ cidx = nullptr, const int* __restrict__ ctab = nullptr,
    int ctab_n = 0, const uint16_t* __restrict__ anc16 = nullptr, const int* __restrict__ abase = nullptr) {
    // PT: per-tile dictionary — this tile's table is ctab[bid * ctab_n ...]; ANC: columns are
    // the row's anchor (abase[tile] + anc16[row]) + table[index] instead of row + table[index]
    static_assert(!PT || CD != 0, "per-tile tables are column dictionaries");
    static_assert(!ANC || PT, "anchored columns in the descriptor kernel come with per-tile tables");
    // C24: the column stream is 3 B/nonzero — per-tile base + 16-bit low part (8 B per lane)
    // + 8-bit high part (4 B per lane) instead of the 16-B int4 of 32-bit ids.
    // VD (opt-in): values are 4-bit indices (2 B per lane) into the tile's 16-value table,
    // read through L1 (the same 128 B for every lane of the tile) — exact fp64 values.
    constexpr int BS = kBlock;
    constexpr int G = TNNZ / (4 * BS);
    static_assert(G >= 1 && TNNZ % (4 * BS) == 0, "tile budget must be a multiple of 4 x block");
    __shared__ __attribute__((aligned(16))) double lprod[TNNZ + 8];
    __shared__ int lrp[kTileRows + 1];
    __shared__ double ldiag[OP == OP_JACOBI ? kTileRows : 1];
    // RL8: row lengths are 8-bit (1 B/row instead of a 4-B row pointer); the row starts are
    // rebuilt from the tile's first nonzero by a wave-level scan + the wave totals (lwt)
    static_assert(kTileRows <= BS, "one row per lane");
    __shared__ int lwt[RL8 ? BS / 64 : 1];
    // CD (column dictionary, 4 or 8 bits per nonzero): column = row + ctab[index], with the
    // tile set's <= 16 / <= 256 distinct offsets (a stencil's 7 for A0) in LDS; every
    // position's row (lrow, tile-local) is marked by the lane that owns the row (RL8 scan)
    static_assert(CD == 0 || (RL8 && !C24), "column dictionary: 8-bit rows");
    __shared__ int ltab[CD != 0 ? BS : 1];
    __shared__ __attribute__((aligned(4))) uint8_t lrow[CD ? TNNZ + 8 : 4];
    __shared__ int lanc[ANC ? BS : 1];

    const int bid = blockIdx.x;
    const int tid = threadIdx.x;
    const int4 t = tiles[bid];
    const int r0 = t.x, nr = t.y - t.x, z0 = t.z, z1 = t.w;
    const int za = z0 & ~3;

    // Load order (vmcnt retires loads in issue order; see k_rows_tm): row bounds, table,
    // column stream and the epilogue operands first, branch-free; the values last.
    const int lr = tid < nr ? tid : (nr > 0 ? nr - 1 : 0);  // clamped own row
    int rlv = 0, rpa = 0, rpb = 0, tabv = 0;
    if constexpr (RL8) {
        rlv = (int)rlen[r0 + lr];
    } else {
        rpa = rowptr[r0 + (tid < nr ? tid : nr)];
        rpb = rowptr[r0 + nr];
    }
    if constexpr (CD != 0) {
        if constexpr (PT) tabv = ctab[(size_t)bid * ctab_n + (tid < ctab_n ? tid : ctab_n - 1)];
        else tabv = ctab[tid];  // the global table is allocated with 256 entries
    }
    int ancv = 0;
    if constexpr (ANC) ancv = abase[bid] + (int)anc16[r0 + lr];
    int4 c4[G];
    double2 va[G], vb[G];
    uint16_t vn[G];  // VD: four 4-bit value indices per lane group
    uint32_t cn[G];  // CD: four 4- or 8-bit column dictionary indices per lane group
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int g = za + 4 * (tid + j * BS);
        const int gs = g < z1 ? g : za;  // clamp: never read past the (padded) arrays
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
            c4[j] = *reinterpret_cast<const int4*>(col + gs);
        }
        if constexpr (VD) vn[j] = *reinterpret_cast<const uint16_t*>(vidx + (gs >> 1));
    }
    // one row per lane: the epilogue's own-row operands (b, old x, y), so their latency
    // hides under the stream instead of trailing the LDS phase
    double pb = 0.0, px = 0.0, py = 0.0;
    {
        const int r = r0 + lr;
        if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[r];
        if constexpr (OP == OP_JACOBI) px = x[r];
        if constexpr (OP == OP_PROLONG) py = y[r];
    }
    asm volatile("" ::: "memory");  // keep the loads above ahead of the value stream
    if constexpr (!VD) {
#pragma unroll
        for (int j = 0; j < G; ++j) {
            const int g = za + 4 * (tid + j * BS);
            const int gs = g < z1 ? g : za;
            va[j] = *reinterpret_cast<const double2*>(val + gs);
            vb[j] = *reinterpret_cast<const double2*>(val + gs + 2);
        }
    }
    int rl_len = 0, rl_inc = 0;  // RL8: this lane's row length and wave-inclusive length sum
    if constexpr (RL8) {
        const int lane = tid & 63;
        rl_len = tid < nr ? rlv : 0;
        rl_inc = wave_incl_scan(rl_len);
        if (lane == 63) lwt[tid >> 6] = rl_inc;
    } else {
        // unconditional stores (lanes past the tile's rows rewrite lrp[nr] with its own value):
        // a conditional store would let the compiler sink the loads behind the values
        lrp[tid < nr ? tid : nr] = rpa;
        lrp[nr] = rpb;
    }
    // row start of this lane's row (RL8, after a barrier has published lwt)
    auto rl_base = [&]() {
        int pre = z0;
#pragma unroll
        for (int q = 0; q < BS / 64; ++q) pre += q < (tid >> 6) ? lwt[q] : 0;
        return pre;
    };
    if constexpr (CD != 0) {
        ltab[tid] = tabv;
        if constexpr (ANC) lanc[tid] = ancv;
        __syncthreads();  // lwt, ltab, lanc
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
                const int rid = (int)((rw >> (8 * e)) & 255u);
                if constexpr (ANC) cc[e] = lanc[rid] + ltab[ix];
                else cc[e] = r0 + rid + ltab[ix];
            }
            c4[j] = make_int4(cc[0], cc[1], cc[2], cc[3]);
        }
    } else if constexpr (OP == OP_JACOBI) {
        __syncthreads();
        if constexpr (RL8) {  // the in-tile diagonal search needs every row's bounds
            const int base = rl_base();
            if (tid == 0) lrp[0] = z0;
            if (tid < kTileRows) lrp[tid + 1] = base + rl_inc;
            __syncthreads();
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
                    if (ok && rl == (int)lrow[k - za]) ldiag[rl] = vv[e];
                } else {
                    if (ok && rl >= 0 && rl < nr && k >= lrp[rl] && k < lrp[rl + 1]) ldiag[rl] = vv[e];
                }
            }
        }
        *reinterpret_cast<double2*>(&lprod[g - za]) = make_double2(p[0], p[1]);
        *reinterpret_cast<double2*>(&lprod[g - za + 2]) = make_double2(p[2], p[3]);
    }
    __syncthreads();
    // every lane computes (lanes past the tile's rows sum an empty range) and only the
    // tile's rows store: with the epilogue unconditional, the compiler keeps the operand
    // loads at entry instead of sinking them into the store branch
    int kb = 0, ke = 0;
    if constexpr (RL8) {
        const int base = rl_base();
        kb = base + rl_inc - rl_len - za;
        ke = base + rl_inc - za;
    } else if (tid < nr) {
        kb = lrp[tid] - za;
        ke = lrp[tid + 1] - za;
    }
    const double s = row_sum_lds(lprod, kb, ke);
    double out;
    if constexpr (OP == OP_SPMV) {
        out = s;
    } else if constexpr (OP == OP_RESID) {
        out = pb - s;
    } else if constexpr (OP == OP_JACOBI) {
        const double u = pb - s;
        const double v = omega * u;
        const double w = v / ldiag[tid < nr ? tid : 0];
        out = px + w;
    } else {
        out = py + s;
    }
    if (tid < nr) y[r0 + tid] = out;
}

// k_rows_tm, tile-major (TileSet::tm): tile t's values, column stream and row lengths live at
// fixed slots of padded per-set arrays — values/columns at t*TNNZ, row lengths at t*rs — so
// every load a block needs before its x gathers is addressed from blockIdx alone and issued
// at entry beside the descriptor load. k_rows_tile2 has to wait for the descriptor (its
// nonzero range) before it can issue the stream, one dependent memory round trip more per
// tile. Columns: CD = 4 / 8, row + table[index] (column dictionary); CD = 0, tile base +
// 24-bit (16-bit low + 8-bit high) offset. Rows: one per lane, starts by a wave scan of the
// lengths; positions are tile-relative (no alignment head: a tile's slot starts at its first
// nonzero). Summation order, epilogues and Jacobi's in-tile diagonal are k_rows_tile2's
// (SPEC §S3).
// XS (x staging, TileSet::xs, row-relative dictionaries only): the tile's x values are the
// runs [r0 + omin_c, r0 + nr - 1 + omin_c + wid_c] of the dictionary's offset clusters; each
// lane loads one element of every run at entry, beside the other independent loads, into LDS
// (segments of xst.stride doubles), and the products read x there at the LDS position the
// table holds at kXsIoff + index. The x gathers — dependent on the column stream and the row
// map, one round trip after them — disappear; Jacobi's diagonal is the entry of offset 0.
// PT (Options::tm_tile_dicts): per-tile row-relative dictionaries (TileSet::pt) in tile-major
// slots — this tile's table is ctab[t * ctab_n ...], addressed from the block index like
// every other pre-gather load.
// VD8 (TileSet::tm_vt): values through the tile's 8-bit dictionary — a byte per nonzero in the
// slot and the tile's table (vt entries, staged into LDS at entry) instead of 8-B values.
template <int OP, int TNNZ, int CD, bool ANC = false, bool XS = false, bool PT = false, bool VD8 = false>
__global__ __launch_bounds__(kBlock) void k_rows_tm(
    const int4* __restrict__ tiles, const double* __restrict__ tval,
    const uint8_t* __restrict__ tcidx, const uint16_t* __restrict__ tclo,
    const uint8_t* __restrict__ tchi, const int* __restrict__ tbase,
    const uint8_t* __restrict__ trlen, int rs, const int* __restrict__ ctab, int ctab_n,
    const double* __restrict__ x, const double* __restrict__ b, double* __restrict__ y,
    double omega, const int* __restrict__ tanc = nullptr, const XStage xst = XStage{},
    const uint8_t* __restrict__ tvidx = nullptr, const double* __restrict__ tvtab = nullptr, int vt = 0) {
    // ANC (anchored dictionary): column = the row's first column (slot anchors, tanc) +
    // table[index] instead of row + table[index]
    static_assert(!ANC || CD != 0, "anchored columns are dictionary columns");
    static_assert(!XS || (CD != 0 && !ANC), "x staging needs row-relative dictionary columns");
    static_assert(!PT || (CD != 0 && !ANC), "per-tile tables: row-relative");
    static_assert(!(XS && PT), "x staging uses the set-wide table");
    constexpr int BS = kBlock;
    constexpr int G = TNNZ / (4 * BS);
    static_assert(G >= 1 && TNNZ % (4 * BS) == 0, "tile budget must be a multiple of 4 x block");
    __shared__ __attribute__((aligned(16))) double lprod[TNNZ + 8];
    __shared__ double ldiag[OP == OP_JACOBI ? BS : 1];
    __shared__ int lwt[BS / 64];
    // XS keeps only the table's LDS positions (kXsIoff + index): 16 / 128 entries, so the
    // staged runs fit beside Jacobi's arrays at 8 blocks per CU
    // 2048-nonzero tiles keep per-tile tables of <= kTmSmallTab entries (checked at upload,
    // build_tile_major), so one more block fits per CU (512^3 A1: residual 7 -> 8, Jacobi 6 -> 7
    // waves per SIMD; -2.4 % / -4.6 %, profiles/r03_lds/)
    constexpr int NTAB = CD == 0 ? 1 : XS ? (CD == 4 ? 16 : kXsIoff) : PT && TNNZ == 2048 ? kTmSmallTab : BS;
    constexpr int NVT = TNNZ == 2048 ? kTmSmallTab : BS;
    __shared__ int ltab[NTAB];
    __shared__ __attribute__((aligned(4))) uint8_t lrow[TNNZ + 8];
    __shared__ int lanc[ANC ? BS : 1];
    __shared__ double lxs[XS ? kXsCap + 1 : 1];  // + 1: the dump slot of lanes past a run
    __shared__ double lvt[VD8 ? NVT : 1];        // the tile's value table (vt <= NVT entries)

    const int t = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int4 d = tiles[t];
    const size_t sb = (size_t)t * TNNZ;
    const int r0 = d.x, nr = d.y - d.x, cnt = d.w - d.z;
    // Load order matters: vmcnt retires loads in issue order, so a wait for a load also waits
    // for every load issued before it. The small loads the dependent phases need first —
    // dictionary table and row anchors, row lengths (scan), column stream (gathers), the
    // epilogue's own-row operands — go out first, branch-free (clamped addresses), and the
    // value stream last: the scan, the row map and the x gathers then proceed while the
    // values are still in flight (previously the scan's wait on the row lengths also waited
    // for the whole value stream, and the gathers' wait on the columns for b / x).
    int tabv = 0, ancv = 0;
    if constexpr (XS) tabv = ctab[kXsIoff + (tid < NTAB ? tid : NTAB - 1)];
    else if constexpr (PT) tabv = ctab[(size_t)t * ctab_n + (tid < ctab_n ? tid : ctab_n - 1)];
    else if constexpr (CD != 0) tabv = ctab[tid];  // the table is allocated with 256 entries
    const size_t rsl = (size_t)t * rs + (tid < rs ? tid : rs - 1);
    if constexpr (ANC) ancv = tanc[rsl];
    const int rlv = (int)trlen[rsl];
    double vtv = 0.0;
    if constexpr (VD8) vtv = tvtab[(size_t)t * vt + (tid < vt ? tid : vt - 1)];
    double2 va[G], vb[G];
    uint32_t vi[G];
    uint32_t cn[G];
    ushort4 clo4[G];
    int cb = 0;
    if constexpr (CD == 0) cb = tbase[t];
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const size_t q = sb + 4 * (tid + j * BS);
        if constexpr (CD == 4) {
            cn[j] = *reinterpret_cast<const uint16_t*>(tcidx + (q >> 1));
        } else if constexpr (CD == 8) {
            cn[j] = *reinterpret_cast<const uint32_t*>(tcidx + q);
        } else {  // 24-bit: low 16 bits per nonzero + the four high bytes packed in cn
            clo4[j] = *reinterpret_cast<const ushort4*>(tclo + q);
            cn[j] = *reinterpret_cast<const uint32_t*>(tchi + q);
        }
    }
    double pb = 0.0, px = 0.0, py = 0.0;
    {
        const int r = r0 + (tid < nr ? tid : 0);  // padding tiles are (0, 0, 0, 0): row 0
        if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[r];
        if constexpr (OP == OP_JACOBI) px = x[r];
        if constexpr (OP == OP_PROLONG) py = y[r];
    }
    double xsv[XS ? kXsMaxClusters : 1];
    if constexpr (XS) {
#pragma unroll
        for (int c = 0; c < kXsMaxClusters; ++c) {
            xsv[c] = 0.0;
            if (c < xst.ncl) {  // uniform
                const int g = r0 + xst.omin[c] + tid;
                const bool ok = tid < nr + xst.wid[c] && g >= 0 && g < xst.ncols;
                xsv[c] = x[ok ? g : 0];
            }
        }
    }
    asm volatile("" ::: "memory");  // keep the loads above ahead of the value stream
    // the whole value slot is loaded at entry (padding included: a load that waits for the
    // descriptor's nonzero count brings its round trip back — measured 2-15 % slower)
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const size_t q = sb + 4 * (tid + j * BS);
        if constexpr (VD8) {
            vi[j] = *reinterpret_cast<const uint32_t*>(tvidx + q);
        } else {
            va[j] = *reinterpret_cast<const double2*>(tval + q);
            vb[j] = *reinterpret_cast<const double2*>(tval + q + 2);
        }
    }
    int rl_len = tid < rs ? rlv : 0;
    if constexpr (VD8) lvt[tid < NVT ? tid : NVT - 1] = vtv;  // every lane (lanes past vt repeat the last entry)
    // every lane stores its entry (unconditionally: a conditional store lets the compiler sink
    // the table load into the branch, behind the value stream)
    if constexpr (XS) ltab[tid < NTAB ? tid : NTAB - 1] = tabv;  // lanes past NTAB rewrite the last entry's value
    else if constexpr (CD != 0) ltab[tid < NTAB ? tid : NTAB - 1] = tabv;  // (lanes past ctab_n: the last entry)
    if constexpr (ANC) lanc[tid] = tid < rs ? ancv : 0;
    if constexpr (XS) {
#pragma unroll
        for (int c = 0; c < kXsMaxClusters; ++c)
            if (c < xst.ncl) lxs[tid < xst.stride ? c * xst.stride + tid : kXsCap] = xsv[c];
    }
    const int rl_inc = wave_incl_scan(rl_len);
    if (lane == 63) lwt[tid >> 6] = rl_inc;
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
    if constexpr (VD8 && !NEED_ROWS) __syncthreads();  // lvt
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
        if constexpr (NEED_ROWS) rw = q < cnt ? *reinterpret_cast<const uint32_t*>(&lrow[q]) : 0u;
        if constexpr (XS) {  // x from the staged runs; cc holds the dictionary index
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int ix = CD == 4 ? (int)((cn[j] >> (4 * e)) & 15u) : (int)((cn[j] >> (8 * e)) & 255u);
                // past the tile's last nonzero the row byte is stale LDS: read slot 0 instead (the
                // product is discarded), so every LDS read stays inside lxs
                const int rid = q + e < cnt ? (int)((rw >> (8 * e)) & 255u) : 0;
                cc[j][e] = ix;
                xv[j][e] = lxs[ltab[ix] + rid];
            }
            continue;
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
                const int rid = (int)((rw >> (8 * e)) & 255u);
                if constexpr (ANC) cc[j][e] = lanc[rid] + ltab[ix];
                else cc[j][e] = r0 + rid + ltab[ix];
            }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[j][e] = x[q + e < cnt ? cc[j][e] : 0];
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
        const int q = 4 * (tid + j * BS);
        uint32_t rw = 0u;
        if constexpr (NEED_ROWS) rw = q < cnt ? *reinterpret_cast<const uint32_t*>(&lrow[q]) : 0u;
        double vv[4];
        if constexpr (VD8) {
#pragma unroll
            for (int e = 0; e < 4; ++e) vv[e] = lvt[(vi[j] >> (8 * e)) & 255u];
        } else {
            vv[0] = va[j].x;
            vv[1] = va[j].y;
            vv[2] = vb[j].x;
            vv[3] = vb[j].y;
        }
        double p[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool ok = q + e < cnt;
            p[e] = ok ? vv[e] * xv[j][e] : 0.0;
            if constexpr (OP == OP_JACOBI) {
                const int rl = (int)((rw >> (8 * e)) & 255u);
                if (ok && (XS ? cc[j][e] == xst.zix : cc[j][e] - r0 == rl)) ldiag[rl] = vv[e];
            }
        }
        *reinterpret_cast<double2*>(&lprod[q]) = make_double2(p[0], p[1]);
        *reinterpret_cast<double2*>(&lprod[q + 2]) = make_double2(p[2], p[3]);
    }
    __syncthreads();
    if constexpr (!NEED_ROWS) re = row_end();
    // unconditional epilogue, conditional store (see k_rows_tile2); lanes past the tile's
    // rows have rl_len = 0 and sum an empty range
    const double s = row_sum_lds(lprod, re - rl_len, re);
    double out;
    if constexpr (OP == OP_SPMV) {
        out = s;
    } else if constexpr (OP == OP_RESID) {
        out = pb - s;
    } else if constexpr (OP == OP_JACOBI) {
        const double u = pb - s;
        const double v = omega * u;
        const double w = v / ldiag[tid < nr ? tid : 0];
        out = px + w;
    } else {
        out = py + s;
    }
    if (tid < nr) y[r0 + tid] = out;
}
// k_rows_sym: the symmetric diagonal-class layout (pamg::SymDia). One row per lane; every
// operand is a coalesced stream over consecutive rows — the diagonal, the NU upper-value
// arrays U_c[i], their mirrors U_c[i - o_c] (the lower values: the same lines a block o_c rows
// earlier read, so L2 / Infinity-Cache hits, not HBM traffic), x[i +- o_c], b, y — with no
// column stream, no row map and no LDS. Products are summed in ascending offset order from
// +0.0, present entries only (mask), which is each row's storage order (checked at upload):
// SPEC §S3 bits. Blocks walk the rows XCD-banded: block b runs on XCD b % 8 (dispatch deals
// blocks round-robin), and XCD k takes the k-th eighth of every band of `band` rows (a grid
// plane), so the mirror and x lines of planes z-1, z, z+1 stay in that XCD's L2.
// The row mask is one byte per row where 2 NU + 1 <= 7 entries fit beside the in-set flag (bit 7;
// the 7-point stencils), else 16 bits (flag bit 15).
template <int NU>
struct SymMask {
    static constexpr bool kByte = 2 * NU + 1 <= 7;
    static constexpr uint32_t kIn = kByte ? 0x80u : 0x8000u;
    __device__ static uint32_t one(const uint8_t* m, int64_t i) {
        if constexpr (kByte) return m[i];
        else return reinterpret_cast<const uint16_t*>(m)[i];
    }
    __device__ static void two(const uint8_t* m, int64_t i, uint32_t (&out)[2]) {  // i even
        if constexpr (kByte) {
            const uint32_t w = *reinterpret_cast<const uint16_t*>(m + i);
            out[0] = w & 0xffu;
            out[1] = w >> 8;
        } else {
            const uint32_t w = *reinterpret_cast<const uint32_t*>(m + 2 * i);
            out[0] = w & 0xffffu;
            out[1] = w >> 16;
        }
    }
};

// the grid plane of band j of a plane-window launch (launch_sym_planes): plane0 + j, the planes from
// gap_at on shifted by gap (two windows in one launch)
__device__ __forceinline__ int sym_plane(const SymDia& sd, int j) {
    const int p = sd.plane0 + j;
    return p >= sd.gap_at ? p + sd.gap : p;
}

template <int OP, int NU>
__global__ __launch_bounds__(kBlock) void k_rows_sym(
    int nrows, int ncols, const uint8_t* __restrict__ mask, const double* __restrict__ dg,
    const double* __restrict__ up, int64_t ld, const SymDia sd, const double* __restrict__ x,
    const double* __restrict__ b, double* __restrict__ y, double omega) {
    const int bid = blockIdx.x, tid = threadIdx.x;
    const int xcd = bid & 7, j = bid >> 3;
    const int plane = sym_plane(sd, j / sd.eighth), blk = xcd * sd.eighth + j % sd.eighth;
    const int64_t lo = (int64_t)plane * sd.band;
    const int64_t i64 = lo + (int64_t)blk * kBlock + tid;
    const int64_t hi = lo + sd.band < nrows ? lo + sd.band : nrows;
    const bool in = blk < sd.band_blocks && i64 < hi;
    const int i = in ? (int)i64 : 0;
    const uint32_t m = SymMask<NU>::one(mask, i);
    // operands in ascending offset order: lower classes (mirrors), diagonal, upper classes
    double v[2 * NU + 1], xv[2 * NU + 1];
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        const int o = sd.off[NU - 1 - c];
        const int jl = i - o >= 0 ? i - o : 0;
        v[c] = up[(size_t)(NU - 1 - c) * ld + jl];
        xv[c] = x[jl];
    }
    v[NU] = dg[i];
    xv[NU] = x[i];
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        const int ju = i + sd.off[c] < ncols ? i + sd.off[c] : i;
        v[NU + 1 + c] = up[(size_t)c * ld + i];
        xv[NU + 1 + c] = x[ju];
    }
    double pb = 0.0;
    if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[i];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 2 * NU + 1; ++k) {
        const double p = v[k] * xv[k];
        const double t = s + p;
        s = ((m >> k) & 1u) ? t : s;
    }
    double out;
    if constexpr (OP == OP_SPMV) {
        out = s;
    } else if constexpr (OP == OP_RESID) {
        out = pb - s;
    } else {
        const double u = pb - s;
        const double w = omega * u;
        const double q = w / v[NU];
        out = xv[NU] + q;
    }
    if (in && (m & SymMask<NU>::kIn)) y[i] = out;
}

// Two consecutive rows per lane (Options::sym_rows = 2): the own-row streams (mask, diagonal,
// upper values, b, x[i]) become 16-byte loads; a mirror or x run at an odd offset is not
// 16-byte aligned and is read as two 8-byte loads (the offsets are uniform, so is the branch).
__device__ __forceinline__ double2 ld_pair(const double* __restrict__ p, int64_t j, int64_t n, bool even) {
    if (even && j >= 0 && j + 1 < n) return *reinterpret_cast<const double2*>(p + j);
    return make_double2(p[j >= 0 && j < n ? j : 0], p[j + 1 >= 0 && j + 1 < n ? j + 1 : 0]);
}

template <int OP, int NU>
__global__ __launch_bounds__(kBlock) void k_rows_sym2(
    int nrows, int ncols, const uint8_t* __restrict__ mask, const double* __restrict__ dg,
    const double* __restrict__ up, int64_t ld, const SymDia sd, const double* __restrict__ x,
    const double* __restrict__ b, double* __restrict__ y, double omega) {
    constexpr int RB = 2 * kBlock;  // rows per block
    const int bid = blockIdx.x, tid = threadIdx.x;
    const int xcd = bid & 7, j = bid >> 3;
    const int plane = sym_plane(sd, j / sd.eighth), blk = xcd * sd.eighth + j % sd.eighth;
    const int64_t lo = (int64_t)plane * sd.band;
    const int64_t i0 = lo + (int64_t)blk * RB + 2 * tid;
    const int64_t hi = lo + sd.band < nrows ? lo + sd.band : nrows;
    const bool blk_ok = blk < sd.band_blocks;
    const bool in0 = blk_ok && i0 < hi, in1 = blk_ok && i0 + 1 < hi;
    const int64_t n = nrows;
    const int64_t ib = in0 ? i0 : 0;  // even
    uint32_t m[2];
    SymMask<NU>::two(mask, ib, m);
    double v[2][2 * NU + 1], xv[2][2 * NU + 1];
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        const int o = sd.off[NU - 1 - c];
        const double2 a = ld_pair(up + (size_t)(NU - 1 - c) * ld, ib - o, n, (o & 1) == 0);
        const double2 xx = ld_pair(x, ib - o, ncols, (o & 1) == 0);
        v[0][c] = a.x;
        v[1][c] = a.y;
        xv[0][c] = xx.x;
        xv[1][c] = xx.y;
    }
    {
        const double2 d = *reinterpret_cast<const double2*>(dg + ib);
        const double2 xx = ld_pair(x, ib, ncols, true);
        v[0][NU] = d.x;
        v[1][NU] = d.y;
        xv[0][NU] = xx.x;
        xv[1][NU] = xx.y;
    }
#pragma unroll
    for (int c = 0; c < NU; ++c) {
        const int o = sd.off[c];
        const double2 a = *reinterpret_cast<const double2*>(up + (size_t)c * ld + ib);
        const double2 xx = ld_pair(x, ib + o, ncols, (o & 1) == 0);
        v[0][NU + 1 + c] = a.x;
        v[1][NU + 1 + c] = a.y;
        xv[0][NU + 1 + c] = xx.x;
        xv[1][NU + 1 + c] = xx.y;
    }
    double2 pb = make_double2(0.0, 0.0);
    if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = ld_pair(b, ib, n, true);
    const double pbv[2] = {pb.x, pb.y};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 2 * NU + 1; ++k) {
            const double p = v[r][k] * xv[r][k];
            const double t = s + p;
            s = ((m[r] >> k) & 1u) ? t : s;
        }
        double out;
        if constexpr (OP == OP_SPMV) {
            out = s;
        } else if constexpr (OP == OP_RESID) {
            out = pbv[r] - s;
        } else {
            const double u = pbv[r] - s;
            const double w = omega * u;
            const double q = w / v[r][NU];
            out = xv[r][NU] + q;
        }
        if ((r == 0 ? in0 : in1) && (m[r] & SymMask<NU>::kIn)) y[ib + r] = out;
    }
}

// k_rows_symd: k_rows_sym2 over the row-class dictionary (SymDia::vd_n): a row's mask, diagonal
// and upper values are its class's (table in LDS), a lower value a(i, i - o_c) is U_c of the
// class of row i - o_c — so the matrix streams one byte per row (its class id; the mirror rows'
// ids are the same bytes a block o_c rows earlier read, cache hits) instead of 33. The products
// and their order are k_rows_sym2's, so are the bits.
template <int NU>
struct SymTab {  // the class table in LDS: values (D, U_0 .. U_{NU-1}) per class, masks, 1 / D
    double v[kSymVdMax][NU + 1];
    uint32_t m[kSymVdMax];
    double r[kSymVdMax];  // RN(1 / D) (div_rn)
};

template <int NU>
__device__ __forceinline__ void symtab_fill(SymTab<NU>& t, const double* __restrict__ vtab,
                                            const uint32_t* __restrict__ mtab, int nv) {
    for (int e = threadIdx.x; e < nv * (NU + 1); e += blockDim.x) (&t.v[0][0])[e] = vtab[e];
    for (int e = threadIdx.x; e < nv; e += blockDim.x) {
        t.m[e] = mtab[e];
        t.r[e] = 1.0 / vtab[e * (NU + 1)];
    }
}

// RN(w / d) given r = RN(1 / d): q0 = RN(w r) and two residual corrections through exact FMA
// residuals (Markstein: q1 is within one ulp of w / d, so q2 = RN(q1 + (w - q1 d) r) is the
// correctly rounded quotient) — 5 f64 operations instead of the ~11 of the IEEE division
// sequence. Outside |w| in [2^-900, 2^900] (zeros — whose sign the sequence could lose —,
// subnormals, huge values, inf, NaN) and for a d whose reciprocal is not a normal number, the
// division itself. Bitwise the same as w / d (checked on 3e8 random and near-midpoint cases,
// tools/div_check.c, and by every oracle test of the kernels that use it).
__device__ __forceinline__ double div_rn(double w, double d, double r) {
    const double aw = fabs(w), ar = fabs(r);
    if (aw >= 0x1p-900 && aw <= 0x1p900 && ar >= 0x1p-900 && ar <= 0x1p900) {
        const double q0 = w * r;
        const double e0 = __builtin_fma(-q0, d, w);
        const double q1 = __builtin_fma(e0, r, q0);
        const double e1 = __builtin_fma(-q1, d, w);
        return __builtin_fma(e1, r, q1);
    }
    return w / d;
}

__device__ __forceinline__ uint16_t tbd_pair_ids(const uint8_t* __restrict__ tid, int64_t j, int64_t n) {
    j = j < 0 ? 0 : (j > n - 2 ? n - 2 : j);  // (even j; clamped ones meet clear mask bits only)
    return *reinterpret_cast<const uint16_t*>(tid + j);
}

__device__ __forceinline__ uint32_t tid_at(const uint8_t* __restrict__ tid, int64_t j, int64_t n) {
    return tid[j >= 0 && j < n ? j : 0];
}

// CH (Options::symd_chunks): a block takes CH consecutive 512-row units of its XCD's eighths
// (unit u = (blockIdx / 8) CH + k, the banded order of k_rows_sym2 otherwise unchanged), so the
// class table is filled and waited for once per CH units; the units' loads go out two at a time.
template <int OP, int NU, int CH = 1>
__global__ __launch_bounds__(kBlock) void k_rows_symd(
    int nrows, int ncols, const uint8_t* __restrict__ tid, const double* __restrict__ vtab,
    const uint32_t* __restrict__ mtab, int nv, const SymDia sd, const double* __restrict__ x,
    const double* __restrict__ b, double* __restrict__ y, double omega) {
    constexpr int RB = 2 * kBlock;  // rows per unit
    constexpr int P = CH < 2 ? CH : 2;
    static_assert(CH % P == 0, "units in pairs");
    __shared__ SymTab<NU> tab;
    const int bid = blockIdx.x, tidx = threadIdx.x;
    const int xcd = bid & 7, u0 = (bid >> 3) * CH;
    const int nunits = sd.nbands * sd.eighth;
    const int64_t n = nrows;
#pragma unroll 1
    for (int k0 = 0; k0 < CH; k0 += P) {
        int64_t ib[P];
        bool in0[P], in1[P];
        uint32_t tw[P], tl[P][2][NU];
        double xv[P][2][2 * NU + 1], pbv[P][2];
#pragma unroll
        for (int q = 0; q < P; ++q) {
            const int u = u0 + k0 + q;
            const int plane = sym_plane(sd, u / sd.eighth), blk = xcd * sd.eighth + u % sd.eighth;
            const int64_t lo = (int64_t)plane * sd.band;
            const int64_t i0 = lo + (int64_t)blk * RB + 2 * tidx;
            const int64_t hi = lo + sd.band < nrows ? lo + sd.band : nrows;
            const bool ok = u < nunits && blk < sd.band_blocks;
            in0[q] = ok && i0 < hi;
            in1[q] = ok && i0 + 1 < hi;
            ib[q] = in0[q] ? i0 : 0;  // even
            // every global load first (ids, mirror ids, x, b), then the table, one barrier
            tw[q] = *reinterpret_cast<const uint16_t*>(tid + ib[q]);
#pragma unroll
            for (int c = 0; c < NU; ++c) {
                const int o = sd.off[NU - 1 - c];
                tl[q][0][c] = tid_at(tid, ib[q] - o, n);
                tl[q][1][c] = tid_at(tid, ib[q] + 1 - o, n);
                const double2 xx = ld_pair(x, ib[q] - o, ncols, (o & 1) == 0);
                xv[q][0][c] = xx.x;
                xv[q][1][c] = xx.y;
            }
            {
                const double2 xx = ld_pair(x, ib[q], ncols, true);
                xv[q][0][NU] = xx.x;
                xv[q][1][NU] = xx.y;
            }
#pragma unroll
            for (int c = 0; c < NU; ++c) {
                const int o = sd.off[c];
                const double2 xx = ld_pair(x, ib[q] + o, ncols, (o & 1) == 0);
                xv[q][0][NU + 1 + c] = xx.x;
                xv[q][1][NU + 1 + c] = xx.y;
            }
            double2 pb = make_double2(0.0, 0.0);
            if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = ld_pair(b, ib[q], n, true);
            pbv[q][0] = pb.x;
            pbv[q][1] = pb.y;
        }
        if (k0 == 0) {  // (uniform)
            symtab_fill<NU>(tab, vtab, mtab, nv);
            __syncthreads();
        }
#pragma unroll
        for (int q = 0; q < P; ++q) {
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const uint32_t t = r == 0 ? (tw[q] & 0xffu) : (tw[q] >> 8);
                const uint32_t m = tab.m[t];
                double v[2 * NU + 1];
#pragma unroll
                for (int c = 0; c < NU; ++c) v[c] = tab.v[tl[q][r][c]][1 + (NU - 1 - c)];
                v[NU] = tab.v[t][0];
#pragma unroll
                for (int c = 0; c < NU; ++c) v[NU + 1 + c] = tab.v[t][1 + c];
                double s = 0.0;
#pragma unroll
                for (int k = 0; k < 2 * NU + 1; ++k) {
                    const double p = v[k] * xv[q][r][k];
                    const double w = s + p;
                    s = ((m >> k) & 1u) ? w : s;
                }
                double out;
                if constexpr (OP == OP_SPMV) {
                    out = s;
                } else if constexpr (OP == OP_RESID) {
                    out = pbv[q][r] - s;
                } else {
                    const double w0 = pbv[q][r] - s;
                    const double w = omega * w0;
                    const double w2 = w / v[NU];
                    out = xv[q][r][NU] + w2;
                }
                if ((r == 0 ? in0[q] : in1[q]) && (m & SymMask<NU>::kIn)) y[ib[q] + r] = out;
            }
        }
    }
}

// ------------------------------------------------------------------ temporally blocked sweeps
// k_sym_tb<S>: S dependent sweeps (Jacobi, [Jacobi,] then Jacobi or the residual) over a 7-point
// grid stencil held in the symmetric layout, in ONE pass over the matrix (Options::jr_fuse):
// the V-cycle's level-0 pre-smoothing + residual (S = 2) and, across a cycle boundary, the
// post-smoothing of one cycle + the pre-smoothing and residual of the next (S = 3).
// 2.5-D temporal blocking: a workgroup owns a kTbX x kTbY column of the grid over a range of
// planes and streams it along z. At step k it computes stage 0 on plane k over the tile plus a
// halo of S-1 lines (and 2 points in x), stage 1 on plane k-1 (halo S-2), ..., each stage reading
// its predecessor's planes k-s-1 .. k-s+1 from a 3-plane LDS ring; the halo is recomputed by
// every workgroup that needs it, so nothing passes between workgroups inside the launch (no
// flags, no cross-XCD visibility question). A thread keeps its row pair's operator values and b
// for the last three planes in registers (the ring c0/c1/c2, rotated by a 3-way unrolled z loop),
// so the matrix streams from HBM once for all S sweeps. Every value is computed by exactly
// k_rows_sym2's expression for its row (ascending class order from +0.0, present entries only,
// SPEC §S3), so halo copies are bit-identical and the outputs equal S separate sweeps.
// Preconditions (runtime.hip build_sym_dia, SymDia::tb_ok): classes {1, nx, nx*ny}, n =
// nx*ny*nz, nx % kTbX == 0, ny % kTbY == 0, every row in the set, and no row has an entry across
// a grid line or plane (so points outside the grid contribute nothing and are held as zeros).
constexpr int kTbPX = (kTbX + 4) / 2;  // row pairs per line: x0-2 .. x0+kTbX+1
constexpr int kTbLW = kTbX + 8;        // LDS line: column x - x0 + 4 (even for even x; pads 0-1, kTbX+6-7)

template <int S, int TY = kTbY>
struct TbShape {                                 // TY: tile height (kTbY)
    static constexpr int H = S - 1;              // stage-0 halo in y and z
    static constexpr int RY = TY + 2 * H;        // grid lines of stage 0
    static constexpr int NT = kTbPX * RY;        // threads with a row pair
    static constexpr int threads = (NT + 63) / 64 * 64;
    static constexpr int XL = RY + 2;            // lines of the in0 window (stage 0's region + 1)
    static constexpr int XPAIRS = XL * (kTbLW / 2);  // its row pairs: x0-4 .. x0+kTbX+3
};

struct TbCoef {        // one row pair on one plane: the 7 values in ascending class order, b, masks
    double v[2][7];
    double b[2];
    uint16_t mw;       // the two rows' mask bytes as loaded (split at use, not right after the load)
};

__device__ __forceinline__ int tb_mod3(int k) { return ((k % 3) + 3) % 3; }

// An aligned pair p[j], p[j+1] (j even) through ONE 16-B load; a pair outside [0, n) is read at
// the nearest end instead: its values only ever meet mask bits that are clear (no row of the
// grid reaches outside it), so they are discarded.
__device__ __forceinline__ double2 tb_pair(const double* __restrict__ p, int64_t j, int64_t n) {
    j = j < 0 ? 0 : (j > n - 2 ? n - 2 : j);
    return *reinterpret_cast<const double2*>(p + j);
}

// prev: the same pair's values one plane down (held in the register ring): its U2 is this
// plane's -M mirror, so only the first plane of a workgroup loads that mirror
template <bool FIRST>
__device__ __forceinline__ void tb_load(TbCoef& c, const TbCoef& prev, const uint8_t* __restrict__ mask,
                                        const double* __restrict__ dg, const double* __restrict__ up, int64_t ld,
                                        const SymDia& sd, const double* __restrict__ b, int64_t i, int64_t n) {
    c.mw = *reinterpret_cast<const uint16_t*>(mask + i);
    // ascending classes -M, -nx, -1, 0, +1, +nx, +M; the lower values from the mirrors
    const double2 u0 = *reinterpret_cast<const double2*>(up + i);
    const double2 u1 = *reinterpret_cast<const double2*>(up + ld + i);
    const double2 u2 = *reinterpret_cast<const double2*>(up + 2 * ld + i);
    const double2 m2 = FIRST ? tb_pair(up + 2 * ld, i - sd.off[2], n) : make_double2(prev.v[0][6], prev.v[1][6]);
    const double2 m1 = tb_pair(up + ld, i - sd.off[1], n);
    const double2 m0 = tb_pair(up, i - 2, n);  // U0[i-1] = a(i, i-1); row i+1's is U0[i]
    const double2 d = *reinterpret_cast<const double2*>(dg + i);
    c.v[0][0] = m2.x; c.v[1][0] = m2.y;
    c.v[0][1] = m1.x; c.v[1][1] = m1.y;
    c.v[0][2] = m0.y; c.v[1][2] = u0.x;
    c.v[0][3] = d.x;  c.v[1][3] = d.y;
    c.v[0][4] = u0.x; c.v[1][4] = u0.y;
    c.v[0][5] = u1.x; c.v[1][5] = u1.y;
    c.v[0][6] = u2.x; c.v[1][6] = u2.y;
    const double2 bb = *reinterpret_cast<const double2*>(b + i);
    c.b[0] = bb.x;
    c.b[1] = bb.y;
}

// the row pair's outputs from its operator values and the 7 neighbour values of each row
__device__ __forceinline__ void tb_rows(const TbCoef& c, const double (&xv)[2][7], bool resid, double omega,
                                        double (&out)[2]) {
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const uint32_t m = r == 0 ? ((uint32_t)c.mw & 0xffu) : ((uint32_t)c.mw >> 8);
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const double p = c.v[r][k] * xv[r][k];
            const double t = s + p;
            s = ((m >> k) & 1u) ? t : s;
        }
        if (resid) {
            out[r] = c.b[r] - s;
        } else {
            const double u = c.b[r] - s;
            const double w = omega * u;
            const double q = w / c.v[r][3];
            out[r] = xv[r][3] + q;
        }
    }
}

template <int S>
struct TbCtx {
    int nx, ny, nz, zs, ze, kend;
    int64_t M, n;
    int ry, col;
    int64_t ixy;          // y * nx + x of the pair's first row
    bool pos_ok, own_xy;
    int x0, y0;           // the tile's first grid point
};

// The workgroup's tile and the thread's row pair (k_sym_tb / k_sym_zc); false: no tile (the
// whole workgroup returns before any barrier). Tiles: consecutive tiles on one XCD (block b runs
// on XCD b % 8; speed only), ordered y-fastest so that the tiles sharing the wide y halos
// (kTbX + 4 points x S-1 lines) sit on one XCD.
template <int S, int TY = kTbY>
__device__ __forceinline__ bool tb_ctx_init(TbCtx<S>& t, const TbGeom& g, int nrows) {
    using Sh = TbShape<S, TY>;
    const int ntiles = g.tiles_x * g.tiles_y * g.zchunks;
    const int per = (ntiles + 7) / 8;
    const int lin = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (lin >= ntiles) return false;
    // y-fastest: an XCD's tiles are one x column of the grid (its y halos shared in its L2); x-fastest
    // (TbGeom::xfast): whole rows of tiles, so the 128-B lines a tile's x halo touches are read once per
    // XCD instead of by two XCDs each
    const int ty = g.xfast ? (lin / g.tiles_x) % g.tiles_y : lin % g.tiles_y;
    const int tx = g.xfast ? lin % g.tiles_x : (lin / g.tiles_y) % g.tiles_x, zc = lin / (g.tiles_x * g.tiles_y);
    if (g.zlo + zc * g.zlen >= g.zhi) return false;  // (a chunk past the output range: uniform)
    const int x0 = tx * kTbX, y0 = ty * TY;
    t.x0 = x0;
    t.y0 = y0;
    t.nx = g.nx;
    t.ny = g.ny;
    t.nz = g.nz;
    t.zs = g.zlo + zc * g.zlen;
    t.ze = min(t.zs + g.zlen, g.zhi);
    t.kend = t.ze + Sh::H;
    t.M = (int64_t)g.nx * g.ny;
    t.n = nrows;
    const int tid = threadIdx.x;
    const bool has = tid < Sh::NT;
    const int px = has ? tid % kTbPX : 0;
    t.ry = has ? tid / kTbPX : -1;
    const int x = x0 - 2 + 2 * px, y = y0 - Sh::H + (has ? t.ry : 0);
    t.col = 2 * px + 2;
    t.ixy = (int64_t)y * g.nx + x;
    t.pos_ok = has && x >= 0 && x < g.nx && y >= 0 && y < g.ny;
    t.own_xy = t.pos_ok && px >= 1 && px <= kTbX / 2 && y >= y0 && y < y0 + TY;
    return true;
}

// The in0 window of plane q (stage 0's region + one point / line around it, zeros outside the
// grid), as the pairs thread tid moves: loads issued now (clamped addresses, no branch), stored
// into the LDS ring later (tb_win_store) so their latency overlaps the step's other work.
template <int S>
struct TbWin {
    double2 v[2];
    bool ok[2];
};
template <int S, int TY = kTbY>
__device__ __forceinline__ void tb_win_load(TbWin<S>& w, const TbCtx<S>& t, const double* __restrict__ in0, int q) {
    using Sh = TbShape<S, TY>;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int p = threadIdx.x + h * Sh::threads;
        const int line = p / (kTbLW / 2), pc = p % (kTbLW / 2);
        const int x = t.x0 - 4 + 2 * pc, y = t.y0 - Sh::H - 1 + line;
        w.ok[h] = p < Sh::XPAIRS && x >= 0 && x < t.nx && y >= 0 && y < t.ny && q >= 0 && q < t.nz;
        w.v[h] = tb_pair(in0, (int64_t)q * t.M + (int64_t)y * t.nx + x, t.n);
    }
}
template <int S, int TY = kTbY>
__device__ __forceinline__ void tb_win_store(const TbWin<S>& w, double (*xin)[TbShape<S, TY>::XL][kTbLW], int slot) {
    using Sh = TbShape<S, TY>;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int p = threadIdx.x + h * Sh::threads;
        if (p < Sh::XPAIRS)
            *reinterpret_cast<double2*>(&xin[slot][p / (kTbLW / 2)][2 * (p % (kTbLW / 2))]) =
                w.ok[h] ? w.v[h] : make_double2(0.0, 0.0);
    }
}

// the 7 neighbour values of a row pair from an LDS plane ring (planes p-1, p, p+1 in slots
// sm, s0, sp; lines ry-1, ry, ry+1)
template <int RY>
__device__ __forceinline__ void tb_gather_lds(const double (*ring)[RY][kTbLW], int sm, int s0, int sp, int ry, int col,
                                              double (&xv)[2][7]) {
    const double2 own = *reinterpret_cast<const double2*>(&ring[s0][ry][col]);
    const double2 lft = *reinterpret_cast<const double2*>(&ring[s0][ry][col - 2]);
    const double2 rgt = *reinterpret_cast<const double2*>(&ring[s0][ry][col + 2]);
    const double2 dn = *reinterpret_cast<const double2*>(&ring[s0][ry - 1][col]);
    const double2 upl = *reinterpret_cast<const double2*>(&ring[s0][ry + 1][col]);
    const double2 zl = *reinterpret_cast<const double2*>(&ring[sm][ry][col]);
    const double2 zh = *reinterpret_cast<const double2*>(&ring[sp][ry][col]);
    xv[0][0] = zl.x;  xv[1][0] = zl.y;
    xv[0][1] = dn.x;  xv[1][1] = dn.y;
    xv[0][2] = lft.y; xv[1][2] = own.x;
    xv[0][3] = own.x; xv[1][3] = own.y;
    xv[0][4] = own.y; xv[1][4] = rgt.x;
    xv[0][5] = upl.x; xv[1][5] = upl.y;
    xv[0][6] = zh.x;  xv[1][6] = zh.y;
}

template <int S, bool FIRST>
__device__ __forceinline__ void tb_step(int k, TbCoef& cA, TbCoef& cB, TbCoef& cC, const TbCtx<S>& t,
                                        const uint8_t* __restrict__ mask, const double* __restrict__ dg,
                                        const double* __restrict__ up, int64_t ld, const SymDia& sd,
                                        const TbArgs& ta, double (*l0)[TbShape<S>::RY][kTbLW],
                                        double (*l1)[TbShape<S>::RY][kTbLW],
                                        double (*xin)[TbShape<S>::XL][kTbLW]) {
    using Sh = TbShape<S>;
    if (k >= t.kend) return;  // uniform: the whole workgroup
    // ---- stage 0 on plane k: a Jacobi sweep from in0 (its window ring in LDS: planes k-1..k+1)
    {
        double o[2] = {0.0, 0.0};
        const bool act0 = t.pos_ok && k >= 0 && k < t.nz;
        const int64_t i = (int64_t)k * t.M + t.ixy;
        // the in0 window of plane k+1 into the slot of plane k-2 (last read by the previous
        // step's stage 0), its loads issued with this plane's operator loads (one latency)
        {
            TbWin<S> win;
            if (act0) tb_load<FIRST>(cA, cB, mask, dg, up, ld, sd, ta.b, i, t.n);
            tb_win_load<S>(win, t, ta.in0, k + 1);
            tb_win_store<S>(win, xin, tb_mod3(k + 1));
        }
        __syncthreads();
        if (act0) {
            double xv[2][7];
            tb_gather_lds<Sh::XL>(xin, tb_mod3(k - 1), tb_mod3(k), tb_mod3(k + 1), t.ry + 1, t.col, xv);
            tb_rows(cA, xv, S == 1 && ta.last_resid, ta.omega, o);
            if (ta.out[0] && t.own_xy && k >= t.zs && k < t.ze)
                *reinterpret_cast<double2*>(ta.out[0] + i) = make_double2(o[0], o[1]);
        }
        if (t.ry >= 0) *reinterpret_cast<double2*>(&l0[tb_mod3(k)][t.ry][t.col]) = make_double2(o[0], o[1]);
    }
    __syncthreads();
    // ---- stage 1 on plane k-1 from stage 0's ring
    {
        const int p = k - 1;
        constexpr bool last = S == 2;
        constexpr int hz = Sh::H - 1;  // planes / lines of halo stage 1 still needs
        double o[2] = {0.0, 0.0};
        const bool act = t.pos_ok && t.ry >= 1 && t.ry < Sh::RY - 1 && p >= 0 && p < t.nz && p >= t.zs - hz &&
                         p < t.ze + hz && (!last || t.own_xy);
        if (act) {
            double xv[2][7];
            tb_gather_lds<Sh::RY>(l0, tb_mod3(p - 1), tb_mod3(p), tb_mod3(p + 1), t.ry, t.col, xv);
            tb_rows(cB, xv, last && ta.last_resid, ta.omega, o);
            if (t.own_xy && p >= t.zs && p < t.ze)
                *reinterpret_cast<double2*>(ta.out[1] + (int64_t)p * t.M + t.ixy) = make_double2(o[0], o[1]);
        }
        if constexpr (S == 3) {
            if (t.ry >= 0) *reinterpret_cast<double2*>(&l1[tb_mod3(p)][t.ry][t.col]) = make_double2(o[0], o[1]);
        }
    }
    __syncthreads();  // S = 3: stage 2 reads l1; S = 2: the next step's stage 0 rewrites l0
    // ---- stage 2 on plane k-2 from stage 1's ring (S = 3)
    if constexpr (S == 3) {
        const int p = k - 2;
        if (t.own_xy && t.ry >= 2 && t.ry < Sh::RY - 2 && p >= t.zs && p < t.ze) {
            double xv[2][7], o[2];
            tb_gather_lds<Sh::RY>(l1, tb_mod3(p - 1), tb_mod3(p), tb_mod3(p + 1), t.ry, t.col, xv);
            tb_rows(cC, xv, ta.last_resid, ta.omega, o);
            *reinterpret_cast<double2*>(ta.out[2] + (int64_t)p * t.M + t.ixy) = make_double2(o[0], o[1]);
        }
    }
}

template <int S>
__global__ __launch_bounds__(TbShape<S>::threads) void k_sym_tb(int nrows, const uint8_t* __restrict__ mask,
                                                                 const double* __restrict__ dg,
                                                                 const double* __restrict__ up, int64_t ld,
                                                                 const SymDia sd, const TbArgs ta) {
    using Sh = TbShape<S>;
    __shared__ __attribute__((aligned(16))) double l0[3][Sh::RY][kTbLW];
    __shared__ __attribute__((aligned(16))) double l1[S == 3 ? 3 : 1][Sh::RY][kTbLW];
    __shared__ __attribute__((aligned(16))) double xin[3][Sh::XL][kTbLW];
    TbCtx<S> t;
    if (!tb_ctx_init<S>(t, sd.tb, nrows)) return;  // the whole workgroup, before any barrier
    TbCoef c0, c1, c2;  // planes k, k-1, k-2 at step k (rotated by the unrolled loop)
    const int k0 = t.zs - Sh::H;
    {  // the in0 windows of planes k0-1 and k0 (each step loads the one above its plane)
        TbWin<S> w;
#pragma unroll
        for (int q = -1; q <= 0; ++q) {
            tb_win_load<S>(w, t, ta.in0, k0 + q);
            tb_win_store<S>(w, xin, tb_mod3(k0 + q));
        }
    }
    tb_step<S, true>(k0, c0, c2, c1, t, mask, dg, up, ld, sd, ta, l0, l1, xin);
    if constexpr (S == 2) {  // two planes of operator values live: a 2-way rotation
        for (int k = k0 + 1; k < t.kend; k += 2) {
            tb_step<S, false>(k, c1, c0, c0, t, mask, dg, up, ld, sd, ta, l0, l1, xin);
            tb_step<S, false>(k + 1, c0, c1, c1, t, mask, dg, up, ld, sd, ta, l0, l1, xin);
        }
    } else {
        for (int k = k0 + 1; k < t.kend; k += 3) {
            tb_step<S, false>(k, c1, c0, c2, t, mask, dg, up, ld, sd, ta, l0, l1, xin);
            tb_step<S, false>(k + 1, c2, c1, c0, t, mask, dg, up, ld, sd, ta, l0, l1, xin);
            tb_step<S, false>(k + 2, c0, c2, c1, t, mask, dg, up, ld, sd, ta, l0, l1, xin);
        }
    }
}

// ---- The row-class dictionary's blocked passes (k_sym_zc below): what a thread holds per row pair
// and plane — the two class ids, the mirror rows' ids (i-1; i-nx, i+1-nx; the -M mirrors are the
// pair's ids one plane down) and b — narrow until use, so no instruction touches a load's result
// before the step that consumes it. Values come from the class table in LDS at use. (Round 4's
// k_sym_tbd — three LDS plane rings and three barriers per plane — is replaced by k_sym_zc.)
struct TbdRow {    // one row pair on one plane, as loaded (narrow types: widened at use, so no
    uint16_t own;  // instruction touches a load's result before the step that consumes it)
    uint8_t m0;    // class ids: own = row i (bits 0-7), row i+1 (8-15); m0 = row i-1;
    uint16_t m1;   // m1 = rows i-nx (0-7), i+1-nx (8-15)
    double b[2];
};


// plane p's entry of the pair at i (even; 0 when the pair or plane is inactive)
__device__ __forceinline__ void tbd_load(TbdRow& c, const uint8_t* __restrict__ tid, const double* __restrict__ b,
                                         const SymDia& sd, int64_t i, int64_t n) {
    c.own = *reinterpret_cast<const uint16_t*>(tid + i);
    c.m0 = tid[i >= 1 ? i - 1 : 0];
    c.m1 = tbd_pair_ids(tid, i - sd.off[1], n);
    const double2 bb = *reinterpret_cast<const double2*>(b + i);
    c.b[0] = bb.x;
    c.b[1] = bb.y;
}

// The pair's outputs: k_rows_symd's values for the 7 classes -M, -nx, -1, 0, +1, +nx, +M (m2: the
// pair's ids one plane down, whose U_2 are this plane's -M values), then k_rows_symd's arithmetic
// without its mask selects and with div_rn — for the kernels whose absent entries meet
// exact zeros (k_sym_zm, k_sym_zc: tb_ok operators, every neighbour outside the grid is held as
// +0.0 and an absent in-grid entry is a +0.0 table value): such an entry's product is +-0, and
// adding +-0 to the running sum leaves its bits unchanged — the sum starts at +0.0 and, rounding
// to nearest, never becomes -0.0 — so every row sum has the masked sum's bits for finite x
// (a non-finite x at an absent entry's neighbour would be discarded by the mask and propagates
// here: an iterate that is already inf / NaN).
__device__ __forceinline__ void zc_rows(const SymTab<3>& tab, const TbdRow& c, uint32_t m2, const double (&xv)[2][7],
                                        bool resid, double omega, double (&out)[2]) {
    const uint32_t t0 = c.own & 0xffu, t1 = (c.own >> 8) & 0xffu;
    const uint32_t tr[2] = {t0, t1}, l0[2] = {c.m0 & 0xffu, t0};
    const uint32_t l1[2] = {c.m1 & 0xffu, (c.m1 >> 8) & 0xffu}, l2[2] = {m2 & 0xffu, (m2 >> 8) & 0xffu};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const uint32_t t = tr[r];
        double v[7];
        v[0] = tab.v[l2[r]][3];  // a(i, i-M)  = U_2 of row i-M
        v[1] = tab.v[l1[r]][2];  // a(i, i-nx) = U_1 of row i-nx
        v[2] = tab.v[l0[r]][1];  // a(i, i-1)  = U_0 of row i-1
        v[3] = tab.v[t][0];
        v[4] = tab.v[t][1];
        v[5] = tab.v[t][2];
        v[6] = tab.v[t][3];
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 7; ++k) {
            const double p = v[k] * xv[r][k];
            s = s + p;
        }
        if (resid) {
            out[r] = c.b[r] - s;
        } else {
            const double u = c.b[r] - s;
            const double w = omega * u;
            out[r] = xv[r][3] + div_rn(w, v[3], tab.r[t]);
        }
    }
}

// ---- k_sym_zc<S>: S dependent sweeps over the row-class dictionary (k_sym_tb's tiles, halos,
// activity ranges and row expressions — so its bits) marching the way k_sym_zm does (round 5): every
// thread owns one row pair of stage 0's region for the whole z range, so the z neighbours of
// every stage (in0 of planes k-1, k+1; stage 0 of k-2, k; stage 1 of k-3, k-1) sit in its own
// registers, and only in-plane neighbours go through LDS — one double-buffered plane per stage.
// A stage's LDS plane is stored at the start of the step AFTER the one that computed it, so the
// three stages of a step (stage 0 on plane k, stage 1 on k-1, stage 2 on k-2) read only data
// stored before the step's single barrier: one barrier per plane instead of three, and the
// stages' loads and arithmetic interleave within a thread. Every global load a step issues
// (in0 of plane k+2, the class ids and b of plane k+1, the in0 halo of plane k+1) is consumed
// one step later.
template <int S>
struct ZcShape {
    static constexpr int H = S - 1;               // stage-0 halo in y (lines) and z (planes)
    static constexpr int RY = kTbY + 2 * H;       // stage-0 lines
    static constexpr int NT = kTbPX * RY;         // stage-0 row pairs (positions), one per thread
    static constexpr int threads = (NT + 63) / 64 * 64;
    static constexpr int XL = RY + 2;             // in0 plane: stage 0's region + one line / pair around
    static constexpr int XW = kTbPX + 2;
    static constexpr int NHALO = 2 * XW + 2 * RY; // in0 halo pairs: lines 0, XL-1; pairs 0, XW-1 of the others
    static_assert(NHALO <= threads, "one halo pair per thread at most");
};

template <int S>
__device__ __forceinline__ void zc_halo_load(double2& v, const TbCtx<S>& t, const double* __restrict__ in0, int q) {
    using Sh = ZcShape<S>;
    const int h = threadIdx.x;
    int line = 0, col = 0;
    if (h < 2 * Sh::XW) {
        line = h < Sh::XW ? 0 : Sh::XL - 1;
        col = h % Sh::XW;
    } else {
        const int u = h - 2 * Sh::XW;
        line = 1 + u % Sh::RY;
        col = u / Sh::RY ? Sh::XW - 1 : 0;
    }
    const int x = t.x0 - 4 + 2 * col, y = t.y0 - Sh::H - 1 + line;
    const bool ok = h < Sh::NHALO && x >= 0 && x < t.nx && y >= 0 && y < t.ny && q >= 0 && q < t.nz;
    v = ok ? *reinterpret_cast<const double2*>(in0 + (int64_t)q * t.M + (int64_t)y * t.nx + x) : make_double2(0.0, 0.0);
}

template <int S>
__device__ __forceinline__ void zc_halo_store(const double2& v, double2 (*sin)[ZcShape<S>::XW]) {
    using Sh = ZcShape<S>;
    const int h = threadIdx.x;
    if (h >= Sh::NHALO) return;
    if (h < 2 * Sh::XW) {
        sin[h < Sh::XW ? 0 : Sh::XL - 1][h % Sh::XW] = v;
    } else {
        const int u = h - 2 * Sh::XW;
        sin[1 + u % Sh::RY][u / Sh::RY ? Sh::XW - 1 : 0] = v;
    }
}

// the 7 neighbour values of the pair at (line, column) of an LDS plane, z from registers
__device__ __forceinline__ void zc_gather(const double2* __restrict__ dn_line, const double2* __restrict__ line,
                                          const double2* __restrict__ up_line, int col, const double2& own,
                                          const double2& zm, const double2& zp, double (&xv)[2][7]) {
    const double2 lft = line[col - 1], rgt = line[col + 1], dn = dn_line[col], up = up_line[col];
    xv[0][0] = zm.x;  xv[1][0] = zm.y;
    xv[0][1] = dn.x;  xv[1][1] = dn.y;
    xv[0][2] = lft.y; xv[1][2] = own.x;
    xv[0][3] = own.x; xv[1][3] = own.y;
    xv[0][4] = own.y; xv[1][4] = rgt.x;
    xv[0][5] = up.x;  xv[1][5] = up.y;
    xv[0][6] = zp.x;  xv[1][6] = zp.y;
}

template <int S, int AH>
__global__ __launch_bounds__(ZcShape<S>::threads) void k_sym_zc(int nrows, const uint8_t* __restrict__ tid,
                                                                 const double* __restrict__ vtab,
                                                                 const uint32_t* __restrict__ mtab, int nv,
                                                                 const SymDia sd, const TbArgs ta) {
    using Sh = ZcShape<S>;
    static_assert(S == 2 || S == 3, "two or three sweeps");
    __shared__ __attribute__((aligned(16))) double2 sin[2][Sh::XL][Sh::XW];
    __shared__ __attribute__((aligned(16))) double2 s0l[2][Sh::RY][Sh::XW];
    __shared__ __attribute__((aligned(16))) double2 s1l[S == 3 ? 2 : 1][S == 3 ? Sh::RY : 1][Sh::XW];
    __shared__ __attribute__((aligned(16))) SymTab<3> tab;
    TbCtx<S> t;
    if (!tb_ctx_init<S>(t, sd.tb, nrows)) return;  // the whole workgroup, before any barrier
    symtab_fill<3>(tab, vtab, mtab, nv);            // (read after the first barrier)
    const int T = threadIdx.x;
    const bool has = t.ry >= 0;                     // a stage-0 position
    const int ry = has ? t.ry : 0, col = has ? (T % kTbPX) + 1 : 1;  // LDS column of the pair
    // the stage planes' pad columns (0, XW-1) are read only by pairs whose affected element is
    // discarded; zero them once so no stale LDS enters even a discarded value
    if (T < 2 * Sh::RY) {
        const int l = T % Sh::RY, c = T < Sh::RY ? 0 : Sh::XW - 1;
        for (int q = 0; q < 2; ++q) {
            s0l[q][l][c] = make_double2(0.0, 0.0);
            if constexpr (S == 3) s1l[q][l][c] = make_double2(0.0, 0.0);
        }
    }
    const int k0 = t.zs - Sh::H;
    auto ldx = [&](int q) {
        return t.pos_ok && q >= 0 && q < t.nz ? *reinterpret_cast<const double2*>(ta.in0 + (int64_t)q * t.M + t.ixy)
                                              : make_double2(0.0, 0.0);
    };
    auto ldrow = [&](TbdRow& e, int q) {
        const bool ok = t.pos_ok && q >= 0 && q < t.nz;
        tbd_load(e, tid, ta.b, sd, ok ? (int64_t)q * t.M + t.ixy : 0, t.n);
    };
    const double2 zero = make_double2(0.0, 0.0);
    // plane rings, indexed by compile-time constants in the 4-way unrolled loop (renaming, not
    // moves: a register that receives a load is read only in the step that consumes it, so no
    // wait for a load is forced before its consumer — a copy at the end of the step would be)
    // X[(u + j) & 3]: in0 of plane k-1+j (j = 0..3: k-1, k, k+1, k+2 in flight); E[(u + j) & 3]:
    // ids + b of plane k-2+j... (j = 3: k+1 in flight); HX[u & 1]: in0 halo of plane k, the
    // other one plane k+1 in flight
    // AH = 2 (ids, b and the in0 halo two planes ahead): E[(u + j) & 3] = plane k-2+j with plane k+2
    // loaded into plane k-2's slot once stage 2's copy of it is taken; HX[(u + j) & 3] = halo of
    // plane k+j (j = 2 loaded this step)
    static_assert(AH == 1 || AH == 2, "one or two planes ahead");
    double2 X[4], HX[AH == 2 ? 4 : 2];
    TbdRow E[4];
    X[0] = ldx(k0 - 1);
    X[1] = ldx(k0);
    X[2] = ldx(k0 + 1);
    X[3] = zero;
    zc_halo_load<S>(HX[0], t, ta.in0, k0);
    HX[1] = zero;
    if constexpr (AH == 2) {
        zc_halo_load<S>(HX[1], t, ta.in0, k0 + 1);
        HX[2] = HX[3] = zero;
    }
    E[0] = TbdRow{};
    ldrow(E[1], k0 - 1);
    ldrow(E[2], k0);
    E[3] = TbdRow{};
    if constexpr (AH == 2) ldrow(E[3], k0 + 1);
    uint32_t e3own = 0;  // class ids of plane k-3 (stage 2's -M mirror)
    double2 s0m1 = zero, s0m2 = zero;  // stage 0 of planes k-1, k-2
    double2 s1m2 = zero, s1m3 = zero;  // stage 1 of planes k-2, k-3
    constexpr int hz = Sh::H - 1;
    for (int kb = k0; kb < t.kend; kb += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = kb + u;
            if (k >= t.kend) break;  // uniform
            double2& xm = X[u & 3];
            double2& xc = X[(u + 1) & 3];
            double2& xp = X[(u + 2) & 3];
            double2& xn = X[(u + 3) & 3];
            double2& hc = HX[u & (AH == 2 ? 3 : 1)];
            double2& hn = HX[(u + AH) & (AH == 2 ? 3 : 1)];
            TbdRow E2 = E[u & 3];         // plane k-2 (AH = 2: a copy, its slot takes plane k+2)
            TbdRow& E1 = E[(u + 1) & 3];  // plane k-1
            TbdRow& E0 = E[(u + 2) & 3];  // plane k
            TbdRow& En = E[(u + (AH == 2 ? 0 : 3)) & 3];  // plane k+AH (loaded this step)
            const int a = k & 1, a1 = (k - 1) & 1, a2 = (k - 2) & 1;
            // this step's LDS planes: in0 of plane k (own pair + halo), stage 0 of k-1, stage 1 of k-2
            if (has) {
                sin[a][ry + 1][col] = xc;
                s0l[a1][ry][col] = s0m1;
                if constexpr (S == 3) s1l[a2][ry][col] = s1m2;
            }
            zc_halo_store<S>(hc, sin[a]);
            const uint32_t e3 = e3own;
            e3own = E2.own;  // (E2 is overwritten by this step's load of plane k+1... next step)
            // next steps' loads
            xn = ldx(k + 2);
            zc_halo_load<S>(hn, t, ta.in0, k + AH);
            ldrow(En, k + AH);
            __syncthreads();
            // ---- stage 0 on plane k: a Jacobi sweep from in0
            double2 s0k = zero;
            if (t.pos_ok && k >= 0 && k < t.nz) {
                double xv[2][7], o[2];
                zc_gather(&sin[a][ry][0], &sin[a][ry + 1][0], &sin[a][ry + 2][0], col, xc, xm, xp, xv);
                zc_rows(tab, E0, E1.own, xv, S == 1 && ta.last_resid, ta.omega, o);
                s0k = make_double2(o[0], o[1]);
                if (ta.out[0] && t.own_xy && k >= t.zs && k < t.ze)
                    *reinterpret_cast<double2*>(ta.out[0] + (int64_t)k * t.M + t.ixy) = s0k;
            }
            // ---- stage 1 on plane k-1 from stage 0 (in-plane: the LDS plane stored this step)
            double2 s1k = zero;
            {
                const int p = k - 1;
                constexpr bool last = S == 2;
                if (t.pos_ok && ry >= 1 && ry < Sh::RY - 1 && p >= 0 && p < t.nz && p >= t.zs - hz && p < t.ze + hz &&
                    (!last || t.own_xy)) {
                    double xv[2][7], o[2];
                    zc_gather(&s0l[a1][ry - 1][0], &s0l[a1][ry][0], &s0l[a1][ry + 1][0], col, s0m1, s0m2, s0k, xv);
                    zc_rows(tab, E1, E2.own, xv, last && ta.last_resid, ta.omega, o);
                    s1k = make_double2(o[0], o[1]);
                    if (t.own_xy && p >= t.zs && p < t.ze)
                        *reinterpret_cast<double2*>(ta.out[1] + (int64_t)p * t.M + t.ixy) = s1k;
                }
            }
            // ---- stage 2 on plane k-2 from stage 1 (S = 3)
            if constexpr (S == 3) {
                const int p = k - 2;
                if (t.own_xy && ry >= 2 && ry < Sh::RY - 2 && p >= t.zs && p < t.ze) {
                    double xv[2][7], o[2];
                    zc_gather(&s1l[a2][ry - 1][0], &s1l[a2][ry][0], &s1l[a2][ry + 1][0], col, s1m2, s1m3, s1k, xv);
                    zc_rows(tab, E2, e3, xv, ta.last_resid, ta.omega, o);
                    *reinterpret_cast<double2*>(ta.out[2] + (int64_t)p * t.M + t.ixy) = make_double2(o[0], o[1]);
                }
            }
            s0m2 = s0m1;
            s0m1 = s0k;
            s1m3 = s1m2;
            s1m2 = s1k;
        }
    }
}

// ---- k_sym_zm<OP>: ONE sweep (SpMV, residual or Jacobi) of a whole one-part 7-point grid operator
// in the row-class dictionary (SymDia::vd_n, tb_ok), marching along z (Options::sym_zm; round 5,
// VERDICT r4 next-3). The shape is the one tools/stencil_ceiling.hip measured closest to the copy
// rate for a 7-point sweep at 512^3 (constant coefficients: 0.39 ms against 0.35 for y = x and
// 0.66-0.81 ms for 7 global loads per row pair, profiles/r05_c/): a 256-thread workgroup owns a
// kTbX x kTbY xy tile over a chunk of planes; each thread holds two row pairs (lines ly, ly + 8)
// and keeps their x of planes k-1, k, k+1 (+ k+2 in flight) and their class ids of planes k-1, k
// in registers, so the z neighbours and the -M mirror class never touch LDS; only plane k's x and
// ids (tile + a one-point / one-line halo) go through a double-buffered LDS plane, one barrier per
// plane. Every load a step issues is consumed one step later. The products, their order (ascending
// class: -M, -nx, -1, 0, +1, +nx, +M), the mask selects and the epilogue are k_rows_symd's, so
// are the bits (SPEC §S3). Preconditions (tb_ok): nx % kTbX == 0, ny % kTbY == 0, every row in
// the set, no row reaching across a grid face (points outside the grid meet clear mask bits).
constexpr int kZmThreads = 256;
constexpr int kZmPX = kTbX / 2;            // row pairs per tile line
constexpr int kZmW = kZmPX + 2;            // LDS line: the left halo pair, 32 pairs, the right halo pair
constexpr int kZmHalo = 2 * kZmPX + 2 * kTbY;  // halo pairs of a plane: lines y0-1, y0+16; pairs x0-2, x0+64

struct ZmHalo {      // one halo item of the next plane, as loaded
    double2 x;
    uint16_t id;
};

__device__ __forceinline__ void zm_halo_load(ZmHalo& h, const double* __restrict__ x, const uint8_t* __restrict__ tid,
                                             int x0, int y0, int nx, int ny, int nz, int64_t M, int q) {
    const int t = threadIdx.x;
    int xh = 0, yh = 0;
    bool ok = false;
    if (t < 2 * kZmPX) {  // lines below / above the tile
        const int top = t / kZmPX;
        xh = x0 + 2 * (t % kZmPX);
        yh = top ? y0 + kTbY : y0 - 1;
        ok = yh >= 0 && yh < ny;
    } else if (t < kZmHalo) {  // the pairs left / right of the tile's lines
        const int u = t - 2 * kZmPX, right = u / kTbY;
        xh = right ? x0 + kTbX : x0 - 2;
        yh = y0 + u % kTbY;
        ok = xh >= 0 && xh < nx;
    }
    ok = ok && q >= 0 && q < nz;
    const int64_t i = ok ? (int64_t)q * M + (int64_t)yh * nx + xh : 0;
    h.x = ok ? *reinterpret_cast<const double2*>(x + i) : make_double2(0.0, 0.0);
    h.id = *reinterpret_cast<const uint16_t*>(tid + i);  // (outside: row 0's ids; they meet clear mask bits)
}

__device__ __forceinline__ void zm_halo_store(const ZmHalo& h, double2 (*sx)[kZmW], uint16_t (*sid)[kZmW]) {
    const int t = threadIdx.x;
    int line = 0, col = 0;
    if (t < 2 * kZmPX) {
        line = t / kZmPX ? kTbY + 1 : 0;
        col = 1 + t % kZmPX;
    } else if (t < kZmHalo) {
        const int u = t - 2 * kZmPX;
        line = 1 + u % kTbY;
        col = u / kTbY ? kZmPX + 1 : 0;
    } else {
        return;
    }
    sx[line][col] = h.x;
    sid[line][col] = h.id;
}

template <int OP>
__global__ __launch_bounds__(kZmThreads) void k_sym_zm(int nrows, const uint8_t* __restrict__ tid,
                                                       const double* __restrict__ vtab, const uint32_t* __restrict__ mtab,
                                                       int nv, const TbGeom g, const double* __restrict__ x,
                                                       const double* __restrict__ b, double* __restrict__ y,
                                                       double omega) {
    __shared__ __attribute__((aligned(16))) double2 sx[2][kTbY + 2][kZmW];
    __shared__ __attribute__((aligned(16))) uint16_t sid[2][kTbY + 2][kZmW];
    __shared__ __attribute__((aligned(16))) SymTab<3> tab;
    const int ntiles = g.tiles_x * g.tiles_y * g.zchunks;
    const int per = (ntiles + 7) / 8;
    const int lin = (blockIdx.x & 7) * per + (blockIdx.x >> 3);  // consecutive tiles on one XCD
    if (lin >= ntiles) return;  // the whole workgroup, before any barrier
    // y-fastest: an XCD's tiles are one x column of the grid (its y halos shared in its L2); x-fastest
    // (TbGeom::xfast): whole rows of tiles, so the 128-B lines a tile's x halo touches are read once per
    // XCD instead of by two XCDs each
    const int ty = g.xfast ? (lin / g.tiles_x) % g.tiles_y : lin % g.tiles_y;
    const int tx = g.xfast ? lin % g.tiles_x : (lin / g.tiles_y) % g.tiles_x, zc = lin / (g.tiles_x * g.tiles_y);
    const int z0 = zc * g.zlen, z1 = min(g.nz, z0 + g.zlen);
    if (z0 >= z1) return;
    const int x0 = tx * kTbX, y0 = ty * kTbY;
    const int64_t M = (int64_t)g.nx * g.ny;
    const int px = threadIdx.x % kZmPX, ly = threadIdx.x / kZmPX;  // ly 0..7: lines ly, ly + 8
    int64_t ixy[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) ixy[h] = (int64_t)(y0 + ly + 8 * h) * g.nx + x0 + 2 * px;
    symtab_fill<3>(tab, vtab, mtab, nv);  // (read after the first barrier)
    auto ldx = [&](int q, int h) {
        return q >= 0 && q < g.nz ? *reinterpret_cast<const double2*>(x + (int64_t)q * M + ixy[h]) : make_double2(0.0, 0.0);
    };
    auto ldid = [&](int q, int h) -> uint32_t {
        return q >= 0 && q < g.nz ? *reinterpret_cast<const uint16_t*>(tid + (int64_t)q * M + ixy[h]) : 0u;
    };
    auto ldb = [&](int q, int h) {
        if constexpr (OP == OP_SPMV) return make_double2(0.0, 0.0);
        return q < g.nz ? *reinterpret_cast<const double2*>(b + (int64_t)q * M + ixy[h]) : make_double2(0.0, 0.0);
    };
    // plane rings indexed by compile-time constants in the 4-way unrolled loop (renaming: no copy
    // of a register with a load in flight, see k_sym_zc): X[(u + j) & 3][h] = x of plane k-1+j
    // (j = 3: k+2 in flight), ID[(u + j) & 3][h] = ids of plane k-1+j (j = 2: k+1 in flight),
    // B[(u + j) & 1][h] = b of plane k+j, HL[(u + j) & 1] = halo of plane k+j
    double2 X[4][2], B[2][2];
    uint32_t ID[4][2];
    ZmHalo HL[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        X[0][h] = ldx(z0 - 1, h);
        X[1][h] = ldx(z0, h);
        X[2][h] = ldx(z0 + 1, h);
        ID[0][h] = ldid(z0 - 1, h);
        ID[1][h] = ldid(z0, h);
        B[0][h] = ldb(z0, h);
    }
    zm_halo_load(HL[0], x, tid, x0, y0, g.nx, g.ny, g.nz, M, z0);
    for (int kb = z0; kb < z1; kb += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = kb + u;
            if (k >= z1) break;  // uniform
            double2(&xm)[2] = X[u & 3];
            double2(&xc)[2] = X[(u + 1) & 3];
            double2(&xp)[2] = X[(u + 2) & 3];
            double2(&xn)[2] = X[(u + 3) & 3];
            uint32_t(&idm)[2] = ID[u & 3];
            uint32_t(&idc)[2] = ID[(u + 1) & 3];
            uint32_t(&idn)[2] = ID[(u + 2) & 3];
            double2(&bc)[2] = B[u & 1];
            double2(&bn)[2] = B[(u + 1) & 1];
            ZmHalo& hc = HL[u & 1];
            ZmHalo& hn = HL[(u + 1) & 1];
            const int sl = k & 1;
            // plane k into LDS (own pairs and halo), then the loads the next step consumes
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                sx[sl][1 + ly + 8 * h][1 + px] = xc[h];
                sid[sl][1 + ly + 8 * h][1 + px] = (uint16_t)idc[h];
            }
            zm_halo_store(hc, sx[sl], sid[sl]);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                xn[h] = ldx(k + 2, h);
                idn[h] = ldid(k + 1, h);
                bn[h] = ldb(k + 1, h);
            }
            zm_halo_load(hn, x, tid, x0, y0, g.nx, g.ny, g.nz, M, k + 1);
            __syncthreads();  // plane k's slot; the slot stored next step was last read a step ago
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ry = 1 + ly + 8 * h, col = 1 + px;
                const double2 lft = sx[sl][ry][col - 1], rgt = sx[sl][ry][col + 1];
                const double2 dn = sx[sl][ry - 1][col], up = sx[sl][ry + 1][col];
                const uint32_t idl = sid[sl][ry][col - 1], idd = sid[sl][ry - 1][col];
                const double xv[2][7] = {{xm[h].x, dn.x, lft.y, xc[h].x, xc[h].y, up.x, xp[h].x},
                                         {xm[h].y, dn.y, xc[h].x, xc[h].y, rgt.x, up.y, xp[h].y}};
                const uint32_t t0 = idc[h] & 0xffu, t1 = idc[h] >> 8;
                const uint32_t tr[2] = {t0, t1}, l0[2] = {idl >> 8, t0};
                const uint32_t l1[2] = {idd & 0xffu, idd >> 8}, l2[2] = {idm[h] & 0xffu, idm[h] >> 8};
                const double bv[2] = {bc[h].x, bc[h].y};
                double o[2];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const uint32_t tc = tr[r];
                    double v[7];
                    v[0] = tab.v[l2[r]][3];  // a(i, i-M)  = U_2 of row i-M
                    v[1] = tab.v[l1[r]][2];  // a(i, i-nx) = U_1 of row i-nx
                    v[2] = tab.v[l0[r]][1];  // a(i, i-1)  = U_0 of row i-1
                    v[3] = tab.v[tc][0];
                    v[4] = tab.v[tc][1];
                    v[5] = tab.v[tc][2];
                    v[6] = tab.v[tc][3];
                    // (absent entries meet exact zeros: no mask select, see zc_rows)
                    double sacc = 0.0;
#pragma unroll
                    for (int q = 0; q < 7; ++q) {
                        const double p = v[q] * xv[r][q];
                        sacc = sacc + p;
                    }
                    if constexpr (OP == OP_SPMV) {
                        o[r] = sacc;
                    } else if constexpr (OP == OP_RESID) {
                        o[r] = bv[r] - sacc;
                    } else {
                        const double u2 = bv[r] - sacc;
                        const double w = omega * u2;
                        o[r] = xv[r][3] + div_rn(w, v[3], tab.r[tc]);
                    }
                }
                *reinterpret_cast<double2*>(y + (int64_t)k * M + ixy[h]) = make_double2(o[0], o[1]);
            }
        }
    }
    (void)nrows;
}

// k_rows_ell: the sliced-ELL layout (pamg::EllSet; round 5, the level-1 operator). One row per
// lane, a workgroup = kEllGroup consecutive rows = 4 slices; the group's two tables (column offsets
// and values, <= 256 entries each) are staged in LDS once; a lane then walks its row in storage
// order, 4 nonzeros per dword pair of index bytes: offset and value from LDS, x gathered at row +
// offset (the k-th entries of 64 consecutive rows are at nearby columns: few lines per wave-load).
// Products rounded and summed left to right from +0.0 in storage order, the padded tail of a
// row (k >= its length) selected away: the bits of every other row kernel (SPEC §S3). Groups in
// XCD-contiguous order: block b on XCD b % 8 takes the (b / 8)-th group of that XCD's eighth, so an
// XCD's L2 holds the x window its consecutive rows reuse.
// PAIR (EllSet::paired): one index byte per nonzero names an (offset, value) pair; no value stream.
template <int OP, bool ANC, bool PAIR>
__global__ __launch_bounds__(kEllGroup) void k_rows_ell(int nrows, const int* __restrict__ gorder,
                                                        const int* __restrict__ anc, const int2* __restrict__ smeta,
                                                        const uint32_t* __restrict__ cw, const uint32_t* __restrict__ vw,
                                                        const uint8_t* __restrict__ len, const int4* __restrict__ gmeta,
                                                        const int* __restrict__ otab, const double* __restrict__ vtab,
                                                        int ngroups, const double* __restrict__ x,
                                                        const double* __restrict__ b, double* __restrict__ y,
                                                        double omega) {
    __shared__ int lo[256];
    __shared__ double lv[256];
    const int per = (ngroups + 7) / 8;
    const int gi = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (gi >= ngroups) return;  // the whole workgroup, before the barrier
    const int g = gorder ? gorder[gi] : gi;  // (a restriction's blocked order: EllSet::d_gorder)
    const int tid = threadIdx.x, lane = tid & 63;
    const int4 gm = gmeta[g];
    const int i = g * kEllGroup + tid;
    const int ic = i < nrows ? i : nrows - 1;
    const int L8 = i < nrows ? (int)len[i] : kEllSkip;
    const bool in = L8 != kEllSkip;  // (a boundary row of a part: the boundary tiles compute it)
    const int2 sm = smeta[ic / kEllW];  // (one slice per wave)
    const int L = in ? L8 : 0;
    const int base = ANC ? anc[ic] : ic;  // offsets from the row (square) or its first column (anchored)
    const uint32_t* __restrict__ cp = cw + sm.x + lane;
    const uint32_t* __restrict__ vp = (PAIR ? cw : vw) + sm.x + lane;
    const int nq = (sm.y + 3) >> 2;
    uint32_t c4 = nq > 0 ? cp[0] : 0u, v4 = PAIR ? 0u : (nq > 0 ? vp[0] : 0u);
    double pb = 0.0, px = 0.0, py = 0.0;
    if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[ic];
    if constexpr (OP == OP_JACOBI) px = x[ic];
    if constexpr (OP == OP_PROLONG) py = y[ic];
    const int ot = gm.x + (tid < gm.y ? tid : 0), vt = gm.z + (tid < gm.w ? tid : 0);
    const int otv = otab[ot];
    const double vtv = vtab[vt];
    if (tid < gm.y) lo[tid] = otv;
    if (tid < gm.w) lv[tid] = vtv;
    __syncthreads();
    double s = 0.0, dg = 0.0;
    for (int q = 0; q < nq; ++q) {
        const uint32_t cq = c4, vq = PAIR ? c4 : v4;
        if (q + 1 < nq) {  // the next dword pair in flight while this one is used
            c4 = cp[(q + 1) * kEllW];
            if constexpr (!PAIR) v4 = vp[(q + 1) * kEllW];
        }
        int of[4];
        double vv[4], xv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            of[e] = lo[(cq >> (8 * e)) & 255u];
            vv[e] = lv[(vq >> (8 * e)) & 255u];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) xv[e] = x[4 * q + e < L ? base + of[e] : base];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const bool ok = 4 * q + e < L;
            const double p = vv[e] * xv[e];
            const double t = s + p;
            s = ok ? t : s;
            if constexpr (OP == OP_JACOBI) dg = ok && of[e] == 0 ? vv[e] : dg;
        }
    }
    double out;
    if constexpr (OP == OP_SPMV) {
        out = s;
    } else if constexpr (OP == OP_RESID) {
        out = pb - s;
    } else if constexpr (OP == OP_JACOBI) {
        const double u = pb - s;
        const double v = omega * u;
        const double w = v / dg;
        out = px + w;
    } else {
        out = py + s;
    }
    if (in) y[i] = out;
}

// k_rows_rpat: pattern-dictionary rows (pamg::RpatSet; round 6, the 512^3 R0). One row per lane, a
// workgroup per kEllGroup rows (the groups in the ELL's blocked order where the columns are a
// registered grid); every workgroup stages the entry, pattern and value tables (<= kRpatEnt + kRpatMax
// + 256 words; 1,249 + 58 + 41 at 512^3) in LDS, then a lane walks its pattern's entries U per step —
// their x gathers issued together, a step past the row's end re-reading its last entry — x at the
// row's first column + offset, products rounded and summed left to right from +0.0 in storage order,
// the entries past the end selected away (SPEC S3: the bits of every other row kernel).
template <int OP, int U>
__global__ __launch_bounds__(kEllGroup) void k_rows_rpat(int nrows, const int* __restrict__ gorder,
                                                         const int* __restrict__ anc, const uint8_t* __restrict__ pid,
                                                         const int2* __restrict__ pmeta, int npat,
                                                         const uint32_t* __restrict__ pent, int nent,
                                                         const double* __restrict__ vtab, int nval, int ngroups,
                                                         const double* __restrict__ x, const double* __restrict__ b,
                                                         double* __restrict__ y, double omega) {
    __shared__ uint32_t le[kRpatEnt];
    __shared__ int2 lm[kRpatMax];
    __shared__ double lv[256];
    const int per = (ngroups + 7) / 8;
    const int gi = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (gi >= ngroups) return;  // the whole workgroup, before the barrier
    const int g = gorder ? gorder[gi] : gi;
    const int tid = threadIdx.x;
    const int i = g * kEllGroup + tid;
    const int ic = i < nrows ? i : nrows - 1;
    const int p = i < nrows ? (int)pid[i] : kRpatSkip;  // (kRpatSkip: a boundary row of a part, or past the end)
    const int a = anc[ic];
    double pb = 0.0, px = 0.0, py = 0.0;
    if constexpr (OP == OP_RESID || OP == OP_JACOBI) pb = b[ic];
    if constexpr (OP == OP_JACOBI) px = x[ic];
    if constexpr (OP == OP_PROLONG) py = y[ic];
    for (int t = tid; t < nent; t += kEllGroup) le[t] = pent[t];
    for (int t = tid; t < npat; t += kEllGroup) lm[t] = pmeta[t];
    for (int t = tid; t < nval; t += kEllGroup) lv[t] = vtab[t];
    __syncthreads();
    const bool in = p != kRpatSkip;
    const int2 m = in ? lm[p] : make_int2(0, 0);
    const int L = m.y;
    double s = 0.0, dg = 0.0;
    for (int q = 0; q < L; q += U) {
        uint32_t w[U];
        double xv[U];
#pragma unroll
        for (int e = 0; e < U; ++e) w[e] = le[m.x + min(q + e, L - 1)];
#pragma unroll
        for (int e = 0; e < U; ++e) xv[e] = x[a + (int)(w[e] & 0xffffffu)];
#pragma unroll
        for (int e = 0; e < U; ++e) {
            const bool ok = q + e < L;
            const double v = lv[w[e] >> 24];
            const double pr = v * xv[e];
            const double t = s + pr;
            s = ok ? t : s;
            if constexpr (OP == OP_JACOBI) dg = ok && a + (int)(w[e] & 0xffffffu) == i ? v : dg;
        }
    }
    double out;
    if constexpr (OP == OP_SPMV) {
        out = s;
    } else if constexpr (OP == OP_RESID) {
        out = pb - s;
    } else if constexpr (OP == OP_JACOBI) {
        const double u = pb - s;
        const double v = omega * u;
        const double w = v / dg;
        out = px + w;
    } else {
        out = py + s;
    }
    if (in) y[i] = out;
}

// k_rows_pnc: the neighbour-coded prolongation (pamg::PncSet; round 5, the 512^3 P0). One row per
// lane, about 8 workgroups per CU, each staging the two global tables (<= 1024 pattern words, <= 128
// values) in LDS once and then walking 256-row blocks: at step t the workgroups of XCD j (block b
// runs on XCD b % 8) take consecutive blocks of the j-th eighth of the rows, so each XCD moves one
// window along its rows and its L2 holds the window's coarse entries and the anchors of the planes
// next to it. A lane loads its row's record and the anchors of its 7 grid points (clamped to the
// row itself off the grid: no code names such a point), takes each entry's column from its code and
// sums value * x[column] left to right from +0.0 in storage order (SPEC S3), as the other row
// kernels do.
// what a lane loads for its row of a block before the pattern is known (k_rows_pnc): the record,
// the anchors of the in-plane neighbours, y / b / x; the z neighbours' anchors come from the
// z-march's registers
struct PncRow {
    uint2 rec;   // the 64-bit record; compact records: rec.x = the 16-bit combination id
    int an[5];   // anchors of the points i, i-1, i+1, i-nx, i+nx (clamped to i off the plane)
    double p0;   // y (prolongate-add), b (residual, Jacobi)
    double p1;   // x_i (Jacobi)
};

template <int OP, bool CP>
__device__ __forceinline__ void pnc_load(PncRow& r, int i, int nrows, int nx, const int* __restrict__ anc,
                                         const uint2* __restrict__ rec, const uint16_t* __restrict__ cid,
                                         const double* __restrict__ x, const double* __restrict__ b,
                                         const double* __restrict__ y) {
    if constexpr (CP) r.rec = make_uint2((uint32_t)cid[i], 0u);
    else r.rec = rec[i];
    r.an[0] = anc[i];
    r.an[1] = anc[i >= 1 ? i - 1 : i];
    r.an[2] = anc[i + 1 < nrows ? i + 1 : i];
    r.an[3] = anc[i >= nx ? i - nx : i];
    r.an[4] = anc[i + nx < nrows ? i + nx : i];
    r.p0 = 0.0;
    r.p1 = 0.0;
    if constexpr (OP == OP_RESID || OP == OP_JACOBI) r.p0 = b[i];
    if constexpr (OP == OP_PROLONG) r.p0 = y[i];
    if constexpr (OP == OP_JACOBI) r.p1 = x[i];
}

// k_rows_pnc: the neighbour-coded prolongation (pamg::PncSet; round 5, the 512^3 P0). One row per
// lane; a workgroup owns a 256-point block of a plane (M % 256 == 0) and marches it along z over a
// chunk of planes — as NS interleaved streams (the chunk cut in as many parts, a plane of each per
// step: independent gather sets in flight per lane) — so the anchors of the z neighbours (i - M,
// i + M) are the ones it loaded for the previous plane and prefetches for the next: each anchor
// leaves HBM once; the in-plane neighbours' anchors (i +- 1: the same lines; i +- nx: the blocks
// next to it, marched by the workgroups beside it on the same XCD) come from the caches. The two
// global tables (<= 1024 pattern words, <= 128 values) sit in LDS. A lane takes each entry's column
// from its code and sums value * x[column] left to right from +0.0 in storage order (SPEC S3), as
// the other row kernels do. The next planes' records, anchors and y are loaded under this step's x
// gathers; every gather is issued (a padded entry reloads the first entry's x), so the loads are
// straight-line and the waits count exactly.
// CP (compact records, PncSet::d_cid): a row holds a 16-bit combination id; the combination's pattern
// word and value indices come from LDS (kPncCombMax entries each).
template <int OP, int NS, bool CP>
__global__ __launch_bounds__(256) void k_rows_pnc(int nrows, int nx, int M, int nz, int zlen,
                                                  const int* __restrict__ anc, const uint2* __restrict__ rec,
                                                  const uint16_t* __restrict__ cid, const uint64_t* __restrict__ pvals,
                                                  const uint32_t* __restrict__ ptab, int npat,
                                                  const double* __restrict__ vtab, int nval,
                                                  const double* __restrict__ x, const double* __restrict__ b,
                                                  double* __restrict__ y, double omega) {
    __shared__ uint32_t lp[CP ? kPncCombMax : kPncPatMax];
    __shared__ uint64_t lw[CP ? kPncCombMax : 1];
    __shared__ double lv[kPncValMax];
    const int nxb = M >> 8;                                    // 256-point blocks of a plane
    const int units = nxb * ((nz + zlen - 1) / zlen);
    const int per = (units + 7) >> 3;
    const int u = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);  // consecutive units on one XCD
    if (u >= units) return;  // the whole workgroup, before the barrier
    for (int t = threadIdx.x; t < npat; t += 256) lp[t] = ptab[t];
    if constexpr (CP)
        for (int t = threadIdx.x; t < npat; t += 256) lw[t] = pvals[t];
    for (int t = threadIdx.x; t < nval; t += 256) lv[t] = vtab[t];
    const int zc0 = (u / nxb) * zlen, zc1 = min(nz, zc0 + zlen);
    const int part = (zc1 - zc0 + NS - 1) / NS;  // planes per stream
    const int ixy = ((u % nxb) << 8) + (int)threadIdx.x;
    int zs[NS], ze[NS], zl[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        zs[q] = zc0 + q * part;
        ze[q] = min(zc1, zs[q] + part);
        zl[q] = ze[q] > zs[q] ? ze[q] - 1 : zc1 - 1;  // a stream's last plane (an empty stream re-walks the chunk's)
    }
    PncRow cur[NS];
    int am[NS], ap[NS];
#pragma unroll
    for (int q = 0; q < NS; ++q) {
        const int z = min(zs[q], zl[q]);
        pnc_load<OP, CP>(cur[q], z * M + ixy, nrows, nx, anc, rec, cid, x, b, y);
        am[q] = anc[z > 0 ? (z - 1) * M + ixy : ixy];          // anchors of planes z - 1 and z + 1
        ap[q] = anc[z + 1 < nz ? (z + 1) * M + ixy : ixy];
    }
    __syncthreads();  // (the tables; the first planes' loads already in flight)
    for (int j = 0; j < part; ++j) {
        int zq[NS], L[NS], col[NS][kPncMaxLen];
        double xv[NS][kPncMaxLen];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            zq[q] = min(zs[q] + j, zl[q]);
            const uint32_t pid = CP ? cur[q].rec.x : cur[q].rec.x & 1023u;
            const uint32_t pw = pid < (uint32_t)npat ? lp[pid] : 0u;  // (kPncSkip / kPncCombSkip: no entries, no store)
            L[q] = (int)(pw & 7u);
#pragma unroll
            for (int k = 0; k < kPncMaxLen; ++k) {
                const uint32_t c = (pw >> (3 + 3 * k)) & 7u;
                // codes 0 self, 1 i-1, 2 i+1, 3 i-nx, 4 i+nx, 5 i-M, 6 i+M: a select chain, no branches
                const int c01 = c & 1u ? cur[q].an[1] : cur[q].an[0];
                const int c23 = c & 1u ? cur[q].an[3] : cur[q].an[2];
                const int c45 = c & 1u ? am[q] : cur[q].an[4];
                const int c03 = c & 2u ? c23 : c01;
                const int c47 = c & 2u ? ap[q] : c45;
                col[q][k] = c & 4u ? c47 : c03;
                xv[q][k] = x[k < L[q] ? col[q][k] : col[q][0]];
            }
        }
        // the next planes (a stream's last plane reloads itself), and the anchors two planes on
        PncRow nxt[NS];
        int ap2[NS];
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int zn = min(zq[q] + 1, zl[q]);
            pnc_load<OP, CP>(nxt[q], zn * M + ixy, nrows, nx, anc, rec, cid, x, b, y);
            ap2[q] = anc[zn + 1 < nz ? (zn + 1) * M + ixy : zn * M + ixy];
        }
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int i = zq[q] * M + ixy;
            // the value indices from bit 0 (compact: the combination's word; else the record's bits 10..)
            uint64_t rr;
            if constexpr (CP) rr = cur[q].rec.x < (uint32_t)npat ? lw[cur[q].rec.x] : 0ull;
            else rr = (((uint64_t)cur[q].rec.y << 32) | cur[q].rec.x) >> 10;
            double s = 0.0, dg = 0.0;
#pragma unroll
            for (int k = 0; k < kPncMaxLen; ++k) {
                const bool ok = k < L[q];
                const double v = lv[(uint32_t)(rr >> (7 * k)) & 127u];
                const double p = v * xv[q][k];
                const double t = s + p;
                s = ok ? t : s;
                if constexpr (OP == OP_JACOBI) dg = ok && col[q][k] == i ? v : dg;
            }
            double out;
            if constexpr (OP == OP_SPMV) {
                out = s;
            } else if constexpr (OP == OP_RESID) {
                out = cur[q].p0 - s;
            } else if constexpr (OP == OP_JACOBI) {
                const double uu = cur[q].p0 - s;
                const double v = omega * uu;
                const double w = v / dg;
                out = cur[q].p1 + w;
            } else {
                out = cur[q].p0 + s;
            }
            const bool in = CP ? cur[q].rec.x != (uint32_t)kPncCombSkip : (cur[q].rec.x & 1023u) != (uint32_t)kPncSkip;
            if (zs[q] + j < ze[q] && in) y[i] = out;
            am[q] = cur[q].an[0];
            cur[q] = nxt[q];
            ap[q] = ap2[q];
        }
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

// Level-0 locality permutation at the V-cycle boundary (pamg_hier_set_perm): gather
// dst[i] = src[perm[i]] (caller -> device numbering) or scatter dst[perm[i]] = src[i].
template <bool SCATTER>
__global__ void k_permute(int64_t n, const int* __restrict__ perm, const double* __restrict__ src,
                          double* __restrict__ dst) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        if constexpr (SCATTER) dst[perm[i]] = src[i];
        else dst[i] = src[perm[i]];
    }
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

// PCG's x += alpha p; r -= alpha q; partials of r.r — one pass instead of two axpby and a
// dot. Each element is computed exactly as k_axpby computes it (a * x + 1.0 * y), and the
// partials walk the same grid-stride order as k_dot_partial on the same grid, so x, r and the
// dot carry the unfused sequence's bits.
__global__ __launch_bounds__(kBlock) void k_cg_update(int64_t n, double alpha, const double* __restrict__ p,
                                                      const double* __restrict__ q, double* __restrict__ x,
                                                      double* __restrict__ r, double* __restrict__ partials) {
    __shared__ double lds[kBlock / 64];
    const double na = -alpha;
    double v = 0.0;
    for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        const double u = alpha * p[i];
        const double w = 1.0 * x[i];
        x[i] = u + w;
        const double u2 = na * q[i];
        const double w2 = 1.0 * r[i];
        const double rn = u2 + w2;
        r[i] = rn;
        v += rn * rn;
    }
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

// descriptor kernel with column dictionaries: global tables, or per-tile (PT) ones, anchored or not
template <int OP, int TNNZ, bool PT>
void launch_tile2_cd(const pamg_mat& A, const TileSet& ts, const double* x, const double* b, double* y,
                     double omega, hipStream_t s) {
    const int n = ts.n_short;
    if (PT && ts.anc) {
        if (ts.cd == 4)
            k_rows_tile2<OP, TNNZ, false, false, true, 4, true, true><<<n, kBlock, 0, s>>>(
                ts.d_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, nullptr, nullptr, nullptr, nullptr, nullptr,
                A.d_rlen, A.d_cidx, ts.d_ctab, ts.ctab_n, A.d_anc16, ts.d_abase);
        else
            k_rows_tile2<OP, TNNZ, false, false, true, 8, true, true><<<n, kBlock, 0, s>>>(
                ts.d_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, nullptr, nullptr, nullptr, nullptr, nullptr,
                A.d_rlen, A.d_cidx, ts.d_ctab, ts.ctab_n, A.d_anc16, ts.d_abase);
    } else if (ts.cd == 4) {
        k_rows_tile2<OP, TNNZ, false, false, true, 4, PT><<<n, kBlock, 0, s>>>(
            ts.d_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, nullptr, nullptr, nullptr, nullptr, nullptr,
            A.d_rlen, A.d_cidx, ts.d_ctab, ts.ctab_n);
    } else {
        k_rows_tile2<OP, TNNZ, false, false, true, 8, PT><<<n, kBlock, 0, s>>>(
            ts.d_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega, nullptr, nullptr, nullptr, nullptr, nullptr,
            A.d_rlen, A.d_cidx, ts.d_ctab, ts.ctab_n);
    }
}

template <int OP, int TNNZ, bool VD8>
void launch_tm(const pamg_mat& A, const TileSet& ts, const double* x, const double* b, double* y, double omega,
               hipStream_t s) {
    (void)A;
    const int n = ts.n_short;
    if (ts.anc && ts.cd == 4)
        k_rows_tm<OP, TNNZ, 4, true, false, false, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr,
                                                         nullptr, ts.d_tm_rlen, ts.tm_rs, ts.d_ctab, ts.ctab_n,
                                                         x, b, y, omega, ts.d_tm_anc, XStage{}, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
    else if (ts.anc)
        k_rows_tm<OP, TNNZ, 8, true, false, false, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr,
                                                         nullptr, ts.d_tm_rlen, ts.tm_rs, ts.d_ctab, ts.ctab_n,
                                                         x, b, y, omega, ts.d_tm_anc, XStage{}, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
    else if (ts.pt && ts.cd == 4)
        k_rows_tm<OP, TNNZ, 4, false, false, true, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, ts.d_tm_cidx,
                                                                      nullptr, nullptr, nullptr, ts.d_tm_rlen,
                                                                      ts.tm_rs, ts.d_ctab, ts.ctab_n, x, b, y,
                                                                      omega, nullptr, XStage{}, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
    else if (ts.pt)
        k_rows_tm<OP, TNNZ, 8, false, false, true, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, ts.d_tm_cidx,
                                                                      nullptr, nullptr, nullptr, ts.d_tm_rlen,
                                                                      ts.tm_rs, ts.d_ctab, ts.ctab_n, x, b, y,
                                                                      omega, nullptr, XStage{}, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
    else if (ts.xs && ts.cd == 4)
        k_rows_tm<OP, TNNZ, 4, false, true, false, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr,
                                                               nullptr, nullptr, ts.d_tm_rlen, ts.tm_rs, ts.d_ctab,
                                                               ts.ctab_n, x, b, y, omega, nullptr, ts.xst, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
    else if (ts.xs)
        k_rows_tm<OP, TNNZ, 8, false, true, false, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr,
                                                               nullptr, nullptr, ts.d_tm_rlen, ts.tm_rs, ts.d_ctab,
                                                               ts.ctab_n, x, b, y, omega, nullptr, ts.xst, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
    else if (ts.cd == 4)
        k_rows_tm<OP, TNNZ, 4, false, false, false, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr,
                                                   nullptr, ts.d_tm_rlen, ts.tm_rs, ts.d_ctab, ts.ctab_n, x,
                                                   b, y, omega, nullptr, XStage{}, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
    else if (ts.cd == 8)
        k_rows_tm<OP, TNNZ, 8, false, false, false, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, ts.d_tm_cidx, nullptr, nullptr,
                                                   nullptr, ts.d_tm_rlen, ts.tm_rs, ts.d_ctab, ts.ctab_n, x,
                                                   b, y, omega, nullptr, XStage{}, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
    else
        k_rows_tm<OP, TNNZ, 0, false, false, false, VD8><<<n, kBlock, 0, s>>>(ts.d_short, ts.d_tm_val, nullptr, ts.d_tm_clo,
                                                   ts.d_tm_chi, ts.d_base, ts.d_tm_rlen, ts.tm_rs, nullptr,
                                                   0, x, b, y, omega, nullptr, XStage{}, ts.d_tm_vidx, ts.d_tm_vtab, ts.tm_vt);
}

template <int OP, int TNNZ>
void launch_tile(const pamg_mat& A, const TileSet& ts, const double* x, const double* b,
                 double* y, double omega, hipStream_t s) {
    const int n = ts.n_short;
    if (ts.tm) {
        if (ts.tm_vt)
            launch_tm<OP, TNNZ, true>(A, ts, x, b, y, omega, s);
        else
            launch_tm<OP, TNNZ, false>(A, ts, x, b, y, omega, s);
    } else if (ts.cd && A.d_cidx && ts.rl8 && A.d_rlen) {
        if (ts.pt)
            launch_tile2_cd<OP, TNNZ, true>(A, ts, x, b, y, omega, s);
        else
            launch_tile2_cd<OP, TNNZ, false>(A, ts, x, b, y, omega, s);
    } else if (ts.c24 && A.d_clo && ts.vd && A.d_vidx && ts.rl8 && A.d_rlen) {
        k_rows_tile2<OP, TNNZ, true, true, true><<<n, kBlock, 0, s>>>(ts.d_short, A.d_rowptr, A.d_col, A.d_val, x, b,
                                                                     y, omega, A.d_clo, A.d_chi, ts.d_base,
                                                                     A.d_vidx, ts.d_vtab, A.d_rlen);
    } else if (ts.c24 && A.d_clo && ts.vd && A.d_vidx) {
        k_rows_tile2<OP, TNNZ, true, true><<<n, kBlock, 0, s>>>(ts.d_short, A.d_rowptr, A.d_col, A.d_val, x, b, y,
                                                               omega, A.d_clo, A.d_chi, ts.d_base, A.d_vidx,
                                                               ts.d_vtab);
    } else if (ts.c24 && A.d_clo && ts.rl8 && A.d_rlen) {
        k_rows_tile2<OP, TNNZ, true, false, true><<<n, kBlock, 0, s>>>(ts.d_short, A.d_rowptr, A.d_col, A.d_val,
                                                                      x, b, y, omega, A.d_clo, A.d_chi,
                                                                      ts.d_base, nullptr, nullptr, A.d_rlen);
    } else if (ts.c24 && A.d_clo) {
        k_rows_tile2<OP, TNNZ, true><<<n, kBlock, 0, s>>>(ts.d_short, A.d_rowptr, A.d_col, A.d_val, x, b, y,
                                                         omega, A.d_clo, A.d_chi, ts.d_base);
    } else {
        k_rows_tile2<OP, TNNZ><<<n, kBlock, 0, s>>>(ts.d_short, A.d_rowptr, A.d_col, A.d_val, x, b, y, omega);
    }
}

template <int OP, int NU>
void launch_sym_nu(const pamg_mat& A, const double* x, const double* b, double* y, double omega, hipStream_t s) {
    const SymDia& sd = A.sym;
    const int grid = sd.nbands * 8 * sd.eighth;
    if constexpr (NU == 3) {
        // the whole one-part grid operator: the z-marching sweep (Options::sym_zm)
        // (plane0 == 0 and the bands covering every row: not a plane window of launch_sym_planes)
        if (sd.vd_n && sd.tb_ok && !sd.tb_part && options().sym_zm && sd.plane0 == 0 &&
            (int64_t)sd.nbands * sd.band >= A.nrows && A.nrows == (int64_t)sd.tb.nx * sd.tb.ny * sd.tb.nz &&
            A.nrows % 2 == 0) {
            TbGeom g = sd.tb;  // (y-fastest tiles: x-fastest measured +-2 %, profiles/r05_l/)
            const int tiles = g.tiles_x * g.tiles_y;
            // z chunks: ~4 workgroups per CU (1024), chunks of >= 16 planes; zm_chunks overrides
            int zc = options().zm_chunks > 0 ? options().zm_chunks : std::min((1024 + tiles - 1) / tiles, g.nz / 16);
            zc = std::max(1, std::min(zc, g.nz));
            g.zlen = (g.nz + zc - 1) / zc;
            g.zchunks = (g.nz + g.zlen - 1) / g.zlen;
            const int gr = (tiles * g.zchunks + 7) / 8 * 8;
            k_sym_zm<OP><<<gr, kZmThreads, 0, s>>>((int)A.nrows, sd.d_tid, sd.d_vtab, sd.d_mtab, sd.vd_n, g, x, b, y,
                                                   omega);
            return;
        }
    }
    if (sd.vd_n) {  // (the upload builds the dictionary only with two rows per lane)
        const int ch = NU <= 3 ? options().symd_chunks : 1;
        const int g = 8 * ((sd.nbands * sd.eighth + ch - 1) / ch);
        if constexpr (NU <= 3) {
            if (ch == 2) {
                k_rows_symd<OP, NU, 2><<<g, kBlock, 0, s>>>((int)A.nrows, (int)A.nrows, sd.d_tid, sd.d_vtab,
                                                            sd.d_mtab, sd.vd_n, sd, x, b, y, omega);
                return;
            }
            if (ch == 4) {
                k_rows_symd<OP, NU, 4><<<g, kBlock, 0, s>>>((int)A.nrows, (int)A.nrows, sd.d_tid, sd.d_vtab,
                                                            sd.d_mtab, sd.vd_n, sd, x, b, y, omega);
                return;
            }
        }
        k_rows_symd<OP, NU><<<grid, kBlock, 0, s>>>((int)A.nrows, (int)A.nrows, sd.d_tid, sd.d_vtab, sd.d_mtab,
                                                  sd.vd_n, sd, x, b, y, omega);
        return;
    }
    if (sd.rpl == 2) {
        k_rows_sym2<OP, NU><<<grid, kBlock, 0, s>>>((int)A.nrows, (int)A.nrows, sd.d_mask, sd.d_diag, sd.d_upper,
                                                  sd.ld, sd, x, b, y, omega);
        return;
    }
    // bound of the upper x index: the own rows (interior rows never read a ghost; rows outside
    // the set are not stored, and must not read the ghost slots an exchange may be writing)
    k_rows_sym<OP, NU><<<grid, kBlock, 0, s>>>((int)A.nrows, (int)A.nrows, sd.d_mask, sd.d_diag, sd.d_upper, sd.ld,
                                             sd, x, b, y, omega);
}

template <int OP>
void launch_sym(const pamg_mat& A, const double* x, const double* b, double* y, double omega, hipStream_t s) {
    if constexpr (OP == OP_PROLONG) {
        return;  // square operators only (the upload never builds the layout for P)
    } else {
        switch (A.sym.nu) {
            case 1: launch_sym_nu<OP, 1>(A, x, b, y, omega, s); break;
            case 2: launch_sym_nu<OP, 2>(A, x, b, y, omega, s); break;
            case 3: launch_sym_nu<OP, 3>(A, x, b, y, omega, s); break;
            case 4: launch_sym_nu<OP, 4>(A, x, b, y, omega, s); break;
            case 5: launch_sym_nu<OP, 5>(A, x, b, y, omega, s); break;
            case 6: launch_sym_nu<OP, 6>(A, x, b, y, omega, s); break;
            default: launch_sym_nu<OP, 7>(A, x, b, y, omega, s); break;
        }
    }
}

// k_rows_pnc's units: one 256-point plane block over kPncZlen planes, two z-streams per workgroup
// (measured at 512^3, profiles/r05_ns/ and r05_zl/: one or three streams 1.33 / 1.16 ms, 8-, 16-plane
// units and units sized to fill the chip in equal rounds 1.14 / 1.12 / 1.11 ms, against 1.09-1.10)
constexpr int kPncZlen = 32, kPncStreams = 2;

template <int OP>
void launch_pnc(const pamg_mat& A, const double* x, const double* b, double* y, double omega, hipStream_t s) {
    const PncSet& P = A.pnc;
    const int zlen = std::min(kPncZlen, P.nz);
    const int nxb = P.nx * P.ny / 256, units = nxb * ((P.nz + zlen - 1) / zlen);
    auto go = [&](auto kern) {
        kern<<<(units + 7) / 8 * 8, 256, 0, s>>>((int)A.nrows, P.nx, P.nx * P.ny, P.nz, zlen, P.d_anc, P.d_rec, P.d_cid,
                                                P.d_pvals, P.d_ptab, P.npat, P.d_vtab, P.nval, x, b, y, omega);
    };
    if (P.d_cid) go(k_rows_pnc<OP, kPncStreams, true>);
    else go(k_rows_pnc<OP, kPncStreams, false>);
}

template <int OP>
void launch_rpat(const pamg_mat& A, const double* x, const double* b, double* y, double omega, hipStream_t s) {
    const RpatSet& R = A.rpat;
    const int grid = (int)((R.ngroups + 7) / 8 * 8);
    auto go = [&](auto kern) {
        kern<<<grid, kEllGroup, 0, s>>>((int)A.nrows, R.d_gorder, R.d_anc, R.d_pid, R.d_pmeta, R.npat, R.d_pent, R.nent,
                                        R.d_vtab, R.nval, (int)R.ngroups, x, b, y, omega);
    };
    // 8 entries per step (512^3 R0: 4 / 8 / 16 per step 0.552 / 0.544 / 0.539-0.548 ms, profiles/r06_m/)
    go(k_rows_rpat<OP, 8>);
}

template <int OP>
void launch_rows_op(const pamg_mat& A, const TileSet& ts, const double* x, const double* b,
                    double* y, double omega, hipStream_t s) {
    if (ts.sym) launch_sym<OP>(A, x, b, y, omega, s);
    if (ts.ell) {
        const EllSet& E = A.ell;
        const int grid = (int)((E.ngroups + 7) / 8 * 8);
        auto go = [&](auto kern) {
            kern<<<grid, kEllGroup, 0, s>>>((int)A.nrows, E.d_gorder, E.d_anc, E.d_smeta, E.d_ci, E.d_vi, E.d_len,
                                            E.d_gmeta, E.d_otab, E.d_vtab, (int)E.ngroups, x, b, y, omega);
        };
        if (E.d_anc) {
            if (E.paired) go(k_rows_ell<OP, true, true>);
            else go(k_rows_ell<OP, true, false>);
        } else {
            if (E.paired) go(k_rows_ell<OP, false, true>);
            else go(k_rows_ell<OP, false, false>);
        }
    }
    if (ts.pnc) launch_pnc<OP>(A, x, b, y, omega, s);
    if (ts.rpat) launch_rpat<OP>(A, x, b, y, omega, s);
    if (ts.n_short > 0) {
        if (ts.tile_nnz == 1024) launch_tile<OP, 1024>(A, ts, x, b, y, omega, s);
        else if (ts.tile_nnz == 4096) launch_tile<OP, 4096>(A, ts, x, b, y, omega, s);
        else launch_tile<OP, 2048>(A, ts, x, b, y, omega, s);
    }
    if (ts.n_long > 0)
        k_rows_long<OP><<<ts.n_long, kBlock, 0, s>>>(ts.d_long, A.d_rowptr, A.d_col, A.d_val, x,
                                                     b, y, omega);
}
}  // namespace

void launch_sym_tb(const pamg_mat& A, const TbArgs& ta, hipStream_t s) {
    SymDia sd = A.sym;
    // output planes: all of a one-part operator's; a part's planes S planes in from a neighbour
    // part, whose stage-0 halo rows stay in the set and in0 planes in the part
    TbGeom& g = sd.tb;
    g.zlo = sd.part_lo == 0 ? 0 : sd.part_lo + ta.nstages - 1;
    g.zhi = sd.part_hi == g.nz ? g.nz : sd.part_hi - (ta.nstages - 1);
    const int span = g.zhi - g.zlo;
    if (span <= 0) return;
    g.zchunks = std::max(1, std::min(g.zchunks, span / 2 > 0 ? span / 2 : 1));
    g.zlen = (span + g.zchunks - 1) / g.zchunks;
    g.zchunks = (span + g.zlen - 1) / g.zlen;
    const int ntiles = g.tiles_x * g.tiles_y * g.zchunks;
    const int grid = (ntiles + 7) / 8 * 8;
    g.xfast = options().tb_xfast;
    if (sd.vd_n) {
        // ids, b and the in0 halo two planes ahead for S = 2 (-2 %), one for S = 3 (two: +2.7 %;
        // same-box A/B, profiles/r06_j/)
        if (ta.nstages == 2)
            k_sym_zc<2, 2><<<grid, ZcShape<2>::threads, 0, s>>>((int)A.nrows, sd.d_tid, sd.d_vtab, sd.d_mtab, sd.vd_n,
                                                                sd, ta);
        else
            k_sym_zc<3, 1><<<grid, ZcShape<3>::threads, 0, s>>>((int)A.nrows, sd.d_tid, sd.d_vtab, sd.d_mtab, sd.vd_n,
                                                                sd, ta);
        return;
    }
    if (ta.nstages == 2)
        k_sym_tb<2><<<grid, TbShape<2>::threads, 0, s>>>((int)A.nrows, sd.d_mask, sd.d_diag, sd.d_upper, sd.ld, sd, ta);
    else
        k_sym_tb<3><<<grid, TbShape<3>::threads, 0, s>>>((int)A.nrows, sd.d_mask, sd.d_diag, sd.d_upper, sd.ld, sd, ta);
}

void launch_sym_planes(const pamg_mat& A, int op, int p0, int p1, const double* x, const double* b, double* y,
                       double omega, hipStream_t s, int p2, int p3) {
    if (p1 < p0) p1 = p0;
    if (p3 < p2) p3 = p2;
    if (p1 == p0) {  // one window: the second
        p0 = p2;
        p1 = p3;
        p2 = p3 = 0;
    }
    if (p1 <= p0) return;
    pamg_mat B = A;  // shallow: the same device arrays, a plane window (or two)
    B.sym.plane0 = p0;
    B.sym.nbands = (p1 - p0) + (p3 - p2);
    if (p3 > p2) {
        B.sym.gap_at = p1;
        B.sym.gap = p2 - p1;
    }
    switch (op) {
        case OP_RESID: launch_sym<OP_RESID>(B, x, b, y, omega, s); break;
        case OP_JACOBI: launch_sym<OP_JACOBI>(B, x, b, y, omega, s); break;
        default: launch_sym<OP_SPMV>(B, x, b, y, omega, s); break;
    }
}

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

void launch_permute(int64_t n, const int* perm, const double* src, double* dst, bool scatter, hipStream_t s) {
    if (n <= 0) return;
    if (scatter) k_permute<true><<<grid_for(n), kBlock, 0, s>>>(n, perm, src, dst);
    else k_permute<false><<<grid_for(n), kBlock, 0, s>>>(n, perm, src, dst);
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

void launch_cg_update(int64_t n, double alpha, const double* p, const double* q, double* x, double* r,
                      double* partials, int np, double* out, hipStream_t s) {
    k_cg_update<<<np, kBlock, 0, s>>>(n, alpha, p, q, x, r, partials);
    k_dot_final<<<1, kBlock, 0, s>>>(np, partials, out);
}

}  // namespace pamg
