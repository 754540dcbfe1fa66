// stencil_ceiling.hip — what a 7-point fp64 stencil sweep y = A x at 512^3 can reach on this
// MI355X with NO matrix bytes at all (constant coefficients: 6 on the diagonal, -1 off it, zero
// across the grid's faces), to bound the library's fine-level sweeps (is the
// limiter of k_rows_symd / k_sym_tbd the class bytes and table lookups, or the 7-point access
// pattern itself?). Each variant moves the same compulsory bytes: x read once + y written once
// (2 x 1.07 GB). Dev tool, not part of libpamg.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/stencil_ceiling tools/stencil_ceiling.hip
//   tools/stencil_ceiling [n=512] [reps=20]
//
// variants (one JSON line each: ms per launch, GB/s on the compulsory bytes):
//   copy        y = x, 16 B per lane (the read+write streaming rate)
//   pair_lin    two rows per lane, 7 neighbours by global loads, blocks in natural order
//   pair_xcd    the same, blocks mapped so that each XCD sweeps one contiguous eighth of the rows
//               (k_rows_symd's banded order in its simplest form: z +- 1 planes stay in one L2)
//   quad_xcd    four rows per lane (two 16-B loads per neighbour line)
//   zmarch      2.5-D: a 256-thread block owns a 64 x 16 xy tile (two rows per lane... 2 pairs
//               per thread), marches z over a chunk of planes, keeps x of planes k-1, k, k+1 of
//               its own points in registers; in-plane neighbours by global loads (L1/L2 hits)
//   zmarch_lds  the same with the plane's x tile (+1 halo) staged in LDS, double-buffered
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));         \
            exit(1);                                                                          \
        }                                                                                     \
    } while (0)

struct Grid {
    int nx, ny, nz;
    long long M, n;
};

__global__ __launch_bounds__(256) void k_copy(const double2* __restrict__ x, double2* __restrict__ y, long long np) {
    const long long i = blockIdx.x * 256ll + threadIdx.x;
    if (i < np) y[i] = x[i];
}

__device__ __forceinline__ double ld(const double* __restrict__ x, long long j, bool ok) { return ok ? x[j] : 0.0; }

// rows i, i+1 (i even) of y = 6 x - sum of the in-grid neighbours
__device__ __forceinline__ void pair_rows(const double* __restrict__ x, double* __restrict__ y, const Grid g,
                                          long long i) {
    const int xi = (int)(i % g.nx);
    const long long r = i / g.nx;
    const int yi = (int)(r % g.ny), zi = (int)(r / g.ny);
    const double2 c = *reinterpret_cast<const double2*>(x + i);
    const double l = ld(x, i - 1, xi > 0), rr = ld(x, i + 2, xi + 2 < g.nx);
    const double2 zero = make_double2(0.0, 0.0);
    const double2 ym = yi > 0 ? *reinterpret_cast<const double2*>(x + i - g.nx) : zero;
    const double2 yp = yi + 1 < g.ny ? *reinterpret_cast<const double2*>(x + i + g.nx) : zero;
    const double2 zm = zi > 0 ? *reinterpret_cast<const double2*>(x + i - g.M) : zero;
    const double2 zp = zi + 1 < g.nz ? *reinterpret_cast<const double2*>(x + i + g.M) : zero;
    double2 o;
    o.x = 6.0 * c.x - zm.x - ym.x - l - c.y - yp.x - zp.x;
    o.y = 6.0 * c.y - zm.y - ym.y - c.x - rr - yp.y - zp.y;
    *reinterpret_cast<double2*>(y + i) = o;
}

template <bool XCD>
__global__ __launch_bounds__(256) void k_pair(const double* __restrict__ x, double* __restrict__ y, const Grid g) {
    const long long np = g.n / 2;
    const long long nb = (np + 255) / 256;
    long long b = blockIdx.x;
    if (XCD) {  // block b runs on XCD b % 8: XCD j sweeps blocks [j per, (j+1) per)
        const long long per = (nb + 7) / 8;
        b = (b & 7) * per + (b >> 3);
        if (b >= nb) return;
    }
    const long long p = b * 256 + threadIdx.x;
    if (p < np) pair_rows(x, y, g, 2 * p);
}

__global__ __launch_bounds__(256) void k_quad(const double* __restrict__ x, double* __restrict__ y, const Grid g) {
    const long long nq = g.n / 4;
    const long long nb = (nq + 255) / 256;
    const long long per = (nb + 7) / 8;
    const long long b = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (b >= nb) return;
    const long long q = b * 256 + threadIdx.x;
    if (q >= nq) return;
    const long long i = 4 * q;
    const int xi = (int)(i % g.nx);
    const long long r = i / g.nx;
    const int yi = (int)(r % g.ny), zi = (int)(r / g.ny);
    const double4 zero = make_double4(0.0, 0.0, 0.0, 0.0);
    auto l4 = [&](long long j, bool ok) { return ok ? *reinterpret_cast<const double4*>(x + j) : zero; };
    const double4 c = l4(i, true), ym = l4(i - g.nx, yi > 0), yp = l4(i + g.nx, yi + 1 < g.ny),
                  zm = l4(i - g.M, zi > 0), zp = l4(i + g.M, zi + 1 < g.nz);
    const double l = ld(x, i - 1, xi > 0), rr = ld(x, i + 4, xi + 4 < g.nx);
    double4 o;
    o.x = 6.0 * c.x - zm.x - ym.x - l - c.y - yp.x - zp.x;
    o.y = 6.0 * c.y - zm.y - ym.y - c.x - c.z - yp.y - zp.y;
    o.z = 6.0 * c.z - zm.z - ym.z - c.y - c.w - yp.z - zp.z;
    o.w = 6.0 * c.w - zm.w - ym.w - c.z - rr - yp.w - zp.w;
    *reinterpret_cast<double4*>(y + i) = o;
}

// 2.5-D: tile 64 x 16 points = 32 x 16 pairs, 256 threads x 2 pairs (lines ly and ly + 8)
constexpr int TX = 64, TY = 16;
template <bool LDS>
__global__ __launch_bounds__(256) void k_zmarch(const double* __restrict__ x, double* __restrict__ y, const Grid g,
                                                int zlen) {
    const int tiles_x = g.nx / TX, tiles_y = g.ny / TY, zch = (g.nz + zlen - 1) / zlen;
    const int ntiles = tiles_x * tiles_y * zch;
    const int per = (ntiles + 7) / 8;
    const int lin = (blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (lin >= ntiles) return;
    const int ty = lin % tiles_y, tx = (lin / tiles_y) % tiles_x, zc = lin / (tiles_x * tiles_y);
    const int z0 = zc * zlen, z1 = min(g.nz, z0 + zlen);
    const int px = threadIdx.x % 32, ly = threadIdx.x / 32;  // ly 0..7
    const int xg = tx * TX + 2 * px;
    __shared__ double2 sx[2][TY + 2][TX / 2 + 2];  // pairs; column 0 / 33: the halo pairs (one value used)
    double2 zm[2], c[2], zp[2];
    const double2 zero = make_double2(0.0, 0.0);
    long long base[2];
    for (int h = 0; h < 2; ++h) {
        const int yg = ty * TY + ly + 8 * h;
        base[h] = (long long)yg * g.nx + xg;
        zm[h] = z0 > 0 ? *reinterpret_cast<const double2*>(x + (z0 - 1) * g.M + base[h]) : zero;
        c[h] = *reinterpret_cast<const double2*>(x + z0 * g.M + base[h]);
    }
    for (int z = z0; z < z1; ++z) {
        for (int h = 0; h < 2; ++h)
            zp[h] = z + 1 < g.nz ? *reinterpret_cast<const double2*>(x + (z + 1) * g.M + base[h]) : zero;
        const long long pl = z * g.M;
        double2 o[2];
        if (LDS) {
            const int s = z & 1;
            for (int h = 0; h < 2; ++h) sx[s][1 + ly + 8 * h][1 + px] = c[h];
            // halo: lines above / below (threads 0..63), pairs left / right (threads 64..95)
            const int t = threadIdx.x;
            if (t < 64) {
                const int hx = t % 32, top = t / 32;
                const int yg = top ? ty * TY + TY : ty * TY - 1;
                const bool ok = yg >= 0 && yg < g.ny;
                sx[s][top ? TY + 1 : 0][1 + hx] =
                    ok ? *reinterpret_cast<const double2*>(x + pl + (long long)yg * g.nx + tx * TX + 2 * hx) : zero;
            } else if (t < 64 + 2 * TY) {
                const int u = t - 64, right = u / TY, yy = u % TY;
                const int xh = right ? tx * TX + TX : tx * TX - 2;
                const bool ok = xh >= 0 && xh < g.nx;
                sx[s][1 + yy][right ? TX / 2 + 1 : 0] =
                    ok ? *reinterpret_cast<const double2*>(x + pl + (long long)(ty * TY + yy) * g.nx + xh) : zero;
            }
            __syncthreads();
            for (int h = 0; h < 2; ++h) {
                const int ry = 1 + ly + 8 * h;
                const double2 l = sx[s][ry][px], r = sx[s][ry][px + 2], dn = sx[s][ry - 1][px + 1],
                              up = sx[s][ry + 1][px + 1];
                o[h].x = 6.0 * c[h].x - zm[h].x - dn.x - l.y - c[h].y - up.x - zp[h].x;
                o[h].y = 6.0 * c[h].y - zm[h].y - dn.y - c[h].x - r.x - up.y - zp[h].y;
            }
        } else {
            for (int h = 0; h < 2; ++h) {
                const long long i = pl + base[h];
                const int yg = ty * TY + ly + 8 * h;
                const double l = ld(x, i - 1, xg > 0), r = ld(x, i + 2, xg + 2 < g.nx);
                const double2 dn = yg > 0 ? *reinterpret_cast<const double2*>(x + i - g.nx) : zero;
                const double2 up = yg + 1 < g.ny ? *reinterpret_cast<const double2*>(x + i + g.nx) : zero;
                o[h].x = 6.0 * c[h].x - zm[h].x - dn.x - l - c[h].y - up.x - zp[h].x;
                o[h].y = 6.0 * c[h].y - zm[h].y - dn.y - c[h].x - r - up.y - zp[h].y;
            }
        }
        for (int h = 0; h < 2; ++h) {
            *reinterpret_cast<double2*>(y + pl + base[h]) = o[h];
            zm[h] = c[h];
            c[h] = zp[h];
        }
    }
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 512;
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    Grid g{N, N, N, (long long)N * N, (long long)N * N * N};
    double *x = nullptr, *y = nullptr, *yref = nullptr;
    CK(hipMalloc(&x, sizeof(double) * (g.n + 8)));
    CK(hipMalloc(&y, sizeof(double) * (g.n + 8)));
    CK(hipMalloc(&yref, sizeof(double) * (g.n + 8)));
    {
        std::vector<double> h(g.n);
        unsigned long long s = 88172645463325252ull;
        for (long long i = 0; i < g.n; ++i) {
            s ^= s << 13; s ^= s >> 7; s ^= s << 17;
            h[i] = (double)(s >> 11) * (1.0 / 9007199254740992.0) - 0.5;
        }
        CK(hipMemcpy(x, h.data(), sizeof(double) * g.n, hipMemcpyHostToDevice));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 16.0 * g.n;  // x once + y once
    auto run = [&](const char* name, auto launch, bool check) {
        launch();
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        long long bad = -1;
        if (check) {
            std::vector<double> a(g.n), b(g.n);
            CK(hipMemcpy(a.data(), y, sizeof(double) * g.n, hipMemcpyDeviceToHost));
            CK(hipMemcpy(b.data(), yref, sizeof(double) * g.n, hipMemcpyDeviceToHost));
            bad = 0;
            for (long long i = 0; i < g.n; ++i) bad += a[i] != b[i];
        }
        printf("{\"variant\": \"%s\", \"n\": %d, \"ms\": %.4f, \"GBps\": %.1f, \"mismatches\": %lld}\n", name, N, ms,
               bytes / (ms * 1e-3) / 1e9, bad);
        fflush(stdout);
    };
    const long long np = g.n / 2, nb2 = (np + 255) / 256;
    run("copy", [&] { k_copy<<<(unsigned)nb2, 256>>>((const double2*)x, (double2*)y, np); }, false);
    // reference output for the checks: the natural-order pair kernel
    k_pair<false><<<(unsigned)nb2, 256>>>(x, yref, g);
    CK(hipDeviceSynchronize());
    run("pair_lin", [&] { k_pair<false><<<(unsigned)nb2, 256>>>(x, y, g); }, true);
    run("pair_xcd", [&] { k_pair<true><<<(unsigned)((nb2 + 7) / 8 * 8), 256>>>(x, y, g); }, true);
    const long long nb4 = (g.n / 4 + 255) / 256;
    run("quad_xcd", [&] { k_quad<<<(unsigned)((nb4 + 7) / 8 * 8), 256>>>(x, y, g); }, true);
    for (int zlen : {512, 128, 64, 32}) {
        const int nt = (g.nx / TX) * (g.ny / TY) * ((g.nz + zlen - 1) / zlen);
        char nm[64];
        snprintf(nm, sizeof nm, "zmarch_z%d", zlen);
        run(nm, [&] { k_zmarch<false><<<(nt + 7) / 8 * 8, 256>>>(x, y, g, zlen); }, true);
        snprintf(nm, sizeof nm, "zmarch_lds_z%d", zlen);
        run(nm, [&] { k_zmarch<true><<<(nt + 7) / 8 * 8, 256>>>(x, y, g, zlen); }, true);
    }
    CK(hipFree(x));
    CK(hipFree(y));
    CK(hipFree(yref));
    return 0;
}
