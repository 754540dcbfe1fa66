// fetch_calib.hip — known-byte kernels to calibrate the rocprofv3 traffic counters on gfx950
// (VERDICT r5 next-2). MI355X_MICROARCH.md: FETCH_SIZE reports 1/2 of a 16-B-per-lane streaming
// read and is uncalibrated for other access widths, while the row kernels also issue 8-B, 4-B,
// 2-B and 1-B loads and 8-B gathers. Each kernel here reads (or writes) a fresh region whose
// byte count is exact and whose lines are each touched once, with a 1 GiB write in between to
// push the previous kernel's lines out of the 256 MiB Infinity Cache:
//
//   r16 r8 r4 r2 r1   coalesced streaming reads, 16 / 8 / 4 / 2 / 1 B per lane, 1 GiB each
//   g8                8-B gathers: lane l of a wave reads element (l * 37) mod 64 of its 64-
//                     element block, so every 512-B block is read whole, in scrambled order
//                     (the shape of k_rows_ell / k_rows_pnc x gathers: nearby, not sequential)
//   s8_64 s8_128      one 8-B element per 64-B / per 128-B segment (strided: what a sparse
//                     gather costs per useful byte); known bytes given as the segments touched
//   w16 w8            coalesced streaming stores, 16 / 8 B per lane, 1 GiB each
//
// Prints one JSON line per kernel: name, useful bytes, bytes of the 64-B / 128-B segments
// touched, ms. The counters come from rocprofv3 passes over this program (tools/gpu_steps.sh
// calib) and tools/calib_analysis.py divides them by these bytes. Dev tool, not part of libpamg.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

// a sum that the compiler must keep: the condition is never true for the zero-filled data, and
// it is one the compiler cannot rule out for any value type (an integer sum compared with a
// non-integer constant would be folded away, and the loads with it)
template <class T>
__device__ __forceinline__ void keep(T s, double* out) {
    if (s == (T)77) out[0] = (double)s;
}

template <class T>
__global__ __launch_bounds__(256) void k_read(const T* __restrict__ a, size_t n, double* __restrict__ out) {
    T s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i];
    keep(s, out);
}

__global__ __launch_bounds__(256) void k_read16(const double2* __restrict__ a, size_t n, double* __restrict__ out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    keep(s, out);
}

// 8-B gathers, every element of each 64-element block read once, lanes scrambled
__global__ __launch_bounds__(256) void k_gather8(const double* __restrict__ a, size_t n, double* __restrict__ out) {
    double s = 0.0;
    const int lane = threadIdx.x & 63;
    const size_t blocks = n / 64, wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
    const size_t waves = (size_t)gridDim.x * blockDim.x / 64;
    for (size_t b = wave; b < blocks; b += waves) s += a[b * 64 + (size_t)((lane * 37) & 63)];
    keep(s, out);
}

// one 8-B element per `stride` elements
__global__ __launch_bounds__(256) void k_strided8(const double* __restrict__ a, size_t n, int stride,
                                                  double* __restrict__ out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i * stride < n; i += (size_t)gridDim.x * blockDim.x)
        s += a[i * stride];
    keep(s, out);
}

__global__ __launch_bounds__(256) void k_flush(double2* __restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_double2(0.0, 0.0);
}

template <class T>
__global__ __launch_bounds__(256) void k_write(T* __restrict__ a, size_t n, T v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = v;
}

int main(int argc, char** argv) {
    const size_t region = (size_t)(argc > 1 ? atof(argv[1]) : 1.0) * (1ull << 30);
    const int nreg = 12;
    char* base = nullptr;
    char* flush = nullptr;
    double* out = nullptr;
    CK(hipMalloc(&base, region * nreg));
    CK(hipMalloc(&flush, region));
    CK(hipMalloc(&out, sizeof(double)));
    CK(hipMemset(base, 0, region * nreg));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grid = 8192, blk = 256;
    int r = 0;
    auto run = [&](const char* name, double useful, double seg64, double seg128, auto launch) {
        k_flush<<<grid, blk>>>(reinterpret_cast<double2*>(flush), region / 16);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\": \"%s\", \"useful_bytes\": %.0f, \"seg64_bytes\": %.0f, \"seg128_bytes\": %.0f, \"ms\": %.4f}\n",
               name, useful, seg64, seg128, ms);
        fflush(stdout);
        ++r;
    };
    auto reg = [&](int k) { return base + (size_t)k * region; };
    const double R = (double)region;
    run("r16", R, R, R, [&] { k_read16<<<grid, blk>>>(reinterpret_cast<const double2*>(reg(0)), region / 16, out); });
    run("r8", R, R, R, [&] { k_read<double><<<grid, blk>>>(reinterpret_cast<const double*>(reg(1)), region / 8, out); });
    run("r4", R, R, R, [&] { k_read<uint32_t><<<grid, blk>>>(reinterpret_cast<const uint32_t*>(reg(2)), region / 4, out); });
    run("r2", R, R, R, [&] { k_read<uint16_t><<<grid, blk>>>(reinterpret_cast<const uint16_t*>(reg(3)), region / 2, out); });
    run("r1", R, R, R, [&] { k_read<uint8_t><<<grid, blk>>>(reinterpret_cast<const uint8_t*>(reg(4)), region, out); });
    run("g8", R, R, R, [&] { k_gather8<<<grid, blk>>>(reinterpret_cast<const double*>(reg(5)), region / 8, out); });
    run("s8_64", R / 8, R, R, [&] { k_strided8<<<grid, blk>>>(reinterpret_cast<const double*>(reg(6)), region / 8, 8, out); });
    run("s8_128", R / 16, R / 2, R, [&] { k_strided8<<<grid, blk>>>(reinterpret_cast<const double*>(reg(7)), region / 8, 16, out); });
    run("w16", R, R, R, [&] { k_write<double2><<<grid, blk>>>(reinterpret_cast<double2*>(reg(8)), region / 16, make_double2(1.0, 1.0)); });
    run("w8", R, R, R, [&] { k_write<double><<<grid, blk>>>(reinterpret_cast<double*>(reg(9)), region / 8, 1.0); });
    CK(hipDeviceSynchronize());
    CK(hipFree(base));
    CK(hipFree(flush));
    CK(hipFree(out));
    return 0;
}
