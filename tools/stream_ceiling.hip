// stream_ceiling.hip — the HBM rates a streaming kernel reaches on this MI355X, as the
// practical ceiling beside the 8 TB/s spec for the row kernels' roofline: pure
// read (16 B per lane, grid-stride, sum kept live), copy (read + write), and a read:write
// mix of 11 : 1 like the level-0 Jacobi (11.85 GB moved, 1.07 GB of it the output). Dev
// tool, not part of libpamg.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/stream_ceiling tools/stream_ceiling.hip
//   tools/stream_ceiling [GiB]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                 \
    do {                                                                      \
        hipError_t e_ = (x);                                                  \
        if (e_ != hipSuccess) {                                               \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                          \
        }                                                                     \
    } while (0)

__global__ __launch_bounds__(256) void k_read(const double4* __restrict__ a, size_t n, double* __restrict__ out) {
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double4 v = a[i];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 1.2345e-300) out[0] = s;  // keeps the loads; never true for the data written below
}

__global__ __launch_bounds__(256) void k_copy(const double4* __restrict__ a, double4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = a[i];
}

// reads `ratio` coalesced streams of a (each nb elements long) per element written to b
__global__ __launch_bounds__(256) void k_mix(const double4* __restrict__ a, double4* __restrict__ b, size_t nb,
                                             int ratio) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nb; i += (size_t)gridDim.x * blockDim.x) {
        double4 s = a[i];
        for (int k = 1; k < ratio; ++k) {
            const double4 v = a[k * nb + i];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        b[i] = s;
    }
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 8.0;
    const size_t bytes = (size_t)(gib * (1ull << 30));
    const size_t n = bytes / sizeof(double4);
    double4 *a = nullptr, *b = nullptr;
    double* out = nullptr;
    CK(hipMalloc(&a, n * sizeof(double4)));
    CK(hipMalloc(&b, n * sizeof(double4)));
    CK(hipMalloc(&out, sizeof(double)));
    CK(hipMemset(a, 0, n * sizeof(double4)));
    CK(hipMemset(b, 0, n * sizeof(double4)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int grids[] = {1024, 2048, 4096, 8192, 16384};
    auto time = [&](auto launch) {
        launch();
        CK(hipDeviceSynchronize());
        float best = 1e30f;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (ms < best) best = ms;
        }
        return best;
    };
    for (int g : grids) {
        const float tr = time([&] { k_read<<<g, 256>>>(a, n, out); });
        const float tc = time([&] { k_copy<<<g, 256>>>(a, b, n / 2); });
        const size_t nb = n / 12;
        const float tm = time([&] { k_mix<<<g, 256>>>(a, b, nb, 11); });
        const double rb = (double)n * 32, cb = (double)(n / 2) * 64, mb = (double)nb * 32 * 12;
        printf("{\"grid\": %d, \"read_TBps\": %.3f, \"copy_TBps\": %.3f, \"mix11to1_TBps\": %.3f, \"GiB\": %.1f}\n", g,
               rb / tr / 1e9, cb / tc / 1e9, mb / tm / 1e9, gib);
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(out));
    return 0;
}
