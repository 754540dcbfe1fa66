// chunk_exp.hip — dev experiment (not part of libpamg): does running two dependent row ops
// (Jacobi sweep, then the residual of its result) chunk-interleaved — the residual of chunk c
// right after the Jacobi of chunk c + lag — reuse A's rows from the Infinity Cache (MALL)?
// Compares against two full passes; checks the residual bits are identical.
//
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -I parallel_amg_amd/csrc tools/chunk_exp.hip \
//       -L parallel_amg_amd -lpamg -Wl,-rpath,$PWD/parallel_amg_amd -o gpurun_ab/chunk_exp
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pamg_device.h"

#define CK(x)                                                              \
    do {                                                                   \
        int rc_ = (x);                                                     \
        if (rc_ != 0) {                                                    \
            fprintf(stderr, "%s:%d %s -> %d %s\n", __FILE__, __LINE__, #x, \
                    rc_, pamg_last_error());                              \
            exit(1);                                                       \
        }                                                                  \
    } while (0)
#define HK(x) CK((x) == hipSuccess ? 0 : -2)

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 512;
    const int64_t N = (int64_t)n * n * n, plane = (int64_t)n * n;
    CK(pamg_set_option("tile_order", 0));
    pamg_hcsr* H;
    CK(pamg_gen_grid(1, n, n, n, 1e-3, 0, N, &H));
    int64_t *rp;
    int32_t* col;
    double* val;
    CK(pamg_hcsr_data(H, &rp, &col, &val));
    pamg_ctx* ctx;
    CK(pamg_ctx_create(0, &ctx));
    pamg_mat* A;
    CK(pamg_mat_upload(ctx, N, N, rp, col, 0, val, 0, nullptr, &A));
    pamg_hcsr_destroy(H);
    pamg_vec *vx, *vb, *vt, *vr, *vr2;
    for (pamg_vec** v : {&vx, &vb, &vt, &vr, &vr2}) CK(pamg_vec_create(ctx, N, 0, v));
    std::vector<double> h(N);
    for (int64_t i = 0; i < N; ++i) h[i] = (double)((i * 2654435761u) % 1000) / 997.0 - 0.5;
    CK(pamg_vec_upload(ctx, vx, h.data()));
    CK(pamg_vec_fill(ctx, vb, 1.0));
    double *x, *b, *t, *r, *r2;
    CK(pamg_vec_device_ptr(vx, &x));
    CK(pamg_vec_device_ptr(vb, &b));
    CK(pamg_vec_device_ptr(vt, &t));
    CK(pamg_vec_device_ptr(vr, &r));
    CK(pamg_vec_device_ptr(vr2, &r2));
    const pamg::TileSet& ts = A->interior;
    std::vector<int4> tiles(ts.n_short);
    HK(hipMemcpy(tiles.data(), ts.d_short, sizeof(int4) * ts.n_short, hipMemcpyDeviceToHost));
    printf("tiles %d long %d\n", ts.n_short, ts.n_long);
    hipStream_t s = ctx->s_comp;
    hipEvent_t e0, e1;
    HK(hipEventCreate(&e0));
    HK(hipEventCreate(&e1));
    const double om = 2.0 / 3.0;
    auto full = [&]() {
        pamg::launch_rows(*A, ts, pamg::OP_JACOBI, x, b, x, t, om, s);
        pamg::launch_rows(*A, ts, pamg::OP_RESID, t, b, t, r, 0.0, s);
    };
    auto timeit = [&](auto&& fn, int reps) {
        fn();
        HK(hipEventRecord(e0, s));
        for (int k = 0; k < reps; ++k) fn();
        HK(hipEventRecord(e1, s));
        HK(hipEventSynchronize(e1));
        float ms;
        HK(hipEventElapsedTime(&ms, e0, e1));
        return ms / reps;
    };
    const float t_full = timeit(full, 5);
    printf("full passes: %.3f ms (jacobi + residual)\n", t_full);
    std::vector<double> ref(N), got(N);
    HK(hipMemcpy(ref.data(), r, 8 * N, hipMemcpyDeviceToHost));
    for (int cp : {1, 2, 4, 8, 16}) {
        // chunk boundaries: first tile starting at or after c * cp planes
        std::vector<int> cut;
        for (int64_t row = 0; row < N; row += cp * plane) {
            int lo = 0, hi = ts.n_short;
            while (lo < hi) {
                int mid = (lo + hi) / 2;
                if (tiles[mid].x < row) lo = mid + 1;
                else hi = mid;
            }
            cut.push_back(lo);
        }
        cut.push_back(ts.n_short);
        const int nch = (int)cut.size() - 1;
        const int lag = 1 + (cp < 2 ? 1 : 0);  // residual rows need t up to one plane ahead
        auto sub = [&](int c) {
            pamg::TileSet q = ts;
            q.d_short = ts.d_short + cut[c];
            q.n_short = cut[c + 1] - cut[c];
            q.n_long = 0;
            return q;
        };
        auto chunked = [&]() {
            for (int c = 0; c < nch + lag; ++c) {
                if (c < nch) {
                    auto q = sub(c);
                    if (q.n_short) pamg::launch_rows(*A, q, pamg::OP_JACOBI, x, b, x, t, om, s);
                }
                if (c - lag >= 0) {
                    auto q = sub(c - lag);
                    if (q.n_short) pamg::launch_rows(*A, q, pamg::OP_RESID, t, b, t, r2, 0.0, s);
                }
            }
        };
        HK(hipMemset(r2, 0, 8 * N));
        const float t_eager = timeit(chunked, 3);
        HK(hipMemcpy(got.data(), r2, 8 * N, hipMemcpyDeviceToHost));
        const bool same = memcmp(got.data(), ref.data(), 8 * N) == 0;
        // graph of the chunked sequence
        hipGraph_t g;
        hipGraphExec_t ge;
        HK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        chunked();
        HK(hipStreamEndCapture(s, &g));
        HK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        const float t_graph = timeit([&]() { HK(hipGraphLaunch(ge, s)); }, 5);
        HK(hipGraphExecDestroy(ge));
        HK(hipGraphDestroy(g));
        printf("chunk %2d planes (%3d chunks, lag %d): eager %.3f ms, graph %.3f ms, bits %s\n", cp,
               nch, lag, t_eager, t_graph, same ? "identical" : "DIFFER");
    }
    fflush(stdout);
    return 0;
}
