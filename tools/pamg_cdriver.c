/* pamg_cdriver.c — a plain-C consumer of the libpamg C-ABI (include/pamg.h), no Python:
 * single-part smoothed-aggregation setup from the setup entry points (SPEC §S4, the same
 * sequence parallel_amg_amd/hierarchy.py runs for one part), device hierarchy, V-cycles.
 * It is what a non-Python host (the reference's Julia over ccall, a C/Fortran code) does.
 *
 *   gcc -O2 -std=c11 -Iinclude tools/pamg_cdriver.c -Lparallel_amg_amd -lpamg \
 *       -Wl,-rpath,$PWD/parallel_amg_amd -o pamg_cdriver
 *   ./pamg_cdriver <kind 0..3> <n> <ncycles> <gpu_products 0|1>
 *
 * Prints one JSON line: levels, rows per level, V-cycles/s, and the residual history both
 * as numbers and as IEEE-754 bit patterns (tests compare those with the Python path).
 */
#define _POSIX_C_SOURCE 199309L
#include <inttypes.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "pamg.h"

#define MAXL 20
#define CK(x)                                                                          \
    do {                                                                               \
        int rc_ = (x);                                                                 \
        if (rc_ != PAMG_OK) {                                                          \
            fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, rc_,      \
                    pamg_last_error());                                                \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static int64_t nrows_of(const pamg_hcsr* M) {
    int64_t nr, nc, nnz;
    CK(pamg_hcsr_info(M, &nr, &nc, &nnz));
    return nr;
}

static pamg_mat* upload(pamg_ctx* ctx, pamg_hcsr* M) {
    int64_t nr, nc, nnz, *rp;
    int32_t* col;
    double* val;
    pamg_mat* D;
    CK(pamg_hcsr_info(M, &nr, &nc, &nnz));
    CK(pamg_hcsr_data(M, &rp, &col, &val));
    CK(pamg_mat_upload(ctx, nr, nc, rp, col, 0, val, 0, NULL, &D));
    return D;
}

int main(int argc, char** argv) {
    const int kind = argc > 1 ? atoi(argv[1]) : 1;
    const int64_t n = argc > 2 ? atoll(argv[2]) : 64;
    const int ncycles = argc > 3 ? atoi(argv[3]) : 10;
    const int gpu_products = argc > 4 ? atoi(argv[4]) : 1;
    const double theta = 0.02, eps = 1e-3;
    const int64_t max_coarse = 1000;
    const int64_t nz = (kind == 0) ? 1 : n;
    const int64_t N = n * n * nz * (kind == 3 ? 3 : 1);

    pamg_ctx* ctx;
    CK(pamg_ctx_create(0, &ctx));
    pamg_hcsr *A[MAXL] = {0}, *P[MAXL] = {0}, *R[MAXL] = {0};
    double omega[MAXL];
    int L = 0;
    const double t0 = now();
    CK(pamg_gen_grid(kind, n, n, nz, eps, 0, N, &A[0]));
    for (;;) {
        double rho;
        CK(pamg_setup_gershgorin(A[L], 0, &rho));
        omega[L] = 4.0 / (3.0 * rho);
        const int64_t nl = nrows_of(A[L]);
        ++L;
        if (nl <= max_coarse || L >= MAXL) break;
        int32_t* agg = malloc(sizeof(int32_t) * (size_t)(nl + 1));
        int64_t nagg;
        CK(pamg_setup_aggregate(A[L - 1], 0, theta, agg, &nagg));
        if (nagg == 0 || nagg >= nl) {
            free(agg);
            break;
        }
        pamg_hcsr *T, *AP;
        CK(pamg_setup_tentative(nl, agg, nagg, 0, nagg, &T));
        free(agg);
        if (gpu_products) CK(pamg_dev_spgemm(ctx, A[L - 1], 0, T, NULL, 0, NULL, &P[L - 1]));
        else CK(pamg_setup_spgemm(A[L - 1], 0, T, NULL, 0, NULL, &P[L - 1]));
        CK(pamg_setup_smooth(A[L - 1], 0, T, P[L - 1], omega[L - 1]));  /* P = T - q A T */
        CK(pamg_hcsr_destroy(T));
        if (gpu_products) {
            CK(pamg_dev_spgemm(ctx, A[L - 1], 0, P[L - 1], NULL, 0, NULL, &AP));
            CK(pamg_dev_transpose(ctx, P[L - 1], 0, 0, nagg, &R[L - 1]));
            CK(pamg_dev_spgemm(ctx, R[L - 1], 0, AP, NULL, 0, NULL, &A[L]));
        } else {
            CK(pamg_setup_spgemm(A[L - 1], 0, P[L - 1], NULL, 0, NULL, &AP));
            CK(pamg_setup_transpose(P[L - 1], 0, 0, nagg, &R[L - 1]));
            CK(pamg_setup_spgemm(R[L - 1], 0, AP, NULL, 0, NULL, &A[L]));
        }
        CK(pamg_hcsr_destroy(AP));
    }
    const int64_t nc = nrows_of(A[L - 1]);
    double* ainv = malloc(sizeof(double) * (size_t)(nc * nc));
    CK(pamg_setup_cholinv(A[L - 1], ainv));
    const double t_setup = now() - t0;

    pamg_mat *dA[MAXL], *dP[MAXL] = {0}, *dR[MAXL] = {0};
    for (int l = 0; l < L; ++l) {
        dA[l] = upload(ctx, A[l]);
        if (l < L - 1) {
            dP[l] = upload(ctx, P[l]);
            dR[l] = upload(ctx, R[l]);
        }
    }
    pamg_hier* H;
    CK(pamg_hier_create(ctx, L, dA, dP, dR, omega, nc, ainv, L - 1, NULL, &H));

    /* b = A x*, x0 = 0 (SPEC §S2) */
    double* xs = malloc(sizeof(double) * (size_t)N);
    CK(pamg_gen_xstar(0, N, 20240807ULL, xs));
    pamg_vec *x, *b, *xst;
    CK(pamg_vec_create(ctx, N, 0, &x));
    CK(pamg_vec_create(ctx, N, 0, &b));
    CK(pamg_vec_create(ctx, N, 0, &xst));
    CK(pamg_vec_upload(ctx, xst, xs));
    CK(pamg_spmv(ctx, dA[0], xst, b));
    CK(pamg_vec_fill(ctx, x, 0.0));
    double hist[1024];
    const int nh = ncycles < 1024 ? ncycles : 1024;
    const double t1 = now();
    CK(pamg_vcycle(ctx, H, x, b, nh, hist));
    const double t_solve = now() - t1;

    printf("{\"kind\": %d, \"n\": %" PRId64 ", \"rows\": %" PRId64 ", \"levels\": %d, \"level_rows\": [",
           kind, n, N, L);
    for (int l = 0; l < L; ++l) printf("%s%" PRId64, l ? ", " : "", nrows_of(A[l]));
    printf("], \"gpu_products\": %d, \"setup_s\": %.3f, \"vcycles_per_s\": %.3f, \"res\": [", gpu_products,
           t_setup, nh / t_solve);
    for (int k = 0; k < nh; ++k) printf("%s%.17g", k ? ", " : "", hist[k]);
    printf("], \"res_bits\": [");
    for (int k = 0; k < nh; ++k) {
        uint64_t u;
        memcpy(&u, &hist[k], 8);
        printf("%s\"%016" PRIx64 "\"", k ? ", " : "", u);
    }
    printf("]}\n");

    CK(pamg_hier_destroy(H));
    for (int l = 0; l < L; ++l) {
        CK(pamg_mat_destroy(dA[l]));
        CK(pamg_hcsr_destroy(A[l]));
        if (l < L - 1) {
            CK(pamg_mat_destroy(dP[l]));
            CK(pamg_mat_destroy(dR[l]));
            CK(pamg_hcsr_destroy(P[l]));
            CK(pamg_hcsr_destroy(R[l]));
        }
    }
    CK(pamg_vec_destroy(x));
    CK(pamg_vec_destroy(b));
    CK(pamg_vec_destroy(xst));
    CK(pamg_ctx_destroy(ctx));
    free(ainv);
    free(xs);
    return 0;
}
