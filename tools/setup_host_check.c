/* setup_host_check.c — host-only consumer of the setup entry points of include/pamg.h (no GPU,
 * no HIP runtime): the single-part SA hierarchy of a grid problem (SPEC §S4), R also built
 * from two transposed row blocks joined by pamg_setup_hstack_rows, and optionally a Matrix
 * Market file. Prints one JSON line with the level sizes and a wrapping uint64 checksum of
 * every level's A, P, R (row pointers + columns + value bits). tests/test_sanitizers.py
 * builds it with setup.cpp / mtx.cpp / errors.cpp under ASan + UBSan and compares the
 * checksums with the Python-driven setup.
 *
 *   ./setup_host_check <kind 0..3> <n> [file.mtx]
 */
#include <inttypes.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

static uint64_t checksum(const pamg_hcsr* M) {
    int64_t nr, nc, nnz, *rp;
    int32_t* col;
    double* val;
    CK(pamg_hcsr_info(M, &nr, &nc, &nnz));
    CK(pamg_hcsr_data((pamg_hcsr*)M, &rp, &col, &val));
    uint64_t s = 0;
    for (int64_t i = 0; i <= nr; ++i) s += (uint64_t)rp[i];
    for (int64_t k = 0; k < nnz; ++k) {
        uint64_t u;
        memcpy(&u, &val[k], 8);
        s += (uint64_t)(int64_t)col[k] + u;
    }
    return s;
}

static int64_t rows_of(const pamg_hcsr* M) {
    int64_t nr, nc, nnz;
    CK(pamg_hcsr_info(M, &nr, &nc, &nnz));
    return nr;
}

int main(int argc, char** argv) {
    const int kind = argc > 1 ? atoi(argv[1]) : 1;
    const int64_t n = argc > 2 ? atoll(argv[2]) : 12;
    const int64_t nz = kind == 0 ? 1 : n, N = n * n * nz * (kind == 3 ? 3 : 1);
    pamg_hcsr *A[MAXL] = {0}, *P[MAXL] = {0}, *R[MAXL] = {0};
    int L = 0;
    CK(pamg_gen_grid(kind, n, n, nz, 1e-3, 0, N, &A[0]));
    for (;;) {
        double rho;
        CK(pamg_setup_gershgorin(A[L], 0, &rho));
        const double omega = 4.0 / (3.0 * rho);
        const int64_t nl = rows_of(A[L]);
        ++L;
        if (nl <= 1000 || L >= MAXL) break;
        int32_t* agg = malloc(sizeof(int32_t) * (size_t)nl);
        int64_t nagg;
        CK(pamg_setup_aggregate(A[L - 1], 0, 0.02, agg, &nagg));
        if (nagg == 0 || nagg >= nl) {
            free(agg);
            break;
        }
        pamg_hcsr *T, *AP, *top, *bot, *Rh;
        CK(pamg_setup_tentative(nl, agg, nagg, 0, nagg, &T));
        free(agg);
        CK(pamg_setup_spgemm(A[L - 1], 0, T, NULL, 0, NULL, &P[L - 1]));
        CK(pamg_setup_smooth(A[L - 1], 0, T, P[L - 1], omega));
        CK(pamg_hcsr_destroy(T));
        CK(pamg_setup_spgemm(A[L - 1], 0, P[L - 1], NULL, 0, NULL, &AP));
        CK(pamg_setup_transpose(P[L - 1], 0, 0, nagg, &R[L - 1]));
        /* the same R from two row blocks of P (how parts assemble R, SPEC §S4.7) */
        {
            int64_t nr, nc, nnz, *rp;
            int32_t* col;
            double* val;
            CK(pamg_hcsr_info(P[L - 1], &nr, &nc, &nnz));
            CK(pamg_hcsr_data(P[L - 1], &rp, &col, &val));
            const int64_t h = nr / 2;
            CK(pamg_hcsr_create(h, nc, rp[h], &top));
            CK(pamg_hcsr_create(nr - h, nc, nnz - rp[h], &bot));
            int64_t *trp, *brp;
            int32_t *tc, *bc;
            double *tv, *bv;
            CK(pamg_hcsr_data(top, &trp, &tc, &tv));
            CK(pamg_hcsr_data(bot, &brp, &bc, &bv));
            memcpy(trp, rp, sizeof(int64_t) * (size_t)(h + 1));
            for (int64_t i = 0; i <= nr - h; ++i) brp[i] = rp[h + i] - rp[h];
            memcpy(tc, col, 4 * (size_t)rp[h]);
            memcpy(tv, val, 8 * (size_t)rp[h]);
            memcpy(bc, col + rp[h], 4 * (size_t)(nnz - rp[h]));
            memcpy(bv, val + rp[h], 8 * (size_t)(nnz - rp[h]));
            pamg_hcsr *pt, *pb;
            CK(pamg_setup_transpose(top, 0, 0, nagg, &pt));
            CK(pamg_setup_transpose(bot, h, 0, nagg, &pb));
            const pamg_hcsr* pieces[2] = {pt, pb};
            CK(pamg_setup_hstack_rows(2, pieces, &Rh));
            if (checksum(Rh) != checksum(R[L - 1])) {
                fprintf(stderr, "hstack of transposed blocks != transpose\n");
                return 2;
            }
            CK(pamg_hcsr_destroy(pt));
            CK(pamg_hcsr_destroy(pb));
            CK(pamg_hcsr_destroy(top));
            CK(pamg_hcsr_destroy(bot));
            CK(pamg_hcsr_destroy(Rh));
        }
        CK(pamg_setup_spgemm(R[L - 1], 0, AP, NULL, 0, NULL, &A[L]));
        CK(pamg_hcsr_destroy(AP));
    }
    const int64_t nc = rows_of(A[L - 1]);
    double* ainv = malloc(sizeof(double) * (size_t)(nc * nc));
    CK(pamg_setup_cholinv(A[L - 1], ainv));
    uint64_t sa = 0;
    for (int64_t k = 0; k < nc * nc; ++k) {
        uint64_t u;
        memcpy(&u, &ainv[k], 8);
        sa += u;
    }
    printf("{\"levels\": %d, \"rows\": [", L);
    for (int l = 0; l < L; ++l) printf("%s%" PRId64, l ? ", " : "", rows_of(A[l]));
    printf("], \"sum\": [");
    for (int l = 0; l < L; ++l) {
        printf("%s[\"%" PRIu64 "\", \"%" PRIu64 "\", \"%" PRIu64 "\"]", l ? ", " : "", checksum(A[l]),
               P[l] ? checksum(P[l]) : 0, R[l] ? checksum(R[l]) : 0);
    }
    printf("], \"ainv\": \"%" PRIu64 "\"", sa);
    if (argc > 3) {
        int64_t ng;
        pamg_hcsr* M;
        CK(pamg_read_mtx(argv[3], 0, -1, &ng, &M));
        int64_t* cnt = malloc(sizeof(int64_t) * (size_t)(ng + 1));
        CK(pamg_mtx_row_counts(argv[3], &ng, cnt));
        printf(", \"mtx_rows\": %" PRId64 ", \"mtx_sum\": \"%" PRIu64 "\"", ng, checksum(M));
        free(cnt);
        CK(pamg_hcsr_destroy(M));
    }
    printf("}\n");
    for (int l = 0; l < L; ++l) {
        CK(pamg_hcsr_destroy(A[l]));
        if (P[l]) CK(pamg_hcsr_destroy(P[l]));
        if (R[l]) CK(pamg_hcsr_destroy(R[l]));
    }
    free(ainv);
    return 0;
}
