/*
 * pamg_oracle.c — CPU restatement of SPEC.md (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the checker, never the product: only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it. The product path (parallel_amg_amd/) never
 * links or calls it.
 *
 * Reference anchoring: the reference (/root/reference/README.md:1-2, "Apply AMG algorithm
 * parallelly using PartitionedArrays.jl") contains no code, tests or golden vectors, and
 * its toolchain (Julia + PartitionedArrays.jl, version unpinned) is absent — PARITY WITH
 * THE REFERENCE IS UNPINNED. This file restates SPEC.md (§S1–§S7), which
 * follows the public smoothed-aggregation algorithm (PyAMG / AlgebraicMultigrid.jl style)
 * named in SURVEY.md §8c. It is pinned instead by (a) scipy.sparse cross-checks,
 * (b) hand-derived known-answer tests and (c) committed golden fixtures (tests/golden/).
 *
 * Deliberately simple: single pass, dense accumulators, qsort; optional OpenMP only on
 * row-independent loops (bit-identical with or without it). Build: oracle/Makefile
 * (-O2 -ffp-contract=off).
 */
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef int64_t i64;

/* ------------------------------------------------------------------ generators §S2 */

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* x*_i for i in [i0, i0+n) (§S2). */
void orc_xstar(i64 i0, i64 n, uint64_t seed, double* out) {
    for (i64 k = 0; k < n; ++k) {
        uint64_t z = mix64(seed + (uint64_t)(i0 + k + 1) * 0x9E3779B97F4A7C15ULL);
        double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
        out[k] = 2.0 * u - 1.0;
    }
}

/* kind: 0 = poisson2d (nz must be 1), 1 = poisson3d, 2 = aniso3d(eps). */
static void stencil_vals(int kind, double eps, double* diag, double* vxy, double* vz) {
    if (kind == 2) { *diag = 4.0 + 2.0 * eps; *vxy = -1.0; *vz = -eps; }
    else if (kind == 1) { *diag = 6.0; *vxy = -1.0; *vz = -1.0; }
    else { *diag = 4.0; *vxy = -1.0; *vz = -1.0; }
}

/* Rows [r0, r1) of the grid operator; rowptr relative (rowptr[0] = 0), global col ids.
 * Returns nnz written. Pass col == NULL to count only. */
/* kind 3 = elastic3d (SPEC §S2): 3 unknowns per node of an nx*ny*nz grid, row 3*node+d,
 * A = L27 (x) B with L27 the 27-point Dirichlet Laplacian (26 / -1) and B = 4I - J (3x3). */
static i64 gen_elastic(i64 nx, i64 ny, i64 nz, i64 r0, i64 r1, i64* rowptr, i64* col, double* val) {
    i64 k = 0;
    if (rowptr) rowptr[0] = 0;
    for (i64 r = r0; r < r1; ++r) {
        const i64 node = r / 3, d = r % 3;
        const i64 x = node % nx, y = (node / nx) % ny, z = node / (nx * ny);
        for (int dz = -1; dz <= 1; ++dz)
            for (int dy = -1; dy <= 1; ++dy)
                for (int dx = -1; dx <= 1; ++dx) {
                    const i64 X = x + dx, Y = y + dy, Z = z + dz;
                    if (X < 0 || Y < 0 || Z < 0 || X >= nx || Y >= ny || Z >= nz) continue;
                    const i64 m = X + nx * (Y + ny * Z);
                    const double l = (m == node) ? 26.0 : -1.0;
                    for (int e = 0; e < 3; ++e) {
                        if (col) { col[k] = 3 * m + e; val[k] = l * ((e == d) ? 3.0 : -1.0); }
                        ++k;
                    }
                }
        if (rowptr) rowptr[r - r0 + 1] = k;
    }
    return k;
}

i64 orc_gen_rows(int kind, i64 nx, i64 ny, i64 nz, double eps, i64 r0, i64 r1,
                 i64* rowptr, i64* col, double* val) {
    if (kind == 3) return gen_elastic(nx, ny, nz, r0, r1, rowptr, col, val);
    double d, vxy, vz;
    stencil_vals(kind, eps, &d, &vxy, &vz);
    const i64 pxy = nx * ny;
    i64 k = 0;
    if (rowptr) rowptr[0] = 0;
    for (i64 r = r0; r < r1; ++r) {
        i64 x = r % nx, y = (r / nx) % ny, z = r / pxy;
        i64 c[7]; double v[7]; int m = 0;
        if (z > 0)      { c[m] = r - pxy; v[m++] = vz; }
        if (y > 0)      { c[m] = r - nx;  v[m++] = vxy; }
        if (x > 0)      { c[m] = r - 1;   v[m++] = vxy; }
        c[m] = r; v[m++] = d;
        if (x < nx - 1) { c[m] = r + 1;   v[m++] = vxy; }
        if (y < ny - 1) { c[m] = r + nx;  v[m++] = vxy; }
        if (z < nz - 1) { c[m] = r + pxy; v[m++] = vz; }
        if (col) for (int t = 0; t < m; ++t) { col[k + t] = c[t]; val[k + t] = v[t]; }
        k += m;
        if (rowptr) rowptr[r - r0 + 1] = k;
    }
    return k;
}

/* ------------------------------------------------------------------ row sums §S3 */

static inline double rowsum(const i64* rp, const i64* col, const double* val,
                            const double* x, i64 i) {
    double s = 0.0;
    for (i64 k = rp[i]; k < rp[i + 1]; ++k) { double p = val[k] * x[col[k]]; s = s + p; }
    return s;
}

static inline double diag_of(const i64* rp, const i64* col, const double* val, i64 i, i64 gi) {
    for (i64 k = rp[i]; k < rp[i + 1]; ++k) if (col[k] == gi) return val[k];
    return 0.0;
}

void orc_spmv(i64 n, const i64* rp, const i64* col, const double* val,
              const double* x, double* y) {
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < n; ++i) y[i] = rowsum(rp, col, val, x, i);
}

void orc_residual(i64 n, const i64* rp, const i64* col, const double* val,
                  const double* x, const double* b, double* r) {
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < n; ++i) r[i] = b[i] - rowsum(rp, col, val, x, i);
}

/* x_new = x + (omega*(b - A x)) / a_ii. Square A (global ids == local). */
void orc_jacobi(i64 n, const i64* rp, const i64* col, const double* val,
                const double* x, const double* b, double omega, double* xn) {
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < n; ++i) {
        double s = rowsum(rp, col, val, x, i);
        double u = b[i] - s, v = omega * u, w = v / diag_of(rp, col, val, i, i);
        xn[i] = x[i] + w;
    }
}

/* ------------------------------------------------------------------ CSR helpers */

typedef struct { i64 nr, nc, nnz; i64* rp; i64* col; double* val; } ocsr;

static void csr_free(ocsr* a) { free(a->rp); free(a->col); free(a->val); memset(a, 0, sizeof *a); }

static ocsr csr_copy(i64 nr, i64 nc, const i64* rp, const i64* col, const double* val) {
    ocsr a; a.nr = nr; a.nc = nc; a.nnz = rp[nr];
    a.rp = malloc(sizeof(i64) * (nr + 1)); a.col = malloc(sizeof(i64) * (a.nnz + 1));
    a.val = malloc(sizeof(double) * (a.nnz + 1));
    memcpy(a.rp, rp, sizeof(i64) * (nr + 1));
    memcpy(a.col, col, sizeof(i64) * a.nnz); memcpy(a.val, val, sizeof(double) * a.nnz);
    return a;
}

static int cmp_i64(const void* a, const void* b) {
    i64 x = *(const i64*)a, y = *(const i64*)b; return (x > y) - (x < y);
}

/* Gustavson C = X*Y (§S4.5): first product initialises, later ones add; row sorted.
 * Rows are independent: blocks of rows run on OpenMP threads, each row computed exactly as in
 * the serial loop (same products, same order), and the blocks are concatenated in row order. */
typedef struct { i64 r0, r1, nnz, cap; i64* col; double* val; i64* len; } gblock;

static void spgemm_rows(const ocsr* X, const ocsr* Y, gblock* g, double* acc, i64* mark, i64* list) {
    g->nnz = 0; g->cap = 1024;
    g->col = malloc(sizeof(i64) * g->cap); g->val = malloc(sizeof(double) * g->cap);
    g->len = malloc(sizeof(i64) * (g->r1 - g->r0 + 1));
    for (i64 i = g->r0; i < g->r1; ++i) {
        i64 m = 0;
        for (i64 a = X->rp[i]; a < X->rp[i + 1]; ++a) {
            i64 k = X->col[a]; double xv = X->val[a];
            for (i64 b = Y->rp[k]; b < Y->rp[k + 1]; ++b) {
                i64 j = Y->col[b]; double p = xv * Y->val[b];
                if (mark[j] != i) { mark[j] = i; acc[j] = p; list[m++] = j; }
                else acc[j] = acc[j] + p;
            }
        }
        qsort(list, (size_t)m, sizeof(i64), cmp_i64);
        if (g->nnz + m > g->cap) {
            while (g->nnz + m > g->cap) g->cap *= 2;
            g->col = realloc(g->col, sizeof(i64) * g->cap); g->val = realloc(g->val, sizeof(double) * g->cap);
        }
        for (i64 t = 0; t < m; ++t) { g->col[g->nnz] = list[t]; g->val[g->nnz] = acc[list[t]]; ++g->nnz; }
        g->len[i - g->r0] = m;
    }
}

static ocsr spgemm(const ocsr* X, const ocsr* Y) {
    ocsr C; C.nr = X->nr; C.nc = Y->nc;
    /* ~32 blocks per thread (a coarse product has few rows, each long) */
    i64 rows_per = X->nr / (32 * (i64)omp_get_max_threads()) + 1;
    if (rows_per > 65536) rows_per = 65536;
    const i64 nb = (X->nr + rows_per - 1) / rows_per;
    gblock* blk = calloc((size_t)nb + 1, sizeof(gblock));
    for (i64 t = 0; t < nb; ++t) { blk[t].r0 = t * rows_per; blk[t].r1 = (t + 1) * rows_per < X->nr ? (t + 1) * rows_per : X->nr; }
#pragma omp parallel
    {
        double* acc = calloc(Y->nc + 1, sizeof(double));
        i64* mark = malloc(sizeof(i64) * (Y->nc + 1));
        for (i64 j = 0; j < Y->nc; ++j) mark[j] = -1;
        i64* list = malloc(sizeof(i64) * (Y->nc + 1));
#pragma omp for schedule(dynamic, 1)
        for (i64 t = 0; t < nb; ++t) spgemm_rows(X, Y, &blk[t], acc, mark, list);
        free(acc); free(mark); free(list);
    }
    i64 nnz = 0;
    for (i64 t = 0; t < nb; ++t) nnz += blk[t].nnz;
    C.rp = malloc(sizeof(i64) * (X->nr + 1)); C.col = malloc(sizeof(i64) * (nnz + 1));
    C.val = malloc(sizeof(double) * (nnz + 1));
    C.rp[0] = 0;
    i64* start = malloc(sizeof(i64) * (nb + 1));
    start[0] = 0;
    for (i64 t = 0; t < nb; ++t) {
        start[t + 1] = start[t] + blk[t].nnz;
        for (i64 i = blk[t].r0; i < blk[t].r1; ++i) C.rp[i + 1] = C.rp[i] + blk[t].len[i - blk[t].r0];
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (i64 t = 0; t < nb; ++t) {
        memcpy(C.col + start[t], blk[t].col, sizeof(i64) * blk[t].nnz);
        memcpy(C.val + start[t], blk[t].val, sizeof(double) * blk[t].nnz);
        free(blk[t].col); free(blk[t].val); free(blk[t].len);
    }
    C.nnz = nnz;
    free(start); free(blk);
    return C;
}

/* R = P^T: entries of each row in ascending fine-row order (§S4.7). Each thread owns a range of
 * R's rows (P's columns) and scans P in fine-row order, so every row of R is filled in that order. */
static ocsr transpose(const ocsr* P) {
    ocsr R; R.nr = P->nc; R.nc = P->nr; R.nnz = P->nnz;
    R.rp = calloc(R.nr + 1, sizeof(i64));
    R.col = malloc(sizeof(i64) * (R.nnz + 1)); R.val = malloc(sizeof(double) * (R.nnz + 1));
    i64* pos = malloc(sizeof(i64) * (R.nr + 1));
#pragma omp parallel
    {
        const i64 nt = omp_get_num_threads(), t = omp_get_thread_num();
        const i64 c0 = R.nr * t / nt, c1 = R.nr * (t + 1) / nt;
        for (i64 a = 0; a < P->nnz; ++a) {
            const i64 c = P->col[a];
            if (c >= c0 && c < c1) R.rp[c + 1]++;
        }
#pragma omp barrier
#pragma omp single
        {
            for (i64 c = 0; c < R.nr; ++c) R.rp[c + 1] += R.rp[c];
            memcpy(pos, R.rp, sizeof(i64) * (R.nr + 1));
        }
        for (i64 i = 0; i < P->nr; ++i)
            for (i64 a = P->rp[i]; a < P->rp[i + 1]; ++a) {
                const i64 c = P->col[a];
                if (c >= c0 && c < c1) { R.col[pos[c]] = i; R.val[pos[c]] = P->val[a]; pos[c]++; }
            }
    }
    free(pos);
    return R;
}

/* ------------------------------------------------------------------ setup §S4 */

static double gershgorin(const ocsr* A) {
    double rho = 0.0;  /* (a max: the same value in any row order) */
#pragma omp parallel for schedule(static) reduction(max : rho)
    for (i64 i = 0; i < A->nr; ++i) {
        double s = 0.0, d = 0.0;
        for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a) {
            s = s + fabs(A->val[a]);
            if (A->col[a] == i) d = A->val[a];
        }
        double q = s / fabs(d);
        if (q > rho) rho = q;
    }
    return rho;
}

/* Standard aggregation (§S4.2-3), decoupled by parts (offs[nparts+1] row ranges).
 * agg[i] = global coarse id or -1; coffs[nparts+1] coarse ranges. Returns n_c. */
static i64 aggregate(const ocsr* A, double theta, int nparts, const i64* offs,
                     i64* agg, i64* coffs) {
    const i64 n = A->nr;
    double* dg = malloc(sizeof(double) * (n + 1));
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < n; ++i) {
        dg[i] = 0.0;
        for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a) if (A->col[a] == i) dg[i] = A->val[a];
    }
    /* strong[a] for each entry (rows independent) */
    char* strong = calloc(A->nnz + 1, 1);
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < n; ++i) {
        int p = 0;  /* the part owning row i */
        while (i >= offs[p + 1]) ++p;
        for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a) {
            i64 j = A->col[a];
            if (j == i || j < offs[p] || j >= offs[p + 1]) continue;
            double t = theta * sqrt(fabs(dg[i] * dg[j]));
            strong[a] = fabs(A->val[a]) >= t;
        }
    }
    enum { UN = -2, ISO = -3 };
    /* state: -2 unassigned, -3 isolated, >=0 local aggregate; pass1 flag */
    char* p1 = calloc(n + 1, 1);
    i64 base = 0;
    coffs[0] = 0;
    for (int q = 0; q < nparts; ++q) {
        i64 lo = offs[q], hi = offs[q + 1], na = 0;
        for (i64 i = lo; i < hi; ++i) agg[i] = UN;
        for (i64 i = lo; i < hi; ++i) {                       /* pass 1 */
            if (agg[i] != UN) continue;
            int has_nb = 0, has_assigned = 0;
            for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a) if (strong[a]) {
                has_nb = 1; if (agg[A->col[a]] != UN) { has_assigned = 1; break; }
            }
            if (!has_nb) { agg[i] = ISO; continue; }
            if (has_assigned) continue;
            agg[i] = na; p1[i] = 1;
            for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a)
                if (strong[a]) { agg[A->col[a]] = na; p1[A->col[a]] = 1; }
            ++na;
        }
        for (i64 i = lo; i < hi; ++i) {                       /* pass 2 */
            if (agg[i] != UN) continue;
            for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a)
                if (strong[a] && p1[A->col[a]]) { agg[i] = agg[A->col[a]]; break; }
        }
        for (i64 i = lo; i < hi; ++i) {                       /* pass 3 */
            if (agg[i] != UN) continue;
            agg[i] = na;
            for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a)
                if (strong[a] && agg[A->col[a]] == UN) agg[A->col[a]] = na;
            ++na;
        }
        for (i64 i = lo; i < hi; ++i) agg[i] = (agg[i] == ISO) ? -1 : agg[i] + base;
        base += na;
        coffs[q + 1] = base;
    }
    free(dg); free(strong); free(p1);
    return base;
}

/* P = T - (omega/a_ii) (A T) (§S4.4, §S4.6). */
static ocsr smoothed_prolongator(const ocsr* A, const i64* agg, i64 nc, double omega) {
    i64* cnt = calloc(nc + 1, sizeof(i64));
    for (i64 i = 0; i < A->nr; ++i) if (agg[i] >= 0) cnt[agg[i]]++;
    ocsr T; T.nr = A->nr; T.nc = nc;
    T.rp = malloc(sizeof(i64) * (A->nr + 1)); T.col = malloc(sizeof(i64) * (A->nr + 1));
    T.val = malloc(sizeof(double) * (A->nr + 1));
    T.rp[0] = 0; i64 m = 0;
    for (i64 i = 0; i < A->nr; ++i) {
        if (agg[i] >= 0) { T.col[m] = agg[i]; T.val[m] = 1.0 / sqrt((double)cnt[agg[i]]); ++m; }
        T.rp[i + 1] = m;
    }
    T.nnz = m;
    ocsr AT = spgemm(A, &T);
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i < AT.nr; ++i) {
        double d = 0.0;
        for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a) if (A->col[a] == i) d = A->val[a];
        double q = omega / d;
        i64 ti = (T.rp[i + 1] > T.rp[i]) ? T.col[T.rp[i]] : -1;
        double tv = (ti >= 0) ? T.val[T.rp[i]] : 0.0;
        for (i64 a = AT.rp[i]; a < AT.rp[i + 1]; ++a) {
            double t = (AT.col[a] == ti) ? tv : 0.0;
            AT.val[a] = t - q * AT.val[a];
        }
    }
    csr_free(&T); free(cnt);
    return AT;
}

/* Cholesky inverse (§S5), column-major output ainv[c*n + i]. Returns 0 or -1. */
static int chol_inverse(const ocsr* A, double* ainv) {
    const i64 n = A->nr;
    double* Ad = calloc((size_t)(n * n) + 1, sizeof(double));  /* row-major dense */
    for (i64 i = 0; i < n; ++i)
        for (i64 a = A->rp[i]; a < A->rp[i + 1]; ++a) Ad[i * n + A->col[a]] = A->val[a];
    double* L = calloc((size_t)(n * n) + 1, sizeof(double));   /* row-major */
    for (i64 j = 0; j < n; ++j) {
        double d = Ad[j * n + j];
        for (i64 k = 0; k < j; ++k) d = d - L[j * n + k] * L[j * n + k];
        if (!(d > 0.0)) { free(Ad); free(L); return -1; }
        L[j * n + j] = sqrt(d);
        for (i64 i = j + 1; i < n; ++i) {
            double s = Ad[i * n + j];
            for (i64 k = 0; k < j; ++k) s = s - L[i * n + k] * L[j * n + k];
            L[i * n + j] = s / L[j * n + j];
        }
    }
    double* y = malloc(sizeof(double) * (n + 1));
    for (i64 c = 0; c < n; ++c) {
        for (i64 i = 0; i < n; ++i) {
            double s = (i == c) ? 1.0 : 0.0;
            for (i64 k = 0; k < i; ++k) s = s - L[i * n + k] * y[k];
            y[i] = s / L[i * n + i];
        }
        double* z = ainv + c * n;
        for (i64 i = n - 1; i >= 0; --i) {
            double s = y[i];
            for (i64 k = n - 1; k > i; --k) s = s - L[k * n + i] * z[k];
            z[i] = s / L[i * n + i];
        }
    }
    free(Ad); free(L); free(y);
    return 0;
}

/* ------------------------------------------------------------------ hierarchy */

#define ORC_MAXL 32
typedef struct {
    int nlev, nparts;
    ocsr A[ORC_MAXL], P[ORC_MAXL], R[ORC_MAXL];
    i64* agg[ORC_MAXL];
    i64* offs[ORC_MAXL];
    double omega[ORC_MAXL], rho[ORC_MAXL];
    double* ainv;
    int status;
    int nu1, nu2;  /* Jacobi sweeps before / after the coarse correction (SPEC §S6); 0 = 1 */
} ohier;

/* SPEC §S6 V(nu1, nu2): sweep counts of the pre- and post-smoothing (default 1, 1). */
void orc_set_sweeps(ohier* h, int nu1, int nu2) { h->nu1 = nu1; h->nu2 = nu2; }

void orc_free(ohier* h) {
    if (!h) return;
    for (int l = 0; l < h->nlev; ++l) {
        csr_free(&h->A[l]); csr_free(&h->P[l]); csr_free(&h->R[l]);
        free(h->agg[l]); free(h->offs[l]);
    }
    free(h->ainv); free(h);
}

/* Setup (§S4). offs: nparts+1 fine row offsets. */
ohier* orc_setup(i64 n, const i64* rp, const i64* col, const double* val, int nparts,
                 const i64* offs, double theta, int max_levels, i64 max_coarse,
                 i64 agglomerate) {
    ohier* h = calloc(1, sizeof(ohier));
    h->nparts = nparts;
    h->A[0] = csr_copy(n, n, rp, col, val);
    h->offs[0] = malloc(sizeof(i64) * (nparts + 1));
    memcpy(h->offs[0], offs, sizeof(i64) * (nparts + 1));
    int l = 0;
    if (max_levels > ORC_MAXL) max_levels = ORC_MAXL;
    for (;;) {
        ocsr* A = &h->A[l];
        h->rho[l] = gershgorin(A);
        h->omega[l] = 4.0 / (3.0 * h->rho[l]);
        /* SPEC §S7 agglomeration: from the first level l >= 1 with <= agglomerate rows on,
         * the whole level is one part (part 0 owns every row; the others are empty) */
        if (l >= 1 && agglomerate > 0 && A->nr <= agglomerate) {
            h->offs[l][0] = 0;
            for (int q = 1; q <= nparts; ++q) h->offs[l][q] = A->nr;
        }
        if (A->nr <= max_coarse || l + 1 >= max_levels) break;
        h->agg[l] = malloc(sizeof(i64) * (A->nr + 1));
        i64* coffs = malloc(sizeof(i64) * (nparts + 1));
        i64 nc = aggregate(A, theta, nparts, h->offs[l], h->agg[l], coffs);
        if (nc == 0 || nc >= A->nr) { free(h->agg[l]); h->agg[l] = NULL; free(coffs); break; }
        h->P[l] = smoothed_prolongator(A, h->agg[l], nc, h->omega[l]);
        h->R[l] = transpose(&h->P[l]);
        ocsr AP = spgemm(A, &h->P[l]);
        h->A[l + 1] = spgemm(&h->R[l], &AP);
        csr_free(&AP);
        h->offs[l + 1] = coffs;
        ++l;
    }
    h->nlev = l + 1;
    const i64 nL = h->A[l].nr;
    h->ainv = malloc(sizeof(double) * (size_t)(nL * nL + 1));
    h->status = chol_inverse(&h->A[l], h->ainv);
    return h;
}

int orc_status(const ohier* h) { return h->status; }
int orc_nlev(const ohier* h) { return h->nlev; }
double orc_omega(const ohier* h, int l) { return h->omega[l]; }
double orc_rho(const ohier* h, int l) { return h->rho[l]; }

/* which: 0 = A, 1 = P, 2 = R. info = {nrows, ncols, nnz}. */
void orc_csr_info(const ohier* h, int l, int which, i64* info) {
    const ocsr* a = which == 0 ? &h->A[l] : which == 1 ? &h->P[l] : &h->R[l];
    info[0] = a->nr; info[1] = a->nc; info[2] = a->nnz;
}
void orc_csr_get(const ohier* h, int l, int which, i64* rp, i64* col, double* val) {
    const ocsr* a = which == 0 ? &h->A[l] : which == 1 ? &h->P[l] : &h->R[l];
    memcpy(rp, a->rp, sizeof(i64) * (a->nr + 1));
    memcpy(col, a->col, sizeof(i64) * a->nnz); memcpy(val, a->val, sizeof(double) * a->nnz);
}
void orc_agg_get(const ohier* h, int l, i64* agg) { memcpy(agg, h->agg[l], sizeof(i64) * h->A[l].nr); }
void orc_offs_get(const ohier* h, int l, i64* offs) {
    memcpy(offs, h->offs[l], sizeof(i64) * (h->nparts + 1));
}
void orc_ainv_get(const ohier* h, double* out) {
    const i64 n = h->A[h->nlev - 1].nr; memcpy(out, h->ainv, sizeof(double) * (size_t)(n * n));
}

/* OpenMP threads of the row-independent loops (bench cpu_baseline: the host's affinity set) */
void orc_set_threads(int n) { if (n > 0) omp_set_num_threads(n); }
int orc_get_threads(void) { return omp_get_max_threads(); }

/* ------------------------------------------------------------------ V-cycle §S6 */

static void vcycle(const ohier* h, int l, double* x, const double* b, int zero_guess) {
    const ocsr* A = &h->A[l];
    const i64 n = A->nr;
    if (l == h->nlev - 1) {
        for (i64 i = 0; i < n; ++i) {
            double s = 0.0;
            for (i64 j = 0; j < n; ++j) { double p = h->ainv[j * n + i] * b[j]; s = s + p; }
            x[i] = s;
        }
        return;
    }
    double* t = malloc(sizeof(double) * (n + 1));
    double* r = malloc(sizeof(double) * (n + 1));
    const int nu1 = h->nu1 > 0 ? h->nu1 : 1, nu2 = h->nu2 > 0 ? h->nu2 : 1;
    for (int sweep = 0; sweep < nu1; ++sweep) {
        if (zero_guess && sweep == 0) {
            for (i64 i = 0; i < n; ++i) {
                double d = diag_of(A->rp, A->col, A->val, i, i);
                double u = b[i] - 0.0, v = h->omega[l] * u, w = v / d;
                x[i] = 0.0 + w;
            }
        } else {
            orc_jacobi(n, A->rp, A->col, A->val, x, b, h->omega[l], t);
            memcpy(x, t, sizeof(double) * n);
        }
    }
    orc_residual(n, A->rp, A->col, A->val, x, b, r);
    const i64 nc = h->A[l + 1].nr;
    double* bc = malloc(sizeof(double) * (nc + 1));
    double* xc = calloc(nc + 1, sizeof(double));
    orc_spmv(nc, h->R[l].rp, h->R[l].col, h->R[l].val, r, bc);
    vcycle(h, l + 1, xc, bc, 1);
    orc_spmv(n, h->P[l].rp, h->P[l].col, h->P[l].val, xc, t);
    for (i64 i = 0; i < n; ++i) x[i] = x[i] + t[i];
    for (int sweep = 0; sweep < nu2; ++sweep) {
        orc_jacobi(n, A->rp, A->col, A->val, x, b, h->omega[l], t);
        memcpy(x, t, sizeof(double) * n);
    }
    free(t); free(r); free(bc); free(xc);
}

/* ncycles stationary V-cycles from x (in/out); res_hist (may be NULL) gets ||b - A x||. */
void orc_solve(const ohier* h, double* x, const double* b, int ncycles, double* res_hist) {
    const ocsr* A = &h->A[0];
    double* r = res_hist ? malloc(sizeof(double) * (A->nr + 1)) : NULL;
    for (int k = 0; k < ncycles; ++k) {
        vcycle(h, 0, x, b, 0);
        if (res_hist) {
            orc_residual(A->nr, A->rp, A->col, A->val, x, b, r);
            double s = 0.0;
            for (i64 i = 0; i < A->nr; ++i) s += r[i] * r[i];
            res_hist[k] = sqrt(s);
        }
    }
    free(r);
}

/* ------------------------------------------------------------------ external hierarchy */
/* Build an oracle hierarchy from given level operators (int32 columns are widened), so the
 * oracle V-cycle can be timed on the very hierarchy the product built (bench cpu_baseline)
 * or checked against it. which: 0 = A, 1 = P, 2 = R. */
ohier* orc_hier_new(int nlev) {
    ohier* h = calloc(1, sizeof(ohier));
    h->nlev = nlev > ORC_MAXL ? ORC_MAXL : nlev;
    h->nparts = 1;
    for (int l = 0; l < h->nlev; ++l) {
        h->offs[l] = calloc(2, sizeof(i64));
    }
    return h;
}

void orc_hier_set(ohier* h, int l, int which, i64 nr, i64 nc, const i64* rp, const int32_t* col,
                  const double* val, double omega) {
    ocsr* a = which == 0 ? &h->A[l] : which == 1 ? &h->P[l] : &h->R[l];
    a->nr = nr; a->nc = nc; a->nnz = rp[nr] - rp[0];
    a->rp = malloc(sizeof(i64) * (nr + 1));
    a->col = malloc(sizeof(i64) * (a->nnz + 1));
    a->val = malloc(sizeof(double) * (a->nnz + 1));
#pragma omp parallel for schedule(static)
    for (i64 i = 0; i <= nr; ++i) a->rp[i] = rp[i] - rp[0];
#pragma omp parallel for schedule(static)
    for (i64 k = 0; k < a->nnz; ++k) { a->col[k] = col[k]; a->val[k] = val[k]; }
    if (which == 0) { h->omega[l] = omega; h->offs[l][1] = nr; }
}

void orc_hier_set_ainv(ohier* h, i64 n, const double* ainv) {
    h->ainv = malloc(sizeof(double) * (size_t)(n * n + 1));
    memcpy(h->ainv, ainv, sizeof(double) * (size_t)(n * n));
}

/* ------------------------------------------------------------------ PCG §S8 */

static double dot_seq(i64 n, const double* x, const double* y) {
    double s = 0.0;
    for (i64 i = 0; i < n; ++i) { double p = x[i] * y[i]; s = s + p; }
    return s;
}

static void axpby(i64 n, double a, const double* x, double b, double* y) {
    for (i64 i = 0; i < n; ++i) { double u = a * x[i], v = b * y[i]; y[i] = u + v; }
}

/* Returns the iteration count; hist (maxit+1, may be NULL) gets ||r_k||. */
int orc_pcg(const ohier* h, double* x, const double* b, double rtol, int maxit, double* hist) {
    const ocsr* A = &h->A[0];
    const i64 n = A->nr;
    double* r = malloc(sizeof(double) * (n + 1));
    double* z = malloc(sizeof(double) * (n + 1));
    double* p = malloc(sizeof(double) * (n + 1));
    double* q = malloc(sizeof(double) * (n + 1));
    orc_residual(n, A->rp, A->col, A->val, x, b, r);
    const double nr0 = sqrt(dot_seq(n, r, r));
    if (hist) hist[0] = nr0;
    int k = 0;
    if (nr0 > 0.0 && maxit > 0) {
        vcycle(h, 0, z, r, 1);
        memcpy(p, z, sizeof(double) * n);
        double rz = dot_seq(n, r, z);
        while (k < maxit) {
            ++k;
            orc_spmv(n, A->rp, A->col, A->val, p, q);
            const double alpha = rz / dot_seq(n, p, q);
            axpby(n, alpha, p, 1.0, x);
            axpby(n, -alpha, q, 1.0, r);
            const double nr = sqrt(dot_seq(n, r, r));
            if (hist) hist[k] = nr;
            if (nr <= rtol * nr0) break;
            vcycle(h, 0, z, r, 1);
            const double rz_new = dot_seq(n, r, z);
            const double beta = rz_new / rz;
            rz = rz_new;
            axpby(n, 1.0, z, beta, p);
        }
    }
    free(r); free(z); free(p); free(q);
    return k;
}
