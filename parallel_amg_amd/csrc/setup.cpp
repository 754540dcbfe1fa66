// setup.cpp — host-side smoothed-aggregation setup of the product (SPEC.md §S2, §S4, §S5).
//
// These are the per-part building blocks an AMG setup written against PartitionedArrays
// (reference README.md:2) would run inside `map(parts) do part ... end`; the host layer
// (parallel_amg_amd/amg.py) sequences them and performs the ghost-row exchanges between
// them. Every floating-point result is bit-identical to oracle/pamg_oracle.c: fixed
// Gustavson accumulation order, no FMA contraction (-ffp-contract=off), OpenMP only over
// independent rows (or a deterministic per-thread split), never over a reduction order.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <memory>

#include "pamg_common.h"

using pamg::fail;

namespace {

constexpr int64_t kMaxDenseCoarse = PAMG_MAX_DENSE_COARSE;

inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// Diagonal of own row i (global row row0 + i); 0 if absent.
inline double diag_of(const pamg_hcsr& A, int64_t i, int64_t row0) {
    const int64_t g = row0 + i;
    for (int64_t a = A.rp[i]; a < A.rp[i + 1]; ++a)
        if (A.col[a] == g) return A.val[a];
    return 0.0;
}

bool valid(const pamg_hcsr* M) { return M && (int64_t)M->rp.size() == M->nr + 1; }

// Row-parallel CSR assembly: `fill(i, cols, vals)` appends row i's entries; rows are
// computed in static per-thread chunks and concatenated in row order (deterministic).
template <class RowFn>
int build_rows(int64_t nr, int64_t nc, pamg_hcsr** out, RowFn&& fill_factory) {
    auto M = std::make_unique<pamg_hcsr>();
    M->nr = nr;
    M->nc = nc;
    M->rp.assign(nr + 1, 0);
    const int nt = std::max(1, omp_get_max_threads());
    std::vector<std::vector<int32_t>> tcol(nt);
    std::vector<std::vector<double>> tval(nt);
    std::vector<int64_t> lo(nt + 1);
    for (int t = 0; t <= nt; ++t) lo[t] = nr * t / nt;
    int err = 0;
#pragma omp parallel num_threads(nt)
    {
        const int t = omp_get_thread_num();
        auto fill = fill_factory();
        auto& C = tcol[t];
        auto& V = tval[t];
        for (int64_t i = lo[t]; i < lo[t + 1]; ++i) {
            if (!fill(i, C, V)) {
#pragma omp atomic write
                err = 1;
            }
            M->rp[i + 1] = (int64_t)C.size();  // local count, fixed below
        }
    }
    if (err) return PAMG_E_SETUP;
    std::vector<int64_t> base(nt + 1, 0);
    for (int t = 0; t < nt; ++t) base[t + 1] = base[t] + (int64_t)tcol[t].size();
    M->col.resize(base[nt]);
    M->val.resize(base[nt]);
#pragma omp parallel for num_threads(nt) schedule(static, 1)
    for (int t = 0; t < nt; ++t) {
        for (int64_t i = lo[t]; i < lo[t + 1]; ++i) M->rp[i + 1] += base[t];
        if (!tcol[t].empty()) {
            std::memcpy(M->col.data() + base[t], tcol[t].data(), tcol[t].size() * 4);
            std::memcpy(M->val.data() + base[t], tval[t].data(), tval[t].size() * 8);
        }
    }
    M->rp[0] = 0;
    *out = M.release();
    return PAMG_OK;
}

// SPEC §S2 elastic3d: 3 unknowns per node (row 3*node + d), A = L27 (x) (4I - J); the
// Flan_1565 stand-in (BASELINE.json configs[4]: ~73-81 nonzeros per row, SPD).
int gen_elastic(int64_t nx, int64_t ny, int64_t nz, int64_t r0, int64_t r1, pamg_hcsr** out) {
    const int64_t n = 3 * nx * ny * nz;
    if (r0 < 0 || r1 > n || r0 > r1) return fail(PAMG_E_ARG, "gen_grid: bad row range");
    if (n >= (int64_t)INT32_MAX) return fail(PAMG_E_OVERFLOW, "gen_grid: n >= 2^31");
    try {
        return build_rows(r1 - r0, n, out, [&]() {
            return [&](int64_t i, std::vector<int32_t>& C, std::vector<double>& V) {
                const int64_t r = r0 + i, node = r / 3, d = r % 3;
                const int64_t x = node % nx, y = (node / nx) % ny, z = node / (nx * ny);
                for (int dz = -1; dz <= 1; ++dz)
                    for (int dy = -1; dy <= 1; ++dy)
                        for (int dx = -1; dx <= 1; ++dx) {
                            const int64_t X = x + dx, Y = y + dy, Z = z + dz;
                            if (X < 0 || Y < 0 || Z < 0 || X >= nx || Y >= ny || Z >= nz) continue;
                            const int64_t m = X + nx * (Y + ny * Z);
                            const double l = (m == node) ? 26.0 : -1.0;
                            for (int e = 0; e < 3; ++e) {
                                C.push_back((int32_t)(3 * m + e));
                                V.push_back(l * ((e == d) ? 3.0 : -1.0));
                            }
                        }
                return true;
            };
        });
    } catch (...) {
        return fail(PAMG_E_NOMEM, "gen_grid: out of host memory");
    }
}

}  // namespace

extern "C" {

int pamg_hcsr_create(int64_t nrows, int64_t ncols, int64_t nnz, pamg_hcsr** out) {
    if (!out || nrows < 0 || ncols < 0 || nnz < 0) return fail(PAMG_E_ARG, "hcsr_create: bad args");
    try {
        auto M = new pamg_hcsr;
        M->nr = nrows;
        M->nc = ncols;
        M->rp.assign(nrows + 1, 0);
        M->col.assign(nnz, 0);
        M->val.assign(nnz, 0.0);
        *out = M;
    } catch (...) {
        return fail(PAMG_E_NOMEM, "hcsr_create: out of host memory");
    }
    return PAMG_OK;
}

int pamg_hcsr_destroy(pamg_hcsr* M) {
    delete M;
    return PAMG_OK;
}

int pamg_hcsr_info(const pamg_hcsr* M, int64_t* nrows, int64_t* ncols, int64_t* nnz) {
    if (!valid(M)) return fail(PAMG_E_ARG, "hcsr_info: invalid handle");
    if (nrows) *nrows = M->nr;
    if (ncols) *ncols = M->nc;
    if (nnz) *nnz = (int64_t)M->col.size();
    return PAMG_OK;
}

int pamg_hcsr_data(pamg_hcsr* M, int64_t** rowptr, int32_t** col, double** val) {
    if (!valid(M)) return fail(PAMG_E_ARG, "hcsr_data: invalid handle");
    if (rowptr) *rowptr = M->rp.data();
    if (col) *col = M->col.data();
    if (val) *val = M->val.data();
    return PAMG_OK;
}

// SPEC §S2. Row entries in ascending column order: z-, y-, x-, diag, x+, y+, z+.
int pamg_gen_grid(int kind, int64_t nx, int64_t ny, int64_t nz, double eps, int64_t r0,
                  int64_t r1, pamg_hcsr** out) {
    if (!out || nx < 1 || ny < 1 || nz < 1 || kind < 0 || kind > 3)
        return fail(PAMG_E_ARG, "gen_grid: bad args");
    if (kind == 3) return gen_elastic(nx, ny, nz, r0, r1, out);
    const int64_t n = nx * ny * nz;
    if (r0 < 0 || r1 > n || r0 > r1) return fail(PAMG_E_ARG, "gen_grid: bad row range");
    if (n >= (int64_t)INT32_MAX) return fail(PAMG_E_OVERFLOW, "gen_grid: n >= 2^31");
    double d = 4.0, vxy = -1.0, vz = -1.0;
    if (kind == 1) d = 6.0;
    if (kind == 2) { d = 4.0 + 2.0 * eps; vz = -eps; }
    const int64_t pxy = nx * ny, m = r1 - r0;
    try {
        // two passes straight into the final arrays: closed-form row lengths, then fill
        auto M = std::make_unique<pamg_hcsr>();
        M->nr = m;
        M->nc = n;
        M->rp.assign(m + 1, 0);
        auto row_len = [&](int64_t r) {
            const int64_t x = r % nx, y = (r / nx) % ny, z = r / pxy;
            return (int64_t)1 + (z > 0) + (y > 0) + (x > 0) + (x < nx - 1) + (y < ny - 1) + (z < nz - 1);
        };
        const int nt = std::max(1, omp_get_max_threads());
        std::vector<int64_t> part(nt + 1, 0);
#pragma omp parallel num_threads(nt)
        {
            const int t = omp_get_thread_num();
            const int64_t lo = m * t / nt, hi = m * (t + 1) / nt;
            int64_t s = 0;
            for (int64_t i = lo; i < hi; ++i) {
                s += row_len(r0 + i);
                M->rp[i + 1] = s;
            }
            part[t + 1] = s;
#pragma omp barrier
#pragma omp single
            for (int u = 0; u < nt; ++u) part[u + 1] += part[u];
            for (int64_t i = lo; i < hi; ++i) M->rp[i + 1] += part[t];
        }
        M->col.resize(M->rp[m]);
        M->val.resize(M->rp[m]);
#pragma omp parallel for schedule(static)
        for (int64_t i = 0; i < m; ++i) {
            const int64_t r = r0 + i, x = r % nx, y = (r / nx) % ny, z = r / pxy;
            int64_t k = M->rp[i];
            int32_t* C = M->col.data();
            double* V = M->val.data();
            if (z > 0) { C[k] = (int32_t)(r - pxy); V[k++] = vz; }
            if (y > 0) { C[k] = (int32_t)(r - nx); V[k++] = vxy; }
            if (x > 0) { C[k] = (int32_t)(r - 1); V[k++] = vxy; }
            C[k] = (int32_t)r; V[k++] = d;
            if (x < nx - 1) { C[k] = (int32_t)(r + 1); V[k++] = vxy; }
            if (y < ny - 1) { C[k] = (int32_t)(r + nx); V[k++] = vxy; }
            if (z < nz - 1) { C[k] = (int32_t)(r + pxy); V[k++] = vz; }
        }
        *out = M.release();
        return PAMG_OK;
    } catch (...) {
        return fail(PAMG_E_NOMEM, "gen_grid: out of host memory");
    }
}

int pamg_gen_xstar(int64_t i0, int64_t n, uint64_t seed, double* out) {
    if (!out || n < 0) return fail(PAMG_E_ARG, "gen_xstar: bad args");
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < n; ++k) {
        const uint64_t z = mix64(seed + (uint64_t)(i0 + k + 1) * 0x9E3779B97F4A7C15ULL);
        const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
        out[k] = 2.0 * u - 1.0;
    }
    return PAMG_OK;
}

// SPEC §S4.1 (local part; the host layer takes the max over parts).
int pamg_setup_gershgorin(const pamg_hcsr* A, int64_t row0, double* rho) {
    if (!valid(A) || !rho) return fail(PAMG_E_ARG, "gershgorin: bad args");
    double best = 0.0;
    int missing = 0;
#pragma omp parallel for schedule(static) reduction(max : best) reduction(+ : missing)
    for (int64_t i = 0; i < A->nr; ++i) {
        double s = 0.0, d = 0.0;
        const int64_t g = row0 + i;
        for (int64_t a = A->rp[i]; a < A->rp[i + 1]; ++a) {
            s = s + std::fabs(A->val[a]);
            if (A->col[a] == g) d = A->val[a];
        }
        if (d == 0.0) { ++missing; continue; }
        const double q = s / std::fabs(d);
        if (q > best) best = q;
    }
    if (missing) return fail(PAMG_E_SETUP, "gershgorin: %d rows without a diagonal", missing);
    *rho = best;
    return PAMG_OK;
}

// SPEC §S4.2-3: decoupled standard aggregation over own columns [row0, row0 + nr).
int pamg_setup_aggregate(const pamg_hcsr* A, int64_t row0, double theta, int32_t* agg,
                         int64_t* n_agg) {
    if (!valid(A) || (!agg && A->nr > 0) || !n_agg) return fail(PAMG_E_ARG, "aggregate: bad args");
    const int64_t n = A->nr, hi = row0 + n;
    std::vector<double> dg(n);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) dg[i] = diag_of(*A, i, row0);
    std::vector<uint8_t> strong(A->col.size(), 0);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
        const int64_t g = row0 + i;
        for (int64_t a = A->rp[i]; a < A->rp[i + 1]; ++a) {
            const int64_t j = A->col[a];
            if (j == g || j < row0 || j >= hi) continue;
            const double t = theta * std::sqrt(std::fabs(dg[i] * dg[j - row0]));
            strong[a] = std::fabs(A->val[a]) >= t;
        }
    }
    constexpr int32_t UN = -2, ISO = -3;
    std::vector<uint8_t> p1(n, 0);
    for (int64_t i = 0; i < n; ++i) agg[i] = UN;
    int32_t na = 0;
    for (int64_t i = 0; i < n; ++i) {  // pass 1
        if (agg[i] != UN) continue;
        bool has_nb = false, has_assigned = false;
        for (int64_t a = A->rp[i]; a < A->rp[i + 1]; ++a)
            if (strong[a]) {
                has_nb = true;
                if (agg[A->col[a] - row0] != UN) { has_assigned = true; break; }
            }
        if (!has_nb) { agg[i] = ISO; continue; }
        if (has_assigned) continue;
        agg[i] = na;
        p1[i] = 1;
        for (int64_t a = A->rp[i]; a < A->rp[i + 1]; ++a)
            if (strong[a]) {
                const int64_t j = A->col[a] - row0;
                agg[j] = na;
                p1[j] = 1;
            }
        ++na;
    }
    for (int64_t i = 0; i < n; ++i) {  // pass 2
        if (agg[i] != UN) continue;
        for (int64_t a = A->rp[i]; a < A->rp[i + 1]; ++a)
            if (strong[a] && p1[A->col[a] - row0]) { agg[i] = agg[A->col[a] - row0]; break; }
    }
    for (int64_t i = 0; i < n; ++i) {  // pass 3
        if (agg[i] != UN) continue;
        agg[i] = na;
        for (int64_t a = A->rp[i]; a < A->rp[i + 1]; ++a)
            if (strong[a] && agg[A->col[a] - row0] == UN) agg[A->col[a] - row0] = na;
        ++na;
    }
    for (int64_t i = 0; i < n; ++i)
        if (agg[i] == ISO) agg[i] = -1;
    *n_agg = na;
    return PAMG_OK;
}

// SPEC §S4.4.
int pamg_setup_tentative(int64_t n, const int32_t* agg, int64_t n_agg, int64_t coarse0,
                         int64_t ncols_global, pamg_hcsr** out) {
    if ((!agg && n > 0) || !out || n < 0 || n_agg < 0) return fail(PAMG_E_ARG, "tentative: bad args");
    std::vector<int64_t> cnt(n_agg, 0);
    for (int64_t i = 0; i < n; ++i)
        if (agg[i] >= 0) {
            if (agg[i] >= n_agg) return fail(PAMG_E_ARG, "tentative: aggregate id out of range");
            cnt[agg[i]]++;
        }
    auto T = std::make_unique<pamg_hcsr>();
    T->nr = n;
    T->nc = ncols_global;
    T->rp.resize(n + 1);
    T->rp[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (agg[i] >= 0) {
            T->col.push_back((int32_t)(coarse0 + agg[i]));
            T->val.push_back(1.0 / std::sqrt((double)cnt[agg[i]]));
        }
        T->rp[i + 1] = (int64_t)T->col.size();
    }
    *out = T.release();
    return PAMG_OK;
}

// SPEC §S4.5: Gustavson C = X * Y with Y = own rows [y0, y0+Yown.nr) + ghost rows.
int pamg_setup_spgemm(const pamg_hcsr* X, int64_t y0, const pamg_hcsr* Yown,
                      const int64_t* ghost_ids, int64_t n_ghost, const pamg_hcsr* Yghost,
                      pamg_hcsr** out) {
    if (!valid(X) || !valid(Yown) || !out) return fail(PAMG_E_ARG, "spgemm: bad args");
    if (n_ghost > 0 && (!ghost_ids || !valid(Yghost) || Yghost->nr != n_ghost))
        return fail(PAMG_E_ARG, "spgemm: ghost rows missing");
    const int64_t nc = Yown->nc;
    if (nc >= (int64_t)INT32_MAX) return fail(PAMG_E_OVERFLOW, "spgemm: ncols >= 2^31");
    const int64_t yhi = y0 + Yown->nr;
    int missing = 0;
    try {
        int rc = build_rows(X->nr, nc, out, [&]() {
            // per-thread dense accumulator over the output columns
            auto pos = std::make_shared<std::vector<int32_t>>(nc, -1);
            auto acc = std::make_shared<std::vector<double>>();
            auto cols = std::make_shared<std::vector<int32_t>>();
            return [&, pos, acc, cols](int64_t i, std::vector<int32_t>& C, std::vector<double>& V) {
                auto& P = *pos;
                auto& S = *acc;
                auto& L = *cols;
                L.clear();
                S.clear();
                for (int64_t a = X->rp[i]; a < X->rp[i + 1]; ++a) {
                    const int64_t k = X->col[a];
                    const double xv = X->val[a];
                    const pamg_hcsr* Y;
                    int64_t r;
                    if (k >= y0 && k < yhi) {
                        Y = Yown;
                        r = k - y0;
                    } else {
                        const int64_t* e = ghost_ids + n_ghost;
                        const int64_t* f = std::lower_bound(ghost_ids, e, k);
                        if (f == e || *f != k) {
#pragma omp atomic
                            missing++;
                            return false;
                        }
                        Y = Yghost;
                        r = f - ghost_ids;
                    }
                    for (int64_t b = Y->rp[r]; b < Y->rp[r + 1]; ++b) {
                        const int32_t j = Y->col[b];
                        const double p = xv * Y->val[b];
                        if (P[j] < 0) {
                            P[j] = (int32_t)L.size();
                            L.push_back(j);
                            S.push_back(p);
                        } else {
                            S[P[j]] = S[P[j]] + p;
                        }
                    }
                }
                // output in column order; P[j] still indexes column j's accumulator
                const size_t m = L.size();
                if (m <= 32) {
                    for (size_t u = 1; u < m; ++u) {
                        const int32_t v = L[u];
                        size_t w = u;
                        for (; w > 0 && L[w - 1] > v; --w) L[w] = L[w - 1];
                        L[w] = v;
                    }
                } else {
                    std::sort(L.begin(), L.end());
                }
                for (int32_t j : L) {
                    C.push_back(j);
                    V.push_back(S[P[j]]);
                    P[j] = -1;
                }
                return true;
            };
        });
        if (rc != PAMG_OK)
            return fail(rc, "spgemm: %d column ids of X reference rows that are neither own nor ghost",
                        missing);
        return PAMG_OK;
    } catch (...) {
        return fail(PAMG_E_NOMEM, "spgemm: out of host memory");
    }
}

// SPEC §S4.6 (in place on AT's values).
int pamg_setup_smooth(const pamg_hcsr* A, int64_t row0, const pamg_hcsr* T, pamg_hcsr* AT,
                      double omega) {
    if (!valid(A) || !valid(T) || !valid(AT) || A->nr != T->nr || A->nr != AT->nr)
        return fail(PAMG_E_ARG, "smooth: bad args");
    int missing = 0;
#pragma omp parallel for schedule(static) reduction(+ : missing)
    for (int64_t i = 0; i < A->nr; ++i) {
        const double d = diag_of(*A, i, row0);
        if (d == 0.0) { ++missing; continue; }
        const double q = omega / d;
        const bool has_t = T->rp[i + 1] > T->rp[i];
        const int64_t ti = has_t ? T->col[T->rp[i]] : -1;
        const double tv = has_t ? T->val[T->rp[i]] : 0.0;
        for (int64_t a = AT->rp[i]; a < AT->rp[i + 1]; ++a) {
            const double t = (AT->col[a] == ti) ? tv : 0.0;
            AT->val[a] = t - q * AT->val[a];
        }
    }
    if (missing) return fail(PAMG_E_SETUP, "smooth: %d rows without a diagonal", missing);
    return PAMG_OK;
}

// SPEC §S4.7, restricted to coarse columns [c0, c1).
int pamg_setup_transpose(const pamg_hcsr* P, int64_t row0, int64_t c0, int64_t c1,
                         pamg_hcsr** out) {
    if (!valid(P) || !out || c1 < c0) return fail(PAMG_E_ARG, "transpose: bad args");
    auto R = std::make_unique<pamg_hcsr>();
    const int64_t m = c1 - c0;
    R->nr = m;
    R->nc = -1;  // global fine columns; caller knows the global size
    R->rp.assign(m + 1, 0);
    for (int64_t a = 0; a < (int64_t)P->col.size(); ++a) {
        const int64_t c = P->col[a];
        if (c >= c0 && c < c1) R->rp[c - c0 + 1]++;
    }
    for (int64_t c = 0; c < m; ++c) R->rp[c + 1] += R->rp[c];
    R->col.resize(R->rp[m]);
    R->val.resize(R->rp[m]);
    std::vector<int64_t> pos(R->rp.begin(), R->rp.end() - 1);
    for (int64_t i = 0; i < P->nr; ++i)
        for (int64_t a = P->rp[i]; a < P->rp[i + 1]; ++a) {
            const int64_t c = P->col[a];
            if (c < c0 || c >= c1) continue;
            const int64_t p = pos[c - c0]++;
            R->col[p] = (int32_t)(row0 + i);
            R->val[p] = P->val[a];
        }
    R->nc = row0 + P->nr;
    *out = R.release();
    return PAMG_OK;
}

int pamg_setup_hstack_rows(int k, const pamg_hcsr* const* pieces, pamg_hcsr** out) {
    if (k < 1 || !pieces || !out) return fail(PAMG_E_ARG, "hstack_rows: bad args");
    const int64_t nr = pieces[0]->nr;
    int64_t nc = 0;
    for (int p = 0; p < k; ++p) {
        if (!valid(pieces[p]) || pieces[p]->nr != nr)
            return fail(PAMG_E_ARG, "hstack_rows: pieces must have equal row counts");
        nc = std::max(nc, pieces[p]->nc);
    }
    auto M = std::make_unique<pamg_hcsr>();
    M->nr = nr;
    M->nc = nc;
    M->rp.assign(nr + 1, 0);
    for (int64_t i = 0; i < nr; ++i) {
        int64_t c = 0;
        for (int p = 0; p < k; ++p) c += pieces[p]->rp[i + 1] - pieces[p]->rp[i];
        M->rp[i + 1] = M->rp[i] + c;
    }
    M->col.resize(M->rp[nr]);
    M->val.resize(M->rp[nr]);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < nr; ++i) {
        int64_t o = M->rp[i];
        for (int p = 0; p < k; ++p) {
            const auto* Q = pieces[p];
            for (int64_t a = Q->rp[i]; a < Q->rp[i + 1]; ++a, ++o) {
                M->col[o] = Q->col[a];
                M->val[o] = Q->val[a];
            }
        }
    }
    *out = M.release();
    return PAMG_OK;
}

// SPEC §S5.
int pamg_setup_cholinv(const pamg_hcsr* A, double* ainv) {
    if (!valid(A) || !ainv || A->nc != A->nr) return fail(PAMG_E_ARG, "cholinv: bad args");
    const int64_t n = A->nr;
    // the dense coarsest solve holds n^2 doubles twice (and the caller's inverse): refuse sizes
    // no coarsest level should have (SPEC §S5: max_coarse <= 2048) instead of exhausting memory
    if (n > kMaxDenseCoarse)
        return fail(PAMG_E_ARG, "cholinv: coarsest level of %lld rows exceeds the dense-solve limit %lld "
                    "(raise max_levels or lower max_coarse)", (long long)n, (long long)kMaxDenseCoarse);
    std::vector<double> Ad((size_t)(n * n), 0.0), L((size_t)(n * n), 0.0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t a = A->rp[i]; a < A->rp[i + 1]; ++a) Ad[i * n + A->col[a]] = A->val[a];
    for (int64_t j = 0; j < n; ++j) {
        double d = Ad[j * n + j];
        for (int64_t k = 0; k < j; ++k) d = d - L[j * n + k] * L[j * n + k];
        if (!(d > 0.0)) return fail(PAMG_E_SETUP, "cholinv: matrix not SPD (pivot %lld)", (long long)j);
        L[j * n + j] = std::sqrt(d);
        const double ljj = L[j * n + j];
#pragma omp parallel for schedule(static)
        for (int64_t i = j + 1; i < n; ++i) {
            double s = Ad[i * n + j];
            for (int64_t k = 0; k < j; ++k) s = s - L[i * n + k] * L[j * n + k];
            L[i * n + j] = s / ljj;
        }
    }
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t c = 0; c < n; ++c) {
        std::vector<double> y(n);
        for (int64_t i = 0; i < n; ++i) {
            double s = (i == c) ? 1.0 : 0.0;
            for (int64_t k = 0; k < i; ++k) s = s - L[i * n + k] * y[k];
            y[i] = s / L[i * n + i];
        }
        double* z = ainv + c * n;
        for (int64_t i = n - 1; i >= 0; --i) {
            double s = y[i];
            for (int64_t k = n - 1; k > i; --k) s = s - L[k * n + i] * z[k];
            z[i] = s / L[i * n + i];
        }
    }
    return PAMG_OK;
}

}  // extern "C"
