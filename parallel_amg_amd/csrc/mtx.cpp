// mtx.cpp — Matrix Market reader for the "SuiteSparse Flan_1565" configuration
// (BASELINE.json configs[4]) and any other SPD matrix handed to the solver as a file.
//
// Reads `%%MatrixMarket matrix coordinate {real|integer|pattern} {general|symmetric}` and
// returns the rows [r0, r1) as host CSR (SPEC §S1: 0-based, columns ascending; duplicate
// (i, j) entries are summed in file order; symmetric files are expanded, the mirrored entry
// of (i, j, v) being (j, i, v)). Each rank of a partitioned run reads only its own rows'
// entries. The file is memory-mapped and parsed without locale-dependent stdio.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>

#include "pamg_common.h"

using pamg::fail;

namespace {

struct Mapped {
    const char* p = nullptr;
    size_t n = 0;
    int fd = -1;
    ~Mapped() {
        if (p) munmap(const_cast<char*>(p), n);
        if (fd >= 0) close(fd);
    }
};

inline const char* skip_ws(const char* s, const char* e) {
    while (s < e && (*s == ' ' || *s == '\t' || *s == '\r')) ++s;
    return s;
}

inline const char* next_line(const char* s, const char* e) {
    while (s < e && *s != '\n') ++s;
    return s < e ? s + 1 : e;
}

struct Entry {
    int64_t r, c;
    double v;
    int64_t seq;  // file order (for duplicate summation)
};

}  // namespace

// Entries per row after symmetric expansion (duplicates counted separately): the weights of
// the nnz-balanced partition (SPEC §S7). counts == NULL: only *n_global is returned.
extern "C" int pamg_mtx_row_counts(const char* path, int64_t* n_global, int64_t* counts) {
    if (!path || !n_global) return fail(PAMG_E_ARG, "mtx_row_counts: bad args");
    Mapped m;
    m.fd = open(path, O_RDONLY);
    if (m.fd < 0) return fail(PAMG_E_ARG, "mtx_row_counts: cannot open %s", path);
    struct stat st;
    if (fstat(m.fd, &st) != 0 || st.st_size == 0) return fail(PAMG_E_ARG, "mtx_row_counts: empty file");
    m.n = (size_t)st.st_size;
    void* mp = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, m.fd, 0);
    if (mp == MAP_FAILED) return fail(PAMG_E_NOMEM, "mtx_row_counts: mmap failed");
    m.p = static_cast<const char*>(mp);
    const char *s = m.p, *e = m.p + m.n;
    std::string banner(s, next_line(s, e) - s);
    for (auto& ch : banner) ch = (char)std::tolower((unsigned char)ch);
    if (banner.rfind("%%matrixmarket", 0) != 0 || banner.find("coordinate") == std::string::npos)
        return fail(PAMG_E_ARG, "mtx_row_counts: not a coordinate Matrix Market file");
    const bool symmetric = banner.find("symmetric") != std::string::npos;
    s = next_line(s, e);
    while (s < e && (*s == '%' || *s == '\n')) s = next_line(s, e);
    char* q = nullptr;
    const long long nr = std::strtoll(s, &q, 10);
    (void)std::strtoll(q, &q, 10);
    const long long nz = std::strtoll(q, &q, 10);
    if (nr <= 0) return fail(PAMG_E_ARG, "mtx_row_counts: bad size line");
    *n_global = nr;
    if (!counts) return PAMG_OK;
    std::fill(counts, counts + nr, 0);
    s = next_line(q, e);
    for (long long k = 0; k < nz && s < e; ++k) {
        s = skip_ws(s, e);
        const long long i = std::strtoll(s, &q, 10) - 1;
        const long long j = std::strtoll(q, &q, 10) - 1;
        if (i < 0 || i >= nr || j < 0 || j >= nr) return fail(PAMG_E_ARG, "mtx_row_counts: entry out of range");
        counts[i]++;
        if (symmetric && i != j) counts[j]++;
        s = next_line(q, e);
    }
    return PAMG_OK;
}

// Rows [r0, r1) of the file (sel == NULL), or the rows sel[0..nsel) in that order (output row
// k = file row sel[k]); columns keep the file's numbering.
static int read_rows(const char* path, int64_t r0, int64_t r1, const int64_t* sel, int64_t nsel,
                     int64_t* n_global, pamg_hcsr** out) {
    if (!path || !out || (sel == nullptr && nsel != 0) || nsel < 0) return fail(PAMG_E_ARG, "read_mtx: bad args");
    Mapped m;
    m.fd = open(path, O_RDONLY);
    if (m.fd < 0) return fail(PAMG_E_ARG, "read_mtx: cannot open %s", path);
    struct stat st;
    if (fstat(m.fd, &st) != 0 || st.st_size == 0) return fail(PAMG_E_ARG, "read_mtx: empty file %s", path);
    m.n = (size_t)st.st_size;
    void* mp = mmap(nullptr, m.n, PROT_READ, MAP_PRIVATE, m.fd, 0);
    if (mp == MAP_FAILED) return fail(PAMG_E_NOMEM, "read_mtx: mmap failed");
    m.p = static_cast<const char*>(mp);
    const char *s = m.p, *e = m.p + m.n;

    // banner
    std::string banner(s, next_line(s, e) - s);
    for (auto& ch : banner) ch = (char)std::tolower((unsigned char)ch);
    if (banner.rfind("%%matrixmarket", 0) != 0 || banner.find("coordinate") == std::string::npos)
        return fail(PAMG_E_ARG, "read_mtx: only '%%%%MatrixMarket matrix coordinate' files are supported");
    const bool pattern = banner.find("pattern") != std::string::npos;
    const bool symmetric = banner.find("symmetric") != std::string::npos;
    if (banner.find("complex") != std::string::npos || banner.find("hermitian") != std::string::npos ||
        banner.find("skew") != std::string::npos)
        return fail(PAMG_E_ARG, "read_mtx: complex / hermitian / skew-symmetric files are not supported");
    s = next_line(s, e);
    while (s < e && (*s == '%' || *s == '\n')) s = next_line(s, e);
    char* q = nullptr;
    const long long nr = std::strtoll(s, &q, 10);
    const long long nc = std::strtoll(q, &q, 10);
    const long long nz = std::strtoll(q, &q, 10);
    if (nr <= 0 || nc != nr || nz < 0) return fail(PAMG_E_ARG, "read_mtx: need a square matrix (got %lld x %lld)", nr, nc);
    if (nr >= INT32_MAX) return fail(PAMG_E_OVERFLOW, "read_mtx: n >= 2^31");
    // pos[file row] = output row, or -1 (selection); a range needs no table
    std::vector<int64_t> pos;
    if (sel) {
        pos.assign(nr, -1);
        for (int64_t k = 0; k < nsel; ++k) {
            if (sel[k] < 0 || sel[k] >= nr || pos[sel[k]] >= 0)
                return fail(PAMG_E_ARG, "read_mtx_rows: row %lld out of range or repeated", (long long)sel[k]);
            pos[sel[k]] = k;
        }
        r0 = 0;
        r1 = nsel;
    } else {
        if (r1 < 0) r1 = nr;
        if (r0 < 0 || r1 > nr || r0 > r1) return fail(PAMG_E_ARG, "read_mtx: bad row range");
    }
    auto out_row = [&](long long i) -> long long {
        if (sel) return pos[i];
        return (i >= r0 && i < r1) ? i : -1;
    };
    s = next_line(q, e);

    std::vector<Entry> ent;
    int64_t seq = 0;
    for (long long k = 0; k < nz; ++k) {
        s = skip_ws(s, e);
        if (s >= e) return fail(PAMG_E_ARG, "read_mtx: file ends after %lld of %lld entries", k, nz);
        const long long i = std::strtoll(s, &q, 10) - 1;
        const long long j = std::strtoll(q, &q, 10) - 1;
        const double v = pattern ? 1.0 : std::strtod(q, &q);
        if (i < 0 || i >= nr || j < 0 || j >= nc) return fail(PAMG_E_ARG, "read_mtx: entry %lld out of range", k + 1);
        const long long oi = out_row(i);
        if (oi >= 0) ent.push_back({sel ? oi + r0 : i, j, v, seq++});
        if (symmetric && i != j) {
            const long long oj = out_row(j);
            if (oj >= 0) ent.push_back({sel ? oj + r0 : j, i, v, seq++});
        }
        s = next_line(q, e);
    }
    std::sort(ent.begin(), ent.end(), [](const Entry& a, const Entry& b) {
        return a.r != b.r ? a.r < b.r : (a.c != b.c ? a.c < b.c : a.seq < b.seq);
    });
    auto M = std::make_unique<pamg_hcsr>();
    M->nr = r1 - r0;
    M->nc = nr;
    M->rp.assign(M->nr + 1, 0);
    for (size_t t = 0; t < ent.size(); ++t) {
        if (t > 0 && ent[t].r == ent[t - 1].r && ent[t].c == ent[t - 1].c) {
            M->val.back() = M->val.back() + ent[t].v;  // duplicates: summed in file order
            continue;
        }
        M->col.push_back((int32_t)ent[t].c);
        M->val.push_back(ent[t].v);
        M->rp[ent[t].r - r0 + 1]++;
    }
    for (int64_t i = 0; i < M->nr; ++i) M->rp[i + 1] += M->rp[i];
    if (n_global) *n_global = nr;
    *out = M.release();
    return PAMG_OK;
}

extern "C" int pamg_read_mtx(const char* path, int64_t r0, int64_t r1, int64_t* n_global,
                             pamg_hcsr** out) {
    return read_rows(path, r0, r1, nullptr, 0, n_global, out);
}

// The rows rows[0..nsel) of the file, in that order (a part's rows under a renumbering, e.g. a
// reverse Cuthill-McKee block: each rank stores only its own rows).
extern "C" int pamg_read_mtx_rows(const char* path, int64_t nsel, const int64_t* rows, int64_t* n_global,
                                  pamg_hcsr** out) {
    if (!rows && nsel > 0) return fail(PAMG_E_ARG, "read_mtx_rows: rows is NULL");
    static const int64_t none = 0;
    return read_rows(path, 0, 0, rows ? rows : &none, nsel, n_global, out);
}

// ------------------------------------------------------------------ graph partitioner (RCM)
// Reverse Cuthill-McKee ordering of a square matrix's graph (its pattern, symmetrised):
// the partitioner for irregularly numbered matrices. A band-limited
// numbering turns the contiguous nnz-balanced row blocks of SPEC §S7 into compact subdomains
// with small interfaces (few ghosts, few neighbours), the role METIS plays for
// PartitionedArrays users, and restores the banded x reuse the tile order relies on.
// Deterministic: start from a pseudo-peripheral node (George-Liu: repeated BFS from a
// minimum-degree node of the last level), visit neighbours by (degree, index); each further
// connected component starts from its minimum-degree unvisited node (lowest index on ties).
namespace {
struct Graph {
    std::vector<int64_t> rp;
    std::vector<int32_t> adj;
    int64_t n = 0;
    int64_t deg(int64_t v) const { return rp[v + 1] - rp[v]; }
};

Graph symmetric_graph(const pamg_hcsr& A) {
    const int64_t n = A.nr;
    std::vector<int64_t> cnt(n + 1, 0);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
            const int64_t j = A.col[k];
            if (j != i) {
                cnt[i + 1]++;
                cnt[j + 1]++;
            }
        }
    Graph g;
    g.n = n;
    g.rp.assign(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) g.rp[i + 1] = g.rp[i] + cnt[i + 1];
    g.adj.resize(g.rp[n]);
    std::vector<int64_t> pos(g.rp.begin(), g.rp.end() - 1);
    for (int64_t i = 0; i < n; ++i)
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
            const int64_t j = A.col[k];
            if (j != i) {
                g.adj[pos[i]++] = (int32_t)j;
                g.adj[pos[j]++] = (int32_t)i;
            }
        }
    // sort + dedupe each list (a symmetric pattern lists every edge twice)
    int64_t w = 0;
    std::vector<int64_t> nrp(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
        auto b = g.adj.begin() + g.rp[i], e = g.adj.begin() + g.rp[i + 1];
        std::sort(b, e);
        const int64_t start = w;
        for (auto it = b; it != e; ++it)
            if (w == start || g.adj[w - 1] != *it) g.adj[w++] = *it;
        nrp[i + 1] = w;
    }
    g.adj.resize(w);
    g.rp.swap(nrp);
    return g;
}

// BFS levels from s over unvisited-in-`mark` nodes (mark == stamp: seen); returns the last level
std::vector<int32_t> bfs_last_level(const Graph& g, int32_t s, std::vector<int32_t>& mark, int32_t stamp,
                                    int* depth) {
    std::vector<int32_t> cur{s}, nxt, last;
    mark[s] = stamp;
    *depth = 0;
    while (!cur.empty()) {
        last = cur;
        nxt.clear();
        for (int32_t v : cur)
            for (int64_t k = g.rp[v]; k < g.rp[v + 1]; ++k) {
                const int32_t u = g.adj[k];
                if (mark[u] != stamp) {
                    mark[u] = stamp;
                    nxt.push_back(u);
                }
            }
        cur.swap(nxt);
        if (!cur.empty()) ++*depth;
    }
    return last;
}
}  // namespace

extern "C" int pamg_rcm_order(const pamg_hcsr* A, int64_t* order) {
    if (!A || !order) return fail(PAMG_E_ARG, "rcm_order: NULL");
    if (A->nr != A->nc) return fail(PAMG_E_ARG, "rcm_order: matrix is %lld x %lld, not square",
                                    (long long)A->nr, (long long)A->nc);
    const int64_t n = A->nr;
    if (n >= INT32_MAX) return fail(PAMG_E_OVERFLOW, "rcm_order: %lld rows exceed int32", (long long)n);
    const Graph g = symmetric_graph(*A);
    std::vector<char> done(n, 0);
    std::vector<int32_t> mark(n, -1);
    int32_t stamp = 0;
    // nodes by (degree, index): start candidates for each component
    std::vector<int32_t> by_deg(n);
    for (int64_t i = 0; i < n; ++i) by_deg[i] = (int32_t)i;
    std::stable_sort(by_deg.begin(), by_deg.end(), [&](int32_t a, int32_t b) { return g.deg(a) < g.deg(b); });
    int64_t out = 0, next_cand = 0;
    std::vector<int32_t> nb;
    while (out < n) {
        while (done[by_deg[next_cand]]) ++next_cand;
        int32_t s = by_deg[next_cand];
        // pseudo-peripheral node: move to a minimum-degree node of the last BFS level while the
        // eccentricity grows (a handful of rounds)
        int depth = 0;
        std::vector<int32_t> last = bfs_last_level(g, s, mark, stamp++, &depth);
        for (int round = 0; round < 8; ++round) {
            int32_t t = last[0];
            for (int32_t v : last)
                if (g.deg(v) < g.deg(t) || (g.deg(v) == g.deg(t) && v < t)) t = v;
            int d2 = 0;
            std::vector<int32_t> l2 = bfs_last_level(g, t, mark, stamp++, &d2);
            if (d2 <= depth) break;
            s = t;
            depth = d2;
            last.swap(l2);
        }
        // Cuthill-McKee from s: neighbours in (degree, index) order
        const int64_t head0 = out;
        order[out++] = s;
        done[s] = 1;
        for (int64_t h = head0; h < out; ++h) {
            const int32_t v = (int32_t)order[h];
            nb.clear();
            for (int64_t k = g.rp[v]; k < g.rp[v + 1]; ++k)
                if (!done[g.adj[k]]) nb.push_back(g.adj[k]);
            std::sort(nb.begin(), nb.end(), [&](int32_t a, int32_t b) {
                return g.deg(a) != g.deg(b) ? g.deg(a) < g.deg(b) : a < b;
            });
            for (int32_t u : nb) {
                done[u] = 1;
                order[out++] = u;
            }
        }
        std::reverse(order + head0, order + out);  // reverse within the component
    }
    return PAMG_OK;
}

// Mean over the rows with entries of (largest - smallest column), the columns read through a
// permutation inv (device column of caller column j = inv[j]; NULL: identity) and the rows
// taken in any order (the span of a row does not depend on where the row goes).
static double mean_row_span(const pamg_hcsr& A, const int64_t* inv) {
    double sum = 0.0;
    int64_t rows = 0;
    // (threads over rows: 938M nonzeros at 512^3; the reduction order is fixed for a thread count,
    // and the figure only gates the auto mode and is reported)
#pragma omp parallel for schedule(static) reduction(+ : sum, rows)
    for (int64_t i = 0; i < A.nr; ++i) {
        if (A.rp[i + 1] == A.rp[i]) continue;
        int64_t lo = INT64_MAX, hi = INT64_MIN;
        for (int64_t k = A.rp[i]; k < A.rp[i + 1]; ++k) {
            const int64_t c = inv ? inv[A.col[k]] : A.col[k];
            lo = std::min(lo, c);
            hi = std::max(hi, c);
        }
        sum += (double)(hi - lo);
        ++rows;
    }
    return rows ? sum / (double)rows : 0.0;
}

// Locality order of one square level operator for the device layout (pamg_mat_upload_perm /
// pamg_hier_set_perm): a scattered numbering (an FE mesh or a random renumbering, and the
// coarse levels aggregated from it) makes every x gather of the row kernels a cache miss.
extern "C" int pamg_locality_order(const pamg_hcsr* A, int mode, int64_t* order, int* applied,
                                   double* span_before, double* span_after) {
    if (!A || !order || mode < 0 || mode > 2) return fail(PAMG_E_ARG, "locality_order: bad args");
    if (A->nr != A->nc) return fail(PAMG_E_ARG, "locality_order: matrix is %lld x %lld, not square",
                                    (long long)A->nr, (long long)A->nc);
    const int64_t n = A->nr;
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) order[i] = i;
    const double before = mean_row_span(*A, nullptr);
    if (span_before) *span_before = before;
    if (span_after) *span_after = before;
    if (applied) *applied = 0;
    // auto: only a numbering whose rows span more than n/32 columns on average is a candidate
    // (grid numberings span ~2 n^(2/3): 0.8 % of n for 512^3, 2.5 % for elastic3d 80^3)
    if (mode == 0 || (mode == 1 && (n < 4096 || before <= (double)n / 32.0))) return PAMG_OK;
    std::vector<int64_t> rcm(n), inv(n);
    const int rc = pamg_rcm_order(A, rcm.data());
    if (rc != PAMG_OK) return rc;
    for (int64_t k = 0; k < n; ++k) inv[rcm[k]] = k;
    const double after = mean_row_span(*A, inv.data());
    // auto: taken when it cuts the mean span at least 4x
    if (mode == 1 && after * 4.0 > before) return PAMG_OK;
    std::copy(rcm.begin(), rcm.end(), order);
    if (span_after) *span_after = after;
    if (applied) *applied = 1;
    return PAMG_OK;
}
