"""ctypes front end of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg may import
this module; the product (``parallel_amg_amd``) never does. It restates SPEC.md (§S1-§S7);
the C source is ``oracle/pamg_oracle.c``. Parity with the Julia reference is unpinned
(the reference, /root/reference/README.md:1-2, holds no code) — see DESIGN.md §Oracle.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libpamg_oracle.so")
SEED = 20240807
KINDS = {"poisson2d": 0, "poisson3d": 1, "aniso3d": 2, "elastic3d": 3}

_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        i64, dbl, vp = C.c_int64, C.c_double, C.c_void_p
        L.orc_xstar.argtypes = [i64, i64, C.c_uint64, _f64p]
        L.orc_gen_rows.restype = i64
        L.orc_gen_rows.argtypes = [C.c_int, i64, i64, i64, dbl, i64, i64, vp, vp, vp]
        for f in ("orc_spmv",):
            getattr(L, f).argtypes = [i64, _i64p, _i64p, _f64p, _f64p, _f64p]
        L.orc_residual.argtypes = [i64, _i64p, _i64p, _f64p, _f64p, _f64p, _f64p]
        L.orc_jacobi.argtypes = [i64, _i64p, _i64p, _f64p, _f64p, _f64p, dbl, _f64p]
        L.orc_setup.restype = vp
        L.orc_setup.argtypes = [i64, _i64p, _i64p, _f64p, C.c_int, _i64p, dbl, C.c_int, i64, i64]
        L.orc_free.argtypes = [vp]
        L.orc_set_threads.argtypes = [C.c_int]
        L.orc_get_threads.restype = C.c_int
        L.orc_set_sweeps.argtypes = [vp, C.c_int, C.c_int]
        L.orc_status.argtypes = [vp]
        L.orc_nlev.argtypes = [vp]
        L.orc_omega.restype = dbl
        L.orc_omega.argtypes = [vp, C.c_int]
        L.orc_rho.restype = dbl
        L.orc_rho.argtypes = [vp, C.c_int]
        L.orc_csr_info.argtypes = [vp, C.c_int, C.c_int, _i64p]
        L.orc_csr_get.argtypes = [vp, C.c_int, C.c_int, _i64p, _i64p, _f64p]
        L.orc_agg_get.argtypes = [vp, C.c_int, _i64p]
        L.orc_offs_get.argtypes = [vp, C.c_int, _i64p]
        L.orc_ainv_get.argtypes = [vp, _f64p]
        L.orc_solve.argtypes = [vp, _f64p, _f64p, C.c_int, vp]
        L.orc_hier_new.restype = vp
        L.orc_hier_new.argtypes = [C.c_int]
        L.orc_hier_set.argtypes = [vp, C.c_int, C.c_int, i64, i64, vp, vp, vp, dbl]
        L.orc_hier_set_ainv.argtypes = [vp, i64, _f64p]
        L.orc_pcg.restype = C.c_int
        L.orc_pcg.argtypes = [vp, _f64p, _f64p, dbl, C.c_int, vp]
        _lib = L
    return _lib


@dataclass
class CSR:
    """Host CSR with int64 indices (SPEC §S1)."""
    rowptr: np.ndarray
    col: np.ndarray
    val: np.ndarray
    ncols: int

    @property
    def nrows(self):
        return len(self.rowptr) - 1

    @property
    def nnz(self):
        return int(self.rowptr[-1])

    def to_scipy(self):
        import scipy.sparse as sp
        return sp.csr_matrix((self.val, self.col, self.rowptr), shape=(self.nrows, self.ncols))


def grid_shape(kind: str, n: int):
    return (n, n, 1) if kind == "poisson2d" else (n, n, n)


def generate(kind: str, nx: int, ny: int, nz: int, eps: float = 1e-3, r0: int = 0, r1=None) -> CSR:
    """Rows [r0, r1) of the SPEC §S2 grid operator (global column ids)."""
    L = lib()
    n = nx * ny * nz * (3 if kind == "elastic3d" else 1)
    r1 = n if r1 is None else r1
    k = KINDS[kind]
    nnz = L.orc_gen_rows(k, nx, ny, nz, eps, r0, r1, None, None, None)
    rp = np.empty(r1 - r0 + 1, np.int64)
    col = np.empty(nnz, np.int64)
    val = np.empty(nnz, np.float64)
    L.orc_gen_rows(k, nx, ny, nz, eps, r0, r1, rp.ctypes.data, col.ctypes.data, val.ctypes.data)
    return CSR(rp, col, val, n)


def xstar(n: int, i0: int = 0, seed: int = SEED) -> np.ndarray:
    out = np.empty(n, np.float64)
    lib().orc_xstar(i0, n, seed, out)
    return out


def spmv(A: CSR, x: np.ndarray) -> np.ndarray:
    y = np.empty(A.nrows, np.float64)
    lib().orc_spmv(A.nrows, A.rowptr, A.col, A.val, np.ascontiguousarray(x, np.float64), y)
    return y


def residual(A: CSR, x, b):
    r = np.empty(A.nrows, np.float64)
    lib().orc_residual(A.nrows, A.rowptr, A.col, A.val, np.ascontiguousarray(x, np.float64),
                       np.ascontiguousarray(b, np.float64), r)
    return r


def jacobi(A: CSR, x, b, omega: float):
    xn = np.empty(A.nrows, np.float64)
    lib().orc_jacobi(A.nrows, A.rowptr, A.col, A.val, np.ascontiguousarray(x, np.float64),
                     np.ascontiguousarray(b, np.float64), omega, xn)
    return xn


def uniform_offsets(n: int, nparts: int) -> np.ndarray:
    """SPEC §S7: part p owns [floor(p n / P), floor((p+1) n / P))."""
    return np.array([(p * n) // nparts for p in range(nparts + 1)], np.int64)


@dataclass
class Hierarchy:
    A: list = field(default_factory=list)
    P: list = field(default_factory=list)
    R: list = field(default_factory=list)
    agg: list = field(default_factory=list)
    offsets: list = field(default_factory=list)
    omega: list = field(default_factory=list)
    rho: list = field(default_factory=list)
    ainv: np.ndarray = None
    _h: int = 0
    _nlev: int = 0

    @property
    def nlevels(self):
        return self._nlev or len(self.A)

    def csr(self, l: int, which: int) -> CSR:
        """Level l's A (which 0), P (1) or R (2), copied out of the C hierarchy."""
        info = np.zeros(3, np.int64)
        lib().orc_csr_info(self._h, l, which, info)
        nr, nc, nnz = (int(v) for v in info)
        rp = np.empty(nr + 1, np.int64); col = np.empty(nnz, np.int64); val = np.empty(nnz)
        lib().orc_csr_get(self._h, l, which, rp, col, val)
        return CSR(rp, col, val, nc)

    def aggregates(self, l: int) -> np.ndarray:
        """Level l's aggregate ids (global coarse ids, -1 isolated)."""
        info = np.zeros(3, np.int64)
        lib().orc_csr_info(self._h, l, 0, info)
        a = np.empty(int(info[0]), np.int64)
        lib().orc_agg_get(self._h, l, a)
        return a

    def set_sweeps(self, nu1: int, nu2: int):
        """SPEC §S6 V(nu1, nu2) (default V(1, 1))."""
        lib().orc_set_sweeps(self._h, int(nu1), int(nu2))

    def solve(self, b, ncycles, x0=None, res_hist=False):
        x = np.zeros(len(b)) if x0 is None else np.array(x0, np.float64, copy=True)
        hist = np.zeros(ncycles) if res_hist else None
        lib().orc_solve(self._h, x, np.ascontiguousarray(b, np.float64), ncycles,
                        hist.ctypes.data if res_hist else None)
        return (x, hist) if res_hist else x

    def pcg(self, b, rtol=1e-8, maxit=100, x0=None):
        """SPEC §S8 PCG with one V-cycle as preconditioner: (x, iterations, history)."""
        x = np.zeros(len(b)) if x0 is None else np.array(x0, np.float64, copy=True)
        hist = np.zeros(maxit + 1)
        k = lib().orc_pcg(self._h, x, np.ascontiguousarray(b, np.float64), rtol, maxit, hist.ctypes.data)
        return x, k, hist[:k + 1]

    def __del__(self):
        if self._h and _lib is not None:
            _lib.orc_free(self._h)
            self._h = 0


def setup(A: CSR, nparts: int = 1, theta: float = 0.02, max_levels: int = 20,
          max_coarse: int = 1000, offsets=None, agglomerate: int = 32768, fetch: bool = True) -> Hierarchy:
    """SPEC §S4-§S5 smoothed-aggregation setup (global view, decoupled by parts; `offsets`
    overrides the uniform partition of SPEC §S7; levels >= 1 with <= `agglomerate` rows are
    one part, SPEC §S7 agglomeration — 0 disables it). fetch=False leaves the level operators
    in the C hierarchy (H.A / H.P / H.R / H.agg stay empty; ``H.csr(l, which)`` and
    ``H.aggregates(l)`` copy one out on demand — for 512^3, where all of them at once would be
    ~50 GB of host memory)."""
    L = lib()
    offs = uniform_offsets(A.nrows, nparts) if offsets is None else np.asarray(offsets, np.int64)
    nparts = len(offs) - 1
    h = L.orc_setup(A.nrows, A.rowptr, A.col, A.val, nparts, offs, theta, max_levels, max_coarse,
                    agglomerate)
    H = Hierarchy(_h=h)
    if L.orc_status(h) != 0:
        raise RuntimeError("oracle setup: coarse Cholesky failed")
    nlev = L.orc_nlev(h)
    info = np.zeros(3, np.int64)
    get = H.csr
    H._nlev = nlev
    for l in range(nlev):
        H.omega.append(L.orc_omega(h, l))
        H.rho.append(L.orc_rho(h, l))
        o = np.empty(nparts + 1, np.int64)
        L.orc_offs_get(h, l, o)
        H.offsets.append(o)
        if fetch:
            H.A.append(get(l, 0))
            if l < nlev - 1:
                H.P.append(get(l, 1))
                H.R.append(get(l, 2))
                H.agg.append(H.aggregates(l))
    L.orc_csr_info(h, nlev - 1, 0, info)
    nL = int(info[0])
    H.ainv = np.empty(nL * nL)
    L.orc_ainv_get(h, H.ainv)
    H.ainv = H.ainv.reshape(nL, nL).T.copy()  # stored column-major -> row-major matrix
    return H


def hierarchy_from_levels(A, P, R, omega, ainv_colmajor) -> Hierarchy:
    """Oracle hierarchy holding the given level operators (objects with rowptr (int64),
    col (int32) and val arrays, e.g. the product's host CSR) — no setup is run. Used to time
    the oracle V-cycle on the product's own hierarchy (bench cpu_baseline)."""
    L = lib()
    h = L.orc_hier_new(len(A))
    H = Hierarchy(_h=h, _nlev=len(A))
    for l, M in enumerate(A):
        for which, X in ((0, M), (1, P[l] if l < len(P) else None), (2, R[l] if l < len(R) else None)):
            if X is None:
                continue
            col = np.ascontiguousarray(X.col, np.int32)
            L.orc_hier_set(h, l, which, X.nrows, X.ncols, X.rowptr.ctypes.data, col.ctypes.data,
                           X.val.ctypes.data, float(omega[l]) if which == 0 else 0.0)
    L.orc_hier_set_ainv(h, int(round(len(ainv_colmajor) ** 0.5)), np.ascontiguousarray(ainv_colmajor))
    return H


# ---------------------------------------------------------------------------------------------
# A second, independent restatement of SPEC §S4.2-3 (strength + standard aggregation), written
# from the SPEC text rather than from pamg_oracle.c: the strength pattern is a scipy matrix built
# with whole-array numpy operations, and the three passes are set operations on per-row
# neighbour lists. It pins the two C implementations (pamg_oracle.c aggregate(), the product's
# csrc/setup.cpp pamg_setup_aggregate), which share one formulation.

def strength_matrix(A, theta: float = 0.02, offsets=None):
    """SPEC §S4.2 as a scipy CSR pattern: entry (i, j) present iff j != i, j is owned by i's
    part, and |a_ij| >= theta * sqrt(|a_ii * a_jj|) (product, then sqrt, then x theta — the
    SPEC's rounding order, evaluated elementwise by numpy in IEEE double). The entries keep A's
    storage order within each row (pass 2 reads "the first strong neighbour in storage order")."""
    import scipy.sparse as sp
    rp = np.asarray(A.rowptr, np.int64)
    col = np.asarray(A.col, np.int64)
    val = np.asarray(A.val, np.float64)
    n = len(rp) - 1
    offs = np.array([0, n], np.int64) if offsets is None else np.asarray(offsets, np.int64)
    row = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
    on_diag = col == row
    d = np.zeros(n)
    d[row[on_diag]] = val[on_diag]            # the stored diagonal (0 if absent)
    part_of = np.searchsorted(offs, np.arange(n), side="right") - 1
    ok = ~on_diag & (col >= 0) & (col < n)
    same = np.zeros(len(col), bool)
    same[ok] = part_of[col[ok]] == part_of[row[ok]]
    jj = np.where(same, col, 0)
    thr = theta * np.sqrt(np.abs(d[row] * d[jj]))
    strong = same & (np.abs(val) >= thr)
    keep_rp = np.concatenate([[0], np.cumsum(np.bincount(row[strong], minlength=n))])
    return sp.csr_matrix((np.ones(int(strong.sum())), col[strong], keep_rp), shape=(n, n))


def aggregate_sets(A, theta: float = 0.02, offsets=None):
    """SPEC §S4.3 standard aggregation on strength_matrix(A), per part in row order, as set
    operations: returns (agg, coarse_offsets) with agg[i] the global coarse id (part offset +
    creation number) or -1 for an isolated row. Pure Python: small and medium sizes only."""
    S = strength_matrix(A, theta, offsets)
    n = S.shape[0]
    offs = np.array([0, n], np.int64) if offsets is None else np.asarray(offsets, np.int64)
    nbrs = [S.indices[S.indptr[i]:S.indptr[i + 1]].tolist() for i in range(n)]
    agg = np.full(n, -1, np.int64)
    coffs = [0]
    for q in range(len(offs) - 1):
        rows = range(int(offs[q]), int(offs[q + 1]))
        members = []                          # aggregate k -> its set of rows
        owner = {}                            # row -> aggregate (assigned rows only)
        isolated = {i for i in rows if not nbrs[i]}
        first = set()                         # rows placed by pass 1
        for i in rows:                        # pass 1: a root and its whole free neighbourhood
            if i in owner or i in isolated:
                continue
            nb = set(nbrs[i])
            if not any(j in owner for j in nb):
                grp = nb | {i}
                members.append(grp)
                owner.update(dict.fromkeys(grp, len(members) - 1))
                first |= grp
        for i in rows:                        # pass 2: join the first pass-1 neighbour's aggregate
            if i in owner or i in isolated:
                continue
            j = next((j for j in nbrs[i] if j in first), None)
            if j is not None:
                owner[i] = owner[j]
                members[owner[j]].add(i)
        for i in rows:                        # pass 3: a new aggregate of the leftovers
            if i in owner or i in isolated:
                continue
            grp = {i} | {j for j in nbrs[i] if j not in owner}
            members.append(grp)
            owner.update(dict.fromkeys(grp, len(members) - 1))
        for k, grp in enumerate(members):
            agg[list(grp)] = coffs[-1] + k
        coffs.append(coffs[-1] + len(members))
    return agg, np.asarray(coffs, np.int64)
