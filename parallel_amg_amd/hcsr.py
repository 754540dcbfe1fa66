"""Host CSR handles of libpamg (pamg_hcsr) with zero-copy numpy views (SPEC.md §S1)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import call, ptr


class HCSR:
    """One part's rows of a sparse matrix on the host: int64 rowptr, int32 global columns,
    fp64 values. Owns a ``pamg_hcsr`` handle; ``rowptr/col/val`` are views into it."""

    __slots__ = ("_h", "nrows", "ncols", "nnz", "rowptr", "col", "val", "__weakref__")

    def __init__(self, handle):
        self._h = handle
        nr, nc, nz = C.c_int64(), C.c_int64(), C.c_int64()
        call("pamg_hcsr_info", handle, C.byref(nr), C.byref(nc), C.byref(nz))
        self.nrows, self.ncols, self.nnz = nr.value, nc.value, nz.value
        rp, col, val = _lib.pi64(), _lib.pi32(), _lib.pdbl()
        call("pamg_hcsr_data", handle, C.byref(rp), C.byref(col), C.byref(val))
        self.rowptr = np.ctypeslib.as_array(rp, (self.nrows + 1,))
        self.col = np.ctypeslib.as_array(col, (self.nnz,)) if self.nnz else np.zeros(0, np.int32)
        self.val = np.ctypeslib.as_array(val, (self.nnz,)) if self.nnz else np.zeros(0)

    @property
    def handle(self):
        return self._h

    def __del__(self):
        h = getattr(self, "_h", None)
        lib = getattr(_lib, "_lib", None) if _lib is not None else None
        if h and lib is not None:
            try:
                lib.pamg_hcsr_destroy(h)
            except Exception:  # pragma: no cover - shutdown ordering
                pass
        self._h = None

    @classmethod
    def from_arrays(cls, rowptr, col, val, ncols) -> "HCSR":
        rowptr = np.asarray(rowptr, np.int64)
        nr = len(rowptr) - 1
        nnz = int(rowptr[-1]) if nr >= 0 else 0
        if nnz and int(np.max(col)) >= 2**31 - 1:
            raise OverflowError("column id exceeds int32")
        h = C.c_void_p()
        call("pamg_hcsr_create", nr, ncols, nnz, C.byref(h))
        M = cls(h)
        M.rowptr[:] = rowptr
        if nnz:
            M.col[:] = np.asarray(col)[:nnz]
            M.val[:] = np.asarray(val, np.float64)[:nnz]
        return M

    def rows(self, idx) -> tuple:
        """(rowptr, col, val) of the local rows ``idx`` (ascending), as new arrays."""
        idx = np.asarray(idx, np.int64)
        starts = self.rowptr[idx]
        counts = self.rowptr[idx + 1] - starts
        rp = np.zeros(len(idx) + 1, np.int64)
        np.cumsum(counts, out=rp[1:])
        tot = int(rp[-1])
        if tot == 0:
            return rp, np.zeros(0, np.int32), np.zeros(0)
        pos = np.arange(tot, dtype=np.int64) - np.repeat(rp[:-1], counts) + np.repeat(starts, counts)
        return rp, self.col[pos], self.val[pos]

    def to_scipy(self, ncols=None):
        import scipy.sparse as sp
        return sp.csr_matrix((self.val.copy(), self.col.astype(np.int64), self.rowptr.copy()),
                             shape=(self.nrows, ncols if ncols is not None else self.ncols))


def gen_grid(kind: int, nx: int, ny: int, nz: int, eps: float, r0: int, r1: int) -> HCSR:
    h = C.c_void_p()
    call("pamg_gen_grid", kind, nx, ny, nz, eps, r0, r1, C.byref(h))
    return HCSR(h)


def read_mtx(path: str, r0: int = 0, r1: int = -1):
    """Rows [r0, r1) of a Matrix Market file -> (HCSR, n_global)."""
    h = C.c_void_p()
    n = C.c_int64()
    call("pamg_read_mtx", str(path).encode(), r0, r1, C.byref(n), C.byref(h))
    return HCSR(h), n.value


def read_mtx_rows(path: str, rows: np.ndarray):
    """File rows ``rows`` (in that order) of a Matrix Market file -> (HCSR in the file's column
    numbering, n_global)."""
    rows = np.ascontiguousarray(rows, np.int64)
    h = C.c_void_p()
    n = C.c_int64()
    call("pamg_read_mtx_rows", str(path).encode(), len(rows), ptr(rows), C.byref(n), C.byref(h))
    return HCSR(h), n.value


def mtx_row_counts(path: str) -> np.ndarray:
    n = C.c_int64()
    call("pamg_mtx_row_counts", str(path).encode(), C.byref(n), None)
    out = np.zeros(n.value, np.int64)
    call("pamg_mtx_row_counts", str(path).encode(), C.byref(n), ptr(out))
    return out


def rcm_order(A: HCSR) -> np.ndarray:
    """Reverse Cuthill-McKee order of a square host matrix (pamg_rcm_order): new row k is old
    row order[k]."""
    out = np.empty(A.nrows, np.int64)
    call("pamg_rcm_order", A.handle, ptr(out))
    return out


def locality_order(A: HCSR, mode: int = 1):
    """Locality order of a square level operator for the device layout (pamg_locality_order):
    mode 0 identity, 1 auto (reverse Cuthill-McKee only where the numbering is scattered and
    RCM cuts the mean row span 4x), 2 always RCM. Returns (order or None for the identity,
    mean row span before, after)."""
    out = np.empty(A.nrows, np.int64)
    applied, before, after = C.c_int(), C.c_double(), C.c_double()
    call("pamg_locality_order", A.handle, int(mode), ptr(out), C.byref(applied), C.byref(before),
         C.byref(after))
    return (out if applied.value else None), before.value, after.value


def gen_xstar(i0: int, n: int, seed: int) -> np.ndarray:
    out = np.empty(n, np.float64)
    call("pamg_gen_xstar", i0, n, seed, ptr(out))
    return out


def gershgorin(A: HCSR, row0: int) -> float:
    r = C.c_double()
    call("pamg_setup_gershgorin", A.handle, row0, C.byref(r))
    return r.value


def aggregate(A: HCSR, row0: int, theta: float):
    agg = np.empty(A.nrows, np.int32)
    na = C.c_int64()
    call("pamg_setup_aggregate", A.handle, row0, theta, ptr(agg), C.byref(na))
    return agg, na.value


def tentative(agg: np.ndarray, n_agg: int, coarse0: int, ncols_global: int) -> HCSR:
    h = C.c_void_p()
    agg = np.ascontiguousarray(agg, np.int32)
    call("pamg_setup_tentative", len(agg), ptr(agg), n_agg, coarse0, ncols_global, C.byref(h))
    return HCSR(h)


def spgemm(X: HCSR, y0: int, Yown: HCSR, ghost_ids=None, Yghost: HCSR | None = None,
           device=None) -> HCSR:
    """C = X * Y (SPEC §S4.5). ``device``: a partitioned.Context -> the GPU routine
    (pamg_dev_spgemm, same result bit for bit), else the host one."""
    h = C.c_void_p()
    fn, pre = ("pamg_dev_spgemm", (device.handle,)) if device is not None else ("pamg_setup_spgemm", ())
    if ghost_ids is None or len(ghost_ids) == 0:
        call(fn, *pre, X.handle, y0, Yown.handle, None, 0, None, C.byref(h))
    else:
        g = np.ascontiguousarray(ghost_ids, np.int64)
        call(fn, *pre, X.handle, y0, Yown.handle, ptr(g), len(g), Yghost.handle, C.byref(h))
    return HCSR(h)


def smooth(A: HCSR, row0: int, T: HCSR, AT: HCSR, omega: float) -> HCSR:
    call("pamg_setup_smooth", A.handle, row0, T.handle, AT.handle, omega)
    return AT


def transpose(P: HCSR, row0: int, c0: int, c1: int, device=None) -> HCSR:
    h = C.c_void_p()
    if device is not None:
        call("pamg_dev_transpose", device.handle, P.handle, row0, c0, c1, C.byref(h))
    else:
        call("pamg_setup_transpose", P.handle, row0, c0, c1, C.byref(h))
    return HCSR(h)


def hstack_rows(pieces) -> HCSR:
    arr = (C.c_void_p * len(pieces))(*[p.handle for p in pieces])
    h = C.c_void_p()
    call("pamg_setup_hstack_rows", len(pieces), arr, C.byref(h))
    return HCSR(h)


MAX_DENSE_COARSE = 16384  # PAMG_MAX_DENSE_COARSE


def cholinv(A: HCSR) -> np.ndarray:
    """Column-major inverse (SPEC §S5) as a flat array of n*n."""
    if A.nrows > MAX_DENSE_COARSE:  # checked before allocating n*n doubles (pamg.h)
        raise _lib.PamgError(-1, "pamg_setup_cholinv",
                             f"coarsest level of {A.nrows} rows exceeds the dense-solve limit {MAX_DENSE_COARSE} "
                             "(raise max_levels or lower max_coarse)")
    out = np.empty(A.nrows * A.nrows, np.float64)
    call("pamg_setup_cholinv", A.handle, ptr(out))
    return out
