"""ctypes binding of libpamg.so (include/pamg.h) — the Python side of the C-ABI boundary.

The library is built in-tree (``parallel_amg_amd/libpamg.so``) by ``build.build()``; there
is deliberately NO fallback: if the shared library is missing or a symbol is absent, every
entry point raises, so a test can never pass on a silent CPU path.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# PAMG_LIB (dev A/B only): load another build of the same ABI, e.g. gpurun_ab/libpamg_a.so
LIB_PATH = os.environ.get("PAMG_LIB") or os.path.join(_HERE, "libpamg.so")

PAMG_OK = 0
ERRORS = {-1: "PAMG_E_ARG", -2: "PAMG_E_HIP", -3: "PAMG_E_RCCL", -4: "PAMG_E_OVERFLOW",
          -5: "PAMG_E_SETUP", -6: "PAMG_E_STATE", -7: "PAMG_E_NOMEM"}


class PamgError(RuntimeError):
    def __init__(self, code, fn, msg):
        super().__init__(f"{fn} -> {ERRORS.get(code, code)}: {msg}")
        self.code = code


vp = C.c_void_p
i32, i64, dbl = C.c_int, C.c_int64, C.c_double
pvp = C.POINTER(C.c_void_p)
pi64 = C.POINTER(C.c_int64)
pdbl = C.POINTER(C.c_double)
pi32 = C.POINTER(C.c_int32)

# name -> argtypes (all return int status unless listed in _RESTYPE)
SIGNATURES = {
    "pamg_version": [],
    "pamg_last_error": [],
    "pamg_ctx_create": [i32, pvp],
    "pamg_ctx_destroy": [vp],
    "pamg_ctx_sync": [vp],
    "pamg_ctx_refcount": [vp, C.POINTER(C.c_int)],
    "pamg_device_count": [C.POINTER(C.c_int)],
    "pamg_device_sync": [i32],
    "pamg_comm_unique_id": [C.c_char_p],
    "pamg_comm_init": [vp, i32, i32, C.c_char_p],
    "pamg_comm_rank": [vp, C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pamg_runtime_versions": [C.POINTER(C.c_int)] * 4,
    "pamg_comm_init_host": [vp, i32, i32, vp, vp],
    "pamg_world_create": [i32, pvp],
    "pamg_world_destroy": [vp],
    "pamg_world_abort": [vp],
    "pamg_world_reset": [vp],
    "pamg_world_state": [vp, vp],
    "pamg_comm_init_local": [vp, vp, i32],
    "pamg_world_spmv": [vp, vp, vp, vp],
    "pamg_world_exchange": [vp, vp, vp],
    "pamg_world_dot": [vp, vp, vp, pdbl],
    "pamg_world_vcycle": [vp, vp, vp, vp, i32, vp],
    "pamg_world_pcg": [vp, vp, vp, vp, dbl, i32, C.POINTER(C.c_int), vp],
    "pamg_plan_create": [vp, i64, i64, i32, vp, vp, vp, vp, pvp],
    "pamg_plan_set_tag": [vp, i64],
    "pamg_plan_destroy": [vp],
    "pamg_vec_create": [vp, i64, i64, pvp],
    "pamg_vec_destroy": [vp],
    "pamg_vec_size": [vp, pi64, pi64],
    "pamg_vec_upload": [vp, vp, vp],
    "pamg_vec_download": [vp, vp, vp],
    "pamg_vec_download_ghosts": [vp, vp, vp],
    "pamg_vec_device_ptr": [vp, pvp],
    "pamg_vec_fill": [vp, vp, dbl],
    "pamg_vec_copy": [vp, vp, vp],
    "pamg_vec_axpby": [vp, dbl, vp, dbl, vp],
    "pamg_vec_dot": [vp, vp, vp, pdbl],
    "pamg_vec_nrm2": [vp, vp, pdbl],
    "pamg_exchange": [vp, vp, vp],
    "pamg_exchange_begin": [vp, vp, vp],
    "pamg_exchange_end": [vp, vp, vp],
    "pamg_mat_upload": [vp, i64, i64, vp, vp, i32, vp, i32, vp, pvp],
    "pamg_mat_upload_perm": [vp, i64, i64, vp, vp, i32, vp, i32, vp, vp, vp, pvp],
    "pamg_mat_destroy": [vp],
    "pamg_mat_info": [vp, pi64, pi64, pi64],
    "pamg_mat_stream_bytes": [vp, pi64],
    "pamg_mat_layout": [vp, i32, C.POINTER(C.c_int)],
    "pamg_spmv": [vp, vp, vp, vp],
    "pamg_residual": [vp, vp, vp, vp, vp, pdbl],
    "pamg_jacobi": [vp, vp, vp, vp, vp, dbl, i32],
    "pamg_jacobi_residual": [vp, vp, vp, vp, vp, vp, dbl, pi32],
    "pamg_hier_create": [vp, i32, vp, vp, vp, vp, i64, vp, i32, vp, pvp],
    "pamg_hier_destroy": [vp],
    "pamg_hier_set_graph": [vp, i32],
    "pamg_hier_set_sweeps": [vp, i32, i32],
    "pamg_hier_set_perm": [vp, i64, vp],
    "pamg_hier_graph_state": [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "pamg_vcycle": [vp, vp, vp, vp, i32, vp],
    "pamg_vcycle_async": [vp, vp, vp, vp, i32],
    "pamg_pcg": [vp, vp, vp, vp, dbl, i32, C.POINTER(C.c_int), vp],
    "pamg_hier_profile": [vp, i32],
    "pamg_hier_profile_read": [vp, vp],
    "pamg_bench_rowop": [vp, vp, i32, vp, vp, vp, dbl, i32, pdbl],
    "pamg_hier_bench_chain": [vp, vp, vp, i32, pdbl],
    "pamg_set_option": [C.c_char_p, i64],
    "pamg_get_option": [C.c_char_p, pi64],
    "pamg_hcsr_create": [i64, i64, i64, pvp],
    "pamg_hcsr_destroy": [vp],
    "pamg_hcsr_info": [vp, pi64, pi64, pi64],
    "pamg_hcsr_data": [vp, C.POINTER(pi64), C.POINTER(pi32), C.POINTER(pdbl)],
    "pamg_gen_grid": [i32, i64, i64, i64, dbl, i64, i64, pvp],
    "pamg_gen_xstar": [i64, i64, C.c_uint64, vp],
    "pamg_read_mtx": [C.c_char_p, i64, i64, pi64, pvp],
    "pamg_mtx_row_counts": [C.c_char_p, pi64, vp],
    "pamg_read_mtx_rows": [C.c_char_p, i64, vp, pi64, pvp],
    "pamg_rcm_order": [vp, vp],
    "pamg_locality_order": [vp, i32, vp, C.POINTER(C.c_int), pdbl, pdbl],
    "pamg_setup_gershgorin": [vp, i64, pdbl],
    "pamg_setup_aggregate": [vp, i64, dbl, vp, pi64],
    "pamg_setup_tentative": [i64, vp, i64, i64, i64, pvp],
    "pamg_setup_spgemm": [vp, i64, vp, vp, i64, vp, pvp],
    "pamg_setup_smooth": [vp, i64, vp, vp, dbl],
    "pamg_setup_transpose": [vp, i64, i64, i64, pvp],
    "pamg_dev_spgemm": [vp, vp, i64, vp, vp, i64, vp, pvp],
    "pamg_dev_transpose": [vp, vp, i64, i64, i64, pvp],
    "pamg_setup_hstack_rows": [i32, vp, pvp],
    "pamg_setup_cholinv": [vp, vp],
}
_RESTYPE = {"pamg_version": C.c_char_p, "pamg_last_error": C.c_char_p}

_lib = None


def lib():
    """Load libpamg.so (raises if it has not been built — no fallback path exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(or `make -C parallel_amg_amd/csrc`). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            f = getattr(L, name)  # AttributeError if the ABI lost a symbol
            f.argtypes = args
            f.restype = _RESTYPE.get(name, C.c_int)
        _lib = L
    return _lib


class _DlInfo(C.Structure):
    _fields_ = [("dli_fname", C.c_char_p), ("dli_fbase", C.c_void_p),
                ("dli_sname", C.c_char_p), ("dli_saddr", C.c_void_p)]


def runtime_providers() -> dict:
    """The files that serve libpamg's HIP and RCCL calls in this process.

    Load order matters: the PyTorch wheel bundles its own ROCm (HIP 7.0, RCCL 2.26) under
    torch/lib with the same sonames as /opt/rocm's (libamdhip64.so.7, librccl.so.1), so if
    torch is imported first, libpamg binds to those copies; loaded first, libpamg binds to
    /opt/rocm (HIP 7.2, RCCL 2.27.7) and torch maps its own copies beside them. Measured on the
    MI355X box: RCCL 2.26.6 segfaults in tests/test_gpu_rccl_self.py where 2.27.7 passes, so
    drivers that use libpamg's RCCL load it before torch and keep torch off the GPU (bench.py).
    """
    L = lib()
    dl = C.CDLL(None)
    dladdr = dl.dladdr
    dladdr.argtypes = [C.c_void_p, C.POINTER(_DlInfo)]
    out = {}
    for key, sym in (("hip", "hipStreamCreateWithFlags"), ("rccl", "ncclCommInitRank")):
        try:
            addr = C.cast(getattr(L, sym), C.c_void_p).value
        except AttributeError:
            continue
        info = _DlInfo()
        if addr and dladdr(addr, C.byref(info)) and info.dli_fname:
            out[key] = os.path.realpath(info.dli_fname.decode())
    return out


def call(name, *args):
    """Call a status-returning entry point; raise PamgError with pamg_last_error on failure."""
    L = lib()
    rc = getattr(L, name)(*args)
    if rc != PAMG_OK:
        msg = L.pamg_last_error().decode(errors="replace")
        raise PamgError(rc, name, msg)
    return rc


def layout_of(M, part_set: int = 0) -> dict:
    """The tile layout libpamg chose at upload for a device matrix (pamg_mat_layout)."""
    out = (C.c_int * 10)()
    call("pamg_mat_layout", M.handle, part_set, out)
    return {"c24": bool(out[0]), "vd": bool(out[1]), "rl8": bool(out[2]), "cd": int(out[3]),
            "cd_offsets": int(out[4]), "tm": bool(out[5]), "tm_rs": int(out[6]),
            "tile_nnz": int(out[7]), "tiles": int(out[8]), "anchored": bool(out[9] & 1), "per_tile": bool(out[9] & 2),
            "x_stage": bool(out[9] & 4), "sym": bool(out[9] & 8), "sym_rows": 2 if out[9] & 16 else 1,
            "jr_fused": bool(out[9] & 32), "tm_vd": bool(out[9] & 64), "sym_vd": bool(out[9] & 128),
            "ell": bool(out[9] & 512), "pnc": bool(out[9] & 1024),
            "rpat": bool(out[9] & 2048), "pnc_compact": bool(out[9] & 4096),
            "ell_pair": bool(out[9] & 8192)}


def last_error() -> str:
    return lib().pamg_last_error().decode(errors="replace")


def ptr(a):
    """Raw data pointer of a numpy array (None for empty arrays)."""
    return C.c_void_p(a.ctypes.data) if a is not None and a.size else None
