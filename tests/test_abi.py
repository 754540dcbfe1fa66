"""C-ABI boundary (include/pamg.h) on CPU: libpamg.so loads, exports every declared entry point,
the ctypes table binds all of them, and the host-side error convention holds (status codes +
pamg_last_error). No device compute here (no GPU in the CPU suite)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pamg.h")


def declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(pamg_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_boundary():
    names = declared()
    for must in ("pamg_ctx_create", "pamg_mat_upload", "pamg_spmv", "pamg_residual", "pamg_jacobi",
                 "pamg_exchange", "pamg_hier_create", "pamg_vcycle", "pamg_comm_init",
                 "pamg_setup_spgemm", "pamg_setup_aggregate"):
        assert must in names
    assert len(names) >= 50


def test_library_exports_every_declared_symbol(built):
    from parallel_amg_amd import _lib
    lib_path = _lib.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (pamg_\w+)", out))
    missing = [n for n in declared() if n not in exported]
    assert not missing, missing
    # the ctypes binding covers the whole boundary (and nothing that is not declared)
    assert sorted(_lib.SIGNATURES) == declared()
    L = _lib.lib()
    for n in declared():
        assert getattr(L, n) is not None


def test_error_convention(built):
    from parallel_amg_amd import _lib
    from parallel_amg_amd._lib import PamgError, call
    L = _lib.lib()
    assert L.pamg_version().startswith(b"pamg")
    rc = L.pamg_hcsr_info(None, None, None, None)
    assert rc == -1 and b"invalid handle" in L.pamg_last_error()
    with pytest.raises(PamgError) as e:
        call("pamg_gen_grid", 7, 4, 4, 4, 0.0, 0, 64, C.byref(C.c_void_p()))
    assert e.value.code == -1
    with pytest.raises(PamgError):
        call("pamg_set_option", b"no_such_key", 1)
    v = C.c_int64()
    call("pamg_set_option", b"tile_nnz", 2048)
    call("pamg_get_option", b"tile_nnz", C.byref(v))
    assert v.value == 2048
    call("pamg_set_option", b"tile_nnz", 1024)


def test_setup_errors_are_reported(built):
    from parallel_amg_amd import hcsr as HC
    from parallel_amg_amd._lib import PamgError
    import numpy as np
    # a row without a diagonal -> PAMG_E_SETUP from the Gershgorin bound (SPEC §S3 needs a_ii)
    M = HC.HCSR.from_arrays(np.array([0, 1, 2]), np.array([1, 1], np.int32), np.array([1.0, 2.0]), 2)
    with pytest.raises(PamgError) as e:
        HC.gershgorin(M, 0)
    assert e.value.code == -5
    # non-SPD coarse matrix -> PAMG_E_SETUP from the Cholesky inverse (SPEC §S5)
    M = HC.HCSR.from_arrays(np.array([0, 2, 4]), np.array([0, 1, 0, 1], np.int32), np.array([1.0, 2.0, 2.0, 1.0]), 2)
    with pytest.raises(PamgError) as e:
        HC.cholinv(M)
    assert e.value.code == -5


def test_product_never_imports_the_oracle():
    """The product package must not touch oracle/ (the checker) — grep its sources."""
    pkg = os.path.join(ROOT, "parallel_amg_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f
                assert "libpamg_oracle" not in txt and not re.search(r"#include\s*[<\"].*oracle", txt), f
                assert not re.search(r"\borc_\w+\(", txt), f


def test_load_order_binds_opt_rocm_runtime(built):
    """libpamg loaded before torch binds to /opt/rocm's HIP and RCCL, not to the copies in the
    torch wheel (same sonames, older RCCL; _lib.runtime_providers). bench.py, conftest.py and
    the multi-process workers rely on this order."""
    import json
    import subprocess
    import sys
    code = ("import json, parallel_amg_amd._lib as L; L.lib(); import torch; "
            "print(json.dumps(L.runtime_providers()))")
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True,
                         check=True).stdout.strip().splitlines()[-1]
    prov = json.loads(out)
    assert set(prov) == {"hip", "rccl"}
    for k, path in prov.items():
        assert "/torch/" not in path and path.startswith("/opt/rocm"), (k, path)


# every pamg_set_option key with its default and another legal value (include/pamg.h, the
# INTEGRATION.md option table)
OPTION_DEFAULTS = {"tile_nnz": (1024, 4096), "tile_order": (1, 0), "col24": (1, 0), "long_tiles": (1, 0),
                   "long_tiles_min": (24, 48), "row_len8": (1, 0), "value_dict": (1, 0), "col_dict": (1, 0),
                   "col_dict_anchor": (1, 0), "col_dict_tile": (1, 0), "x_stage": (1, 0), "tm_tile_dicts": (1, 0),
                   "band_pct": (100, 50), "band_pct_restrict": (50, 100), "tile_major": (1, 2), "poison_ghosts": (0, 1),
                   "sym_dia": (1, 0), "sym_rows": (2, 1), "jr_fuse": (1, 0), "sym_vd": (1, 0),
                   "symd_chunks": (2, 4), "chain_store_x": (0, 1), "sym_zm": (1, 0), "zm_chunks": (0, 16),
                   "tb_xfast": (1, 0), "ell": (1, 0), "ell_restrict": (1, 0), "ell_min_rows": (65536, 1024), "pnc": (1, 0), "rpat": (1, 0), "pnc_compact": (1, 0), "ell_pair": (1, 0),
                   "ell_yblock": (16, 0)}


def test_option_keys_defaults_and_docs(built):
    """Each knob reads back its documented default, takes another legal value, rejects an
    illegal one, and is listed in INTEGRATION.md's table and pamg.h's option comment."""
    import os
    from parallel_amg_amd._lib import PamgError, call
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    integ = open(os.path.join(root, "INTEGRATION.md")).read()
    header = open(os.path.join(root, "include", "pamg.h")).read()
    v = C.c_int64()
    for k, (default, other) in OPTION_DEFAULTS.items():
        call("pamg_get_option", k.encode(), C.byref(v))
        assert v.value == default, k
        call("pamg_set_option", k.encode(), other)
        call("pamg_get_option", k.encode(), C.byref(v))
        assert v.value == other, k
        with pytest.raises(PamgError):
            call("pamg_set_option", k.encode(), -7)
        call("pamg_set_option", k.encode(), default)
        assert f"`{k}`" in integ, k
        assert f'"{k}"' in header, k
