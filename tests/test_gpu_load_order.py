"""Library load order guard.

The torch wheel bundles HIP 7.0 + RCCL 2.26.6 under the sonames /opt/rocm uses
(libamdhip64.so.7, librccl.so.1). A process that imports torch before loading libpamg binds
libpamg's HIP/RCCL calls to those copies; round 1 saw that combination segfault in the first
captured V-cycle with RCCL nodes. `pamg_comm_init` now compares the RCCL it resolved with the
one it was built against and returns PAMG_E_RCCL (naming the library file) instead of letting
the process run into the crash. Each order runs in its own child process, so a fault could
only end that child: the test asserts on its exit status as well.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import ctypes as C, json, sys
sys.path.insert(0, {root!r})
if {torch_first}:
    import torch  # noqa: F401  (maps torch/lib's libamdhip64 / librccl first)
from parallel_amg_amd import _lib
L = _lib.lib()
v = [C.c_int() for _ in range(4)]
assert L.pamg_runtime_versions(*[C.byref(x) for x in v]) == 0
ctx = C.c_void_p()
assert L.pamg_ctx_create(0, C.byref(ctx)) == 0, _lib.last_error()
uid = C.create_string_buffer(128)
assert L.pamg_comm_unique_id(uid) == 0, _lib.last_error()
rc = L.pamg_comm_init(ctx, 1, 0, uid)
msg = _lib.last_error() if rc else ""
L.pamg_ctx_destroy(ctx)
print(json.dumps({{"rc": rc, "msg": msg, "versions": [x.value for x in v],
                  "providers": _lib.runtime_providers()}}))
"""


@pytest.mark.parametrize("torch_first", [False, True])
def test_comm_init_checks_the_bound_rccl(torch_first):
    code = CHILD.format(root=ROOT, torch_first=torch_first)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, f"child ended with {p.returncode}:\n{p.stderr[-3000:]}"
    out = json.loads(p.stdout.strip().splitlines()[-1])
    hip_rt, hip_built, rccl_rt, rccl_built = out["versions"]
    print(out)
    if rccl_rt < rccl_built:
        assert out["rc"] == -3, out  # PAMG_E_RCCL, not a crash
        assert "older than" in out["msg"] and "librccl" in out["msg"], out["msg"]
    else:
        assert out["rc"] == 0, out
    if not torch_first:  # libpamg first: /opt/rocm's RCCL, the one it was built against
        assert rccl_rt == rccl_built and out["rc"] == 0, out
