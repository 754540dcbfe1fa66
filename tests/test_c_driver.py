"""The C-ABI from plain C (tools/pamg_cdriver.c): the header compiles as C11 and links against
libpamg.so (CPU), and the C driver's setup + V-cycles reproduce the Python path's residual
history bit for bit (GPU) — the boundary does not depend on the Python host layer."""
import json
import os
import subprocess

import numpy as np
import pytest

import parallel_amg_amd as pa
from parallel_amg_amd._lib import LIB_PATH

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _build(tmp_path):
    exe = str(tmp_path / "pamg_cdriver")
    cmd = ["gcc", "-O2", "-std=c11", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tools", "pamg_cdriver.c"), "-L", os.path.dirname(LIB_PATH), "-lpamg",
           f"-Wl,-rpath,{os.path.dirname(LIB_PATH)}", "-o", exe]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_c_driver_builds(tmp_path, built):
    assert os.access(_build(tmp_path), os.X_OK)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,gpu_products", [(1, 20, 1), (1, 20, 0), (2, 16, 1), (0, 64, 1)])
def test_c_driver_matches_python(tmp_path, ctx, kind, n, gpu_products):
    from parallel_amg_amd.partitioned import PVector, mul
    from parallel_amg_amd.solver import AMGSolver
    exe = _build(tmp_path)
    ncycles = 6
    out = subprocess.run([exe, str(kind), str(n), str(ncycles), str(gpu_products)], check=True,
                         capture_output=True, text=True, timeout=300)
    res = json.loads(out.stdout.strip().splitlines()[-1])
    name = {0: "poisson2d", 1: "poisson3d", 2: "aniso3d", 3: "elastic3d"}[kind]
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, name, n)
    H = pa.build_hierarchy(be, A, offs, pa.SAParams(), device=ctx if gpu_products else None)
    assert res["levels"] == H.nlevels
    assert res["level_rows"] == [H.levels[l][0].A.nrows for l in range(H.nlevels)]
    S = AMGSolver(ctx, H)
    b = PVector(ctx, S.A[0].nrows)
    mul(b, S.A[0], PVector(ctx, S.A[0].nrows, 0, xs[0]))
    hist = S.vcycle(S.new_vector(), b, ncycles, res_hist=True)
    assert [f"{v:016x}" for v in np.asarray(hist).view(np.uint64)] == res["res_bits"]
