"""Host code under the sanitizers (SURVEY §5 "race detection / sanitizers": ASan/UBSan builds
of the C++ CPU path). setup.cpp, mtx.cpp and errors.cpp are compiled with
-fsanitize=address,undefined (no HIP runtime involved) together with the plain-C driver
tools/setup_host_check.c, which runs the single-part setup and the Matrix Market reader;
any sanitizer report aborts it. Its checksums must equal those of the normal build driven
from Python."""
import json
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import scipy.io

import parallel_amg_amd as pa
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "parallel_amg_amd", "csrc")
SAN = ["-g", "-O1", "-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer"]


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    d = tmp_path_factory.mktemp("san")
    jobs = [["gcc", "-std=c11", *SAN, "-I", os.path.join(ROOT, "include"), "-c",
             os.path.join(ROOT, "tools", "setup_host_check.c"), "-o", str(d / "drv.o")]]
    for f in ("setup", "mtx", "errors"):
        jobs.append(["g++", "-std=c++17", "-fopenmp", "-ffp-contract=off", *SAN, "-c",
                     os.path.join(CSRC, f + ".cpp"), "-o", str(d / (f + ".o"))])
    with ThreadPoolExecutor(4) as ex:
        for r in ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs):
            assert r.returncode == 0, r.stderr
    exe = str(d / "setup_host_check")
    subprocess.run(["g++", *SAN, "-fopenmp", *(str(d / f) for f in ("drv.o", "setup.o", "mtx.o", "errors.o")),
                    "-o", exe], check=True, capture_output=True, text=True)
    return exe


def _sum(M):
    if M is None:
        return "0"
    s = (M.rowptr.astype(np.uint64).sum(dtype=np.uint64) + M.col.astype(np.uint64).sum(dtype=np.uint64)
         + np.ascontiguousarray(M.val).view(np.uint64).sum(dtype=np.uint64))
    return str(int(s))


@pytest.mark.parametrize("kind,n", [(1, 20), (0, 80), (2, 14), (3, 7)])
def test_setup_clean_under_asan_ubsan(checker, tmp_path, kind, n, built):
    A = O.generate("poisson3d", 6, 6, 6).to_scipy()
    mtx = str(tmp_path / "m.mtx")
    scipy.io.mmwrite(mtx, A.tocoo(), symmetry="symmetric")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", OMP_NUM_THREADS="4")
    r = subprocess.run([checker, str(kind), str(n), mtx], capture_output=True, text=True, env=env,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    got = json.loads(r.stdout.strip().splitlines()[-1])
    name = {0: "poisson2d", 1: "poisson3d", 2: "aniso3d", 3: "elastic3d"}[kind]
    be = pa.SequentialBackend(1)
    Ap, offs, _ = pa.generate_problem(be, name, n)
    H = pa.build_hierarchy(be, Ap, offs, pa.SAParams())
    assert got["levels"] == H.nlevels
    assert got["rows"] == [H.levels[l][0].A.nrows for l in range(H.nlevels)]
    for l in range(H.nlevels):
        lp = H.levels[l][0]
        assert got["sum"][l] == [_sum(lp.A), _sum(lp.P), _sum(lp.R)]
    assert got["ainv"] == str(int(np.ascontiguousarray(H.ainv).view(np.uint64).sum(dtype=np.uint64)))
    assert got["mtx_rows"] == A.shape[0]
