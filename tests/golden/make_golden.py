#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the CPU oracle (oracle/).

The reference (/root/reference/README.md:1-2) holds no code, tests or data, so these vectors
are produced by this repo's SPEC.md restatement and pinned independently by
tests/test_oracle.py (scipy.sparse cross-checks + hand-derived known answers). They guard the
oracle, the product's host setup and the GPU path against drift. Re-run only when SPEC.md
changes on purpose:

    python tests/golden/make_golden.py
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import oracle as O  # noqa: E402

# (name, kind, n, nparts, max_coarse, ncycles, full arrays?)
CASES = [
    ("poisson2d_32_p1", "poisson2d", 32, 1, 60, 10, True),
    ("poisson3d_12_p1", "poisson3d", 12, 1, 40, 10, True),
    ("aniso3d_12_p2", "aniso3d", 12, 2, 60, 10, True),
    # BASELINE.json configs[0]: 2D 5-pt 256x256, 2 parts on CPU (plumbing config)
    ("poisson2d_256_p2", "poisson2d", 256, 2, 1000, 10, False),
]


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def make(name, kind, n, nparts, max_coarse, ncycles, full):
    A = O.generate(kind, *O.grid_shape(kind, n))
    b = O.spmv(A, O.xstar(A.nrows))
    H = O.setup(A, nparts=nparts, max_coarse=max_coarse, agglomerate=0)  # decoupled on every level
    x, hist = H.solve(b, ncycles, res_hist=True)
    out = {"kind": kind, "n": n, "nparts": nparts, "max_coarse": max_coarse, "ncycles": ncycles,
           "nlevels": H.nlevels, "b_sha": sha(b), "x_sha": sha(x), "x": x if full else x[:64],
           "res_hist": hist, "omega": np.asarray(H.omega), "rho": np.asarray(H.rho),
           "ainv_sha": sha(H.ainv)}
    for l in range(H.nlevels):
        out[f"offsets_{l}"] = H.offsets[l]
        mats = [("A", H.A[l])] + ([("P", H.P[l]), ("R", H.R[l])] if l < H.nlevels - 1 else [])
        for tag, M in mats:
            out[f"{tag}{l}_shape"] = np.array([M.nrows, M.ncols, M.nnz])
            for part in ("rowptr", "col", "val"):
                arr = getattr(M, part)
                out[f"{tag}{l}_{part}_sha"] = sha(arr)
                if full:
                    out[f"{tag}{l}_{part}"] = arr
        if l < H.nlevels - 1:
            out[f"agg_{l}"] = H.agg[l].astype(np.int32)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print(name, H.nlevels, "levels", [a.nrows for a in H.A], "res", hist[-1])


if __name__ == "__main__":
    for c in CASES:
        make(*c)
