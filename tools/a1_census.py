#!/usr/bin/env python3
"""Distinct values of the 512^3 hierarchy's level-1..2 operators (A1, P0, R0, ...): in total and
per 1024 / 4096-nonzero tile, to size value dictionaries. Dev tool."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import parallel_amg_amd as pa
from parallel_amg_amd.partitioned import Context

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
t = time.time()
ctx = Context(0)
be = pa.SequentialBackend(1)
A, offs, xs = pa.generate_problem(be, "poisson3d", n)
H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
print("setup", round(time.time() - t, 1), "levels", H.nlevels, flush=True)
for l in range(1, min(3, H.nlevels)):
    for name, M in (("A", H.levels[l][0].A), ("P", H.levels[l - 1][0].P), ("R", H.levels[l - 1][0].R)):
        rp = np.asarray(M.rowptr); val = np.asarray(M.val)
        nr = len(rp) - 1; nnz = int(rp[-1])
        u = np.unique(val)
        out = {"mat": f"{name}{l if name == 'A' else l - 1}", "rows": nr, "nnz": nnz, "distinct": len(u)}
        for tn in (1024, 4096):
            cuts = np.searchsorted(rp, np.arange(0, nnz, tn))
            b = np.unique(np.concatenate([cuts, [nr]]))
            cnts = np.array([len(np.unique(val[rp[a]:rp[c]])) for a, c in zip(b[:-1], b[1:])])
            out[f"t{tn}_max"] = int(cnts.max())
            out[f"t{tn}_le256"] = round(float((cnts <= 256).mean()), 3)
        print(out, flush=True)
