#!/usr/bin/env python3
"""Census of the 512^3 level-1 operator's per-tile x runs (k_rows_xsr sizing). Dev tool.

For 2048- and 4096-nonzero tiles (<= 256 rows, as build_tiles cuts them) and several gap
thresholds: runs per tile (offsets sorted, a new run where the gap exceeds G or a run would need
more than 256 doubles) and staged doubles per tile, as distribution quantiles."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import parallel_amg_amd as pa  # noqa: E402
from parallel_amg_amd.partitioned import Context  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
t = time.time()
ctx = Context(0)
be = pa.SequentialBackend(1)
A, offs, xs = pa.generate_problem(be, "poisson3d", n)
H = pa.build_hierarchy(be, A, offs, pa.SAParams(max_coarse=1000), device=ctx)
print("setup", round(time.time() - t, 1), flush=True)
M = H.levels[1][0].A
rp = np.asarray(M.rowptr)
col = np.asarray(M.col).astype(np.int64)
nr_all = len(rp) - 1
rows = np.repeat(np.arange(nr_all), np.diff(rp))
off = col - rows
for tn in (2048, 4096):
    cuts = []
    r = 0
    while r < nr_all:
        e = min(nr_all, r + 256)
        e = min(e, int(np.searchsorted(rp, rp[r] + tn, side="right")) - 1)
        e = max(e, r + 1)
        cuts.append((r, e))
        r = e
    idx = np.random.default_rng(0).choice(len(cuts), size=min(4000, len(cuts)), replace=False)
    for G in (16, 48, 128):
        ncl, tot = [], []
        for i in idx:
            a, e = cuts[i]
            nr = e - a
            o = np.unique(off[rp[a]:rp[e]])
            c, cm, cx, t_ = 0, None, None, 0
            for v in o:
                if cm is None or v - cx > G or nr + (v - cm) > 256:
                    if cm is not None:
                        c += 1
                        t_ += nr + (cx - cm)
                    cm = v
                cx = v
            c += 1
            t_ += nr + (cx - cm)
            ncl.append(c)
            tot.append(t_)
        q = lambda v: [int(np.quantile(v, z)) for z in (0.5, 0.9, 0.99, 1.0)]  # noqa: E731
        print(f"tiles {tn}: G={G} runs p50/p90/p99/max {q(ncl)} staged {q(tot)} (tiles {len(cuts)})", flush=True)
