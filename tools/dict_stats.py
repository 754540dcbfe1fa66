#!/usr/bin/env python3
"""Dictionary-size census of the level operators (dev tool, GPU box: 512^3 needs its memory):
per greedy 1024-nonzero tile, distinct row-relative (col - row) and anchored (col - first col)
offsets, and distinct columns; decides which compressed column formats could fit.

    gpurun -- 'python3 tools/dict_stats.py --n 512 > gpurun_out/dict_stats.json'
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import parallel_amg_amd as pa  # noqa: E402
from parallel_amg_amd.partitioned import Context  # noqa: E402


def census(M, ntiles=20000):
    rp, col = M.rowptr, M.col.astype(np.int64)
    nr = M.nrows
    starts = np.linspace(0, nr - 1, ntiles).astype(np.int64)
    rel, anc, dc, fill = [], [], [], []
    for i in starts:
        j, nz = i, 0
        while j < nr and j - i < 256 and nz + (rp[j + 1] - rp[j]) <= 1024:
            nz += rp[j + 1] - rp[j]
            j += 1
        j = max(j, i + 1)
        c = col[rp[i]:rp[j]]
        lens = np.diff(rp[i:j + 1])
        rows = np.repeat(np.arange(i, j, dtype=np.int64), lens)
        first = np.repeat(col[rp[i:j]], lens) if len(c) else c
        rel.append(len(np.unique(c - rows)))
        anc.append(len(np.unique(c - first)))
        dc.append(len(np.unique(c)))
        fill.append(len(c))
    out = {}
    for k, v in (("rowrel", rel), ("anchored", anc), ("columns", dc)):
        v = np.array(v)
        out[k] = {"mean": float(v.mean()), "p99": float(np.percentile(v, 99)), "max": int(v.max()),
                  "frac_over_256": float(np.mean(v > 256))}
    out["nnz_per_tile"] = float(np.mean(fill))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--kind", default="poisson3d")
    a = ap.parse_args()
    ctx = Context(0)
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, a.kind, a.n)
    H = pa.build_hierarchy(be, A, offs, device=ctx)
    res = {}
    for l in range(2):
        lp = H.levels[l][0]
        for w in "APR":
            res[f"{w}{l}"] = census(getattr(lp, w))
            print(w, l, json.dumps(res[f"{w}{l}"]), file=sys.stderr, flush=True)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
