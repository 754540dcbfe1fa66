#!/usr/bin/env python3
"""Host census of the repetition the round-6 layouts rely on (CPU only, no GPU):

* R0 = P0^T rows as (column - first column, value bits) sequences: distinct patterns and their
  entries (the pattern-dictionary rows, `rpat`: <= 255 patterns, <= 4096 entries);
* P0 rows as (neighbour-code pattern, value indices) combinations (the compact neighbour-coded
  records, `pnc_compact`: <= 1024), the codes as build_pnc assigns them (first neighbour of
  i, i-1, i+1, i-nx, i+nx, i-M, i+M whose anchor is the column);
* A1's 256-row groups: distinct (col - row, value bits) pairs per group (the paired ELL,
  `ell_pair`: <= 256).

The level-0 products come from the library's own host setup (aggregation, tentative prolongator,
smoothing, transpose), A1 from the full host hierarchy (skipped with --no-a1, e.g. at 512^3 where
the host Galerkin product needs ~40 GB).

    python tools/pattern_census.py --n 128            # seconds
    python tools/pattern_census.py --n 512 --no-a1    # ~2 min, ~30 GB of host memory
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import parallel_amg_amd as pa  # noqa: E402
from parallel_amg_amd import hcsr as H  # noqa: E402


def row_patterns(rp, col, val):
    """Distinct (col - first col, value bits) row sequences: (count, total entries)."""
    lens = np.diff(rp)
    first = col[rp[:-1]]
    vb = val.view(np.int64)
    npat = ent = 0
    for L in np.unique(lens):
        rows = np.nonzero(lens == L)[0]
        idx = rp[rows][:, None] + np.arange(L)[None, :]
        key = np.concatenate([col[idx] - first[rows][:, None], vb[idx]], axis=1)
        u = np.unique(key, axis=0)
        npat += len(u)
        ent += len(u) * int(L)
    return npat, ent


def p0_combinations(P, n):
    rp, col, val = P.rowptr, P.col.astype(np.int64), P.val
    N = len(rp) - 1
    M = n * n
    lens = np.diff(rp)
    rows = np.repeat(np.arange(N), lens)
    order = np.lexsort((-val, rows))          # per row: the largest value first (the anchor)
    anc = col[order[rp[:-1]]]
    i = np.arange(N)
    x, y, z = i % n, (i // n) % n, i // M
    d = [0, -1, 1, -n, n, -M, M]
    inb = [np.ones(N, bool), x > 0, x < n - 1, y > 0, y < n - 1, z > 0, z < n - 1]
    code = np.full(len(col), 7, np.int64)
    for c in range(6, -1, -1):               # the first matching neighbour wins
        nb = np.clip(i + d[c], 0, N - 1)
        ok = inb[c][rows] & (anc[nb][rows] == col)
        code[ok] = c
    _, vi = np.unique(val.view(np.int64), return_inverse=True)
    k = np.arange(len(col)) - np.repeat(rp[:-1], lens)
    w1 = lens.astype(np.int64).copy()
    w2 = np.zeros(N, np.int64)
    np.add.at(w1, rows, code << (3 + 3 * k))
    np.add.at(w2, rows, vi.astype(np.int64) << (9 * k))
    return int(np.count_nonzero(code == 7)), len(np.unique(np.stack([w1, w2], axis=1), axis=0))


def a1_pairs(A1):
    rp, col, val = A1.rowptr, A1.col.astype(np.int64), A1.val
    rows = np.repeat(np.arange(len(rp) - 1), np.diff(rp))
    key = np.stack([rows // 256, col - rows, val.view(np.int64)], axis=1)
    cnt = np.bincount(np.unique(key, axis=0)[:, 0])
    return int(cnt.max()), float(cnt.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=128)
    ap.add_argument("--kind", default="poisson3d")
    ap.add_argument("--no-a1", action="store_true")
    a = ap.parse_args()
    be = pa.SequentialBackend(1)
    A, offs, xs = pa.generate_problem(be, a.kind, a.n)
    out = {"n": a.n, "kind": a.kind}
    if a.no_a1:
        A0 = A[0]
        omega = 4.0 / (3.0 * H.gershgorin(A0, 0))
        agg, nc = H.aggregate(A0, 0, 0.02)
        T = H.tentative(agg, nc, 0, nc)
        AT = H.spgemm(A0, 0, T, np.zeros(0, np.int64), None)
        P = H.smooth(A0, 0, T, AT, omega)
        del AT, T
        R = H.transpose(P, 0, 0, nc)
        del A, A0
    else:
        Hh = pa.build_hierarchy(be, A, offs, pa.SAParams())
        lp = Hh.levels[0][0]
        P, R = lp.P, lp.R
        out["A1_pairs_per_group_max"], out["A1_pairs_per_group_mean"] = a1_pairs(Hh.levels[1][0].A)
    out["R0_patterns"], out["R0_pattern_entries"] = row_patterns(R.rowptr, R.col.astype(np.int64), R.val)
    del R
    if a.kind != "aniso3d":
        out["P0_unmatched_entries"], out["P0_combinations"] = p0_combinations(P, a.n)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
