"""Hierarchy dump / load (SURVEY §5 checkpoint/resume: "a hierarchy dump/load (binary CSR) to
skip setup"). The parts a process holds (all of them for SequentialBackend, its own for
DistributedBackend) go to one ``.npz`` of plain arrays — no pickle — and load back into a
HostHierarchy that AMGSolver uploads exactly like a freshly built one.

    save_hierarchy(H, "h512.npz")                        # SequentialBackend: every part in one file
    save_hierarchy(H, "h512_{rank}.npz")                 # DistributedBackend: one file per rank
    H = load_hierarchy("h512_{rank}.npz", backend=be)    # checks the parts match be.parts

A hierarchy that holds only some of its parts (DistributedBackend) must be saved under a path
with a ``{rank}`` placeholder (filled with the first part it holds), so ranks on a shared
filesystem never overwrite each other's file.
"""
from __future__ import annotations

import numpy as np

from .hcsr import HCSR
from .hierarchy import HostHierarchy, HostPlan, LevelPart

_VERSION = 1


def _put_csr(d, key, M: HCSR | None):
    if M is None:
        return
    d[key + "_rp"], d[key + "_col"], d[key + "_val"] = M.rowptr, M.col, M.val
    d[key + "_nc"] = np.int64(M.ncols)


def _get_csr(z, key):
    if key + "_rp" not in z:
        return None
    return HCSR.from_arrays(z[key + "_rp"], z[key + "_col"], z[key + "_val"], int(z[key + "_nc"]))


def _put_plan(d, key, P: HostPlan | None):
    if P is None:
        return
    d[key + "_meta"] = np.array([P.n_own, P.col0], np.int64)
    d[key + "_ghost"] = np.asarray(P.ghost_ids, np.int64)
    d[key + "_nbrs"] = np.asarray(P.nbrs, np.int64)
    d[key + "_recv"] = np.asarray(P.recv_counts, np.int64)
    d[key + "_send"] = np.asarray(P.send_counts, np.int64)
    d[key + "_sidx"] = (np.asarray(P.send_idx, np.int64) if P.send_idx is not None
                        else np.zeros(0, np.int64))


def _get_plan(z, key):
    if key + "_meta" not in z:
        return None
    n_own, col0 = (int(v) for v in z[key + "_meta"])
    P = HostPlan(n_own=n_own, col0=col0, ghost_ids=z[key + "_ghost"])
    P.nbrs = [int(q) for q in z[key + "_nbrs"]]
    P.recv_counts = [int(c) for c in z[key + "_recv"]]
    P.send_counts = [int(c) for c in z[key + "_send"]]
    P.send_idx = z[key + "_sidx"]
    P._recv = {q: c for q, c in zip(P.nbrs, P.recv_counts) if c}
    off = np.concatenate([[0], np.cumsum(P.send_counts)]).astype(np.int64)
    P._send = {q: P.send_idx[off[k]:off[k + 1]] for k, q in enumerate(P.nbrs) if P.send_counts[k]}
    return P


def _resolve(path: str, parts) -> str:
    if "{rank}" in path:
        return path.replace("{rank}", str(min(parts)))
    return path


def save_hierarchy(H: HostHierarchy, path: str) -> None:
    parts = sorted(H.levels[0])
    if len(parts) < H.nparts and "{rank}" not in path:
        raise ValueError(f"{path}: this hierarchy holds parts {parts} of {H.nparts}; save it under a "
                         "path with a '{rank}' placeholder so every rank writes its own file")
    path = _resolve(path, parts)
    d = {"version": np.int64(_VERSION), "nparts": np.int64(H.nparts), "nlevels": np.int64(H.nlevels),
         "parts": np.asarray(sorted(H.levels[0]), np.int64), "ainv": np.asarray(H.ainv, np.float64),
         "n_coarse": np.int64(H.n_coarse), "rep_level": np.int64(H.rep_level),
         "rep_offsets": np.asarray(H.rep_offsets if H.rep_offsets is not None else [], np.int64)}
    for l, lev in enumerate(H.levels):
        for p, lp in lev.items():
            k = f"l{l}_p{p}"
            d[k + "_offsets"] = np.asarray(lp.offsets, np.int64)
            d[k + "_scal"] = np.array([lp.omega, lp.rho, float(lp.whole)], np.float64)
            if lp.agg is not None:
                d[k + "_agg"] = np.asarray(lp.agg)
            for w in ("A", "P", "R"):
                _put_csr(d, f"{k}_{w}", getattr(lp, w))
            for w in ("planA", "planP", "planR"):
                _put_plan(d, f"{k}_{w}", getattr(lp, w))
    with open(path, "wb") as f:
        np.savez(f, **d)


def load_hierarchy(path: str, backend=None) -> HostHierarchy:
    """Load a saved hierarchy; with ``backend`` the file must hold exactly ``backend.parts``
    (and ``{rank}`` in the path is filled with the backend's first part)."""
    if backend is not None:
        path = _resolve(path, backend.parts)
    elif "{rank}" in path:
        raise ValueError(f"{path}: a '{{rank}}' path needs the backend to resolve it")
    with np.load(path, allow_pickle=False) as z:
        if int(z["version"]) != _VERSION:
            raise ValueError(f"{path}: hierarchy file version {int(z['version'])} != {_VERSION}")
        parts = [int(p) for p in z["parts"]]
        if backend is not None and sorted(backend.parts) != parts:
            raise ValueError(f"{path}: holds parts {parts}, the backend has {sorted(backend.parts)}")
        levels = []
        for l in range(int(z["nlevels"])):
            lev = {}
            for p in parts:
                k = f"l{l}_p{p}"
                omega, rho, whole = (float(v) for v in z[k + "_scal"])
                lev[p] = LevelPart(A=_get_csr(z, k + "_A"), offsets=z[k + "_offsets"], omega=omega,
                                   rho=rho, planA=_get_plan(z, k + "_planA"),
                                   agg=z[k + "_agg"] if k + "_agg" in z else None,
                                   P=_get_csr(z, k + "_P"), R=_get_csr(z, k + "_R"),
                                   planP=_get_plan(z, k + "_planP"), planR=_get_plan(z, k + "_planR"),
                                   whole=bool(whole))
            levels.append(lev)
        ro = z["rep_offsets"]
        return HostHierarchy(int(z["nparts"]), parts, levels, z["ainv"], int(z["n_coarse"]),
                             rep_level=int(z["rep_level"]), rep_offsets=ro if len(ro) else None)
