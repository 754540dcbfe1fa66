"""Host-side smoothed-aggregation setup over a partitioned matrix (SPEC.md §S4, §S5, §S7).

Written the way an AMG setup on top of PartitionedArrays (reference README.md:2) is written:
per-part kernels (the C++ routines of ``csrc/setup.cpp``, bound in ``hcsr.py``) separated by
neighbour exchanges of ghost rows (``backend.exchange``). The result is bit-identical to the
global-view oracle for any number of parts because every product of §S4 is defined on the
global matrices and evaluated in the same order (§S4.5).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import hcsr as H
from .hcsr import HCSR

KIND = {"poisson2d": 0, "poisson3d": 1, "aniso3d": 2, "elastic3d": 3}
SEED = 20240807


@dataclass
class SAParams:
    theta: float = 0.02
    max_levels: int = 20
    max_coarse: int = 1000
    # SPEC §S7 agglomeration: levels >= 1 with <= this many global rows are built as one part
    # and replicated on every part; 0 = decoupled on every level
    agglomerate: int = 32768


@dataclass
class HostPlan:
    """One part's ghost layout of a column space (a PartitionedArrays PRange part): ghost
    global ids (ascending, so grouped by owner), plus the neighbour lists of the exchange."""
    n_own: int
    col0: int
    ghost_ids: np.ndarray
    nbrs: list = field(default_factory=list)          # union of send/recv neighbours, ascending
    recv_counts: list = field(default_factory=list)   # per nbr: ghosts owned by nbr
    send_counts: list = field(default_factory=list)   # per nbr: own entries nbr needs
    send_idx: np.ndarray = None                       # local own indices, concatenated per nbr
    _send: dict = field(default_factory=dict)         # nbr -> local own indices
    _recv: dict = field(default_factory=dict)         # nbr -> number of ghosts it owns

    @property
    def n_ghost(self):
        return len(self.ghost_ids)

    def localize(self, col: np.ndarray) -> np.ndarray:
        """Global column ids -> local ids (own first, then ghosts), int32."""
        col = np.asarray(col, np.int64)
        out = col - self.col0
        g = (out < 0) | (out >= self.n_own)
        if np.any(g):
            out[g] = self.n_own + np.searchsorted(self.ghost_ids, col[g])
        return out.astype(np.int32)


def owners_of(ids: np.ndarray, offsets: np.ndarray) -> np.ndarray:
    return np.searchsorted(offsets, ids, side="right") - 1


def ghost_ids(M: HCSR, lo: int, hi: int) -> np.ndarray:
    c = M.col
    if M.nnz == 0:
        return np.zeros(0, np.int64)
    m = (c < lo) | (c >= hi)
    return np.unique(c[m]).astype(np.int64)


def build_plans(backend, ghosts: dict, offsets: np.ndarray) -> dict:
    """Request exchange: every part tells each owner which of its rows it holds as ghosts."""
    plans, reqs = {}, {}
    for p in backend.parts:
        g = ghosts[p]
        own = owners_of(g, offsets)
        nb, cnt = np.unique(own, return_counts=True)
        plans[p] = HostPlan(n_own=int(offsets[p + 1] - offsets[p]), col0=int(offsets[p]), ghost_ids=g)
        plans[p]._recv = dict(zip(nb.tolist(), cnt.tolist()))
        reqs[p] = {int(q): (g[own == q],) for q in nb.tolist()}
    got = backend.exchange(reqs)
    for p in backend.parts:
        P = plans[p]
        P._send = {q: (ids - offsets[p]).astype(np.int64) for q, (ids,) in got[p].items()}
        nbrs = sorted(set(P._recv) | set(P._send))
        P.nbrs = nbrs
        P.recv_counts = [P._recv.get(q, 0) for q in nbrs]
        P.send_counts = [len(P._send.get(q, ())) for q in nbrs]
        P.send_idx = (np.concatenate([P._send[q] for q in nbrs if q in P._send])
                      if P._send else np.zeros(0, np.int64))
    return plans


def fetch_rows(backend, plans: dict, mats: dict) -> dict:
    """Ghost rows of ``mats`` for every part's plan (the response half of the exchange)."""
    resp = {p: {q: mats[p].rows(idx) for q, idx in plans[p]._send.items()} for p in backend.parts}
    got = backend.exchange(resp)
    out = {}
    for p in backend.parts:
        P = plans[p]
        if P.n_ghost == 0:
            out[p] = None
            continue
        rps, cols, vals = [np.zeros(1, np.int64)], [], []
        base = 0
        for q in sorted(got[p]):
            rp, c, v = got[p][q]
            rps.append(rp[1:] + base)
            base += int(rp[-1])
            cols.append(c)
            vals.append(v)
        rp = np.concatenate(rps)
        if len(rp) - 1 != P.n_ghost:
            raise RuntimeError("fetch_rows: ghost row count mismatch")
        ncols = max((m.ncols for m in mats.values()), default=0)
        out[p] = HCSR.from_arrays(rp, np.concatenate(cols) if cols else np.zeros(0, np.int32),
                                  np.concatenate(vals) if vals else np.zeros(0), ncols)
    return out


@dataclass
class LevelPart:
    A: HCSR
    offsets: np.ndarray
    omega: float
    rho: float
    planA: HostPlan = None
    agg: np.ndarray = None          # local aggregate ids (-1 isolated)
    P: HCSR = None                  # own fine rows x global coarse cols
    R: HCSR = None                  # own coarse rows (next level) x global fine cols
    planP: HostPlan = None          # column space: next level
    planR: HostPlan = None          # column space: this level
    whole: bool = False             # agglomerated level: every part holds all rows (§S7)


@dataclass
class HostHierarchy:
    nparts: int
    parts: list
    levels: list            # list of dict part -> LevelPart
    ainv: np.ndarray        # column-major n_c x n_c (SPEC §S5)
    n_coarse: int
    # first level held whole on every part (agglomerated tail; the coarsest level otherwise)
    # and how the restriction into it distributes its rows over the parts
    rep_level: int = 0
    rep_offsets: np.ndarray = None

    @property
    def nlevels(self):
        return len(self.levels)

    def offsets(self, l):
        return next(iter(self.levels[l].values())).offsets

    def nnz(self, l, which="A"):
        lps = list(self.levels[l].values())
        if lps[0].whole:
            lps = lps[:1]
        return sum(getattr(lp, which).nnz for lp in lps if getattr(lp, which) is not None)

    def part_rows(self, l, which="A"):
        """The level's matrix as the list of distinct row blocks in part order (one block for a
        whole, agglomerated level)."""
        lps = [self.levels[l][p] for p in sorted(self.levels[l])]
        return [getattr(lps[0], which)] if lps[0].whole else [getattr(lp, which) for lp in lps]


def generate_problem(backend, kind: str, n: int, eps: float = 1e-3):
    """Partitioned rows of the SPEC §S2 operator and the right-hand side b = A x*.

    Returns (A_parts, offsets, xstar_parts). b is formed by the caller's SpMV (device, §S3),
    or with ``spmv_host`` for CPU use."""
    nx, ny, nz = (n, n, 1) if kind == "poisson2d" else (n, n, n)
    N = nx * ny * nz * (3 if kind == "elastic3d" else 1)
    offs = np.array([(p * N) // backend.nparts for p in range(backend.nparts + 1)], np.int64)
    A = {p: H.gen_grid(KIND[kind], nx, ny, nz, eps, int(offs[p]), int(offs[p + 1])) for p in backend.parts}
    xs = {p: H.gen_xstar(int(offs[p]), int(offs[p + 1] - offs[p]), SEED) for p in backend.parts}
    return A, offs, xs


def permutation(n: int, seed: int) -> np.ndarray:
    """The seeded random permutation ``permute_problem`` applies: new row i is old row perm[i]."""
    return np.random.default_rng(seed).permutation(n).astype(np.int64)


def reorder(M: HCSR, perm: np.ndarray) -> HCSR:
    """Symmetric permutation Q M Q^T of a square host matrix: new row i is old row perm[i];
    rows keep their columns sorted ascending (SPEC §S1)."""
    n = M.nrows
    inv = np.empty(n, np.int64)
    inv[perm] = np.arange(n, dtype=np.int64)
    lens = np.diff(M.rowptr)[perm]
    rp = np.zeros(n + 1, np.int64)
    np.cumsum(lens, out=rp[1:])
    src = np.repeat(M.rowptr[perm], lens) + (np.arange(rp[-1], dtype=np.int64) - np.repeat(rp[:-1], lens))
    col = inv[M.col[src]]
    val = M.val[src]
    # sort each row's columns: one global stable sort on (row, col)
    row = np.repeat(np.arange(n, dtype=np.int64), lens)
    order = np.lexsort((col, row))
    return HCSR.from_arrays(rp, col[order].astype(np.int32), val[order], M.ncols)


def permute_problem(A: dict, xs: dict, seed: int):
    """Symmetric permutation Q A Q^T of a one-part problem, x* permuted alike (bench
    ``--permute``). A grid operator renumbered at random keeps its values and nonzero counts
    but loses the banded, row-relative column pattern that the column dictionaries and the
    banded tile order exploit, as an FE mesh numbering would (a Flan_1565 proxy)."""
    if set(A) != {0}:
        raise ValueError("permute_problem: one part only")
    perm = permutation(A[0].nrows, seed)
    return {0: reorder(A[0], perm)}, {0: np.ascontiguousarray(xs[0][perm])}


def rcm_problem(A: dict, xs: dict):
    """Reverse Cuthill-McKee renumbering of a one-part problem (the graph partitioner,
    pamg_rcm_order), x* permuted alike; split it afterwards with ``split_problem``."""
    if set(A) != {0}:
        raise ValueError("rcm_problem: one part only")
    perm = H.rcm_order(A[0])
    return {0: reorder(A[0], perm)}, {0: np.ascontiguousarray(xs[0][perm])}, perm


def split_problem(backend, A: dict, xs: dict, partition: str = "nnz"):
    """Cut a whole (one-part) problem into the backend's parts: contiguous row blocks, uniform
    or nnz-balanced (SPEC §S7). Every rank holds the whole problem and keeps its own rows."""
    M = A[0]
    if partition == "nnz":
        offs = balanced_offsets(np.diff(M.rowptr), backend.nparts)
    else:
        offs = np.array([(p * M.nrows) // backend.nparts for p in range(backend.nparts + 1)], np.int64)
    parts = {}
    for p in backend.parts:
        a, b = int(offs[p]), int(offs[p + 1])
        lo, hi = int(M.rowptr[a]), int(M.rowptr[b])
        parts[p] = HCSR.from_arrays(M.rowptr[a:b + 1] - lo, M.col[lo:hi].copy(), M.val[lo:hi].copy(), M.ncols)
    return parts, offs, {p: np.ascontiguousarray(xs[0][offs[p]:offs[p + 1]]) for p in backend.parts}


def balanced_offsets(row_counts: np.ndarray, nparts: int) -> np.ndarray:
    """SPEC §S7 nnz-balanced partition: o_p = first row r with sum_{i<r} len_i >= floor(p*nnz/P)."""
    pre = np.zeros(len(row_counts) + 1, np.int64)
    np.cumsum(row_counts, out=pre[1:])
    tot = int(pre[-1])
    targets = np.array([(p * tot) // nparts for p in range(nparts + 1)], np.int64)
    offs = np.searchsorted(pre, targets, side="left").astype(np.int64)
    offs[0], offs[-1] = 0, len(row_counts)
    return offs


def load_problem(backend, path: str, partition: str = "uniform"):
    """Partitioned rows of a Matrix Market matrix (pamg_read_mtx; BASELINE.json configs[4],
    SuiteSparse Flan_1565) and the SPEC §S2 synthetic solution x* for b = A x*. Each part reads
    only its own rows; the partition is SPEC §S7's uniform one, or nnz-balanced
    (``partition="nnz"``: equal nonzeros per part, for matrices with irregular rows), or
    ``partition="rcm"``: the graph partitioner — rank 0 reads the whole matrix and computes the
    reverse Cuthill-McKee order and the nnz-balanced blocks of the renumbered rows, broadcasts
    them, and every rank reads only its own block's rows (pamg_read_mtx_rows) and renumbers
    their columns; x* is drawn in the new numbering (so it differs from other partitions')."""
    if partition == "rcm":
        if not backend.distributed:  # every part in this process: one read, one renumbering
            M, N = H.read_mtx(path)
            perm = H.rcm_order(M)
            R = reorder(M, perm)
            del M
            return split_problem(backend, {0: R}, {0: H.gen_xstar(0, N, SEED)}, "nnz")
        me = backend.rank
        perm = offs = None
        if me == 0:
            M, N = H.read_mtx(path)
            perm = H.rcm_order(M)
            offs = balanced_offsets(np.diff(M.rowptr)[perm], backend.nparts)
            del M
        perm = backend.broadcast_array(perm, np.int64)
        offs = backend.broadcast_array(offs, np.int64)
        N = len(perm)
        inv = np.empty(N, np.int64)
        inv[perm] = np.arange(N, dtype=np.int64)
        Mp, _ = H.read_mtx_rows(path, perm[offs[me]:offs[me + 1]])
        # columns into the new numbering, each row sorted ascending (as reorder() leaves them)
        lens = np.diff(Mp.rowptr)
        row = np.repeat(np.arange(Mp.nrows, dtype=np.int64), lens)
        col = inv[Mp.col]
        order = np.lexsort((col, row))
        A = {me: HCSR.from_arrays(Mp.rowptr.copy(), col[order].astype(np.int32), Mp.val[order], N)}
        return A, offs, {me: H.gen_xstar(int(offs[me]), int(offs[me + 1] - offs[me]), SEED)}
    head = H.read_mtx(path, 0, 0)
    N = head[1]
    if partition == "nnz" and backend.nparts > 1:
        offs = balanced_offsets(H.mtx_row_counts(path), backend.nparts)
    else:
        offs = np.array([(p * N) // backend.nparts for p in range(backend.nparts + 1)], np.int64)
    A = {p: H.read_mtx(path, int(offs[p]), int(offs[p + 1]))[0] for p in backend.parts}
    xs = {p: H.gen_xstar(int(offs[p]), int(offs[p + 1] - offs[p]), SEED) for p in backend.parts}
    return A, offs, xs


def build_hierarchy(backend, A: dict, offsets: np.ndarray, params: SAParams = SAParams(),
                    log=None, device=None, _level0: int = 0) -> HostHierarchy:
    """SPEC §S4: levels until n <= max_coarse / max_levels / stalled coarsening.

    ``device`` (a partitioned.Context): the Galerkin products (A T, A P, R (A P)) and the
    transposes run on that GPU (spgemm.hip) — bit-identical to the host routines;
    strength, aggregation and the coarsest inverse stay on the host (§8f-4)."""
    dv = device
    parts = backend.parts
    offs = np.asarray(offsets, np.int64)
    levels = []
    while True:
        n = int(offs[-1])
        if backend.nparts > 1 and levels and 0 < params.agglomerate and n <= params.agglomerate:
            return _replicated_tail(backend, A, offs, levels, params, log, device)
        rho = backend.allreduce_max({p: H.gershgorin(A[p], int(offs[p])) for p in parts})
        omega = 4.0 / (3.0 * rho)
        ghosts = {p: (ghost_ids(A[p], int(offs[p]), int(offs[p + 1])) if backend.nparts > 1
                      else np.zeros(0, np.int64)) for p in parts}
        planA = build_plans(backend, ghosts, offs)
        lev = {p: LevelPart(A=A[p], offsets=offs, omega=omega, rho=rho, planA=planA[p]) for p in parts}
        levels.append(lev)
        if n <= params.max_coarse or len(levels) >= params.max_levels:
            break
        aggs = {p: H.aggregate(A[p], int(offs[p]), params.theta) for p in parts}
        nagg = backend.allgather({p: aggs[p][1] for p in parts})
        coffs = np.zeros(backend.nparts + 1, np.int64)
        np.cumsum(nagg, out=coffs[1:])
        nc = int(coffs[-1])
        if nc == 0 or nc >= n:
            break
        T = {p: H.tentative(aggs[p][0], aggs[p][1], int(coffs[p]), nc) for p in parts}
        Tg = fetch_rows(backend, planA, T)
        P = {}
        for p in parts:
            AT = H.spgemm(A[p], int(offs[p]), T[p], planA[p].ghost_ids, Tg[p], device=dv)
            P[p] = H.smooth(A[p], int(offs[p]), T[p], AT, omega)
        del T, Tg
        Pg = fetch_rows(backend, planA, P)
        AP = {p: H.spgemm(A[p], int(offs[p]), P[p], planA[p].ghost_ids, Pg[p], device=dv) for p in parts}
        del Pg
        # R = P^T: each part transposes its rows per coarse owner and ships the pieces
        pieces_local, sends = {}, {}
        for p in parts:
            qs = (np.unique(owners_of(np.unique(P[p].col).astype(np.int64), coffs)).tolist()
                  if backend.nparts > 1 else [p])
            sends[p] = {}
            for q in qs:
                piece = H.transpose(P[p], int(offs[p]), int(coffs[q]), int(coffs[q + 1]), device=dv)
                if q == p:
                    pieces_local[p] = piece
                else:
                    sends[p][q] = (piece.rowptr.copy(), piece.col.copy(), piece.val.copy())
        got = backend.exchange(sends)
        R = {}
        for q in parts:
            nrows_q = int(coffs[q + 1] - coffs[q])
            plist = []
            for p in sorted(set(got[q]) | ({q} if q in pieces_local else set())):
                if p == q:
                    plist.append(pieces_local[q])
                else:
                    rp, c, v = got[q][p]
                    plist.append(HCSR.from_arrays(rp, c, v, n))
            if not plist:
                plist = [HCSR.from_arrays(np.zeros(nrows_q + 1, np.int64), np.zeros(0, np.int32), np.zeros(0), n)]
            R[q] = plist[0] if len(plist) == 1 else H.hstack_rows(plist)
        ghR = {q: (ghost_ids(R[q], int(offs[q]), int(offs[q + 1])) if backend.nparts > 1
                   else np.zeros(0, np.int64)) for q in parts}
        planR = build_plans(backend, ghR, offs)
        APg = fetch_rows(backend, planR, AP)
        Ac = {q: H.spgemm(R[q], int(offs[q]), AP[q], planR[q].ghost_ids, APg[q], device=dv) for q in parts}
        del AP, APg
        ghP = {p: (ghost_ids(P[p], int(coffs[p]), int(coffs[p + 1])) if backend.nparts > 1
                   else np.zeros(0, np.int64)) for p in parts}
        planP = build_plans(backend, ghP, coffs)
        for p in parts:
            lp = lev[p]
            lp.agg, lp.P, lp.R, lp.planP, lp.planR = aggs[p][0], P[p], R[p], planP[p], planR[p]
        if log:
            log(f"level {_level0 + len(levels) - 1}: n={n} nnz={sum(A[p].nnz for p in parts)} -> n_c={nc}")
        A, offs = Ac, coffs
    # coarsest level: every part assembles the full matrix and the same Cholesky inverse
    last = levels[-1]
    if backend.nparts == 1:
        full = last[parts[0]].A
    else:
        full = _gather_full(backend, {p: last[p].A for p in parts}, offs)
    ainv = H.cholinv(full)
    return HostHierarchy(backend.nparts, parts, levels, ainv, int(offs[-1]),
                         rep_level=len(levels) - 1, rep_offsets=offs)


def _replicated_tail(backend, A: dict, offs, levels: list, params: SAParams, log, device):
    """SPEC §S7 agglomeration: gather the level on every part and set up the rest of the
    hierarchy as one part (the same work on every part, so the replicas are identical)."""
    from dataclasses import replace
    from .backend import SequentialBackend
    n = int(offs[-1])
    full = _gather_full(backend, A, offs)
    # the tail's products run where the rest of the setup's do (device or host: the same bits).
    # Round 3 kept them on the host after a tail level came out without its diagonal (8 ranks
    # sharing one GPU); the cause was spgemm.hip's overflow-row path, whose table offsets were
    # copied asynchronously from a host vector freed before the copy had run (fixed; DESIGN.md,
    # Correctness tooling) — these wide rows are the ones that overflow the LDS tables
    sub = build_hierarchy(SequentialBackend(1), {0: full}, np.array([0, n], np.int64),
                          replace(params, agglomerate=0, max_levels=params.max_levels - len(levels)),
                          (lambda m: log(m + " (whole on every part)")) if log else None, device,
                          _level0=len(levels))
    for p in backend.parts:  # the prolongation into the tail reads the whole vector
        levels[-1][p].planP = None
    for l in range(sub.nlevels):
        lp = sub.levels[l][0]
        lp.offsets = np.array([0] + [lp.A.nrows] * backend.nparts, np.int64)
        lp.whole = True
        levels.append({p: lp for p in backend.parts})
    return HostHierarchy(backend.nparts, backend.parts, levels, sub.ainv, sub.n_coarse,
                         rep_level=len(levels) - sub.nlevels, rep_offsets=np.asarray(offs, np.int64))


def _gather_full(backend, A: dict, offs) -> HCSR:
    from .backend import pack_arrays, unpack_arrays
    n = int(offs[-1])
    if not backend.distributed:
        pieces = [(A[p].rowptr, A[p].col, A[p].val) for p in range(backend.nparts)]
    else:
        me = backend.rank
        bufs = backend.allgather_bytes(pack_arrays((A[me].rowptr, A[me].col, A[me].val)))
        pieces = [unpack_arrays(b) for b in bufs]
    rps, cols, vals, base = [np.zeros(1, np.int64)], [], [], 0
    for rp, c, v in pieces:
        rps.append(np.asarray(rp[1:]) + base)
        base += int(rp[-1])
        cols.append(c)
        vals.append(v)
    return HCSR.from_arrays(np.concatenate(rps), np.concatenate(cols), np.concatenate(vals), n)


def spmv_host(A: HCSR, x_full: np.ndarray) -> np.ndarray:
    """Host row sums in SPEC §S3 order via scipy would not match bit for bit; this helper is
    only used for sizes where the per-row Python loop is cheap (tests)."""
    y = np.zeros(A.nrows)
    for i in range(A.nrows):
        s = 0.0
        for k in range(A.rowptr[i], A.rowptr[i + 1]):
            s = s + A.val[k] * x_full[A.col[k]]
        y[i] = s
    return y
