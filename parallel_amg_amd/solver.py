"""Device AMG solver: uploads one part of a ``HostHierarchy`` and runs V-cycles (SPEC §S6).

``AMGSolver`` is the preconditioner object an AMG-on-PartitionedArrays driver would pass
around (``ldiv!``-style ``vcycle``); the cycle itself is one C-ABI call (``pamg_vcycle``),
replayed as a hipGraph on one part.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import call, ptr
from .hierarchy import HostHierarchy
from .partitioned import Context, PSparseMatrix, PVector, _release

OPS = ("jacobi_pre", "residual", "restrict", "prolong", "jacobi_post", "coarse")


REORDER = {"off": 0, "auto": 1, "on": 2, "agg": 3}


def plan_tag(level: int, op: str) -> int:
    """Tag of a hierarchy's column plan (pamg_plan_set_tag): 1 + 3 level + (A 0, P 1, R 2)."""
    return 1 + 3 * int(level) + "APR".index(op)


class _LevelOps:
    """Read-only sequence view of an AMGSolver's level operators: index 0 resolves through
    ``fine_operator()`` (the caller's numbering), every other index is ``A_dev[l]``."""

    def __init__(self, solver):
        self._s = solver

    def __len__(self):
        return len(self._s.A_dev)

    def __getitem__(self, l):
        if isinstance(l, slice):
            return [self[i] for i in range(*l.indices(len(self)))]
        l = range(len(self))[l]
        return self._s.fine_operator() if l == 0 else self._s.A_dev[l]

    def __iter__(self):
        return (self[i] for i in range(len(self)))


class AMGSolver:
    def __init__(self, ctx: Context, H: HostHierarchy, part: int = 0, graph: bool | None = None,
                 reorder: str = "auto"):
        """``reorder`` (one part only): a locality permutation of every level but the coarsest
        inside the device layout (pamg_locality_order / pamg_mat_upload_perm): "auto" takes
        reverse Cuthill-McKee on the levels whose numbering is scattered (FE meshes, random
        renumberings and the levels aggregated from them), "on" on every level, "off" never.
        A_l, P_l and R_l are uploaded through the fine and coarse permutations with each row
        in its storage order, and the V-cycle gathers / scatters the caller's level-0 vectors
        (pamg_hier_set_perm), so every result keeps the unpermuted hierarchy's bits."""
        self.ctx, self.part, self.L = ctx, part, H.nlevels
        # the level operators as the hierarchy holds them (device numbering where permuted);
        # ``A`` (below) gives level 0 in the caller's numbering
        self.A_dev, self.P, self.R, self.omega = [], [], [], []
        self._A0_caller = None
        self._H = H
        # levels >= rep are whole on every part (agglomerated tail / coarsest level): the
        # prolongation into rep - 1 reads that whole vector, so its columns stay global
        rep = H.rep_level if H.nparts > 1 else H.nlevels - 1
        mode = REORDER[reorder]
        if H.nparts > 1 and mode == 2:
            raise ValueError("reorder='on' needs a one-part hierarchy (renumber a partitioned "
                             "matrix before setup: partition='rcm')")
        # per level: device row i = host row perm[l][i] (None: identity); the coarsest level
        # keeps its numbering (its dense inverse sums in column order)
        self.perm = [None] * H.nlevels
        self.span = [None] * H.nlevels
        if H.nparts == 1 and mode == REORDER["agg"]:
            # levels 1 .. L-2 in the order of their coarse aggregates: the nodes
            # of one level-(l+1) aggregate become a contiguous run — R_l's rows read runs of the
            # level-l vector instead of ~25 scattered lines — each aggregate's nodes in their own
            # order, the aggregates in coarse-row order; level 0 keeps its grid layout
            for l in range(1, H.nlevels - 1):
                agg = H.levels[l][part].agg
                if agg is None or len(agg) != H.levels[l][part].A.nrows:
                    continue
                agg = np.asarray(agg, np.int64)
                key = np.where(agg < 0, np.int64(1) << 40, agg)
                self.perm[l] = np.argsort(key, kind="stable").astype(np.int64)
        elif H.nparts == 1 and mode:
            from .hcsr import locality_order
            for l in range(H.nlevels - 1):
                order, before, after = locality_order(H.levels[l][part].A, mode)
                self.perm[l] = order
                self.span[l] = (round(before, 1), round(after, 1))
        for l in range(H.nlevels):
            lp = H.levels[l][part]
            pl = self.perm[l]
            pn = self.perm[l + 1] if l + 1 < H.nlevels else None
            # plan tags (pamg_plan_set_tag): level and operator, the same on every part
            self.A_dev.append(PSparseMatrix(ctx, lp.A, lp.planA, row_perm=pl, col_perm=pl, tag=plan_tag(l, "A")))
            self.omega.append(lp.omega)
            if l < H.nlevels - 1:
                self.P.append(PSparseMatrix(ctx, lp.P, None if l + 1 >= rep else lp.planP,
                                            row_perm=pl, col_perm=pn, tag=plan_tag(l, "P")))
                self.R.append(PSparseMatrix(ctx, lp.R, lp.planR, row_perm=pn, col_perm=pl, tag=plan_tag(l, "R")))
        self.level_rows = [int(H.levels[l][part].A.nrows) for l in range(H.nlevels)]
        self.n_coarse = H.n_coarse
        L = self.L
        arrA = (C.c_void_p * L)(*[a.handle for a in self.A_dev])
        arrP = (C.c_void_p * L)(*([p.handle for p in self.P] + [None]))
        arrR = (C.c_void_p * L)(*([r.handle for r in self.R] + [None]))
        om = np.asarray(self.omega, np.float64)
        roffs = np.asarray(H.rep_offsets, np.int64) if H.nparts > 1 else None
        self.rep_level = rep
        self._ainv = np.ascontiguousarray(H.ainv, np.float64)
        h = C.c_void_p()
        call("pamg_hier_create", ctx.handle, L, arrA, arrP, arrR, ptr(om), H.n_coarse,
             ptr(self._ainv), int(rep), ptr(roffs) if roffs is not None else None, C.byref(h))
        self._h = h
        if self.perm[0] is not None:
            p0 = np.ascontiguousarray(self.perm[0], np.int64)
            call("pamg_hier_set_perm", h, len(p0), ptr(p0))
        if graph is not None:
            self.set_graph(graph)

    @property
    def A(self) -> "_LevelOps":
        """The level operators, level 0 in the CALLER's numbering (b = A[0] x, residuals of the
        caller's vectors): the hierarchy's own A_0 when level 0 is not permuted, else an
        unpermuted upload made on first use of index 0 (``fine_operator``; ADVICE r4: ``A[l]``
        for l >= 1 never triggers it). Levels >= 1 are internal to the cycle and listed as the
        hierarchy holds them (``A_dev``)."""
        return _LevelOps(self)

    @property
    def reordered(self) -> list:
        """Levels whose device layout carries a locality permutation."""
        return [l for l, p in enumerate(self.perm) if p is not None]

    def fine_operator(self) -> PSparseMatrix:
        """The level-0 operator in the caller's numbering (for b = A x and residuals of the
        caller's vectors): the hierarchy's own A_0 when level 0 is not permuted, else an
        unpermuted upload (made once, kept)."""
        if self.perm[0] is None:
            return self.A_dev[0]
        if self._A0_caller is None:
            lp = self._H.levels[0][self.part]
            self._A0_caller = PSparseMatrix(self.ctx, lp.A, lp.planA)
        return self._A0_caller

    @property
    def handle(self):
        return self._h

    def set_graph(self, enable: bool):
        call("pamg_hier_set_graph", self._h, int(bool(enable)))

    def set_sweeps(self, nu1: int, nu2: int):
        """V(nu1, nu2) weighted-Jacobi sweeps (SPEC §S6; default V(1, 1))."""
        call("pamg_hier_set_sweeps", self._h, int(nu1), int(nu2))

    def graph_state(self) -> dict:
        e, c, f = C.c_int(), C.c_int(), C.c_int()
        call("pamg_hier_graph_state", self._h, C.byref(e), C.byref(c), C.byref(f))
        return {"enabled": bool(e.value), "captured": bool(c.value), "failed": bool(f.value)}

    def new_vector(self) -> PVector:
        """A level-0 vector with room for the fine-level ghosts."""
        return self.A_dev[0].new_input_vector()

    def vcycle(self, x: PVector, b: PVector, ncycles: int = 1, res_hist: bool = False):
        if res_hist:
            hist = np.zeros(ncycles)
            call("pamg_vcycle", self.ctx.handle, self._h, x.handle, b.handle, ncycles, ptr(hist))
            return hist
        call("pamg_vcycle", self.ctx.handle, self._h, x.handle, b.handle, ncycles, None)
        return None

    def pcg(self, x: PVector, b: PVector, rtol: float = 1e-8, maxit: int = 100):
        """CG preconditioned by one V-cycle (SPEC §S8); returns (iterations, ||r_k|| history)."""
        hist = np.zeros(maxit + 1)
        it = C.c_int()
        call("pamg_pcg", self.ctx.handle, self._h, x.handle, b.handle, float(rtol), int(maxit),
             C.byref(it), ptr(hist))
        return it.value, hist[: it.value + 1]

    def vcycle_async(self, x: PVector, b: PVector, ncycles: int = 1):
        call("pamg_vcycle_async", self.ctx.handle, self._h, x.handle, b.handle, ncycles)

    def bench_chain(self, x: PVector, b: PVector, reps: int = 10):
        """ms per launch of the cross-cycle pipeline's level-0 chain kernel (None when the
        hierarchy does not run the pipeline); x is overwritten."""
        from ._lib import PamgError
        ms = C.c_double()
        try:
            call("pamg_hier_bench_chain", self._h, x.handle, b.handle, int(reps), C.byref(ms))
        except PamgError:
            return None
        return ms.value

    def profile(self, x: PVector, b: PVector, ncycles: int) -> np.ndarray:
        """Eager V-cycles with HIP events around every op; returns ms per (level, op) summed
        over the cycles (shape L x 6, columns = OPS)."""
        call("pamg_hier_profile", self._h, 1)
        try:
            call("pamg_vcycle_async", self.ctx.handle, self._h, x.handle, b.handle, ncycles)
            out = np.zeros(self.L * 6)
            call("pamg_hier_profile_read", self._h, ptr(out))
        finally:
            call("pamg_hier_profile", self._h, 0)
        return out.reshape(self.L, 6)

    # ---- algorithmic byte model (SURVEY.md §8d / BASELINE.md) --------------------------
    @staticmethod
    def rowsum_bytes(M, extra_vec_rw: int) -> int:
        """Algorithmic bytes of one row operation of the device matrix M: the
        matrix stream in its uploaded layout (pamg_mat_stream_bytes: 8 B values + 4 B, or 3 B
        in 24-bit column tiles, columns per nonzero + row pointers + tile descriptors) + 8 B per
        x entry read once + 8 B per output row + 8 B per extra own vector read or written."""
        return M.stream_bytes + 8 * (M.n_own_cols + M.n_ghost) + 8 * M.nrows + 8 * M.nrows * extra_vec_rw

    @staticmethod
    def csr_bytes(M, extra_vec_rw: int) -> int:
        """SURVEY §8(d)'s algorithmic bytes of one row operation, independent of the device
        layout: plain CSR with 32-bit indices (12 B per nonzero + 4 B per row pointer) + 8 B
        per x entry read once + 8 B per output row + 8 B per extra own vector read or written
        (b; the diagonal is read inline). The layouts libpamg uploads (24-bit columns, 8-bit
        row lengths, column dictionaries) stream fewer bytes than this (rowsum_bytes)."""
        return (12 * M.nnz + 4 * (M.nrows + 1) + 8 * (M.n_own_cols + M.n_ghost) + 8 * M.nrows
                + 8 * M.nrows * extra_vec_rw)

    def op_bytes(self, model: str = "format") -> np.ndarray:
        """Bytes per (level, op) of one V-cycle on this part (L x 6): model "format" = what
        the uploaded layout streams (rowsum_bytes), "csr" = SURVEY §8(d)'s CSR model."""
        rb = self.rowsum_bytes if model == "format" else self.csr_bytes
        out = np.zeros((self.L, 6))
        for l in range(self.L):
            n = self.level_rows[l]
            if l == self.L - 1:
                nc = self.n_coarse
                out[l, 5] = 8 * nc * n + 8 * nc + 8 * n
                continue
            A, P, R = self.A_dev[l], self.P[l], self.R[l]
            # jacobi: x (read once), b, x' ; zero-guess form on l >= 1 reads b, diag, writes x'
            out[l, 0] = rb(A, 1) if l == 0 else 24 * n
            out[l, 1] = rb(A, 1)
            out[l, 2] = rb(R, 0)
            out[l, 3] = rb(P, 1)
            out[l, 4] = rb(A, 1)
        return out

    def __del__(self):
        _release(self, "pamg_hier_destroy")
