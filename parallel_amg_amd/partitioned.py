"""Device PartitionedArrays surface over libpamg (reference README.md:2).

PartitionedArrays.jl names → this module:

=========================================  ==========================================
``PRange`` part (own + ghost ids)          ``HostPlan`` (hierarchy.py) → ``DevicePlan``
``PVector``                                ``PVector`` (own values then ghost slots)
``PSparseMatrix`` part                     ``PSparseMatrix`` (own rows, local columns)
``mul!(y, A, x)``                          ``mul(y, A, x)``
``consistent!(x) |> wait``                 ``consistent(x, plan)``
``t = consistent!(x); …; wait(t)``         ``t = consistent_async(x, plan); …; t.wait()``
``own_values(x)``                          ``x.own_values()``
``dot(x, y)`` / ``norm(x)``                ``dot(x, y)`` / ``norm(x)``
``axpy!`` / ``copy!`` / ``fill!``          ``axpby`` / ``copy`` / ``fill``
=========================================  ==========================================

One process drives one GPU and one part (the ``with_mpi`` shape); with more than one part
the context owns an RCCL communicator and ``mul`` overlaps the RCCL ghost exchange with the
interior rows. ``LocalWorld`` is the ``with_debug`` shape: every part in this process, one
context per part (on one GPU or several), exchanges by device-to-device copies between sibling
vectors. Everything here calls the C-ABI; there is no host fallback.
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from . import _lib as _L
from ._lib import call, ptr
from .hcsr import HCSR
from .hierarchy import HostPlan


def _release(obj, fn):
    """Destroy a libpamg handle once. During interpreter shutdown nothing is called: the
    process is ending, and objects a failed test's traceback kept alive are collected after the
    HIP runtime has begun its own teardown (a destroy call then can abort the process)."""
    h = getattr(obj, "_h", None)
    lib = getattr(_L, "_lib", None) if _L is not None else None
    if sys is None or sys.is_finalizing():
        obj._h = None
        return
    if h and lib is not None:
        try:
            getattr(lib, fn)(h)
        except Exception:  # pragma: no cover - shutdown ordering
            pass
    obj._h = None


HOST_COMM_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_int32),
                           C.POINTER(C.c_int64), C.POINTER(C.c_double), C.POINTER(C.c_int64),
                           C.POINTER(C.c_double))


def _host_comm_callback(backend):
    """pamg_host_comm_fn over torch.distributed (gloo): op 0 neighbour exchange, 1 all-gather,
    2 all-reduce (see include/pamg.h)."""
    import torch
    dist, group = backend.dist, backend.group

    def view(p, n):
        return np.ctypeslib.as_array(p, (n,)) if n else np.zeros(0)

    def fn(_user, op, n, peer, sc, sbuf, rc, rbuf):
        try:
            if op == 0:
                ns = sum(sc[k] for k in range(n))
                nr = sum(rc[k] for k in range(n))
                s_all, r_all = view(sbuf, ns), view(rbuf, nr)
                reqs, so, ro = [], 0, 0
                recvs = []
                for k in range(n):
                    q = int(peer[k])
                    if sc[k]:
                        t = torch.from_numpy(s_all[so:so + sc[k]].copy())
                        reqs.append(dist.isend(t, dst=q, group=group))
                    if rc[k]:
                        t = torch.empty(rc[k], dtype=torch.float64)
                        reqs.append(dist.irecv(t, src=q, group=group))
                        recvs.append((ro, t))
                    so += sc[k]
                    ro += rc[k]
                for r in reqs:
                    r.wait()
                for o, t in recvs:
                    r_all[o:o + len(t)] = t.numpy()
            elif op == 1:
                cnt = sc[0]
                t = torch.from_numpy(view(sbuf, cnt).copy())
                outs = [torch.empty(cnt, dtype=torch.float64) for _ in range(backend.nparts)]
                dist.all_gather(outs, t, group=group)
                r_all = view(rbuf, cnt * backend.nparts)
                for q, o in enumerate(outs):
                    r_all[q * cnt:(q + 1) * cnt] = o.numpy()
            elif op == 2:
                cnt = sc[0]
                t = torch.from_numpy(view(sbuf, cnt).copy())
                dist.all_reduce(t, group=group)
                view(rbuf, cnt)[:] = t.numpy()
            else:
                return -1
            return 0
        except Exception:  # pragma: no cover - reported as PAMG_E_RCCL by the library
            import traceback
            traceback.print_exc()
            return -1

    return HOST_COMM_FN(fn)


class Context:
    """A GPU (``pamg_ctx``) plus, for multi-part runs, its RCCL communicator (or the host
    debug transport)."""

    def __init__(self, device: int = 0, backend=None, transport: str = "rccl"):
        h = C.c_void_p()
        call("pamg_ctx_create", device, C.byref(h))
        self._h = h
        self.device = device
        self.rank, self.nranks = 0, 1
        self._hostfn = None
        if backend is not None and backend.nparts > 1:
            if not backend.distributed:
                raise ValueError("several parts in one process: use LocalWorld(nparts) (one context per part)")
            if transport == "rccl":
                self._init_comm(backend)
            elif transport == "host":
                self._init_host_comm(backend)
            else:
                raise ValueError(f"unknown transport {transport!r}")

    def _init_host_comm(self, backend):
        """Debug transport: ghost exchanges staged through host memory over the backend's gloo
        group (several ranks may then share one GPU; RCCL refuses that)."""
        self._hostfn = _host_comm_callback(backend)
        call("pamg_comm_init_host", self._h, backend.nparts, backend.rank,
             C.cast(self._hostfn, C.c_void_p), None)
        self.rank, self.nranks = backend.rank, backend.nparts

    def _init_comm(self, backend):
        import torch
        uid = C.create_string_buffer(128)
        if backend.rank == 0:
            call("pamg_comm_unique_id", uid)
        t = torch.frombuffer(bytearray(uid.raw), dtype=torch.uint8).clone()
        backend.dist.broadcast(t, src=0, group=backend.group)
        raw = bytes(t.numpy().tobytes())
        call("pamg_comm_init", self._h, backend.nparts, backend.rank, raw)
        self.rank, self.nranks = backend.rank, backend.nparts

    @property
    def handle(self):
        return self._h

    def sync(self):
        call("pamg_ctx_sync", self._h)

    def refcount(self) -> int:
        """References held on the context (pamg_ctx_refcount): this handle + one per live plan,
        vector, matrix and hierarchy made on it."""
        v = C.c_int()
        call("pamg_ctx_refcount", self._h, C.byref(v))
        return v.value

    def close(self):
        _release(self, "pamg_ctx_destroy")

    def __del__(self):
        self.close()


class LocalWorld:
    """PartitionedArrays ``with_debug`` on the device (pamg_world, pamg_comm_init_local): the
    parts of a ``SequentialBackend(n)`` in this process, part p on ``ctxs[p]`` (devices[p %
    len(devices)]; several parts may share a GPU). A collective operation (``mul``, ``vcycle``,
    ``pcg``, dots, exchanges) is issued for all parts at once with ``run``, one host thread per
    part: each thread drives its own context (libpamg calls release the GIL) and the parts meet
    inside the library at every exchange."""

    def __init__(self, nparts: int, devices=(0,)):
        h = C.c_void_p()
        call("pamg_world_create", int(nparts), C.byref(h))
        self._h = h
        self.nparts = nparts
        self.ctxs = []
        try:
            for r in range(nparts):
                c = Context(devices[r % len(devices)])
                call("pamg_comm_init_local", c.handle, h, r)
                c.rank, c.nranks = r, nparts
                self.ctxs.append(c)
        except Exception:
            for c in self.ctxs:
                c.close()
            self.close()
            raise

    def run(self, fn, parts=None):
        """[fn(p) for p in parts], one thread per part, concurrently; the exception of the part
        that failed first is raised after every thread has ended. A failing part breaks the world at once (its
        siblings stop waiting for it); a run over all the parts resets it before raising, so the
        world stays usable for the next run."""
        import threading
        parts = list(range(self.nparts)) if parts is None else list(parts)
        out, err, failed = {}, {}, []  # failed: the parts in the order they failed

        def body(p):
            try:
                out[p] = fn(p)
            except BaseException as e:  # noqa: BLE001 - re-raised below
                err[p] = e
                failed.append(p)  # (list.append is atomic under the GIL)

        def guarded(p):
            body(p)
            if p in err and self._h:
                # a part that fails outside a collective would leave its siblings
                # waiting 300 s for it; mark the world broken so they fail now
                call("pamg_world_abort", self._h)

        th = [threading.Thread(target=guarded, args=(p,), daemon=True) for p in parts]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if err:
            if self._h and set(parts) == set(range(self.nparts)):
                # every part has returned: clear the break that released the siblings, so one
                # part's error fails this call only (a run over some of the parts
                # leaves that to the caller's reset(), the others may still be inside a call)
                call("pamg_world_reset", self._h)
            p = failed[0]  # the first to fail: the cause (the others failed because the world broke)
            raise RuntimeError(f"part {p}: {err[p]!r}") from err[p]
        return [out[p] for p in parts]

    @property
    def broken(self) -> bool:
        v = C.c_int()
        call("pamg_world_state", self._h, C.byref(v))
        return bool(v.value)

    def reset(self):
        """Clear a broken world (pamg_world_reset) once every part has returned."""
        call("pamg_world_reset", self._h)

    def close(self):
        # drop this object's references only: a context is destroyed when its last user (a
        # vector, a matrix) is, and the library keeps the world until its last context is gone
        self.ctxs = []
        _release(self, "pamg_world_destroy")

    def __del__(self):
        self.close()


class DevicePlan:
    """Device exchange plan built from a ``HostPlan`` (``pamg_plan``)."""

    def __init__(self, ctx: Context, plan: HostPlan, tag: int = 0):
        """``tag``: the identity of the index space (pamg_plan_set_tag), the same on every part —
        the in-process world refuses to pair exchanges of plans with different tags."""
        self.ctx, self.host = ctx, plan
        nb = np.asarray(plan.nbrs, np.int32)
        rc = np.asarray(plan.recv_counts, np.int64)
        sc = np.asarray(plan.send_counts, np.int64)
        si = np.asarray(plan.send_idx if plan.send_idx is not None else [], np.int64)
        h = C.c_void_p()
        call("pamg_plan_create", ctx.handle, plan.n_own, plan.n_ghost, len(nb), ptr(nb), ptr(rc),
             ptr(sc), ptr(si), C.byref(h))
        self._h = h
        if tag:
            call("pamg_plan_set_tag", h, int(tag))
        self.n_own, self.n_ghost, self.tag = plan.n_own, plan.n_ghost, int(tag)

    @property
    def handle(self):
        return self._h

    def __del__(self):
        _release(self, "pamg_plan_destroy")


class PVector:
    """Device vector of one part: ``n_own`` own values followed by ``n_ghost`` ghost slots."""

    def __init__(self, ctx: Context, n_own: int, n_ghost: int = 0, values=None):
        h = C.c_void_p()
        call("pamg_vec_create", ctx.handle, n_own, n_ghost, C.byref(h))
        self._h, self.ctx, self.n_own, self.n_ghost = h, ctx, n_own, n_ghost
        if values is not None:
            self.set(values)

    @property
    def handle(self):
        return self._h

    def set(self, own):
        own = np.ascontiguousarray(own, np.float64)
        if own.shape != (self.n_own,):
            raise ValueError(f"expected {self.n_own} own values, got {own.shape}")
        call("pamg_vec_upload", self.ctx.handle, self._h, ptr(own))

    def own_values(self) -> np.ndarray:
        out = np.empty(self.n_own, np.float64)
        call("pamg_vec_download", self.ctx.handle, self._h, ptr(out))
        return out

    def ghost_values(self) -> np.ndarray:
        """PartitionedArrays ``ghost_values(x)``: the ghost slots, as last exchanged."""
        out = np.empty(self.n_ghost)
        call("pamg_vec_download_ghosts", self.ctx.handle, self._h, ptr(out))
        return out

    def device_ptr(self) -> int:
        p = C.c_void_p()
        call("pamg_vec_device_ptr", self._h, C.byref(p))
        return p.value

    def fill(self, v: float):
        call("pamg_vec_fill", self.ctx.handle, self._h, float(v))

    def __del__(self):
        _release(self, "pamg_vec_destroy")


class PSparseMatrix:
    """Device CSR of one part: own rows, columns local to ``plan`` (own, then ghosts)."""

    def __init__(self, ctx: Context, M: HCSR, plan: HostPlan | None = None,
                 dplan: DevicePlan | None = None, row_perm=None, col_perm=None, tag: int = 0):
        """``row_perm`` / ``col_perm`` (pamg_mat_upload_perm): device row i is row
        ``row_perm[i]`` of M, device own column k is own column ``col_perm[k]`` (None: the
        identity); rows keep their storage order, so row sums keep their bits. ``tag``: the
        column plan's identity (DevicePlan)."""
        self.ctx = ctx
        if plan is not None and dplan is None and plan.nbrs:
            dplan = DevicePlan(ctx, plan, tag)
        self.plan = dplan
        if plan is not None:
            col = plan.localize(M.col) if (plan.n_ghost or plan.col0) else M.col
            ncols = plan.n_own + plan.n_ghost
        else:
            col, ncols = M.col, M.ncols
        col = np.ascontiguousarray(col, np.int32)
        h = C.c_void_p()
        if row_perm is None and col_perm is None:
            call("pamg_mat_upload", ctx.handle, M.nrows, ncols, ptr(M.rowptr), ptr(col), 0,
                 ptr(M.val), 0, dplan.handle if dplan is not None else None, C.byref(h))
        else:
            rperm = None if row_perm is None else np.ascontiguousarray(row_perm, np.int64)
            cperm = None if col_perm is None else np.ascontiguousarray(col_perm, np.int64)
            call("pamg_mat_upload_perm", ctx.handle, M.nrows, ncols, ptr(M.rowptr), ptr(col), 0,
                 ptr(M.val), 0, dplan.handle if dplan is not None else None,
                 ptr(rperm) if rperm is not None else None, ptr(cperm) if cperm is not None else None,
                 C.byref(h))
        self._h = h
        self.nrows, self.ncols, self.nnz = M.nrows, ncols, M.nnz
        self.n_own_cols = plan.n_own if plan is not None else ncols
        self.n_ghost = plan.n_ghost if plan is not None else 0
        sb = C.c_int64()
        call("pamg_mat_stream_bytes", h, C.byref(sb))
        self.stream_bytes = sb.value  # matrix bytes one row operation reads (uploaded layout)

    @property
    def handle(self):
        return self._h

    def new_input_vector(self) -> PVector:
        return PVector(self.ctx, self.n_own_cols, self.n_ghost)

    def new_output_vector(self) -> PVector:
        return PVector(self.ctx, self.nrows)

    def __del__(self):
        _release(self, "pamg_mat_destroy")


def mul(y: PVector, A: PSparseMatrix, x: PVector) -> PVector:
    """``mul!(y, A, x)``: ghost exchange of x (overlapped with interior rows), y = A x."""
    call("pamg_spmv", A.ctx.handle, A.handle, x.handle, y.handle)
    return y


def residual(r: PVector, A: PSparseMatrix, x: PVector, b: PVector, with_norm=False):
    nrm = C.c_double()
    call("pamg_residual", A.ctx.handle, A.handle, x.handle, b.handle, r.handle,
         C.byref(nrm) if with_norm else None)
    return nrm.value if with_norm else r


def jacobi(x: PVector, A: PSparseMatrix, b: PVector, tmp: PVector, omega: float, nsweeps: int = 1):
    call("pamg_jacobi", A.ctx.handle, A.handle, x.handle, b.handle, tmp.handle, float(omega), nsweeps)
    return x


def jacobi_residual(t: PVector, r: PVector, A: PSparseMatrix, x: PVector, b: PVector, omega: float) -> bool:
    """t = x + omega D^-1 (b - A x); r = b - A t. Returns whether the fused pass ran."""
    f = C.c_int(0)
    call("pamg_jacobi_residual", A.ctx.handle, A.handle, x.handle, b.handle, t.handle, r.handle, float(omega),
         C.byref(f))
    return bool(f.value)


def consistent(x: PVector, plan: DevicePlan) -> PVector:
    """``consistent!(x) |> wait``: owners' values into x's ghost slots."""
    call("pamg_exchange", x.ctx.handle, plan.handle, x.handle)
    return x


class ExchangeTask:
    """``t = consistent!(x)`` ... ``wait(t)``: the exchange runs on the comm stream until
    ``wait`` (pamg_exchange_begin / pamg_exchange_end)."""

    def __init__(self, x: PVector, plan: DevicePlan):
        self.x, self.plan, self.done = x, plan, False
        call("pamg_exchange_begin", x.ctx.handle, plan.handle, x.handle)

    def wait(self) -> PVector:
        if not self.done:
            call("pamg_exchange_end", self.x.ctx.handle, self.plan.handle, self.x.handle)
            self.done = True
        return self.x


def consistent_async(x: PVector, plan: DevicePlan) -> ExchangeTask:
    """``consistent!(x)`` returning the task to ``wait`` on (overlap your own work with it)."""
    return ExchangeTask(x, plan)


def dot(x: PVector, y: PVector) -> float:
    out = C.c_double()
    call("pamg_vec_dot", x.ctx.handle, x.handle, y.handle, C.byref(out))
    return out.value


def norm(x: PVector) -> float:
    out = C.c_double()
    call("pamg_vec_nrm2", x.ctx.handle, x.handle, C.byref(out))
    return out.value


def axpby(a: float, x: PVector, b: float, y: PVector) -> PVector:
    call("pamg_vec_axpby", x.ctx.handle, float(a), x.handle, float(b), y.handle)
    return y


def copy(dst: PVector, src: PVector) -> PVector:
    call("pamg_vec_copy", src.ctx.handle, src.handle, dst.handle)
    return dst
