"""Part backends — the PartitionedArrays execution models (reference README.md:2).

PartitionedArrays runs the same driver either with ``with_debug`` (all parts in one process,
messages are in-memory copies) or ``with_mpi`` (one part per MPI rank). This module has the
same two shapes for the host-side setup of the hierarchy:

* ``SequentialBackend(nparts)`` — every part in this process; used by the CPU tests and for
  the ``BASELINE.json`` plumbing config (2D 256^2, 2 parts on CPU).
* ``DistributedBackend()`` — one part per ``torch.distributed`` rank; host messages go over a
  gloo process group (the device ghost exchange of the solve phase is RCCL, in libpamg).

Both expose ``parts`` (the part ids held here), ``nparts``, and three collective operations
whose arguments/results are dicts keyed by the local part ids:
``allreduce_max``, ``allgather`` and ``exchange`` (sparse neighbour messages).
"""
from __future__ import annotations

import numpy as np

_DTYPES = [np.dtype(t) for t in ("int8", "uint8", "int32", "int64", "float64")]


def pack_arrays(arrays) -> np.ndarray:
    """Serialise a tuple of 1-D numpy arrays into one uint8 buffer."""
    head = [len(arrays)]
    for a in arrays:
        a = np.asarray(a)
        head += [_DTYPES.index(a.dtype), a.size]
    h = np.asarray(head, np.int64).view(np.uint8)
    parts = [np.asarray(len(h), np.int64).reshape(1).view(np.uint8), h]
    parts += [np.ascontiguousarray(a).reshape(-1).view(np.uint8) for a in arrays]
    return np.concatenate(parts) if parts else np.zeros(0, np.uint8)


def unpack_arrays(buf: np.ndarray):
    buf = np.asarray(buf, np.uint8)
    hl = int(buf[:8].view(np.int64)[0])
    head = buf[8:8 + hl].view(np.int64)
    n = int(head[0])
    off = 8 + hl
    out = []
    for k in range(n):
        dt = _DTYPES[int(head[1 + 2 * k])]
        cnt = int(head[2 + 2 * k])
        nb = cnt * dt.itemsize
        out.append(buf[off:off + nb].copy().view(dt))
        off += nb
    return tuple(out)


class SequentialBackend:
    """All parts in one process (PartitionedArrays ``with_debug``)."""

    def __init__(self, nparts: int):
        if nparts < 1:
            raise ValueError("nparts must be >= 1")
        self.nparts = nparts
        self.parts = list(range(nparts))
        self.rank = 0
        self.distributed = False

    def allreduce_max(self, vals: dict) -> float:
        return max(float(v) for v in vals.values())

    def allgather(self, vals: dict) -> list:
        return [vals[p] for p in range(self.nparts)]

    def exchange(self, sends: dict) -> dict:
        """sends[p][q] = tuple of arrays from part p to part q -> recv[q][p]."""
        recv = {p: {} for p in self.parts}
        for p, msgs in sends.items():
            for q, arrays in msgs.items():
                recv[q][p] = tuple(np.array(a, copy=True) for a in arrays)
        return recv


class DistributedBackend:
    """One part per torch.distributed rank (PartitionedArrays ``with_mpi``); host messages
    travel over a gloo group so the setup also runs (and is tested) without GPUs."""

    def __init__(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("DistributedBackend needs torch.distributed to be initialised")
        self.dist = dist
        self.nparts = dist.get_world_size()
        self.rank = dist.get_rank()
        self.parts = [self.rank]
        self.distributed = True
        if group is None:
            group = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else None
        self.group = group

    def _tensor(self, a):
        import torch
        return torch.from_numpy(np.ascontiguousarray(a))

    def allreduce_max(self, vals: dict) -> float:
        import torch
        t = torch.tensor([float(vals[self.rank])], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX, group=self.group)
        return float(t.item())

    def allgather(self, vals: dict) -> list:
        import torch
        t = torch.tensor([int(vals[self.rank])], dtype=torch.int64)
        out = [torch.zeros(1, dtype=torch.int64) for _ in range(self.nparts)]
        self.dist.all_gather(out, t, group=self.group)
        return [int(o.item()) for o in out]

    def allgather_bytes(self, buf: np.ndarray) -> list:
        import torch
        sizes = self.allgather({self.rank: len(buf)})
        m = max(sizes) if sizes else 0
        pad = np.zeros(max(m, 1), np.uint8)
        pad[:len(buf)] = buf
        out = [torch.zeros(max(m, 1), dtype=torch.uint8) for _ in range(self.nparts)]
        self.dist.all_gather(out, self._tensor(pad), group=self.group)
        return [o.numpy()[:s].copy() for o, s in zip(out, sizes)]

    def allgather_array(self, a: np.ndarray) -> list:
        """Every rank's float64 array (any lengths), in rank order."""
        bufs = self.allgather_bytes(np.ascontiguousarray(a, np.float64).view(np.uint8))
        return [b.view(np.float64) for b in bufs]

    def broadcast_array(self, a, dtype, root: int = 0) -> np.ndarray:
        """Rank root's array (of dtype) on every rank; the others pass None."""
        buf = np.ascontiguousarray(a, dtype).view(np.uint8) if self.rank == root else np.zeros(0, np.uint8)
        return self.allgather_bytes(buf)[root].view(dtype)

    def exchange(self, sends: dict) -> dict:
        import torch
        me = self.rank
        msgs = sends.get(me, {})
        # who sends to whom: all-gather a row of the message-size matrix
        row = np.zeros(self.nparts, np.int64)
        bufs = {}
        for q, arrays in msgs.items():
            bufs[q] = pack_arrays(arrays)
            row[q] = len(bufs[q])
        rows = [torch.zeros(self.nparts, dtype=torch.int64) for _ in range(self.nparts)]
        self.dist.all_gather(rows, self._tensor(row), group=self.group)
        incoming = {p: int(rows[p][me].item()) for p in range(self.nparts) if int(rows[p][me].item()) > 0}
        reqs = []
        recv_t = {}
        for p, n in incoming.items():
            recv_t[p] = torch.empty(n, dtype=torch.uint8)
            reqs.append(self.dist.irecv(recv_t[p], src=p, group=self.group))
        for q, b in bufs.items():
            if len(b):
                reqs.append(self.dist.isend(self._tensor(b), dst=q, group=self.group))
        for r in reqs:
            r.wait()
        return {me: {p: unpack_arrays(t.numpy()) for p, t in recv_t.items()}}
