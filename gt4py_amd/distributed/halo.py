"""IJ domain decomposition + halo neighbour exchange for gt:mi355x stencils.

The reference has no multi-device support: users decompose
externally and pass ``origin``/``domain`` per call (``stencil_object.py:155-175``). This module
adds the missing piece the north star asks for: one process per GPU, the global IJ plane cut
into J strips (K is never split: K sweeps carry dependencies), and a per-call exchange of
the ``halo``-wide J faces with the two neighbours through ``torch.distributed``
(backend ``nccl`` = RCCL over xGMI on MI355X; ``gloo`` on CPU for tests).

In the I-first layout ``(2,1,0)`` a J face ``[:, j0:j1, :]`` is ``j1-j0`` contiguous rows per
K plane, so packing is one strided copy per face; messages are a few MB (SURVEY.md §8(e):
2 x (8192+4) x 160 x 4 B = 10.5 MB per face for C5), i.e. one point-to-point xGMI transfer
per neighbour -- there are no reductions, so no ring collective is involved.
Global boundaries are plain input cells (no periodicity, as in the reference).
"""

from __future__ import annotations

import dataclasses
from typing import List, Optional, Tuple


@dataclasses.dataclass(frozen=True)
class JStrips:
    """Split ``nj_global`` rows into ``world_size`` contiguous strips (first ranks get +1)."""

    nj_global: int
    world_size: int

    def bounds(self, rank: int) -> Tuple[int, int]:
        base, extra = divmod(self.nj_global, self.world_size)
        j0 = rank * base + min(rank, extra)
        j1 = j0 + base + (1 if rank < extra else 0)
        return j0, j1

    def size(self, rank: int) -> int:
        j0, j1 = self.bounds(rank)
        return j1 - j0


class JHaloExchange:
    """Exchange the J halo of one or more fields stored as [I, J_local + 2h, K] tensors.

    Local row ``h + r`` holds global row ``j0 + r``; rows ``[0, h)`` and ``[h + nj, 2h + nj)``
    are the halos filled from the previous / next rank. On the first/last rank the outer halo
    is left untouched (it holds the global boundary input).
    """

    def __init__(self, nj_local: int, halo: int, rank: int, world_size: int, group=None):
        self.nj = nj_local
        self.h = halo
        self.rank = rank
        self.world = world_size
        self.group = group
        self.prev = rank - 1 if rank > 0 else None
        self.next = rank + 1 if rank < world_size - 1 else None
        self._bufs = {}

    def _buffers(self, t):
        key = (t.data_ptr(), tuple(t.shape), t.dtype)
        if key not in self._bufs:
            import torch

            ni, _, nk = t.shape
            mk = lambda: torch.empty((ni, self.h, nk), dtype=t.dtype, device=t.device)  # noqa: E731
            self._bufs[key] = {"send_lo": mk(), "send_hi": mk(), "recv_lo": mk(), "recv_hi": mk()}
        return self._bufs[key]

    def start(self, fields: List) -> List:
        """Pack faces and post the sends/receives; returns the pending work handles."""
        import torch.distributed as dist

        ops = []
        h, nj = self.h, self.nj
        self._pending = []
        for t in fields:
            b = self._buffers(t)
            if self.prev is not None:
                b["send_lo"].copy_(t[:, h : 2 * h, :])
                ops.append(dist.P2POp(dist.isend, b["send_lo"], self.prev, self.group))
                ops.append(dist.P2POp(dist.irecv, b["recv_lo"], self.prev, self.group))
            if self.next is not None:
                b["send_hi"].copy_(t[:, nj : nj + h, :])
                ops.append(dist.P2POp(dist.isend, b["send_hi"], self.next, self.group))
                ops.append(dist.P2POp(dist.irecv, b["recv_hi"], self.next, self.group))
            self._pending.append((t, b))
        if not ops:
            return []
        return dist.batch_isend_irecv(ops)

    def finish(self, works) -> None:
        """Wait for the transfers and unpack the received faces into the halos."""
        for w in works:
            w.wait()
        h, nj = self.h, self.nj
        for t, b in self._pending:
            if self.prev is not None:
                t[:, 0:h, :].copy_(b["recv_lo"])
            if self.next is not None:
                t[:, nj + h : nj + 2 * h, :].copy_(b["recv_hi"])
        self._pending = []

    def exchange(self, fields: List) -> None:
        self.finish(self.start(fields))


def init_process_group(backend: Optional[str] = None):
    """Initialise torch.distributed from the torchrun environment (127.0.0.1 rendezvous)."""
    import os

    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(lr)
        dist.init_process_group(backend, device_id=torch.device("cuda", lr))
    else:
        dist.init_process_group(backend)
    return dist.get_rank(), dist.get_world_size()
