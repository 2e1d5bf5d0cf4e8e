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

``HaloStencil`` overlaps the exchange with compute: the rows that do not read the halo run
while RCCL moves the faces (RCCL's own stream waits on the packing kernel; the compute stream
waits on the transfers only before unpacking), then the two boundary strips run.
"""

from __future__ import annotations

import dataclasses
import os
from typing import Dict, List, Optional, Sequence, Tuple


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


def _backend_name(group=None) -> str:
    import torch.distributed as dist

    return str(dist.get_backend(group)).lower()


class JHaloExchange:
    """Exchange the J halo of fields stored as ``[I, J_local + 2h, K]`` tensors.

    Local row ``h + r`` holds global row ``j0 + r``; rows ``[0, h)`` and ``[h + nj, 2h + nj)``
    are the halos filled from the previous / next rank. On the first/last rank the outer halo
    is left untouched (it holds the global boundary input).
    """

    def __init__(self, nj_local: int, halo: int, rank: int, world_size: int, group=None,
                 periodic: bool = False, force_comm: bool = False):
        """``periodic``: the J axis wraps (ranks 0 and N-1 are neighbours; one rank copies its own
        faces). ``force_comm``: a rank that is its own neighbour still goes through the
        communicator (one GPU can exercise the RCCL path end to end)."""
        self.nj = nj_local
        self.h = halo
        self.rank = rank
        self.world = world_size
        self.group = group
        self.force_comm = force_comm
        if periodic:
            self.prev = (rank - 1) % world_size
            self.next = (rank + 1) % world_size
        else:
            self.prev = rank - 1 if rank > 0 else None
            self.next = rank + 1 if rank < world_size - 1 else None
        self._bufs: Dict[Tuple, Dict] = {}
        self._pending: List = []
        self._stage_host: Optional[bool] = None
        self._copies: Dict[Tuple, Tuple] = {}
        self._pending_device = None

    def _global_rank(self, r):
        import torch.distributed as dist

        return dist.get_global_rank(self.group, r) if self.group is not None else r

    def _buffers(self, t):
        key = (t.data_ptr(), tuple(t.shape), t.dtype)
        if key not in self._bufs:
            import torch

            ni, _, nk = t.shape
            dev = "cpu" if self._stage_host else t.device
            mk = lambda: torch.empty((ni, self.h, nk), dtype=t.dtype, device=dev)  # noqa: E731
            self._bufs[key] = {"send_lo": mk(), "send_hi": mk(), "recv_lo": mk(), "recv_hi": mk()}
        return self._bufs[key]

    def _device_copies(self, fields):
        """Batched pack/unpack descriptors (one launch each) for this list of device fields."""
        from gt4py_amd.distributed.halo_copy import BatchedCopy

        key = tuple((t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype) for t in fields)
        if key not in self._copies:
            h, nj = self.h, self.nj
            pack, unpack = [], []
            for t in fields:
                b = self._buffers(t)
                ni, _, nk = t.shape
                if self.next is not None:
                    pack.append((t, (0, nj, 0), (ni, h, nk), b["send_hi"]))
                    unpack.append((t, (0, nj + h, 0), (ni, h, nk), b["recv_hi"]))
                if self.prev is not None:
                    pack.append((t, (0, h, 0), (ni, h, nk), b["send_lo"]))
                    unpack.append((t, (0, 0, 0), (ni, h, nk), b["recv_lo"]))
            self._copies[key] = (BatchedCopy(pack), BatchedCopy(unpack))
        return self._copies[key]

    def start(self, fields: Sequence) -> List:
        """Pack faces and post the sends/receives; returns the pending work handles.

        Every send is posted before every receive, sends hi-face first and receives lo-halo
        first: with one peer on both sides (two ranks on a periodic axis, or one rank and
        ``force_comm``) the k-th receive from a peer then matches that peer's k-th send.
        Device fields are packed by ONE batched kernel launch (``halo_copy.py``).
        """
        import torch.distributed as dist

        if self._stage_host is None:
            # gloo moves host memory only: stage device faces through the host (tests / CPU runs)
            self._stage_host = _backend_name(self.group) == "gloo"
        h, nj = self.h, self.nj
        self._pending = []
        device = (not self._stage_host) and len(fields) > 0 and getattr(fields[0], "is_cuda", False)
        if device:
            pack, _ = self._device_copies(fields)
            pack.run(0)
        sends, recvs = [], []
        local = lambda peer: peer == self.rank and not self.force_comm  # noqa: E731
        for t in fields:
            b = self._buffers(t)
            if not device:
                if self.next is not None:
                    b["send_hi"].copy_(t[:, nj : nj + h, :])
                if self.prev is not None:
                    b["send_lo"].copy_(t[:, h : 2 * h, :])
            if self.next is not None and not local(self.next):
                sends.append(dist.P2POp(dist.isend, b["send_hi"], self._global_rank(self.next), self.group))
            if self.prev is not None and not local(self.prev):
                sends.append(dist.P2POp(dist.isend, b["send_lo"], self._global_rank(self.prev), self.group))
            if self.prev is not None:
                if local(self.prev):
                    b["recv_lo"].copy_(b["send_hi"])
                else:
                    recvs.append(dist.P2POp(dist.irecv, b["recv_lo"], self._global_rank(self.prev), self.group))
            if self.next is not None:
                if local(self.next):
                    b["recv_hi"].copy_(b["send_lo"])
                else:
                    recvs.append(dist.P2POp(dist.irecv, b["recv_hi"], self._global_rank(self.next), self.group))
            self._pending.append((t, b))
        self._pending_device = fields if device else None
        ops = sends + recvs
        if not ops:
            return []
        return dist.batch_isend_irecv(ops)

    def finish(self, works) -> None:
        """Wait for the transfers and unpack the received faces into the halos."""
        for w in works:
            w.wait()
        if self._pending_device is not None:
            _, unpack = self._device_copies(self._pending_device)
            unpack.run(1)
            self._pending = []
            self._pending_device = None
            return
        h, nj = self.h, self.nj
        for t, b in self._pending:
            if self.prev is not None:
                t[:, 0:h, :].copy_(b["recv_lo"])
            if self.next is not None:
                t[:, nj + h : nj + 2 * h, :].copy_(b["recv_hi"])
        self._pending = []

    def exchange(self, fields: Sequence) -> None:
        self.finish(self.start(fields))


class HaloStencil:
    """Run a stencil on one J strip of a decomposed domain, overlapping the halo exchange.

    ``halo_fields`` are the arguments read at J offsets; they carry ``halo`` extra rows on
    each side. The call splits the local domain into the interior rows (no halo read,
    computed while the faces are in flight) and the two boundary strips (computed after).
    """

    def __init__(self, stencil, halo_fields: Sequence[str], nj_local: int, halo: int, rank: int, world_size: int,
                 group=None, overlap: bool = True, periodic: bool = False, force_comm: bool = False,
                 stream_mode: Optional[str] = None, split: Optional[int] = None, bands_on_halo: Optional[bool] = None):
        """GPU scheduling knobs (defaults from ``GTMI_HALO_STREAM`` / ``GTMI_HALO_SPLIT`` /
        ``GTMI_HALO_BANDS``; measurements in DESIGN.md §6): ``stream_mode`` "side" (exchange on a
        high-priority halo stream, default) or "main" (pack/unpack on the caller's stream);
        ``split``: interior launched as that many row bands; ``GTMI_HALO_BANDS``: "unpack_main"
        (default: the caller's stream waits on RCCL, unpacks and runs the boundary strips),
        "halo" (unpack and strips on the halo stream) or "main" (unpack on the halo stream,
        strips on the caller's); ``bands_on_halo`` given explicitly selects between the last two."""
        self.stencil = stencil
        self.halo_fields = list(halo_fields)
        self.exchange = JHaloExchange(nj_local, halo, rank, world_size, group, periodic, force_comm)
        self.h = halo
        self.nj = nj_local
        # the overlap packs the halo fields' edge rows while the interior kernel runs: only sound
        # when the stencil never writes them
        self.overlap = (overlap and (world_size > 1 or force_comm) and nj_local > 2 * halo
                        and halo_fields_read_only(stencil, self.halo_fields))
        self._stream = None
        self.stream_mode = stream_mode or os.environ.get("GTMI_HALO_STREAM", "side")
        if self.stream_mode not in ("side", "main"):
            raise ValueError(f"stream_mode must be 'side' or 'main', got {self.stream_mode!r}")
        self.split = max(1, int(split if split is not None else os.environ.get("GTMI_HALO_SPLIT", "1")))
        # gate (``GTMI_HALO_GATE``: 1, 0, or auto = on when the neighbours are other ranks): the
        # interior waits for the pack, so RCCL's kernel and the interior become ready together and
        # RCCL's high-priority queue is dispatched first -- otherwise the interior's workgroups fill
        # every CU and RCCL's kernel completes only at the interior's tail, which puts the whole
        # transfer on the critical path. With the gate the unpack and the strips default to the
        # halo stream and run as soon as the faces land, beside the interior (when the stencil has
        # no scratch temporaries the two launches would share). One GPU as its own neighbour
        # (a transfer of ~25 us) measures the gate's hand-offs, not its gain: +3.4 % against +2.5 %
        # per step (profiles/r06/r06c_halo_gate_*), so auto keeps it off there.
        gate = os.environ.get("GTMI_HALO_GATE", "auto")
        self.gate = (world_size > 1 and not force_comm) if gate == "auto" else gate == "1"
        bands = os.environ.get("GTMI_HALO_BANDS", "halo" if self.gate else "unpack_main")
        self.bands_on_halo = bands_on_halo if bands_on_halo is not None else bands == "halo"
        # "unpack_main" (default): the caller's stream itself waits on RCCL's stream, unpacks and
        # computes the strips -- one cross-queue hand-off after the transfer instead of two
        # (+2.0-2.1 % vs +2.2-2.7 % per step)
        self.unpack_on_main = bands_on_halo is None and bands == "unpack_main"
        self.fuse_strips = os.environ.get("GTMI_HALO_STRIPS", "fused") == "fused"

    def schedule(self) -> Dict[str, object]:
        """The GPU schedule this runner uses (reported in the bench line's ``dist``)."""
        return {"overlap": self.overlap, "transport": _backend_name(self.exchange.group), "stream": self.stream_mode,
                "gate": self.gate, "split": self.split,
                "strips": "halo stream" if self.bands_on_halo else ("caller's stream after the unpack"
                                                                     if self.unpack_on_main else "caller's stream")}

    def _shifted(self, origin: Dict[str, Tuple[int, int, int]], dj: int) -> Dict[str, Tuple[int, int, int]]:
        return {k: (o[0], o[1] + dj, *o[2:]) for k, o in origin.items()}

    def __call__(self, args: Dict, origin: Dict[str, Tuple[int, int, int]], domain: Tuple[int, int, int],
                 **params) -> None:
        ni, nj, nk = domain
        assert nj == self.nj, (nj, self.nj)
        fields = [args[n] for n in self.halo_fields]
        kw = dict(args)
        kw.update(params)
        if not self.overlap:
            self.exchange.exchange(fields)
            self.stencil(**kw, origin=origin, domain=domain, validate_args=False)
            return
        h = self.h
        on_gpu = bool(fields) and getattr(fields[0], "is_cuda", False) and _backend_name(self.exchange.group) != "gloo"
        if on_gpu and self.stream_mode == "side":
            # default on the GPU: pack -> RCCL -> unpack on a HIGH-priority halo stream (never the
            # caller's hardware queue, see rccl_options), queued BEFORE the interior so that the
            # transfer is posted first; the interior (rows [h, nj - h)) runs on the caller's
            # stream meanwhile, the two boundary strips after it waits on the halo stream.
            # Measured per-rank cost (rank = own periodic neighbour): +2.0 % with
            # the unpack on the caller's stream, +2.5 % for the all-caller's-stream ordering
            # ("main") and +3.0 % for no overlap.
            import torch

            dev = fields[0].device
            if self._stream is None:
                self._stream = torch.cuda.Stream(device=dev, priority=-1)
            main = torch.cuda.current_stream(dev)
            ready = main.record_event()
            self._stream.wait_event(ready)
            with torch.cuda.stream(self._stream):
                works = self.exchange.start(fields)
            if self.gate:
                main.wait_event(self._stream.record_event())
            # the transfers are posted before the interior is enqueued; with split > 1 the interior
            # runs as that many row bands, so CU slots free up between launches
            rows = nj - 2 * h
            cuts = [h + rows * q // self.split for q in range(self.split + 1)]
            for a, b in zip(cuts[:-1], cuts[1:]):
                if b > a:
                    self.stencil(**kw, origin=self._shifted(origin, a), domain=(ni, b - a, nk), validate_args=False)
            if self.unpack_on_main:
                self.exchange.finish(works)
                self._strips(kw, origin, ni, nj, nk)
                return
            interior_done = main.record_event() if self.bands_on_halo else None
            with torch.cuda.stream(self._stream):
                self.exchange.finish(works)
                if self.bands_on_halo:
                    # the two boundary strips follow the unpack on the halo stream (they write rows
                    # the interior does not) -- but only after the interior when both may use the
                    # launcher's per-domain scratch buffers (a band as tall as the interior)
                    if not (self.gate and not _uses_scratch(self.stencil)):
                        self._stream.wait_event(interior_done)
                    self._strips(kw, origin, ni, nj, nk)
            main.wait_stream(self._stream)
            if self.bands_on_halo:
                return
        else:
            # "main" (and the CPU/gloo path): pack on the caller's stream, post the transfers
            # (RCCL's stream waits on the pack), enqueue the interior (rows [h, nj - h): reads rows
            # [0, nj) of the halo'ed fields only), then wait on the transfers and unpack
            works = self.exchange.start(fields)
            self.stencil(**kw, origin=self._shifted(origin, h), domain=(ni, nj - 2 * h, nk), validate_args=False)
            self.exchange.finish(works)
        self._strips(kw, origin, ni, nj, nk)

    def _strips(self, kw, origin, ni, nj, nk):
        """The two boundary strips: one call over both row ranges when the stencil object offers
        it (gt:mi355x: one launch per kernel, ``gtmi_stencil_run_jsplit``), else two calls."""
        h = self.h
        call_rows = getattr(self.stencil, "call_rows", None)
        if call_rows is not None and self.fuse_strips:
            call_rows(h, nj - 2 * h, domain=(ni, nj, nk), origin=origin, validate_args=False, **kw)
            return
        self.stencil(**kw, origin=origin, domain=(ni, h, nk), validate_args=False)
        self.stencil(**kw, origin=self._shifted(origin, nj - h), domain=(ni, h, nk), validate_args=False)


def _uses_scratch(stencil) -> bool:
    """Does the stencil's library allocate scratch temporaries (shared by concurrent calls)?
    Unknown backends count as yes."""
    compiled = getattr(getattr(stencil, "_gt_run_impl_", None), "compiled", None)
    plan = getattr(compiled, "plan", None)
    return plan is None or bool(plan.scratch)


def halo_fields_read_only(stencil, names) -> bool:
    """Every halo field is only read by ``stencil`` (``field_info`` access kind READ)."""
    from gt4py_amd.definitions import AccessKind

    info = getattr(stencil, "field_info", None) or {}
    for n in names:
        fi = info.get(n)
        if fi is not None and fi.access & AccessKind.WRITE:
            return False
    return True


def rccl_options():
    """ProcessGroupNCCL options for the halo exchange: RCCL on HIGH-priority streams. HIP pools
    hardware queues per priority (GPU_MAX_HW_QUEUES = 4 per process), so a high-priority RCCL
    stream never shares an in-order hardware queue with the caller's compute stream -- sharing
    one serialises the transfer behind (or ahead of) the interior kernel."""
    import torch.distributed as dist

    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


def init_process_group(backend: Optional[str] = None):
    """Initialise torch.distributed from the torchrun environment (127.0.0.1 rendezvous)."""
    import os

    import torch
    import torch.distributed as dist

    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = os.environ.get("GTMI_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    import datetime

    # a rank that never arrives fails the job in minutes instead of hanging it (GTMI_DIST_TIMEOUT s)
    timeout = datetime.timedelta(seconds=float(os.environ.get("GTMI_DIST_TIMEOUT", "300")))
    if backend == "nccl":
        lr = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(lr)
        dist.init_process_group(backend, device_id=torch.device("cuda", lr), pg_options=rccl_options(),
                                timeout=timeout)
    else:
        dist.init_process_group(backend, timeout=timeout)
    return dist.get_rank(), dist.get_world_size()
