"""2-D IJ decomposition with corner-correct halo exchange.

The global IJ plane is cut into a ``pi x pj`` process grid (K is never split). Every field
that stencils read at horizontal offsets is stored per rank as ``[ni + 2*hi, nj + 2*hj, nk]``
(I-first layout), interior at ``[hi:hi+ni, hj:hj+nj]``.

Corners: hdiff reads the diagonal neighbours of ``lap`` (``lap[i+1, j+1]`` needs
``in[i+1, j+1]`` etc.), so the halo corners must hold the diagonal rank's cells. They are
filled without diagonal messages by exchanging in two phases (the classic dimension-by-
dimension scheme): phase 1 moves the I faces over the interior rows (and over the halo rows of
a global J boundary), phase 2 moves the J faces over the FULL I width including the
just-received I halos -- the corners arrive transitively.

Batching: in every phase each rank sends ONE message per neighbour holding the faces of all
exchanged fields (packed back to back into a flat buffer), so a call costs at most 4 messages
regardless of how many fields are exchanged -- on MI355X each lands on one xGMI link.

Periodic boundaries (optional per axis) wrap the neighbour ranks; a periodic axis with a single
rank copies its own opposite face. Non-periodic global boundaries keep the caller's halo cells
(plain input, as in the reference).

Overlap: phase 1 (the I faces, small) completes first; the interior ``[0, ni) x [hj, nj-hj)``
-- full width, it reads only filled I halos -- then runs while phase 2 moves the J faces, and
the south/north bands follow the unpack. Default ``stream_mode="main"`` (``GTMI_HALO2D_STREAM``):
packs and unpacks on the caller's stream, RCCL on its own high-priority stream; ``"side"`` puts
the packs/unpacks on a high-priority halo stream (``halo.rccl_options``; three more cross-queue
hand-offs per step). ``ifirst=False`` instead overlaps both phases with an interior that also
excludes west/east bands, run after both phases (measured slower: DESIGN.md §6).
"""

from __future__ import annotations

import dataclasses
import os
from typing import Dict, List, Optional, Sequence, Tuple

from gt4py_amd.distributed.halo import halo_fields_read_only


def _split(n: int, parts: int, idx: int) -> Tuple[int, int]:
    base, extra = divmod(n, parts)
    a = idx * base + min(idx, extra)
    return a, a + base + (1 if idx < extra else 0)


@dataclasses.dataclass(frozen=True)
class Decomposition2D:
    """``pi x pj`` ranks over an ``ni x nj`` plane; rank = ci + pi * cj."""

    ni: int
    nj: int
    pi: int
    pj: int
    periodic: Tuple[bool, bool] = (False, False)

    @property
    def size(self) -> int:
        return self.pi * self.pj

    def coords(self, rank: int) -> Tuple[int, int]:
        return rank % self.pi, rank // self.pi

    def rank_of(self, ci: int, cj: int) -> Optional[int]:
        if self.periodic[0]:
            ci %= self.pi
        if self.periodic[1]:
            cj %= self.pj
        if not (0 <= ci < self.pi and 0 <= cj < self.pj):
            return None
        return ci + self.pi * cj

    def bounds(self, rank: int) -> Tuple[Tuple[int, int], Tuple[int, int]]:
        ci, cj = self.coords(rank)
        return _split(self.ni, self.pi, ci), _split(self.nj, self.pj, cj)

    def local_shape(self, rank: int) -> Tuple[int, int]:
        (i0, i1), (j0, j1) = self.bounds(rank)
        return i1 - i0, j1 - j0

    @staticmethod
    def balanced(ni: int, nj: int, world: int, periodic=(False, False)) -> "Decomposition2D":
        """The factorisation of ``world`` with the least halo perimeter per rank."""
        best = None
        for pi in range(1, world + 1):
            if world % pi:
                continue
            pj = world // pi
            cost = ni / pi + nj / pj  # halo cells per unit width ~ local perimeter
            if best is None or cost < best[0] - 1e-12:
                best = (cost, pi, pj)
        return Decomposition2D(ni, nj, best[1], best[2], tuple(periodic))


def _backend_name(group=None) -> str:
    import torch.distributed as dist

    return str(dist.get_backend(group)).lower()


class HaloExchange2D:
    """Batched halo exchange of ``[ni+2hi, nj+2hj, nk]`` fields: two phases (I faces, then J
    faces over the full width), or with ``diagonal=True`` ONE phase that also sends the four
    corner boxes to the diagonal neighbours (8 messages, one pack, one unpack)."""

    def __init__(self, decomp: Decomposition2D, rank: int, halo: Tuple[int, int], group=None,
                 force_comm: bool = False, diagonal: bool = False):
        """``force_comm``: send to oneself through the communicator instead of copying locally
        (a periodic axis with one rank); lets one GPU exercise the RCCL path end to end."""
        self.force_comm = force_comm
        self.diagonal = diagonal
        self.d = decomp
        self.rank = rank
        self.hi, self.hj = halo
        self.ni, self.nj = decomp.local_shape(rank)
        self.group = group
        ci, cj = decomp.coords(rank)
        self.nbr = {
            "W": decomp.rank_of(ci - 1, cj) if self.hi else None,
            "E": decomp.rank_of(ci + 1, cj) if self.hi else None,
            "S": decomp.rank_of(ci, cj - 1) if self.hj else None,
            "N": decomp.rank_of(ci, cj + 1) if self.hj else None,
        }
        both = bool(self.hi and self.hj)
        for d, (dx, dy) in (("SW", (-1, -1)), ("SE", (1, -1)), ("NW", (-1, 1)), ("NE", (1, 1))):
            self.nbr[d] = decomp.rank_of(ci + dx, cj + dy) if both else None
        self._host = None
        self._copies: Dict[Tuple, Tuple] = {}
        self._bufs: Dict[Tuple, object] = {}
        self._stream = None

    # -- face geometry (local index ranges of what is sent / received, per direction) -----
    def _faces(self, phase: int):
        hi, hj, ni, nj = self.hi, self.hj, self.ni, self.nj
        if phase == 0:
            # I faces over the interior rows, plus the halo rows of a global (non-periodic) J
            # boundary: no J neighbour will fill those corners in phase 2
            js = slice(0 if self.nbr["S"] is None else hj, hj + nj + (hj if self.nbr["N"] is None else 0))
            return {
                "W": ((slice(hi, 2 * hi), js), (slice(0, hi), js)),
                "E": ((slice(ni, ni + hi), js), (slice(ni + hi, ni + 2 * hi), js)),
            }
        if phase == 1:
            is_ = slice(0, ni + 2 * hi)  # J faces over the full width: corners travel along
            return {
                "S": ((is_, slice(hj, 2 * hj)), (is_, slice(0, hj))),
                "N": ((is_, slice(nj, nj + hj)), (is_, slice(nj + hj, nj + 2 * hj))),
            }
        # phase 2 = the single diagonal phase: faces over the interior, extended over the halo of
        # a global (non-periodic) boundary of the other axis, whose corner no diagonal rank owns
        nb = self.nbr
        js = slice(0 if nb["S"] is None else hj, hj + nj + (hj if nb["N"] is None else 0))
        is_ = slice(0 if nb["W"] is None else hi, hi + ni + (hi if nb["E"] is None else 0))
        lo_i, hi_i = slice(hi, 2 * hi), slice(ni, ni + hi)  # sent: first / last interior columns
        lo_j, hi_j = slice(hj, 2 * hj), slice(nj, nj + hj)
        hw, he = slice(0, hi), slice(ni + hi, ni + 2 * hi)  # received: west / east halo columns
        hs, hn = slice(0, hj), slice(nj + hj, nj + 2 * hj)
        return {
            "W": ((lo_i, js), (hw, js)),
            "E": ((hi_i, js), (he, js)),
            "S": ((is_, lo_j), (is_, hs)),
            "N": ((is_, hi_j), (is_, hn)),
            "SW": ((lo_i, lo_j), (hw, hs)),
            "SE": ((hi_i, lo_j), (he, hs)),
            "NW": ((lo_i, hi_j), (hw, hn)),
            "NE": ((hi_i, hi_j), (he, hn)),
        }

    _OPPOSITE = {"W": "E", "E": "W", "S": "N", "N": "S", "SW": "NE", "NE": "SW", "SE": "NW", "NW": "SE"}

    def _buffer(self, key, numel, like):
        import torch

        if key not in self._bufs or self._bufs[key].numel() < numel:
            dev = "cpu" if self._host else like.device
            self._bufs[key] = torch.empty(numel, dtype=like.dtype, device=dev)
        return self._bufs[key][:numel]

    def _phase(self, fields: Sequence, phase: int) -> None:
        self._phase_finish(self._phase_start(fields, phase))

    def _phase_start(self, fields: Sequence, phase: int):
        """Pack the phase's faces and post its transfers; returns the state ``_phase_finish`` needs."""
        import torch.distributed as dist

        faces = self._faces(phase)
        dirs = [d for d in faces if self.nbr[d] is not None]
        if not dirs:
            return None
        sizes = {d: [t[faces[d][0][0], faces[d][0][1], :].numel() for t in fields] for d in dirs}
        sbuf, rbuf = {}, {}
        for d in dirs:
            total = sum(sizes[d])
            sbuf[d] = self._buffer(("s", phase, d, fields[0].dtype), total, fields[0])
            rbuf[d] = self._buffer(("r", phase, d, fields[0].dtype), total, fields[0])
        device = (not self._host) and getattr(fields[0], "is_cuda", False)
        if device:  # one batched launch packs every face of the phase
            pack, unpack_dev = self._device_copies(fields, phase, faces, dirs, sizes, sbuf, rbuf)
            pack.run(0)
        else:
            for d in dirs:
                off = 0
                for t, n in zip(fields, sizes[d]):
                    face = t[faces[d][0][0], faces[d][0][1], :]
                    sbuf[d][off : off + n].view(face.shape).copy_(face)
                    off += n
        # my d-halo receives the neighbour's opposite face. Receives are posted in the canonical
        # direction order, sends toward opposite(d) in the same order: a peer that is my
        # neighbour in several directions (two ranks on a periodic axis) then matches its k-th
        # send to me with my k-th receive from it (neighbourhood is symmetric).
        ops, unpack = [], []
        local = lambda peer: peer == self.rank and not self.force_comm  # noqa: E731
        for d in [self._OPPOSITE[x] for x in faces if self._OPPOSITE[x] in dirs]:
            peer = self.nbr[d]
            if not local(peer):
                gpeer = dist.get_global_rank(self.group, peer) if self.group is not None else peer
                ops.append(dist.P2POp(dist.isend, sbuf[d], gpeer, self.group))
        for d in dirs:
            peer = self.nbr[d]
            if local(peer):  # periodic axis with one rank: my own opposite face
                unpack.append((d, sbuf[self._OPPOSITE[d]]))
                continue
            gpeer = dist.get_global_rank(self.group, peer) if self.group is not None else peer
            ops.append(dist.P2POp(dist.irecv, rbuf[d], gpeer, self.group))
            unpack.append((d, rbuf[d]))
        works = dist.batch_isend_irecv(ops) if ops else []
        return fields, faces, sizes, rbuf, unpack, works, (unpack_dev if device else None)

    def _phase_finish(self, state) -> None:
        """Wait for the phase's transfers and unpack the received faces."""
        if state is None:
            return
        fields, faces, sizes, rbuf, unpack, works, unpack_dev = state
        for w in works:
            w.wait()
        if unpack_dev is not None:
            for d, buf in unpack:
                if buf is not rbuf[d]:  # local periodic wrap: my own opposite face
                    rbuf[d].copy_(buf)
            unpack_dev.run(1)
            return
        for d, buf in unpack:
            off = 0
            for t, n in zip(fields, sizes[d]):
                face = t[faces[d][1][0], faces[d][1][1], :]
                face.copy_(buf[off : off + n].view(face.shape))
                off += n

    def _device_copies(self, fields, phase, faces, dirs, sizes, sbuf, rbuf):
        from gt4py_amd.distributed.halo_copy import BatchedCopy

        key = (phase,) + tuple((t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype) for t in fields) + tuple(
            (sbuf[d].data_ptr(), rbuf[d].data_ptr()) for d in dirs
        )  # buffers included: a re-allocated message buffer never meets a stale descriptor
        if key not in self._copies:
            pack, unpack = [], []
            for d in dirs:
                soff = roff = 0
                for t, n in zip(fields, sizes[d]):
                    nk = t.shape[2]
                    (si, sj), (ri, rj) = faces[d]
                    pack.append((t, (si.start, sj.start, 0), (si.stop - si.start, sj.stop - sj.start, nk),
                                 sbuf[d][soff : soff + n]))
                    unpack.append((t, (ri.start, rj.start, 0), (ri.stop - ri.start, rj.stop - rj.start, nk),
                                   rbuf[d][roff : roff + n]))
                    soff += n
                    roff += n
            self._copies[key] = (BatchedCopy(pack), BatchedCopy(unpack))
        return self._copies[key]

    def _groups(self, fields):
        if self._host is None:
            self._host = _backend_name(self.group) == "gloo"
        dtypes = []
        for t in fields:
            if t.dtype not in dtypes:
                dtypes.append(t.dtype)
        return [[t for t in fields if t.dtype == dt] for dt in dtypes]  # one batched message per neighbour and dtype

    def exchange(self, fields: Sequence) -> None:
        """Fill the halos (and corners) of ``fields``; must be called by every rank."""
        if not fields:
            return
        for group in self._groups(fields):
            if self.diagonal:
                self._phase(group, 2)
            else:
                self._phase(group, 0)
                self._phase(group, 1)

    def exchange_phase(self, fields: Sequence, phase: int) -> None:
        """Only phase ``phase`` (0: I faces, 1: J faces incl. corners) of every dtype group."""
        if not fields:
            return
        for group in self._groups(fields):
            self._phase(group, phase)

    def start_phase(self, fields: Sequence, phase: int):
        """Post phase ``phase`` of every dtype group; ``finish_phase`` completes it."""
        return [(group, self._phase_start(group, phase)) for group in self._groups(fields)] if fields else []

    def finish_phase(self, pending) -> None:
        for _group, state in pending:
            self._phase_finish(state)

    def start(self, fields: Sequence):
        """Post phase 0 (I faces) of every dtype group; ``finish`` completes both phases."""
        if not fields:
            return []
        return [(group, self._phase_start(group, 0)) for group in self._groups(fields)]

    def finish(self, pending) -> None:
        for group, state in pending:
            self._phase_finish(state)
            self._phase(group, 1)


class HaloStencil2D:
    """Run a stencil on one tile of a 2-D decomposition, overlapping the halo exchange.

    ``halo_fields`` carry ``(hi, hj)`` halo cells on every side. The interior
    ``[hi, ni-hi) x [hj, nj-hj)`` reads no halo and is computed while the exchange runs on the
    halo stream; the four boundary bands follow.
    """

    def __init__(self, stencil, halo_fields: Sequence[str], decomp: Decomposition2D, rank: int,
                 halo: Tuple[int, int], group=None, overlap: bool = True, force_comm: bool = False,
                 stream_mode: Optional[str] = None, ifirst: Optional[bool] = None, scheme: Optional[str] = None):
        """``ifirst`` (default ``GTMI_HALO2D_IFIRST``, on): exchange the I faces
        before the interior, which then spans the full I width and overlaps only the J-face
        phase; off: the interior excludes west/east bands that run after both phases."""
        self.stencil = stencil
        self.halo_fields = list(halo_fields)
        # "two_phase" (default, GTMI_HALO2D_SCHEME): I faces then J faces, overlapped as below;
        # "diagonal": one exchange phase with corner messages to the diagonal neighbours, then the
        # whole tile in one launch -- measured slower on MI355X (+7.9-8.2 % vs +6.5 %): RCCL splits
        # the 16-operation group into three kernels and starts it ~100 us after the pack
        # 
        self.scheme = scheme or os.environ.get("GTMI_HALO2D_SCHEME", "two_phase")
        if self.scheme not in ("diagonal", "two_phase"):
            raise ValueError(f"scheme must be 'diagonal' or 'two_phase', got {self.scheme!r}")
        self.ex = HaloExchange2D(decomp, rank, halo, group, force_comm=force_comm,
                                 diagonal=self.scheme == "diagonal")
        self.hi, self.hj = halo
        self.ni, self.nj = decomp.local_shape(rank)
        self.overlap = (
            overlap and (decomp.size > 1 or force_comm) and self.ni > 2 * self.hi and self.nj > 2 * self.hj
            and halo_fields_read_only(stencil, self.halo_fields)
        )
        self._stream = None
        # default "main": with the I faces first nothing overlaps phase 1 anyway, and keeping the
        # packs/unpacks on the caller's stream saves three cross-queue hand-offs per step
        # (+6.3-6.7 % vs +6.6-7.2 % for "side")
        self.stream_mode = stream_mode or os.environ.get("GTMI_HALO2D_STREAM", "main")
        if self.stream_mode not in ("side", "main"):
            raise ValueError(f"stream_mode must be 'side' or 'main', got {self.stream_mode!r}")
        self.ifirst = (os.environ.get("GTMI_HALO2D_IFIRST", "1") != "0") if ifirst is None else bool(ifirst)

    def _run(self, kw, origin, i0, j0, ni, nj, nk):
        if ni <= 0 or nj <= 0:
            return
        org = {k: (o[0] + i0, o[1] + j0, *o[2:]) for k, o in origin.items()}
        self.stencil(**kw, origin=org, domain=(ni, nj, nk), validate_args=False)

    def _south_north(self, kw, origin, ni, nj, nk):
        """The two full-width J bands, in one call over both row ranges when the stencil object
        offers it (gt:mi355x: ``gtmi_stencil_run_jsplit``)."""
        call_rows = getattr(self.stencil, "call_rows", None)
        if call_rows is not None:
            call_rows(self.hj, nj - 2 * self.hj, domain=(ni, nj, nk), origin=origin, validate_args=False, **kw)
            return
        for i0, j0, bi, bj in self.bands()[:2]:
            self._run(kw, origin, i0, j0, bi, bj, nk)

    def band_width_i(self) -> int:
        """Width of the west/east bands. The halo width itself would leave bands a few columns
        wide, and a plane-kernel wave (one I strip of ~112-224 outputs) would then compute a
        handful of them per row (measured: +28.6 % per step for 2-column bands on hdiff
        2048^2x160). So the bands take ``BAND_I`` columns (>= the halo), whole strips of the plane
        kernel, and the interior shrinks by as much; the work is the same, only its split changes."""
        w = max(self.hi, self.BAND_I)
        return w if self.ni > 2 * w else self.hi

    BAND_I = 224  # two f64 / one f32 plane-kernel strip of outputs

    def bands(self) -> List[Tuple[int, int, int, int]]:
        """(i0, j0, ni, nj) of the boundary bands around the interior (disjoint, covering)."""
        hj, ni, nj = self.hj, self.ni, self.nj
        wi = self.band_width_i()
        return [
            (0, 0, ni, hj),  # south band, full width
            (0, nj - hj, ni, hj),  # north band, full width
            (0, hj, wi, nj - 2 * hj),  # west band
            (ni - wi, hj, wi, nj - 2 * hj),  # east band
        ]

    def __call__(self, args: Dict, origin: Dict[str, Tuple[int, int, int]], domain: Tuple[int, int, int],
                 **params) -> None:
        ni, nj, nk = domain
        assert (ni, nj) == (self.ni, self.nj), ((ni, nj), (self.ni, self.nj))
        fields = [args[n] for n in self.halo_fields]
        kw = dict(args)
        kw.update(params)
        if not self.overlap or self.scheme == "diagonal":
            # diagonal: the exchange is one pack, one RCCL group, one unpack; overlapping it buys
            # nothing while RCCL's kernel waits for CUs behind the interior (measured for the
            # two-phase scheme: overlapped +6.1-6.5 %, not overlapped +6.4-6.8 %)
            self.ex.exchange(fields)
            self.stencil(**kw, origin=origin, domain=domain, validate_args=False)
            return
        hi, hj = self.hi, self.hj
        wi = self.band_width_i()
        on_gpu = fields and getattr(fields[0], "is_cuda", False) and not _backend_name(self.ex.group) == "gloo"
        if on_gpu and self.stream_mode == "side":
            import torch

            if self._stream is None:
                self._stream = torch.cuda.Stream(device=fields[0].device, priority=-1)
            main = torch.cuda.current_stream(fields[0].device)
            self._stream.wait_stream(main)  # the fields' producers
            if self.ifirst:
                # the I faces are ~1/(2 nj) of the field: moving them first costs a few tens of us
                # unhidden, and in exchange the interior runs full-width (no narrow west/east
                # bands, which a J-streaming plane kernel computes at a fraction of its rate)
                with torch.cuda.stream(self._stream):
                    self.ex.exchange_phase(fields, 0)
                main.wait_stream(self._stream)
                with torch.cuda.stream(self._stream):
                    self.ex.exchange_phase(fields, 1)
                self._run(kw, origin, 0, hj, ni, nj - 2 * hj, nk)
                main.wait_stream(self._stream)
                self._south_north(kw, origin, ni, nj, nk)
                return
            with torch.cuda.stream(self._stream):
                self.ex.exchange(fields)
            self._run(kw, origin, wi, hj, ni - 2 * wi, nj - 2 * hj, nk)
            main.wait_stream(self._stream)
        elif self.ifirst:
            # caller's stream (and the CPU/gloo path): phase 0 whole (pack, RCCL, unpack), then
            # phase 1 posted, the full-width interior enqueued while it moves, unpack and the
            # south/north bands -- every hand-off is between the caller's and RCCL's streams
            self.ex.exchange_phase(fields, 0)
            pending = self.ex.start_phase(fields, 1)
            self._run(kw, origin, 0, hj, ni, nj - 2 * hj, nk)
            self.ex.finish_phase(pending)
            self._south_north(kw, origin, ni, nj, nk)
            return
        else:
            # phase 0 (I faces) is packed and posted on the caller's stream, the interior runs
            # while RCCL moves it; phase 1 (J faces incl. the received I halos) follows
            pending = self.ex.start(fields)
            self._run(kw, origin, wi, hj, ni - 2 * wi, nj - 2 * hj, nk)
            self.ex.finish(pending)
        for i0, j0, bi, bj in self.bands():
            self._run(kw, origin, i0, j0, bi, bj, nk)
