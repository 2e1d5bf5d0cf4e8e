"""Kernel planning for gt:mi355x.

Splits a typed stencil (``passes.StencilAnalysis``) into HIP launches of two hand-written
execution patterns (SURVEY.md §2.1 N1 -> K1/K2):

- ``PlaneKernel`` (K1): one PARALLEL interval section that has horizontal offsets. Lowered to
  the J-streaming skeleton: a wavefront owns a 64-wide I strip and walks a chunk of J rows at
  one K level; every value (field load, temporary version) lives in a register ring of the
  depth its J offsets need, and I offsets are wave shuffles. No LDS, no barriers.
- ``ColumnKernel`` (K2): a run of vertical loops without horizontal offsets on values produced
  inside the run (FORWARD/BACKWARD sweeps, and PARALLEL loops that are pointwise in IJ). One
  thread per (i, j) column walks the K levels in loop order with a register K-window per
  accessed (name, di, dj) -- the register-carried K-cache of the reference's
  ``KCacheDetection`` (``gtc/passes/oir_optimizations/caches.py:92``).

Temporaries used by more than one launch (or by more than one vertical loop of a column
kernel) become global *scratch* fields (I-first, allocated per domain by the host); all other
temporaries live in registers only.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional, Set, Tuple

from gt4py_amd import ir
from gt4py_amd.passes import ZERO_EXTENT, StencilAnalysis, iter_accesses


class UnsupportedStencil(NotImplementedError):
    pass


@dataclasses.dataclass
class PlaneKernel:
    loop: int
    section: int

    @property
    def items(self):
        return [(self.loop, self.section)]


@dataclasses.dataclass
class ColumnKernel:
    loops: List[int]
    # tile mode (one sequential loop): blocks own overlapping 2-D tiles of columns with the loop's
    # IJ extent as halo, and the values in ``lds`` -- produced in the loop and read at IJ offsets
    # at the same level -- are exchanged through an LDS plane per level (codegen/column.py)
    tile: bool = False
    lds: Tuple[str, ...] = ()

    def items(self, stencil):
        return [(li, si) for li in self.loops for si in range(len(stencil.vertical_loops[li].sections))]


@dataclasses.dataclass
class KernelPlan:
    kernels: List[object]
    scratch: List[str]  # temporaries materialised in global memory
    scratch_extent: Dict[str, Tuple[Tuple[int, int], Tuple[int, int]]]


def _loop_accesses(vl: ir.VerticalLoop):
    for sec in vl.sections:
        yield from iter_accesses(sec.body)


def _has_horizontal_offsets(vl: ir.VerticalLoop) -> bool:
    for acc, _ in _loop_accesses(vl):
        if isinstance(acc, ir.FieldAccess) and (acc.offset[0] != 0 or acc.offset[1] != 0):
            return True
    for sec in vl.sections:
        for n in ir.walk(sec.body):
            if isinstance(n, ir.HorizontalRegion):
                return True
    return False


def _pointwise_plane_ok(vl: ir.VerticalLoop) -> bool:
    """A PARALLEL loop without horizontal offsets that K1 can stream (no value written and read at
    a K offset, no run-time K offsets)."""
    written = {a.name for a, w in _loop_accesses(vl) if w}
    for a, w in _loop_accesses(vl):
        if isinstance(a, ir.FieldAccess) and (a.k_offset is not None or (not w and a.name in written and a.offset[2])):
            return False
    return True


def sections_contiguous(vl: ir.VerticalLoop) -> bool:
    """Consecutive sections (in sweep order) share their boundary: no level is skipped between them."""
    fwd = vl.loop_order != ir.LoopOrder.BACKWARD
    for s0, s1 in zip(vl.sections, vl.sections[1:]):
        a, b = (s0.interval.end, s1.interval.start) if fwd else (s0.interval.start, s1.interval.end)
        if a.level != b.level or a.offset != b.offset:
            return False
    return True


def _tile_lds_names(vl: ir.VerticalLoop) -> Optional[List[str]]:
    """Names a sequential loop produces and reads at IJ offsets, if a tile kernel can take the
    loop (every such read at K offset 0, no run-time K offsets on them); None otherwise."""
    written = {acc.name for acc, w in _loop_accesses(vl) if w}
    names: List[str] = []
    for acc, w in _loop_accesses(vl):
        if w or not isinstance(acc, ir.FieldAccess) or acc.name not in written:
            continue
        if acc.offset[0] or acc.offset[1]:
            if acc.offset[2] != 0 or acc.k_offset is not None:
                return None
            if acc.name not in names:
                names.append(acc.name)
    return names


def make_plan(analysis: StencilAnalysis, column_only: bool = False, pointwise_plane: bool = False,
              tile: bool = False) -> KernelPlan:
    """``column_only``: every computation runs in column kernels (the staged fallback, after
    ``lowering.split_phases``); otherwise PARALLEL computations with horizontal offsets become
    J-streaming plane kernels. ``tile``: a sequential computation that reads its own products at
    IJ offsets (same level) becomes a tile-mode column kernel instead of being rejected."""
    st = analysis.stencil
    temps = {t.name for t in st.temporaries}
    api = {p.name for p in st.field_params()}

    kernels: List[object] = []
    run: List[int] = []

    def flush():
        if run:
            kernels.append(ColumnKernel(list(run)))
            run.clear()
        run_written.clear()
        run_read_ij.clear()

    run_written: Set[str] = set()
    run_read_ij: Set[str] = set()
    for li, vl in enumerate(st.vertical_loops):
        plane = vl.loop_order == ir.LoopOrder.PARALLEL and (
            _has_horizontal_offsets(vl) or (pointwise_plane and _pointwise_plane_ok(vl))
        )
        if not column_only and plane:
            if any(isinstance(a, ir.FieldAccess) and a.k_offset is not None for a, _ in _loop_accesses(vl)):
                raise UnsupportedStencil("run-time K offsets in a PARALLEL computation with horizontal offsets")
            flush()
            for si in range(len(vl.sections)):
                kernels.append(PlaneKernel(li, si))
        else:
            lds = _tile_lds_names(vl) if (tile and vl.loop_order != ir.LoopOrder.PARALLEL) else None
            if lds:
                # a tile kernel of its own: its products cross columns through LDS, every level
                flush()
                kernels.append(ColumnKernel([li], tile=True, lds=tuple(lds)))
                continue
            if vl.loop_order != ir.LoopOrder.PARALLEL:
                # sequential loops: values produced in the loop may not be read at IJ offsets
                written = set()
                for acc, w in _loop_accesses(vl):
                    if w:
                        written.add(acc.name)
                for acc, w in _loop_accesses(vl):
                    if (
                        not w
                        and isinstance(acc, ir.FieldAccess)
                        and acc.name in written
                        and (acc.offset[0] or acc.offset[1])
                    ):
                        raise UnsupportedStencil(
                            f"'{acc.name}' is written in a {vl.loop_order.name} loop and read at a horizontal "
                            f"offset {acc.offset[:2]} in the same loop"
                        )
            # a column kernel may not consume values at IJ offsets produced earlier in the same run
            # (RAW across columns), nor overwrite values an earlier loop of the run read at IJ
            # offsets (WAR across columns): either needs a grid-wide barrier -> new kernel
            accs = list(_loop_accesses(vl))
            if any(
                not w and isinstance(a, ir.FieldAccess) and a.name in run_written and (a.offset[0] or a.offset[1])
                for a, w in accs
            ) or any(w and a.name in run_read_ij for a, w in accs):
                flush()
            run.append(li)
            run_written.update(a.name for a, w in accs if w)
            run_read_ij.update(
                a.name for a, w in accs if not w and isinstance(a, ir.FieldAccess) and (a.offset[0] or a.offset[1])
            )
    flush()

    # which kernel(s) / loops touch each temporary
    touch_kernels: Dict[str, Set[int]] = {}
    touch_loops: Dict[str, Set[int]] = {}
    read_ij_offset: Set[str] = set()
    for ki, k in enumerate(kernels):
        loops = [k.loop] if isinstance(k, PlaneKernel) else k.loops
        for li in loops:
            vl = st.vertical_loops[li]
            secs = [vl.sections[k.section]] if isinstance(k, PlaneKernel) else vl.sections
            for sec in secs:
                for acc, _ in iter_accesses(sec.body):
                    if isinstance(acc, ir.FieldAccess) and acc.name in temps:
                        touch_kernels.setdefault(acc.name, set()).add(ki)
                        touch_loops.setdefault(acc.name, set()).add(li)
                        if acc.offset[0] or acc.offset[1]:
                            read_ij_offset.add(acc.name)
    # a temporary read at a K offset in a loop whose sections leave gaps: the gap levels never run,
    # so a register window cannot carry the value across them -- it goes through memory
    gap_read: Set[str] = set()
    for vl in st.vertical_loops:
        if not sections_contiguous(vl):
            for acc, w in _loop_accesses(vl):
                if not w and isinstance(acc, ir.FieldAccess) and acc.name in temps and acc.offset[2] != 0:
                    gap_read.add(acc.name)
    def section_local(name: str, li: int) -> bool:
        """Every section of loop ``li`` that touches ``name`` writes it and reads it at its own
        level only: the plane kernels of the sections never hand a value to each other."""
        for sec in st.vertical_loops[li].sections:
            accs = [(a, w) for a, w in iter_accesses(sec.body) if a.name == name]
            if not accs:
                continue
            if not any(w for _, w in accs):
                return False
            if any(isinstance(a, ir.FieldAccess) and (a.offset[2] != 0 or a.k_offset is not None) for a, _ in accs):
                return False
        return True

    scratch = []
    for t in st.temporaries:
        kk = touch_kernels.get(t.name, set())
        ll = touch_loops.get(t.name, set())
        if len(kk) > 1 and len(ll) == 1 and t.name not in gap_read and all(
            isinstance(kernels[ki], PlaneKernel) for ki in kk
        ) and section_local(t.name, next(iter(ll))):
            continue  # per-section plane kernels of one loop, each producing its own values
        if len(kk) > 1 or len(ll) > 1 or t.name in gap_read:
            scratch.append(t.name)
    # column kernels must not read scratch temporaries written inside the same kernel at IJ offsets
    for k in kernels:
        if isinstance(k, ColumnKernel) and not k.tile:
            written = set()
            for li in k.loops:
                for acc, w in _loop_accesses(st.vertical_loops[li]):
                    if w:
                        written.add(acc.name)
            for li in k.loops:
                for acc, w in _loop_accesses(st.vertical_loops[li]):
                    if (
                        not w
                        and isinstance(acc, ir.FieldAccess)
                        and acc.name in written
                        and (acc.offset[0] or acc.offset[1])
                    ):
                        raise UnsupportedStencil(
                            f"'{acc.name}' is produced and read at an IJ offset inside one column kernel"
                        )
    # PARALLEL plane kernels: K offsets only on values not written in the same section
    for k in kernels:
        if isinstance(k, PlaneKernel):
            sec = st.vertical_loops[k.loop].sections[k.section]
            written = set()
            for acc, w in iter_accesses(sec.body):
                if w:
                    written.add(acc.name)
            for acc, w in iter_accesses(sec.body):
                if not w and isinstance(acc, ir.FieldAccess) and acc.offset[2] and acc.name in written:
                    raise UnsupportedStencil(
                        f"'{acc.name}' is written in a PARALLEL section and read at a K offset in the same section"
                    )
    scratch_extent = {t: analysis.extents.fields.get(t, ZERO_EXTENT) for t in scratch}
    del api
    return KernelPlan(kernels, scratch, scratch_extent)
