"""IR lowerings applied before kernel planning (gt:mi355x only).

Data dimensions (``Field[(dtype, (n,))]``, ``GlobalTable``) are lowered to *component fields*:
every distinct data index of a field becomes one virtual 3-D field whose base address is the
field's address plus ``sum(index_d * data_stride_d)``, computed by the host code at launch time.
With the ``(2, 1, 0)`` I-first layout the data dimensions are the outermost ones
(``storage/layout.py``), so each component is itself a dense I-first 3-D array: the plane and
column kernels stream it like any other field.

The indices must be launch-uniform (integer literals and scalar parameters, e.g.
``vec[0, 0, 0][2]`` or ``vec[0, 0, 0][idx]``; reference ``test_code_generation.py:309-361,
463-510, 664-716, 894-917, 1096-1109``). A written data-dimension field must use literal indices
only (or a single index), so that two components never alias.
"""

from __future__ import annotations

import dataclasses
from typing import Dict, List, Tuple

from gt4py_amd import ir, passes
from gt4py_amd.codegen.plan import UnsupportedStencil
from gt4py_amd.passes import StencilAnalysis


@dataclasses.dataclass
class Component:
    base: str  # API field name
    index: List[ir.Expr]  # launch-uniform index expression per data dimension


def _uniform(e: ir.Expr) -> bool:
    for n in ir.walk(e):
        if isinstance(n, (ir.FieldAccess, ir.AxisIndex)):
            return False
    return True


def _key(index: List[ir.Expr]) -> str:
    return repr([(type(x).__name__, dataclasses.astuple(x) if dataclasses.is_dataclass(x) else x) for x in index])


def lower_data_dims(analysis: StencilAnalysis) -> Tuple[StencilAnalysis, Dict[str, Component]]:
    st = analysis.stencil
    dd_fields = {p.name: p for p in st.field_params() if p.data_dims}
    dd_temps = {t.name: t for t in st.temporaries if t.data_dims}
    if not dd_fields and not dd_temps:
        return analysis, {}
    temp_comps: Dict[Tuple[str, Tuple[int, ...]], str] = {}

    def temp_comp(acc: ir.FieldAccess) -> str:
        if not all(isinstance(x, ir.Literal) for x in acc.data_index):
            raise UnsupportedStencil(f"run-time data index into temporary '{acc.name}'")
        idx = tuple(int(x.value) for x in acc.data_index)
        k = (acc.name, idx)
        if k not in temp_comps:
            temp_comps[k] = f"{acc.name}__t{'_'.join(str(i) for i in idx)}"
        return temp_comps[k]

    comps: Dict[str, Component] = {}
    by_key: Dict[Tuple[str, str], str] = {}
    written: Dict[str, set] = {}

    def comp_name(acc: ir.FieldAccess) -> str:
        if not all(_uniform(x) for x in acc.data_index):
            raise UnsupportedStencil(f"data index of '{acc.name}' varies across grid points")
        k = (acc.name, _key(acc.data_index))
        if k not in by_key:
            vname = f"{acc.name}__c{sum(1 for b in by_key if b[0] == acc.name)}"
            by_key[k] = vname
            comps[vname] = Component(acc.name, list(acc.data_index))
        return by_key[k]

    def fn(e):
        if isinstance(e, ir.FieldAccess) and e.name in dd_fields:
            return ir.FieldAccess(comp_name(e), e.offset, e.dtype, [], e.k_offset)
        if isinstance(e, ir.FieldAccess) and e.name in dd_temps:
            return ir.FieldAccess(temp_comp(e), e.offset, e.dtype, [], e.k_offset)
        return e

    # a written field: its components must be provably distinct (literal indices) or just one
    keys: Dict[str, set] = {}
    runtime: Dict[str, bool] = {}
    for vl in st.vertical_loops:
        for sec in vl.sections:
            for acc, w in passes.iter_accesses(sec.body):
                if isinstance(acc, ir.FieldAccess) and acc.name in dd_fields:
                    keys.setdefault(acc.name, set()).add(_key(acc.data_index))
                    if not all(isinstance(x, ir.Literal) for x in acc.data_index):
                        runtime[acc.name] = True
                    if w:
                        written[acc.name] = set()
    for name in written:
        if runtime.get(name) and len(keys[name]) > 1:
            raise UnsupportedStencil(f"'{name}' is written with run-time data indices that may alias")

    loops = [ir.map_expr(vl, fn) for vl in st.vertical_loops]
    params = []
    virtual_decls = []
    for p in st.params:
        if isinstance(p, ir.FieldDecl) and p.name in dd_fields:
            for vname, c in comps.items():
                if c.base == p.name:
                    virtual_decls.append(ir.FieldDecl(vname, p.dtype, p.axes, (), False))
            continue
        params.append(p)
    params += virtual_decls
    temps = [t for t in st.temporaries if t.name not in dd_temps]
    temps += [ir.FieldDecl(v, dd_temps[n].dtype, dd_temps[n].axes, (), True) for (n, _), v in temp_comps.items()]
    lowered = ir.Stencil(st.name, st.api_signature, params, temps, loops, st.externals, st.docstring)
    extents = passes.compute_extents(lowered)
    out = StencilAnalysis(
        lowered,
        passes.compute_access_kinds(lowered),
        extents,
        passes.compute_k_boundary(lowered),
        analysis.min_k_size,
    )
    return out, comps


# ------------------------------------------------------------------------------------------
# phase splitting: the general multi-stage lowering (column kernels + scratch temporaries)
# ------------------------------------------------------------------------------------------


def _stmt_accesses(s):
    reads, writes = [], []
    for acc, w in passes.iter_accesses([s]):
        if isinstance(acc, ir.FieldAccess):
            (writes if w else reads).append(acc)
    return reads, writes


def _loop_phases(vl: ir.VerticalLoop) -> List[int]:
    """Phase of every top-level statement (flattened over sections, program order).

    Splitting a computation into phases (one sub-computation per phase, same order and intervals)
    is legal when every value a statement reads is still produced before (RAW) or after (WAR) the
    read, as in the original order; an access at a horizontal offset (another column) or, inside one
    column, at a vertical offset the sweep has not reached, needs the two statements in different
    phases. Constraints ``phase(b) >= phase(a) + d`` are solved by longest paths; a positive cycle
    means the computation cannot be staged.
    """
    stmts = [s for sec in vl.sections for s in sec.body]
    n = len(stmts)
    acc = [_stmt_accesses(s) for s in stmts]
    fwd = vl.loop_order != ir.LoopOrder.BACKWARD
    par = vl.loop_order == ir.LoopOrder.PARALLEL
    edges = []  # (a, b, d): phase[b] >= phase[a] + d
    for si in range(n):
        for r in acc[si][0]:
            for wi in range(n):
                for w in acc[wi][1]:
                    if w.name != r.name:
                        continue
                    di, dj, dk = r.offset
                    dk -= w.offset[2]
                    ij = bool(di or dj)
                    var_k = r.k_offset is not None or w.k_offset is not None
                    if par:
                        raw = wi < si
                        d = 1 if (ij or dk or var_k) else 0
                    else:
                        if var_k:
                            # unknown level: keep reader and writer in one column sweep
                            if ij:
                                raise UnsupportedStencil(f"'{r.name}': run-time K offset across columns")
                            if wi != si:
                                edges.append((wi, si, 0))
                                edges.append((si, wi, 0))
                            continue
                        before = dk < 0 if fwd else dk > 0
                        raw = before or (dk == 0 and wi < si)
                        d = 1 if ij else 0
                    if wi == si:
                        if raw and d:
                            raise UnsupportedStencil(f"'{r.name}' feeds itself at a horizontal offset")
                        continue
                    edges.append((wi, si, d) if raw else (si, wi, d))
    for a in range(n):  # writers of one name keep their order
        for b in range(a + 1, n):
            if {w.name for w in acc[a][1]} & {w.name for w in acc[b][1]}:
                edges.append((a, b, 0))
    phase = [0] * n
    for _ in range(n + 1):
        changed = False
        for a, b, d in edges:
            if phase[b] < phase[a] + d:
                phase[b] = phase[a] + d
                changed = True
        if not changed:
            return phase
    raise UnsupportedStencil("statements depend on each other across columns in both directions")


def split_phases(analysis: StencilAnalysis) -> StencilAnalysis:
    """Split every computation into its phases (``_loop_phases``) so that each piece can run as
    a column kernel; temporaries crossing pieces become scratch fields in the plan."""
    st = analysis.stencil
    loops: List[ir.VerticalLoop] = []
    for vl in st.vertical_loops:
        phases = _loop_phases(vl)
        if not phases or max(phases) == 0:
            loops.append(vl)
            continue
        for p in range(max(phases) + 1):
            secs = []
            t = 0
            for sec in vl.sections:
                body = []
                for s in sec.body:
                    if phases[t] == p:
                        body.append(s)
                    t += 1
                if body:
                    secs.append(ir.Section(sec.interval, body))
            if secs:
                loops.append(ir.VerticalLoop(vl.loop_order, secs))
    if len(loops) == len(st.vertical_loops):
        return analysis
    new = dataclasses.replace(st, vertical_loops=loops)
    return StencilAnalysis(
        new,
        passes.compute_access_kinds(new),
        passes.compute_extents(new),
        passes.compute_k_boundary(new),
        analysis.min_k_size,
    )


# ------------------------------------------------------------------------------------------
# fusion of adjacent PARALLEL computations
# ------------------------------------------------------------------------------------------


def _same_intervals(a: ir.VerticalLoop, b: ir.VerticalLoop) -> bool:
    if len(a.sections) != len(b.sections):
        return False
    for sa, sb in zip(a.sections, b.sections):
        for x, y in ((sa.interval.start, sb.interval.start), (sa.interval.end, sb.interval.end)):
            if x.level != y.level or x.offset != y.offset:
                return False
    return True


def _fusable(a: ir.VerticalLoop, b: ir.VerticalLoop, api: set) -> bool:
    """Can computation ``b`` run inside computation ``a`` (statements appended per section)
    without changing any result? Both PARALLEL over the same intervals, and the merged loop obeys
    the parallel model: nothing written by one is read by the other at a K offset (levels of one
    PARALLEL loop run in any order), no API field written in either is read at an IJ offset in
    either (the merged loop would read a field it writes across columns), ``a`` reads nothing
    ``b`` writes, and no run-time K offsets."""
    if a.loop_order != ir.LoopOrder.PARALLEL or b.loop_order != ir.LoopOrder.PARALLEL:
        return False
    if not _same_intervals(a, b):
        return False
    acc_a = [x for sec in a.sections for x in passes.iter_accesses(sec.body)]
    acc_b = [x for sec in b.sections for x in passes.iter_accesses(sec.body)]
    for acc, _ in acc_a + acc_b:
        if isinstance(acc, ir.FieldAccess) and acc.k_offset is not None:
            return False
    wa = {acc.name for acc, w in acc_a if w}
    wb = {acc.name for acc, w in acc_b if w}
    for acc, w in acc_b:
        if not w and isinstance(acc, ir.FieldAccess) and acc.name in wa and acc.offset[2] != 0:
            return False
    for acc, w in acc_a:
        if not w and acc.name in wb:
            return False
    written_api = (wa | wb) & api
    for acc, w in acc_a + acc_b:
        if not w and isinstance(acc, ir.FieldAccess) and acc.name in written_api and (acc.offset[0] or acc.offset[1]):
            return False
    return True


def fuse_parallel_loops(analysis: StencilAnalysis) -> StencilAnalysis:
    """Merge consecutive PARALLEL computations over identical intervals into one, so that a
    temporary one computation produces and the next reads at IJ offsets lives in the plane
    kernel's register rings instead of a scratch field round trip through HBM (e.g. hdiff
    written as lap / flux / update blocks runs as ONE launch, like the single-block form).
    The reference keeps such computations as separate vertical loops (its AdjacentLoopMerging,
    ``gtc/passes/oir_optimizations/vertical_loop_merging.py:16-29``, only joins loops whose
    intervals touch); merging here changes no result (same statements, same order per point)."""
    st = analysis.stencil
    api = {p.name for p in st.field_params()}
    loops: List[ir.VerticalLoop] = []
    for vl in st.vertical_loops:
        if loops and _fusable(loops[-1], vl, api):
            prev = loops[-1]
            loops[-1] = ir.VerticalLoop(
                prev.loop_order,
                [ir.Section(sa.interval, list(sa.body) + list(sb.body), sa.def_index)
                 for sa, sb in zip(prev.sections, vl.sections)],
            )
        else:
            loops.append(vl)
    if len(loops) == len(st.vertical_loops):
        return analysis
    new = dataclasses.replace(st, vertical_loops=loops)
    return StencilAnalysis(
        new,
        passes.compute_access_kinds(new),
        passes.compute_extents(new),
        passes.compute_k_boundary(new),
        analysis.min_k_size,
    )


# ------------------------------------------------------------------------------------------
# fusion of consecutive sequential computations (for the tile kernel)
# ------------------------------------------------------------------------------------------


def _whole_range(vl: ir.VerticalLoop) -> bool:
    if len(vl.sections) != 1:
        return False
    itv = vl.sections[0].interval
    return (itv.start.level == ir.LevelMarker.START and itv.start.offset == 0
            and itv.end.level == ir.LevelMarker.END and itv.end.offset == 0)


def _covers_range(vl: ir.VerticalLoop) -> bool:
    """Sections contiguous from START+0 to END+0 (taken in level order: a BACKWARD
    computation usually lists its top interval first)."""
    rank = {ir.LevelMarker.START: 0, ir.LevelMarker.END: 1}
    secs = sorted(vl.sections, key=lambda s: (rank[s.interval.start.level], s.interval.start.offset))
    if not secs:
        return False
    s0, s1 = secs[0].interval.start, secs[-1].interval.end
    if not (s0.level == ir.LevelMarker.START and s0.offset == 0 and s1.level == ir.LevelMarker.END and s1.offset == 0):
        return False
    for a, b in zip(secs, secs[1:]):
        if a.interval.end.level != b.interval.start.level or a.interval.end.offset != b.interval.start.offset:
            return False
    return True


def _aligned_sections(a: ir.VerticalLoop, b: ir.VerticalLoop):
    """Pairs of (interval, body_a, body_b) over a common partition of the levels, or None."""
    if _same_intervals(a, b):
        return [(sa.interval, sa.body, sb.body, sa.def_index) for sa, sb in zip(a.sections, b.sections)]
    if _whole_range(b) and _covers_range(a):
        return [(sa.interval, sa.body, b.sections[0].body, sa.def_index) for sa in a.sections]
    if _whole_range(a) and _covers_range(b):
        return [(sb.interval, a.sections[0].body, sb.body, sb.def_index) for sb in b.sections]
    return None


def _seq_fusable(a: ir.VerticalLoop, b: ir.VerticalLoop, api: set) -> bool:
    """Can sequential computation ``b`` run inside ``a``'s K sweep (statements appended per
    level) without changing any result? Same order (FORWARD or BACKWARD), aligned intervals, no
    run-time K offsets, no name written by both, ``a`` reads nothing ``b`` writes, and every
    read in ``b`` of a value ``a`` produces is at a level the fused sweep has already produced
    (K offset <= 0 forward, >= 0 backward), at the same level when it is read across columns
    (the tile kernel exchanges one level through LDS), never an API field across columns."""
    if a.loop_order != b.loop_order or a.loop_order == ir.LoopOrder.PARALLEL:
        return False
    if _aligned_sections(a, b) is None:
        return False
    fwd = a.loop_order == ir.LoopOrder.FORWARD
    acc_a = [x for sec in a.sections for x in passes.iter_accesses(sec.body)]
    acc_b = [x for sec in b.sections for x in passes.iter_accesses(sec.body)]
    for acc, _ in acc_a + acc_b:
        if isinstance(acc, ir.FieldAccess) and acc.k_offset is not None:
            return False
    wa = {acc.name for acc, w in acc_a if w}
    wb = {acc.name for acc, w in acc_b if w}
    if wa & wb:
        return False
    for acc, w in acc_a:
        if not w and acc.name in wb:
            return False
    for acc, w in acc_b:
        if w or not isinstance(acc, ir.FieldAccess) or acc.name not in wa:
            continue
        di, dj, dk = acc.offset
        if (dk > 0) if fwd else (dk < 0):
            return False
        if (di or dj) and (dk != 0 or acc.name in api):
            return False
    return True


def fuse_sequential_loops(analysis: StencilAnalysis) -> StencilAnalysis:
    """Merge consecutive FORWARD (or BACKWARD) computations into one K sweep when legal
    (``_seq_fusable``), so that a column recurrence feeding a temporary that a later computation
    reads across columns (``staged_forward_ij_temp``) needs neither a scratch field for the
    recurrence nor a second sweep: the tile kernel (``codegen/column.py``, tile mode) then runs
    the whole sweep with the cross-column temporary in an LDS plane per level. Used only when the
    two skeletons cannot take the computations as written; per column and level the statements
    run in the original order, so no result changes."""
    st = analysis.stencil
    api = {p.name for p in st.field_params()}
    loops: List[ir.VerticalLoop] = []
    for vl in st.vertical_loops:
        if loops and _seq_fusable(loops[-1], vl, api):
            prev = loops[-1]
            loops[-1] = ir.VerticalLoop(
                prev.loop_order,
                [ir.Section(itv, list(ba) + list(bb), di) for itv, ba, bb, di in _aligned_sections(prev, vl)],
            )
        else:
            loops.append(vl)
    if len(loops) == len(st.vertical_loops):
        return analysis
    new = dataclasses.replace(st, vertical_loops=loops)
    return StencilAnalysis(
        new,
        passes.compute_access_kinds(new),
        passes.compute_extents(new),
        passes.compute_k_boundary(new),
        analysis.min_k_size,
    )
