"""Analysis and typing passes over ``gt4py_amd.ir``.

Each pass restates the reference semantics it follows:

- ``resolve_dtypes``: ``gtc/passes/gtir_dtype_resolver.py:17-84`` (temporaries take the dtype
  of the right-hand side of their FIRST assignment) with the non-strict propagation of
  ``gtc/common.py:285-305, 511-631`` (arithmetic -> max dtype, comparison -> bool, ...).
- ``upcast``: ``gtc/passes/gtir_upcaster.py:42-147`` -- explicit ``Cast`` nodes chosen with the
  NumPy-ufunc loop rule on the gt4py ``DataType`` ordering.
- ``compute_access_kinds``: ``gtc/passes/oir_access_kinds.py:20-70`` (first access decides,
  READ then WRITE -> READ_WRITE).
- ``compute_extents``: ``gtc/passes/oir_optimizations/utils.py:250-330`` (reverse sweep over
  horizontal executions; an execution's extent is the union of its written fields' extents).
- ``compute_k_boundary`` / ``compute_min_k_size``: ``gtc/passes/gtir_k_boundary.py:24-109``.
- ``validate_memory_accesses``: ``gtc/gtir_to_oir.py:19-47``.
"""

from __future__ import annotations

import dataclasses
import functools
import math
from typing import Dict, List, Optional, Set, Tuple

import numpy as np

from gt4py_amd import ir
from gt4py_amd.definitions import AccessKind
from gt4py_amd.ir import DataType

# --------------------------------------------------------------------------------------
# dtype propagation
# --------------------------------------------------------------------------------------


def _node_dtype(e: ir.Expr) -> DataType:
    """(Re)compute the dtype of an expression node from its (typed) children."""
    if isinstance(e, (ir.Literal, ir.FieldAccess, ir.ScalarAccess, ir.Cast, ir.AxisIndex)):
        return e.dtype
    if isinstance(e, ir.BinaryOp):
        lt, rt = e.left.dtype, e.right.dtype
        if e.op in ir.COMPARE_OPS:
            return DataType.BOOL
        if e.op in ir.LOGICAL_OPS:
            if lt != DataType.BOOL or rt != DataType.BOOL:
                raise TypeError("Arithmetic expression is not allowed in boolean operation.")
            return DataType.BOOL
        common = max(lt, rt)
        if common == DataType.BOOL:
            raise TypeError("Boolean expression is not allowed with arithmetic operation.")
        return common
    if isinstance(e, ir.UnaryOp):
        if e.op == "not":
            return DataType.BOOL
        return e.expr.dtype
    if isinstance(e, ir.TernaryOp):
        return max(e.true_expr.dtype, e.false_expr.dtype)
    if isinstance(e, ir.NativeCall):
        f = e.func
        if f in ("isfinite", "isinf", "isnan"):
            return DataType.BOOL
        if f in ("int32", "int64", "float32", "float64"):
            return DataType[f.upper()]
        return max(a.dtype for a in e.args)
    raise TypeError(type(e))


def resolve_dtypes(stencil: ir.Stencil) -> ir.Stencil:
    """Propagate declaration dtypes to accesses and resolve temporaries (AUTO) in order."""
    decls: Dict[str, object] = {p.name: p for p in stencil.params}
    temp_dtype: Dict[str, DataType] = {}
    declared = getattr(stencil, "temp_declared_dtype", {}) or {}
    for t in stencil.temporaries:
        decls[t.name] = t
        if t.name in declared:
            temp_dtype[t.name] = declared[t.name]

    def type_expr(e: ir.Expr) -> ir.Expr:
        if isinstance(e, ir.FieldAccess):
            d = decls[e.name]
            if getattr(d, "is_temporary", False):
                if e.name not in temp_dtype:
                    raise TypeError(f"Temporary '{e.name}' is read before being assigned")
                return dataclasses.replace(e, dtype=temp_dtype[e.name])
            return dataclasses.replace(e, dtype=d.dtype)
        if isinstance(e, ir.ScalarAccess):
            return dataclasses.replace(e, dtype=decls[e.name].dtype)
        return _retype(e)

    def visit_stmts(stmts):
        out = []
        for s in stmts:
            if isinstance(s, ir.Assign):
                value = ir.map_expr(s.value, type_expr)
                name = s.target.name
                d = decls[name]
                if getattr(d, "is_temporary", False) and name not in temp_dtype:
                    temp_dtype[name] = value.dtype
                tgt = dataclasses.replace(
                    s.target,
                    dtype=temp_dtype[name] if getattr(d, "is_temporary", False) else d.dtype,
                    data_index=[ir.map_expr(x, type_expr) for x in s.target.data_index],
                    k_offset=None if s.target.k_offset is None else ir.map_expr(s.target.k_offset, type_expr),
                )
                out.append(ir.Assign(tgt, value))
            elif isinstance(s, ir.If):
                cond = ir.map_expr(s.cond, type_expr)
                out.append(ir.If(cond, visit_stmts(s.body), visit_stmts(s.orelse)))
            elif isinstance(s, ir.While):
                cond = ir.map_expr(s.cond, type_expr)
                out.append(ir.While(cond, visit_stmts(s.body)))
            elif isinstance(s, ir.HorizontalRegion):
                out.append(ir.HorizontalRegion(s.masks, visit_stmts(s.body)))
            else:
                raise TypeError(type(s))
        return out

    loops = []
    for vl in stencil.vertical_loops:
        secs = [ir.Section(sec.interval, visit_stmts(sec.body)) for sec in vl.sections]
        loops.append(ir.VerticalLoop(vl.loop_order, secs))
    temps = [dataclasses.replace(t, dtype=temp_dtype.get(t.name, DataType.FLOAT64)) for t in stencil.temporaries]
    new = dataclasses.replace(stencil, vertical_loops=loops, temporaries=temps)
    return new


def _retype(e: ir.Expr) -> ir.Expr:
    if isinstance(e, (ir.Literal, ir.FieldAccess, ir.ScalarAccess, ir.AxisIndex, ir.Cast)):
        return e
    return dataclasses.replace(e, dtype=_node_dtype(e))


# --------------------------------------------------------------------------------------
# upcasting (NumPy ufunc loop rule on the gt4py DataType ordering)
# --------------------------------------------------------------------------------------

_CUSTOM_UFUNC_TYPES = {
    # gtc/ufuncs.py: scipy.special / custom functions registered with these loops
    "gamma": ["f->f", "d->d"],
    "erf": ["f->f", "d->d"],
    "erfc": ["f->f", "d->d"],
    "round": ["f->f", "d->d"],
    "round_away_from_zero": ["f->f", "d->d"],
}

_OP_TO_UFUNC = {
    "+": "add",
    "-": "subtract",
    "*": "multiply",
    "/": "true_divide",
    ">": "greater",
    "<": "less",
    ">=": "greater_equal",
    "<=": "less_equal",
    "==": "equal",
    "!=": "not_equal",
    "and": "logical_and",
    "or": "logical_or",
}
_UNARY_TO_UFUNC = {"+": "positive", "-": "negative", "not": "logical_not"}
_NATIVE_TO_UFUNC = {
    "abs": "absolute",
    "min": "minimum",
    "max": "maximum",
    "mod": "remainder",
    "sin": "sin",
    "cos": "cos",
    "tan": "tan",
    "arcsin": "arcsin",
    "arccos": "arccos",
    "arctan": "arctan",
    "sinh": "sinh",
    "cosh": "cosh",
    "tanh": "tanh",
    "arcsinh": "arcsinh",
    "arccosh": "arccosh",
    "arctanh": "arctanh",
    "sqrt": "sqrt",
    "exp": "exp",
    "log": "log",
    "log10": "log10",
    "cbrt": "cbrt",
    "isfinite": "isfinite",
    "isinf": "isinf",
    "isnan": "isnan",
    "floor": "floor",
    "ceil": "ceil",
    "trunc": "trunc",
}


def _typechar_to_dt(ch: str) -> DataType:
    try:
        return DataType.from_np(np.dtype(ch))
    except TypeError:
        return DataType.INVALID


@functools.lru_cache(maxsize=None)
def _ufunc_types(name: str) -> Tuple[Tuple[Tuple[DataType, ...], DataType], ...]:
    if name in _CUSTOM_UFUNC_TYPES:
        types = _CUSTOM_UFUNC_TYPES[name]
    else:
        types = getattr(np, name).types
    out = []
    for t in types:
        ins, outs = t.split("->")
        out.append((tuple(_typechar_to_dt(c) for c in ins), _typechar_to_dt(outs[0])))
    return tuple(out)


@functools.lru_cache(maxsize=None)
def ufunc_upcast(name: str, dtypes: Tuple[DataType, ...]) -> Tuple[DataType, ...]:
    """``_numpy_ufunc_upcasting_rule`` (gtir_upcaster.py:42-70)."""
    matched = {}
    for ins, _ in _ufunc_types(name):
        if len(ins) != len(dtypes):
            continue
        if any(c == DataType.INVALID for c in ins):
            continue
        if all(a <= c for a, c in zip(dtypes, ins)):
            matched[sum(int(c) for c in ins)] = ins
    if not matched:
        raise TypeError(f"No '{name}' implementation for argument types {[d.name for d in dtypes]}")
    return matched[min(matched)]


def _cast(target: DataType, e: ir.Expr) -> ir.Expr:
    return e if e.dtype == target else ir.Cast(target, e)


def _upcast_expr(e: ir.Expr) -> ir.Expr:
    if isinstance(e, ir.BinaryOp):
        l, r = _upcast_expr(e.left), _upcast_expr(e.right)
        tl, tr = ufunc_upcast(_OP_TO_UFUNC[e.op], (l.dtype, r.dtype))
        return _retype(ir.BinaryOp(e.op, _cast(tl, l), _cast(tr, r)))
    if isinstance(e, ir.UnaryOp):
        x = _upcast_expr(e.expr)
        (t,) = ufunc_upcast(_UNARY_TO_UFUNC[e.op], (x.dtype,))
        return _retype(ir.UnaryOp(e.op, _cast(t, x)))
    if isinstance(e, ir.TernaryOp):
        c = _upcast_expr(e.cond)
        t, f = _upcast_expr(e.true_expr), _upcast_expr(e.false_expr)
        common = max(t.dtype, f.dtype)
        return _retype(ir.TernaryOp(c, _cast(common, t), _cast(common, f)))
    if isinstance(e, ir.NativeCall):
        args = [_upcast_expr(a) for a in e.args]
        if e.func in ("int32", "int64", "float32", "float64", "pow"):
            return _retype(ir.NativeCall(e.func, args))
        targets = ufunc_upcast(_NATIVE_TO_UFUNC.get(e.func, e.func), tuple(a.dtype for a in args))
        return _retype(ir.NativeCall(e.func, [_cast(t, a) for t, a in zip(targets, args)]))
    if isinstance(e, ir.Cast):
        return ir.Cast(e.dtype, _upcast_expr(e.expr))
    if isinstance(e, ir.FieldAccess) and (e.data_index or e.k_offset is not None):
        return dataclasses.replace(
            e,
            data_index=[_upcast_expr(x) for x in e.data_index],
            k_offset=None if e.k_offset is None else _upcast_expr(e.k_offset),
        )
    return e


def upcast(stencil: ir.Stencil) -> ir.Stencil:
    def visit_stmts(stmts):
        out = []
        for s in stmts:
            if isinstance(s, ir.Assign):
                v = _upcast_expr(s.value)
                out.append(ir.Assign(_upcast_expr(s.target), _cast(s.target.dtype, v)))
            elif isinstance(s, ir.If):
                out.append(ir.If(_upcast_expr(s.cond), visit_stmts(s.body), visit_stmts(s.orelse)))
            elif isinstance(s, ir.While):
                out.append(ir.While(_upcast_expr(s.cond), visit_stmts(s.body)))
            elif isinstance(s, ir.HorizontalRegion):
                out.append(ir.HorizontalRegion(s.masks, visit_stmts(s.body)))
            else:
                raise TypeError(type(s))
        return out

    loops = [
        ir.VerticalLoop(vl.loop_order, [ir.Section(sec.interval, visit_stmts(sec.body)) for sec in vl.sections])
        for vl in stencil.vertical_loops
    ]
    return dataclasses.replace(stencil, vertical_loops=loops)


# --------------------------------------------------------------------------------------
# access helpers
# --------------------------------------------------------------------------------------


def stmt_writes(stmts) -> List[str]:
    """Names assigned in a statement list (recursively), in program order."""
    out: List[str] = []
    for n in ir.walk(list(stmts)):
        if isinstance(n, ir.Assign) and n.target.name not in out:
            out.append(n.target.name)
    return out


def iter_accesses(stmts):
    """Yield (FieldAccess|ScalarAccess, is_write) in the reference visiting order.

    AssignStmt: right side first (READ), then the target (WRITE); If: condition, then
    bodies; While: condition, then body (``oir_access_kinds.py:36-52``).
    """

    def expr_accesses(e):
        for n in ir.walk(e):
            if isinstance(n, (ir.FieldAccess, ir.ScalarAccess)):
                yield n, False

    def visit(s):
        if isinstance(s, ir.Assign):
            yield from expr_accesses(s.value)
            for sub in list(s.target.data_index) + ([s.target.k_offset] if s.target.k_offset is not None else []):
                yield from expr_accesses(sub)
            yield s.target, True
        elif isinstance(s, ir.If):
            yield from expr_accesses(s.cond)
            for x in s.body:
                yield from visit(x)
            for x in s.orelse:
                yield from visit(x)
        elif isinstance(s, ir.While):
            yield from expr_accesses(s.cond)
            for x in s.body:
                yield from visit(x)
        elif isinstance(s, ir.HorizontalRegion):
            for x in s.body:
                yield from visit(x)

    for s in stmts:
        yield from visit(s)


def compute_access_kinds(stencil: ir.Stencil) -> Dict[str, AccessKind]:
    """First access decides READ / WRITE, a later write makes READ_WRITE; the body of a horizontal
    region that cannot overlap its statement's (signed) extent is not visited
    (``oir_access_kinds.py:43-48``)."""
    access: Dict[str, AccessKind] = {}
    blocks: dict = {}
    compute_signed_extents(stencil, blocks)

    def visible(stmts, he):
        for s in stmts:
            if isinstance(s, ir.HorizontalRegion):
                if any(mask_overlap(m, he) is not None for m in s.masks):
                    yield from visible(s.body, he)
            elif isinstance(s, (ir.If, ir.While)):
                yield type(s)(s.cond, [], []) if isinstance(s, ir.If) else type(s)(s.cond, [])
                yield from visible(s.body, he)
                if isinstance(s, ir.If):
                    yield from visible(s.orelse, he)
            else:
                yield s

    for li, vl in enumerate(stencil.vertical_loops):
        for si, sec in enumerate(vl.sections):
            stmts = [x for ti, s in enumerate(sec.body)
                     for x in visible([s], blocks.get((li, si, ti), ((0, 0), (0, 0))))]
            for acc, is_write in iter_accesses(stmts):
                kind = AccessKind.WRITE if is_write else AccessKind.READ
                if kind == AccessKind.WRITE and access.get(acc.name) == AccessKind.READ:
                    access[acc.name] = AccessKind.READ_WRITE
                elif acc.name not in access:
                    access[acc.name] = kind
    for p in stencil.params:
        access.setdefault(p.name, AccessKind.NONE)
    return access


# --------------------------------------------------------------------------------------
# horizontal extents
# --------------------------------------------------------------------------------------

Extent = Tuple[Tuple[int, int], Tuple[int, int]]  # ((i_lo, i_hi), (j_lo, j_hi)) halo sizes >= 0
ZERO_EXTENT: Extent = ((0, 0), (0, 0))


def extent_union(a: Extent, b: Extent) -> Extent:
    return ((max(a[0][0], b[0][0]), max(a[0][1], b[0][1])), (max(a[1][0], b[1][0]), max(a[1][1], b[1][1])))


def extent_shift(e: Extent, offset) -> Extent:
    di, dj = offset[0], offset[1]
    return ((max(0, e[0][0] - di), max(0, e[0][1] + di)), (max(0, e[1][0] - dj), max(0, e[1][1] + dj)))


def _overlap_along_axis(ext, itv) -> Optional[Tuple[int, int]]:
    """Distances of a region interval to the edges of a (signed) extent, or None when the region
    cannot overlap it (reference ``gtc/passes/horizontal_masks.py:15-47``)."""
    if itv.start is None:
        start_diff = 1000
    elif itv.start.level == ir.LevelMarker.START:
        start_diff = ext[0] - itv.start.offset
    else:
        start_diff = None
    if itv.end is None:
        end_diff = -1000
    elif itv.end.level == ir.LevelMarker.END:
        end_diff = ext[1] - itv.end.offset
    else:
        end_diff = None
    if start_diff is not None and start_diff > 0 and end_diff is None and itv.end is not None:
        if itv.end.offset <= ext[0]:
            return None
    elif end_diff is not None and end_diff < 0 and start_diff is None and itv.start is not None:
        if itv.start.offset > ext[1]:
            return None
    start_diff = min(start_diff, 0) if start_diff is not None else -10000
    end_diff = max(end_diff, 0) if end_diff is not None else 10000
    return start_diff, end_diff


def mask_overlap(mask, he_signed) -> Optional[Extent]:
    """``mask_overlap_with_extent`` (horizontal_masks.py:50-58) on a signed extent."""
    di = _overlap_along_axis(he_signed[0], mask.i)
    dj = _overlap_along_axis(he_signed[1], mask.j)
    return None if di is None or dj is None else (di, dj)


def region_access_extent(masks, he_signed, di: int, dj: int) -> Optional[Extent]:
    """Signed extent of a read at (di, dj) inside horizontal regions ``masks`` of a statement
    with signed horizontal extent ``he_signed``: ``((he - dist_from_edge) + offset) | zeros``
    per mask (``GenericAccess.to_extent``, oir_optimizations/utils.py:50-75), unioned; None when
    no mask overlaps (the access then reads nothing)."""
    out = None
    for m in masks:
        d = mask_overlap(m, he_signed)
        if d is None:
            continue
        e = ((min(he_signed[0][0] - d[0][0] + di, 0), max(he_signed[0][1] - d[0][1] + di, 0)),
             (min(he_signed[1][0] - d[1][0] + dj, 0), max(he_signed[1][1] - d[1][1] + dj, 0)))
        out = e if out is None else ((min(out[0][0], e[0][0]), max(out[0][1], e[0][1])),
                                     (min(out[1][0], e[1][0]), max(out[1][1], e[1][1])))
    return out


def _to_signed(e: Extent) -> Extent:
    return ((-e[0][0], e[0][1]), (-e[1][0], e[1][1]))


def _to_centered(e: Extent) -> Extent:
    return ((max(0, -e[0][0]), max(0, e[0][1])), (max(0, -e[1][0]), max(0, e[1][1])))


@dataclasses.dataclass
class ExtentInfo:
    fields: Dict[str, Extent]
    blocks: Dict[Tuple[int, int, int], Extent]  # (loop, section, statement) -> extent


def compute_extents(stencil: ir.Stencil) -> ExtentInfo:
    fields: Dict[str, Extent] = {}
    blocks: Dict[Tuple[int, int, int], Extent] = {}
    for li in reversed(range(len(stencil.vertical_loops))):
        vl = stencil.vertical_loops[li]
        for si in reversed(range(len(vl.sections))):
            sec = vl.sections[si]
            for ti in reversed(range(len(sec.body))):
                stmt = sec.body[ti]
                accesses = list(iter_accesses([stmt]))
                he = ZERO_EXTENT
                for acc, is_write in accesses:
                    if is_write:
                        he = extent_union(he, fields.setdefault(acc.name, ZERO_EXTENT))
                blocks[(li, si, ti)] = he
                for acc, is_write, masks in _accesses_with_region([stmt]):
                    if isinstance(acc, ir.FieldAccess):
                        if masks is None:
                            ext = extent_shift(he, acc.offset)
                        else:  # inside a horizontal region: clipped by its mask (reference semantics)
                            se = region_access_extent(masks, _to_signed(he), acc.offset[0], acc.offset[1])
                            if se is None:
                                continue
                            ext = _to_centered(se)
                        fields[acc.name] = extent_union(fields.get(acc.name, ZERO_EXTENT), ext)
    for p in stencil.params:
        fields.setdefault(p.name, ZERO_EXTENT)
    return ExtentInfo(fields, blocks)


def _accesses_with_region(stmts, in_region=None):
    """(access, is_write, masks of the enclosing horizontal region or None) in
    :func:`iter_accesses` order."""
    for s in stmts:
        if isinstance(s, ir.HorizontalRegion):
            yield from _accesses_with_region(s.body, s.masks)
        elif isinstance(s, (ir.If, ir.While)):
            for acc, w in iter_accesses([type(s)(s.cond, [], []) if isinstance(s, ir.If) else type(s)(s.cond, [])]):
                yield acc, w, in_region
            yield from _accesses_with_region(s.body, in_region)
            if isinstance(s, ir.If):
                yield from _accesses_with_region(s.orelse, in_region)
        else:
            for acc, w in iter_accesses([s]):
                yield acc, w, in_region


def compute_signed_extents(stencil: ir.Stencil, blocks_out: Optional[dict] = None) -> Dict[str, Extent]:
    """Per-field extents as signed offset ranges ``((i_min, i_max), (j_min, j_max))``, the
    non-centered extents the reference reports in ``FieldInfo.boundary``
    (``oir_optimizations/utils.py:250-315``: a read at ``he + offset`` is NOT widened to include
    offset 0, so a field read only at ``[1, 0, 0]`` gets the boundary ``(-1, 1)`` in I and may be
    called with origin -1; accesses inside horizontal regions are clipped by the region's mask and
    widened to 0, ``GenericAccess.to_extent``). Code generation keeps using the centered halo
    sizes of :func:`compute_extents`. ``blocks_out``: filled with the signed statement extents
    ((loop, section, statement) -> extent, ``compute_horizontal_block_extents``)."""
    zero = ((0, 0), (0, 0))

    def union(a, b):
        return ((min(a[0][0], b[0][0]), max(a[0][1], b[0][1])), (min(a[1][0], b[1][0]), max(a[1][1], b[1][1])))

    fields: Dict[str, Extent] = {}
    for li in reversed(range(len(stencil.vertical_loops))):
        vl = stencil.vertical_loops[li]
        for si in reversed(range(len(vl.sections))):
            sec = vl.sections[si]
            for ti in reversed(range(len(sec.body))):
                stmt = sec.body[ti]
                accesses = list(_accesses_with_region([stmt]))
                he = zero
                for acc, is_write, _ in accesses:
                    if is_write:
                        he = union(he, fields.setdefault(acc.name, zero))
                if blocks_out is not None:
                    blocks_out[(li, si, ti)] = he
                for acc, _, masks in accesses:
                    if not isinstance(acc, ir.FieldAccess):
                        continue
                    di, dj = acc.offset[0], acc.offset[1]
                    if masks is None:
                        ext = ((he[0][0] + di, he[0][1] + di), (he[1][0] + dj, he[1][1] + dj))
                    else:
                        ext = region_access_extent(masks, he, di, dj)
                        if ext is None:
                            continue
                    fields[acc.name] = union(fields[acc.name], ext) if acc.name in fields else ext
    for p in stencil.params:
        fields.setdefault(p.name, zero)
    return fields


# --------------------------------------------------------------------------------------
# K boundary and minimal K size
# --------------------------------------------------------------------------------------


def _outer_field_accesses(stmts):
    """FieldAccess nodes that are not nested in another access's run-time offset or data index
    (the reference's KBoundaryVisitor does not descend into a visited FieldAccess)."""
    stack = list(reversed(list(stmts)))
    while stack:
        n = stack.pop()
        if isinstance(n, ir.FieldAccess):
            yield n
            continue
        stack.extend(reversed(list(ir.iter_children(n))))


def compute_k_boundary(stencil: ir.Stencil) -> Dict[str, Tuple[int, int]]:
    temps = {t.name for t in stencil.temporaries}
    bounds: Dict[str, List[float]] = {}
    for vl in stencil.vertical_loops:
        for sec in vl.sections:
            itv = sec.interval
            for acc in _outer_field_accesses(sec.body):
                b = bounds.setdefault(acc.name, [-math.inf, -math.inf])
                if acc.k_offset is not None:
                    continue  # run-time offsets do not enter the boundary (gtir_k_boundary.py:55)
                k = acc.offset[2]
                if itv.start.level == ir.LevelMarker.START:
                    b[0] = max(-itv.start.offset - k, b[0])
                if itv.end.level == ir.LevelMarker.END:
                    b[1] = max(itv.end.offset + k, b[1])
                if acc.name in temps and (b[0] > 0 or b[1] > 0):
                    raise TypeError(f"Invalid access with offset in k to temporary field {acc.name}.")
    out = {}
    for name, b in bounds.items():
        out[name] = (int(b[0]) if b[0] != -math.inf else 0, int(b[1]) if b[1] != -math.inf else 0)
    for p in stencil.params:
        out.setdefault(p.name, (0, 0))
    return out


def compute_min_k_size(stencil: ir.Stencil) -> int:
    min_size_start = 0
    min_size_end = 0
    biggest_offset = 0
    for vl in stencil.vertical_loops:
        for sec in vl.sections:
            s, e = sec.interval.start, sec.interval.end
            if s.level == ir.LevelMarker.START and e.level == ir.LevelMarker.END:
                if not (s.offset == 0 and e.offset == 0):
                    biggest_offset = max(biggest_offset, s.offset - e.offset + 1)
            elif s.level == ir.LevelMarker.START and e.level == ir.LevelMarker.START:
                min_size_start = max(min_size_start, e.offset)
                biggest_offset = max(biggest_offset, e.offset)
            else:
                min_size_end = max(min_size_end, -s.offset)
                biggest_offset = max(biggest_offset, -s.offset)
    return max(min_size_start + min_size_end, biggest_offset)


def validate_memory_accesses(stencil: ir.Stencil, extents: ExtentInfo) -> None:
    field_names = {p.name for p in stencil.field_params()}
    written: Set[str] = set()
    for vl in stencil.vertical_loops:
        for sec in vl.sections:
            written.update(stmt_writes(sec.body))
    bad = sorted(n for n in written & field_names if extents.fields[n] != ZERO_EXTENT)
    if bad:
        raise ValueError(f"Found non-zero read extent on written fields: {', '.join(bad)}")


# --------------------------------------------------------------------------------------
# Pipeline
# --------------------------------------------------------------------------------------


@dataclasses.dataclass
class StencilAnalysis:
    stencil: ir.Stencil
    access: Dict[str, AccessKind]
    extents: ExtentInfo
    k_boundary: Dict[str, Tuple[int, int]]
    min_k_size: int

    signed_extents: Optional[Dict[str, Extent]] = None

    def boundary(self, name: str):
        """``FieldInfo.boundary``: (-min, max) of the signed I/J extents, the K boundary."""
        if self.signed_extents is not None and name in self.signed_extents:
            (a, b), (c, d) = self.signed_extents[name]
            return ((-a, b), (-c, d), self.k_boundary.get(name, (0, 0)))
        e = self.extents.fields.get(name, ZERO_EXTENT)
        return (e[0], e[1], self.k_boundary.get(name, (0, 0)))


def prune_unused_fields(stencil: ir.Stencil) -> ir.Stencil:
    return stencil


def _cartesian_h_reads(node) -> Set[str]:
    """Names read at a non-zero I/J offset (run-time K offsets excluded, ``gtir.py:326-348``)."""
    return {
        a.name for a in ir.walk(node)
        if isinstance(a, ir.FieldAccess) and a.k_offset is None and (a.offset[0] or a.offset[1])
    }


def _assign_writes(stmts) -> Set[str]:
    out: Set[str] = set()
    for n in ir.walk(stmts):
        if isinstance(n, ir.Assign):
            out |= {a.name for a in ir.walk(n.target) if isinstance(a, ir.FieldAccess)}
    return out


def validate_parallel_model(stencil: ir.Stencil) -> None:
    """The GTScript parallel-model rules the reference checks while building GTIR.

    Per statement (``gtc/gtir.py:95-109``): no assignment reads its own target at an I/J offset.
    Per while loop (``:152-166``) and per computation block (``:226-240``; temporaries first
    assigned in the block exempt): no field is both written and read at an I/J offset. Per
    PARALLEL block of more than one static level (``:242-300``): a written field is read at its
    write's K offset only, and never through a run-time K offset or an absolute K index.
    Blocks are checked in definition order, statements bottom-up, as the validators fire.
    """
    temps = {t.name for t in stencil.temporaries}
    declared: Set[str] = set()

    def check_stmt(s):
        for child in ir.iter_children(s):
            if isinstance(child, ir.Stmt):
                check_stmt(child)
        if isinstance(s, ir.Assign):
            if s.target.name in _cartesian_h_reads(s.value):
                raise ValueError("Self-assignment with offset in I or J is illegal.")
        elif isinstance(s, ir.While):
            names = _assign_writes(s.body) & _cartesian_h_reads(s.body)
            if names:
                raise ValueError(f"Illegal write and read with horizontal offset detected for {names}.")

    for vl in stencil.vertical_loops:
        secs = list(vl.sections)
        if all(sec.def_index >= 0 for sec in secs):
            # the frontend stores sections in sweep order; the temporary a block declares is
            # decided in definition order, as the reference builds GTIR
            secs.sort(key=lambda sec: sec.def_index)
        for sec in secs:
            for s in sec.body:
                check_stmt(s)
            written = _assign_writes(sec.body)
            local = (written & temps) - declared
            declared |= local
            bad = (written & _cartesian_h_reads(sec.body)) - local
            if bad:
                raise ValueError(f"Illegal write and read with horizontal offset detected for {bad}.")
            iv = sec.interval
            size_one = iv.start.level == iv.end.level and abs(iv.end.offset - iv.start.offset) == 1
            if vl.loop_order != ir.LoopOrder.PARALLEL or size_one:
                continue
            writes = [n.target for n in ir.walk(sec.body) if isinstance(n, ir.Assign)]
            write_ids = {id(w) for w in writes}
            for node in ir.walk(sec.body):
                if not isinstance(node, ir.FieldAccess) or id(node) in write_ids:
                    continue
                for w in writes:
                    if node.name != w.name:
                        continue
                    if node.k_offset is not None or w.k_offset is not None:
                        raise ValueError(
                            "Not allowed to write and read with `VariableKOffset` and/or "
                            f"`AbsoluteKIndex` in PARALLEL loops: `{node.name}`"
                        )
                    if node.offset[2] != w.offset[2]:
                        raise ValueError(f"Not allowed to write and read with k-offsets in PARALLEL loops: `{node.name}`")


def run_pipeline(stencil: ir.Stencil) -> StencilAnalysis:
    validate_parallel_model(stencil)
    stencil = resolve_dtypes(stencil)
    stencil = upcast(stencil)
    extents = compute_extents(stencil)
    validate_memory_accesses(stencil, extents)
    access = compute_access_kinds(stencil)
    kb = compute_k_boundary(stencil)
    min_k = compute_min_k_size(stencil)
    return StencilAnalysis(stencil, access, extents, kb, min_k, compute_signed_extents(stencil))
