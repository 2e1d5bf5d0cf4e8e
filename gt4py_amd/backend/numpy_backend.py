"""``numpy`` backend: a vectorised numpy executor of the gt4py_amd IR (host only).

Executes the same semantics as the reference numpy backend
(``src/gt4py/cartesian/gtc/numpy/npir_codegen.py:320-368``): every top-level statement
(one OIR horizontal execution) is applied over ``domain + its extent`` for the whole K range
of a PARALLEL section, or level by level inside a Python K loop for FORWARD/BACKWARD
(``npir_codegen.py:243-248``); ``if``/``else`` become masks evaluated once
(``gtir_to_oir.py:146-188``); temporaries are full 3-D arrays. Arithmetic runs under
``np.errstate(ignore)``.

This backend is a product backend for host arrays (the reference's plumbing config C1); it
is unrelated to the parity oracle under ``oracle/`` and is never a fallback of ``gt:mi355x``.
"""

from __future__ import annotations

import math
from typing import Any, Dict, Tuple

import numpy as np

from gt4py_amd import ir
from gt4py_amd.backend.base import BaseBackend, register
from gt4py_amd.ir import DataType
from gt4py_amd.storage.layout import layout_checker_factory, layout_maker_factory

try:  # same source of gamma/erf/erfc as gtc/ufuncs.py:15-28
    from scipy.special import erf as _erf, erfc as _erfc, gamma as _gamma
except ImportError:  # pragma: no cover
    _gamma = np.vectorize(math.gamma, otypes=[np.float64])
    _erf = np.vectorize(math.erf, otypes=[np.float64])
    _erfc = np.vectorize(math.erfc, otypes=[np.float64])


def _round_away_from_zero(x):
    return np.copysign(np.floor(np.abs(x) + 0.5), x)


_NATIVE = {
    "abs": np.abs,
    "min": np.minimum,
    "max": np.maximum,
    "mod": np.mod,
    "sin": np.sin,
    "cos": np.cos,
    "tan": np.tan,
    "arcsin": np.arcsin,
    "arccos": np.arccos,
    "arctan": np.arctan,
    "sinh": np.sinh,
    "cosh": np.cosh,
    "tanh": np.tanh,
    "arcsinh": np.arcsinh,
    "arccosh": np.arccosh,
    "arctanh": np.arctanh,
    "sqrt": np.sqrt,
    "pow": np.power,
    "exp": np.exp,
    "log": np.log,
    "log10": np.log10,
    "gamma": _gamma,
    "cbrt": np.cbrt,
    "isfinite": np.isfinite,
    "isinf": np.isinf,
    "isnan": np.isnan,
    "floor": np.floor,
    "ceil": np.ceil,
    "trunc": np.trunc,
    "erf": _erf,
    "erfc": _erfc,
    "round": np.round,
    "round_away_from_zero": _round_away_from_zero,
}

_BINOP = {
    "+": np.add,
    "-": np.subtract,
    "*": np.multiply,
    "/": np.true_divide,
    ">": np.greater,
    "<": np.less,
    ">=": np.greater_equal,
    "<=": np.less_equal,
    "==": np.equal,
    "!=": np.not_equal,
    "and": np.logical_and,
    "or": np.logical_or,
}
_UNOP = {"-": np.negative, "+": np.positive, "not": np.logical_not}


class _Arr:
    """A field (API or temporary) viewed in logical (i, j, k) coordinates."""

    def __init__(self, array: np.ndarray, origin, mask):
        self.array = array
        self.origin = tuple(origin)
        self.mask = tuple(mask)  # which of I, J, K the array has

    def view(self, i0, i1, j0, j1, k0, k1):
        idx = []
        for (lo, hi), o, m in zip(((i0, i1), (j0, j1), (k0, k1)), self.origin, self.mask):
            if m:
                idx.append(slice(o + lo, o + hi))
        idx = tuple(idx)
        v = self.array[idx]
        # broadcast lower-dimensional fields to (I, J, K)
        shape = []
        for m in self.mask:
            shape.append(slice(None) if m else None)
        return v[tuple(shape)] if not all(self.mask) else v


class NumpyExecutor:
    def __init__(self, analysis):
        self.analysis = analysis
        self.stencil = analysis.stencil

    def run(self, domain, origins: Dict[str, Tuple[int, ...]], args: Dict[str, Any]):
        st = self.stencil
        ni, nj, nk = (int(d) for d in domain)
        fields: Dict[str, _Arr] = {}
        scalars: Dict[str, Any] = {}
        for p in st.params:
            v = args.get(p.name)
            if isinstance(p, ir.FieldDecl):
                if v is None:
                    continue
                arr = np.asarray(v) if not isinstance(v, np.ndarray) else v
                org = tuple(origins[p.name])
                mask = p.mask
                full = [0, 0, 0]
                it = iter(org)
                for d in range(3):
                    if mask[d]:
                        full[d] = next(it)
                fields[p.name] = _Arr(arr, full, mask)
            else:
                scalars[p.name] = None if v is None else p.dtype.np_dtype.type(v)
        for t in st.temporaries:
            (ilo, ihi), (jlo, jhi) = self.analysis.extents.fields.get(t.name, ((0, 0), (0, 0)))
            mask = t.mask
            shape = [n for n, m in zip((ni + ilo + ihi, nj + jlo + jhi, nk), mask) if m]
            arr = np.zeros(tuple(shape) + tuple(t.data_dims), dtype=t.dtype.np_dtype)
            fields[t.name] = _Arr(arr, (ilo, jlo, 0), mask)
        self.fields, self.scalars, self.domain = fields, scalars, (ni, nj, nk)
        self.api = {p.name for p in st.field_params()}
        errs = "ignore" if getattr(self, "ignore_errstate", True) else "warn"
        with np.errstate(divide=errs, over=errs, under="ignore", invalid=errs):
            for li, vl in enumerate(st.vertical_loops):
                for si, sec in enumerate(vl.sections):
                    k0, k1 = sec.interval.resolve(nk)
                    k0, k1 = max(k0, 0), min(k1, nk)
                    if k1 <= k0:
                        continue
                    if vl.loop_order == ir.LoopOrder.PARALLEL:
                        self._section(li, si, sec, k0, k1)
                    else:
                        ks = range(k0, k1) if vl.loop_order == ir.LoopOrder.FORWARD else range(k1 - 1, k0 - 1, -1)
                        for k in ks:
                            self._section(li, si, sec, k, k + 1)

    def _section(self, li, si, sec, k0, k1):
        ni, nj, _ = self.domain
        for ti, stmt in enumerate(sec.body):
            (ilo, ihi), (jlo, jhi) = self.analysis.extents.blocks[(li, si, ti)]
            reg = (-ilo, ni + ihi, -jlo, nj + jhi, k0, k1)
            self._stmt(stmt, reg, None)

    # -------------------------------------------------------------- statements
    def _stmt(self, s, reg, mask):
        if isinstance(s, ir.Assign):
            self._assign(s, reg, mask)
        elif isinstance(s, ir.If):
            c = np.broadcast_to(self._ev(s.cond, reg), _shape(reg))
            m_true = c if mask is None else (mask & c)
            for x in s.body:
                self._stmt(x, reg, m_true)
            if s.orelse:
                m_false = ~c if mask is None else (mask & ~c)
                for x in s.orelse:
                    self._stmt(x, reg, m_false)
        elif isinstance(s, ir.While):
            while True:
                c = np.broadcast_to(self._ev(s.cond, reg), _shape(reg))
                m = c if mask is None else (mask & c)
                if not m.any():
                    break
                for x in s.body:
                    self._stmt(x, reg, m)
        elif isinstance(s, ir.HorizontalRegion):
            # each mask in turn over its own sub-box of ``reg`` (the reference numpy backend's
            # relative masks, gtc/passes/horizontal_masks.py:98-115): the body only touches points
            # inside the region, so fields need no halo beyond the region's clipped extent
            for hm in s.masks:
                sub = self._region_box(hm, reg)
                if sub is None:
                    continue
                m = None
                if mask is not None:
                    i0, _, j0, _, _, _ = reg
                    m = np.broadcast_to(mask, _shape(reg))[sub[0] - i0:sub[1] - i0, sub[2] - j0:sub[3] - j0]
                for x in s.body:
                    self._stmt(x, sub, m)
        else:
            raise TypeError(type(s))

    def _region_box(self, hm, reg):
        """``reg`` restricted to the rectangle of horizontal mask ``hm`` (None if empty)."""
        ni, nj, _ = self.domain
        i0, i1, j0, j1, k0, k1 = reg

        def lim(itv, n, a, b):
            if itv.start is not None:
                a = max(a, itv.start.offset if itv.start.level == ir.LevelMarker.START else n + itv.start.offset)
            if itv.end is not None:
                b = min(b, itv.end.offset if itv.end.level == ir.LevelMarker.START else n + itv.end.offset)
            return a, b

        a0, a1 = lim(hm.i, ni, i0, i1)
        b0, b1 = lim(hm.j, nj, j0, j1)
        if a1 <= a0 or b1 <= b0:
            return None
        return (a0, a1, b0, b1, k0, k1)

    def _region_mask(self, masks, reg):
        ni, nj, _ = self.domain
        i0, i1, j0, j1, k0, k1 = reg
        ii = np.arange(i0, i1)[:, None, None]
        jj = np.arange(j0, j1)[None, :, None]

        def rng(itv, n, idx):
            m = np.ones_like(idx, dtype=bool)
            if itv.start is not None:
                lo = itv.start.offset if itv.start.level == ir.LevelMarker.START else n + itv.start.offset
                m &= idx >= lo
            if itv.end is not None:
                hi = itv.end.offset if itv.end.level == ir.LevelMarker.START else n + itv.end.offset
                m &= idx < hi
            return m

        out = np.zeros(_shape(reg), dtype=bool)
        for hm in masks:
            out |= np.broadcast_to(rng(hm.i, ni, ii) & rng(hm.j, nj, jj), _shape(reg))
        return out

    # -------------------------------------------------------------- data dims / run-time K offsets
    def _index_scalar(self, e, reg):
        v = self._ev(e, reg)
        if isinstance(v, np.ndarray):
            if v.size != 1 and not np.all(v == v.reshape(-1)[0]):
                return v
            v = v.reshape(-1)[0]
        return int(v)

    def _data_select(self, v, data_index, reg):
        """``v[..., d0, d1, ...]`` for the trailing data dimensions of a field view."""
        idx = [self._index_scalar(d, reg) for d in data_index]
        if all(isinstance(x, int) for x in idx):
            return v[(Ellipsis,) + tuple(idx)]
        shp = _shape(reg)
        lead = np.broadcast_to(v[(Ellipsis,) + (0,) * len(idx)], shp).shape
        grids = list(np.indices(lead, sparse=True))
        full = [np.broadcast_to(x, lead) if isinstance(x, np.ndarray) else x for x in idx]
        return np.broadcast_to(v, lead + v.shape[v.ndim - len(idx):])[tuple(grids) + tuple(full)]

    def _gather_index(self, e: ir.FieldAccess, f: "_Arr", reg):
        """Fancy index of ``f.array`` for an access with a run-time K offset over ``reg``."""
        i0, i1, j0, j1, k0, k1 = reg
        di, dj, dk = e.offset
        shp = _shape(reg)
        ii = np.arange(i0 + di, i1 + di)[:, None, None] + f.origin[0]
        jj = np.arange(j0 + dj, j1 + dj)[None, :, None] + f.origin[1]
        kv = self._ev(e.k_offset, reg)
        kk = np.arange(k0 + dk, k1 + dk)[None, None, :] + f.origin[2] + np.asarray(kv).astype(np.int64)
        if f.mask[2]:
            # out-of-range levels are clipped to the array (utils/field.py:53-57)
            kk = np.clip(kk, 0, f.array.shape[sum(f.mask[:2])] - 1)
        ii, jj, kk = (np.broadcast_to(x, shp) for x in (ii, jj, kk))
        sel = [x for x, m in zip((ii, jj, kk), f.mask) if m]
        for d in e.data_index:
            sel.append(np.broadcast_to(np.asarray(self._ev(d, reg)).astype(np.int64), shp))
        return tuple(sel)

    def _assign_indexed(self, s: ir.Assign, reg, mask, value):
        """Assignment whose target has a K offset, a run-time K offset or a data index."""
        t = s.target
        f = self.fields[t.name]
        i0, i1, j0, j1, k0, k1 = reg
        ni, nj, _ = self.domain
        ci0, ci1, cj0, cj1 = max(i0, 0), min(i1, ni), max(j0, 0), min(j1, nj)
        if ci1 <= ci0 or cj1 <= cj0:
            return
        sub = (slice(ci0 - i0, ci1 - i0), slice(cj0 - j0, cj1 - j0), slice(None))
        creg = (ci0, ci1, cj0, cj1, k0, k1)
        value = np.broadcast_to(value, _shape(reg))[sub]
        if mask is not None:
            mask = np.broadcast_to(mask, _shape(reg))[sub]
        if t.k_offset is not None:
            idx = self._gather_index(t, f, creg)
        else:
            dk = t.offset[2]
            lo = [ci0 + f.origin[0], cj0 + f.origin[1], k0 + dk + f.origin[2]]
            hi = [ci1 + f.origin[0], cj1 + f.origin[1], k1 + dk + f.origin[2]]
            idx = [slice(a, b) for a, b, m in zip(lo, hi, f.mask) if m]
            didx = [self._index_scalar(d, creg) for d in t.data_index]
            if any(not isinstance(x, int) for x in didx):
                raise NotImplementedError("field-valued data index in an assignment target")
            idx = tuple(idx) + tuple(didx)
        cur = f.array[idx]
        if all(f.mask):
            val = np.broadcast_to(value, cur.shape)
        else:  # lower-dimensional target: the (broadcast) values of the missing axis collapse
            sel = tuple(slice(None) if m else 0 for m in f.mask)
            val = np.broadcast_to(value, _shape(creg))[sel]
            if mask is not None:
                mask = mask[sel]
        f.array[idx] = val if mask is None else np.where(mask, val, cur)

    def _assign(self, s: ir.Assign, reg, mask):
        name = s.target.name
        f = self.fields[name]
        value = self._ev(s.value, reg)
        if s.target.k_offset is not None or s.target.offset[2] != 0 or s.target.data_index:
            return self._assign_indexed(s, reg, mask, value)
        i0, i1, j0, j1, k0, k1 = reg
        if name in self.api:
            ni, nj, _ = self.domain
            ci0, ci1, cj0, cj1 = max(i0, 0), min(i1, ni), max(j0, 0), min(j1, nj)
            if ci1 <= ci0 or cj1 <= cj0:
                return
            sub = (slice(ci0 - i0, ci1 - i0), slice(cj0 - j0, cj1 - j0), slice(None))
            value = np.broadcast_to(value, _shape(reg))[sub]
            if mask is not None:
                mask = mask[sub]
            i0, i1, j0, j1 = ci0, ci1, cj0, cj1
        view = f.view(i0, i1, j0, j1, k0, k1)
        if not all(f.mask):
            # lower-dimensional target: write the (broadcast) last level (as numpy does)
            idx = tuple(slice(None) if m else 0 for m in f.mask)
            target = view[idx]
            val = np.broadcast_to(value, _shape((i0, i1, j0, j1, k0, k1)))[idx]
            if mask is not None:
                val = np.where(mask[idx], val, target)
            target[...] = val
            return
        dt = f.array.dtype
        if mask is None:
            view[...] = value
        else:
            view[...] = np.where(mask, value, view)
        del dt

    # -------------------------------------------------------------- expressions
    def _ev(self, e, reg):
        if isinstance(e, ir.Literal):
            return e.dtype.np_dtype.type(e.value)
        if isinstance(e, ir.ScalarAccess):
            v = self.scalars.get(e.name)
            if v is None:
                raise TypeError(f"The type of parameter '{e.name}' is '{type(None)}' instead of '{e.dtype.np_dtype}'")
            return v
        if isinstance(e, ir.FieldAccess):
            f = self.fields[e.name]
            if e.k_offset is not None:
                return f.array[self._gather_index(e, f, reg)]
            di, dj, dk = e.offset
            i0, i1, j0, j1, k0, k1 = reg
            v = f.view(i0 + di, i1 + di, j0 + dj, j1 + dj, k0 + dk, k1 + dk)
            if e.data_index:
                v = self._data_select(v, e.data_index, reg)
            return v
        if isinstance(e, ir.Cast):
            v = self._ev(e.expr, reg)
            t = e.dtype.np_dtype
            return v.astype(t) if isinstance(v, np.ndarray) else t.type(v)
        if isinstance(e, ir.BinaryOp):
            return _BINOP[e.op](self._ev(e.left, reg), self._ev(e.right, reg))
        if isinstance(e, ir.UnaryOp):
            return _UNOP[e.op](self._ev(e.expr, reg))
        if isinstance(e, ir.TernaryOp):
            return np.where(self._ev(e.cond, reg), self._ev(e.true_expr, reg), self._ev(e.false_expr, reg))
        if isinstance(e, ir.NativeCall):
            args = [self._ev(a, reg) for a in e.args]
            if e.func in ("int32", "int64", "float32", "float64"):
                t = np.dtype(e.func)
                a = args[0]
                return a.astype(t) if isinstance(a, np.ndarray) else t.type(a)
            return _NATIVE[e.func](*args)
        if isinstance(e, ir.AxisIndex):
            i0, i1, j0, j1, k0, k1 = reg
            r = [(i0, i1), (j0, j1), (k0, k1)][e.axis]
            shape = [1, 1, 1]
            shape[e.axis] = r[1] - r[0]
            return np.arange(r[0], r[1], dtype=np.int64).reshape(shape)
        raise TypeError(type(e))


def _shape(reg):
    i0, i1, j0, j1, k0, k1 = reg
    return (i1 - i0, j1 - j0, k1 - k0)


@register
class NumpyBackend(BaseBackend):
    name = "numpy"
    options = {
        "oir_pipeline": {"versioning": True, "type": object},
        "verbose": {"versioning": False, "type": bool},
        # numpy_backend.py:36,43: False runs the computation under numpy's default error state
        "ignore_np_errstate": {"versioning": True, "type": bool},
    }
    _layout = layout_maker_factory((0, 1, 2))
    storage_info = {
        "alignment": 1,
        "device": "cpu",
        "layout_map": _layout,
        "is_optimal_layout": layout_checker_factory(_layout),
    }
    languages = {"computation": "python", "bindings": ["python"]}

    def make_run_impl(self):
        executor = NumpyExecutor(self.builder.analysis)
        executor.ignore_errstate = bool(self.builder.options.backend_opts.get("ignore_np_errstate", True))

        def run_impl(domain, origin, exec_info, kwargs):
            executor.run(domain, origin, kwargs)

        return run_impl
