"""Shared pieces of the gt:mi355x HIP code generators: C names and literals, the typed-IR
expression renderer (numpy-faithful casts and native functions), the field-argument model
(``FieldSlot`` -> kernel parameters / host packing) and launch constants."""

from __future__ import annotations

import dataclasses
import math
from typing import Dict, List, Optional, Set, Tuple

from gt4py_amd import ir
from gt4py_amd.codegen.plan import ColumnKernel, KernelPlan, PlaneKernel, UnsupportedStencil
from gt4py_amd.ir import DataType
from gt4py_amd.passes import ZERO_EXTENT, StencilAnalysis, iter_accesses

WAVE = 64
PLANE_BLOCK_WAVES = 4
PLANE_TARGET_BLOCKS = 60000  # auto J-chunk: aim for at least this many workgroups
PLANE_MIN_JCHUNK = 4
PLANE_ORDER_AUTO = 6  # plane work order chosen per launch: level-synchronous (5) for small launches, else XCD ranges (0)
PLANE_LVLSYNC_MAX_PLANE = 1 << 20  # ... when the plane has at most this many cells
PLANE_LVLSYNC_MAX_LEVELS = 80  # ... and the launch at most this many levels
COLUMN_BLOCK = (64, 4)


def cname(name: str) -> str:
    out = "".join(c if c.isalnum() else "_" for c in name)
    return out


# ------------------------------------------------------------------------------------------
# expression rendering
# ------------------------------------------------------------------------------------------


def literal(value, dtype: DataType) -> str:
    if dtype == DataType.BOOL:
        return "true" if value else "false"
    if dtype.isinteger():
        v = int(value)
        if dtype == DataType.INT64:
            if v == -(2**63):
                return "((int64_t)(-9223372036854775807LL - 1))"
            return f"((int64_t){v}LL)"
        return f"(({dtype.ctype}){v})"
    v = float(value)
    if math.isnan(v):
        s = "__builtin_nan(\"\")"
    elif math.isinf(v):
        s = "__builtin_inf()" if v > 0 else "(-__builtin_inf())"
    else:
        s = v.hex()
    return f"(({dtype.ctype})({s}))"


_MATH1 = {
    "sin": "sin",
    "cos": "cos",
    "tan": "tan",
    "arcsin": "asin",
    "arccos": "acos",
    "arctan": "atan",
    "sinh": "sinh",
    "cosh": "cosh",
    "tanh": "tanh",
    "arcsinh": "asinh",
    "arccosh": "acosh",
    "arctanh": "atanh",
    "sqrt": "sqrt",
    "exp": "exp",
    "log": "log",
    "log10": "log10",
    "gamma": "tgamma",
    "cbrt": "cbrt",
    "floor": "floor",
    "ceil": "ceil",
    "trunc": "trunc",
    "erf": "erf",
    "erfc": "erfc",
}


def _exactly_widened(e) -> bool:
    """``e`` is an f64 value cast from a type whose every value, times a power of two of modest
    exponent, is exact in f64 (f32, integers of at most 32 bits)."""
    if not isinstance(e, ir.Cast) or e.dtype != DataType.FLOAT64:
        return False
    src = getattr(e.expr, "dtype", None)
    return src in (DataType.FLOAT32, DataType.INT8, DataType.INT16, DataType.INT32)


def _pow2_literal(e):
    """The value of an f64 power-of-two literal (possibly behind casts) with |exponent| <= 64."""
    while isinstance(e, ir.Cast):
        e = e.expr
    if not isinstance(e, ir.Literal) or e.dtype == DataType.BOOL:
        return None
    try:
        v = float(e.value)
    except (TypeError, ValueError):
        return None
    if v == 0.0 or not math.isfinite(v):
        return None
    m, x = math.frexp(abs(v))
    return v if (m == 0.5 and -64 <= x <= 64) else None


class ExprRenderer:
    """Renders typed IR expressions to C++; ``resolve(FieldAccess) -> str`` is supplied.

    ``exact_fma``: an f64 ``p +- c`` / ``c - p`` whose product ``p`` = power-of-two literal x value
    widened from f32 (or a <= 32-bit integer) is rendered as one ``fma``. The product is exact, so
    the single rounding of the fma equals the rounding of the separate add: bit-identical results,
    one instruction fewer (the f32 hdiff cast tree's ``4.0 * f64(u) - f64(sum)``)."""

    exact_fma = True

    def __init__(self, resolve, scalar_name, axis_index=None):
        self.resolve = resolve
        self.scalar_name = scalar_name
        self.axis_index = axis_index

    def _exact_product(self, e):
        """(literal C text, other factor C text) when ``e`` is such an exact f64 product."""
        if not (self.exact_fma and isinstance(e, ir.BinaryOp) and e.op == "*" and e.dtype == DataType.FLOAT64):
            return None
        for lit, other in ((e.left, e.right), (e.right, e.left)):
            v = _pow2_literal(lit)
            if v is not None and _exactly_widened(other):
                return v, self.r(other)
        return None

    def _fma(self, e):
        if e.op not in ("+", "-") or e.dtype != DataType.FLOAT64:
            return None
        lp, rp = self._exact_product(e.left), self._exact_product(e.right)
        if lp is not None:  # p + c, p - c
            c = self.r(e.right)
            return f"__builtin_fma({literal(lp[0], DataType.FLOAT64)}, {lp[1]}, {c if e.op == '+' else f'(-{c})'})"
        if rp is not None:  # c + p, c - p
            v = rp[0] if e.op == "+" else -rp[0]
            return f"__builtin_fma({literal(v, DataType.FLOAT64)}, {rp[1]}, {self.r(e.left)})"
        return None

    def __call__(self, e: ir.Expr) -> str:
        return self.r(e)

    def r(self, e) -> str:
        if isinstance(e, ir.Literal):
            return literal(e.value, e.dtype)
        if isinstance(e, ir.FieldAccess):
            return self.resolve(e)
        if isinstance(e, ir.ScalarAccess):
            return self.scalar_name(e.name)
        if isinstance(e, ir.Cast):
            return f"(({e.dtype.ctype})({self.r(e.expr)}))"
        if isinstance(e, ir.BinaryOp):
            f = self._fma(e)
            if f is not None:
                return f
            a, b = self.r(e.left), self.r(e.right)
            if e.op in ("and", "or"):
                return f"({a} {'&&' if e.op == 'and' else '||'} {b})"
            if e.op in ir.COMPARE_OPS:
                return f"({a} {e.op} {b})"
            expr = f"({a} {e.op} {b})"
            if not e.dtype.isfloat():
                return f"(({e.dtype.ctype}){expr})"
            return expr
        if isinstance(e, ir.UnaryOp):
            a = self.r(e.expr)
            if e.op == "not":
                return f"(!{a})"
            if e.op == "-":
                return f"(({e.dtype.ctype})(-{a}))" if not e.dtype.isfloat() else f"(-{a})"
            return f"(+{a})" if e.dtype.isfloat() else f"(({e.dtype.ctype})(+{a}))"
        if isinstance(e, ir.TernaryOp):
            return f"({self.r(e.cond)} ? {self.r(e.true_expr)} : {self.r(e.false_expr)})"
        if isinstance(e, ir.NativeCall):
            return self.native(e)
        if isinstance(e, ir.AxisIndex):
            return self.axis_index(e.axis)
        raise TypeError(type(e))

    def native(self, e: ir.NativeCall) -> str:
        f = e.func
        args = [self.r(a) for a in e.args]
        t = e.dtype.ctype
        if f in ("int32", "int64", "float32", "float64"):
            return f"(({t})({args[0]}))"
        if f == "abs":
            return f"gtmi::absolute({args[0]})"
        if f == "min":
            return f"gtmi::minimum<{t}>({args[0]}, {args[1]})"
        if f == "max":
            return f"gtmi::maximum<{t}>({args[0]}, {args[1]})"
        if f == "mod":
            return f"gtmi::remainder_(({t}){args[0]}, ({t}){args[1]})"
        if f == "pow":
            if e.dtype.isfloat():
                ex = e.args[1]
                while isinstance(ex, ir.Cast):
                    ex = ex.expr
                if isinstance(ex, ir.Literal) and float(ex.value) == 2.0:
                    # x ** 2: glibc's pow (numpy's float power loop) is correctly rounded, so it
                    # equals the correctly rounded product; ocml's pow is not (1 ULP off)
                    return f"gtmi::square<{t}>(({t})({args[0]}))"
                return f"(({t})pow(({t})({args[0]}), ({t})({args[1]})))"
            return f"gtmi::ipow<{t}>(({t})({args[0]}), ({t})({args[1]}))"
        if f in ("isfinite", "isinf", "isnan"):
            at = e.args[0].dtype
            if not at.isfloat():
                return "true" if f == "isfinite" else "false"
            return f"((bool)__builtin_{f}({args[0]}))"
        if f == "round":
            return f"gtmi::round_half_even({args[0]})"
        if f == "round_away_from_zero":
            return f"gtmi::round_away({args[0]})"
        if f in _MATH1:
            at = e.args[0].dtype
            if not at.isfloat():
                return f"(({t}){_MATH1[f]}((double)({args[0]})))"
            return f"(({t}){_MATH1[f]}({args[0]}))"
        raise UnsupportedStencil(f"native function {f}")


# ------------------------------------------------------------------------------------------
# shared field-argument model
# ------------------------------------------------------------------------------------------


@dataclasses.dataclass
class FieldSlot:
    """A memory-backed field visible to kernels: an API field or a scratch temporary."""

    name: str
    index: int  # index in the gtmi_field array
    dtype: DataType
    is_scratch: bool
    data_index: Tuple[str, ...] = ()  # host C expressions: component of a data-dimension field

    @property
    def c(self) -> str:
        return cname(self.name)


def kparam_decl(slot: FieldSlot, writable: bool) -> List[str]:
    c = slot.c
    const = "" if writable else "const "
    return [
        f"{const}{slot.dtype.ctype}* __restrict__ p_{c};",
        f"int64_t sI_{c}, sJ_{c}, sK_{c};",
        f"int32_t ilo_{c}, ihi_{c}, jlo_{c}, jhi_{c}, klo_{c}, khi_{c};",
    ]


def host_fill(slot: FieldSlot, pvar: str, writable: bool) -> List[str]:
    c = slot.c
    t = slot.dtype.ctype
    cast = f"({t}*)" if writable else f"(const {t}*)"
    f = f"f[{slot.index}]"
    comp = "".join(
        f" + (int64_t)gtmi_clamp_index((int64_t)({x}), {f}.data_shape[{d}]) * {f}.data_strides[{d}]"
        for d, x in enumerate(slot.data_index)
    )
    return [
        f"{pvar}.p_{c} = {cast}{f}.data + ({f}.origin[0] * {f}.strides[0] + {f}.origin[1] * {f}.strides[1] + "
        f"{f}.origin[2] * {f}.strides[2]{comp});",
        f"{pvar}.sI_{c} = {f}.strides[0]; {pvar}.sJ_{c} = {f}.strides[1]; {pvar}.sK_{c} = {f}.strides[2];",
        f"{pvar}.ilo_{c} = (int32_t)(-{f}.origin[0]); {pvar}.ihi_{c} = (int32_t)({f}.shape[0] - {f}.origin[0] - 1);",
        f"{pvar}.jlo_{c} = (int32_t)(-{f}.origin[1]); {pvar}.jhi_{c} = (int32_t)({f}.shape[1] - {f}.origin[1] - 1);",
        f"{pvar}.klo_{c} = (int32_t)(-{f}.origin[2]); {pvar}.khi_{c} = (int32_t)({f}.shape[2] - {f}.origin[2] - 1);",
    ]


def interval_bounds(itv: ir.Interval) -> Tuple[str, str]:
    def b(x):
        return f"{x.offset}" if x.level == ir.LevelMarker.START else f"(nk + ({x.offset}))"

    return b(itv.start), b(itv.end)


# ------------------------------------------------------------------------------------------
# K1: J-streaming plane kernel

def region_condition(masks, iv, jv, ni, nj) -> str:
    def bound(b, n):
        return f"{b.offset}" if b.level == ir.LevelMarker.START else f"({n} + ({b.offset}))"

    parts = []
    for m in masks:
        conds = []
        for itv, var, n in ((m.i, iv, ni), (m.j, jv, nj)):
            if itv.start is not None:
                conds.append(f"({var} >= {bound(itv.start, n)})")
            if itv.end is not None:
                conds.append(f"({var} < {bound(itv.end, n)})")
        parts.append("(" + (" && ".join(conds) if conds else "true") + ")")
    return " || ".join(parts) if parts else "false"
