"""Stencil IR of gt4py_amd.

A small, OIR-like IR (reference: ``src/gt4py/cartesian/gtc/oir.py:305-362`` and
``gtc/gtir.py``): a stencil is a list of vertical loops (loop order + interval sections),
each section a list of statements over IJ-parallel points. Temporaries are 3-D fields
(``gtir_to_oir.py:225-253``); all dtype transitions are explicit ``Cast`` nodes after
``passes.upcast`` (``gtc/passes/gtir_upcaster.py:80-143``).
"""

from __future__ import annotations

import dataclasses
import enum
from typing import Any, List, Optional, Tuple, Union

import numpy as np


class DataType(enum.IntEnum):
    """Same ids (and therefore the same ordering) as ``gtc/common.py:105-118``.

    The ordering matters: the upcasting rule compares dtypes by these ids.
    """

    INVALID = -1
    AUTO = 0
    DEFAULT = 1
    BOOL = 10
    INT8 = 11
    INT16 = 12
    INT32 = 14
    INT64 = 18
    FLOAT32 = 104
    FLOAT64 = 108

    def isbool(self):
        return self == DataType.BOOL

    def isinteger(self):
        return self in (DataType.INT8, DataType.INT16, DataType.INT32, DataType.INT64)

    def isfloat(self):
        return self in (DataType.FLOAT32, DataType.FLOAT64)

    @property
    def np_dtype(self) -> np.dtype:
        return np.dtype(_DT_TO_NP[self])

    @property
    def ctype(self) -> str:
        return _DT_TO_C[self]

    @property
    def itemsize(self) -> int:
        return self.np_dtype.itemsize

    @staticmethod
    def from_np(dtype) -> "DataType":
        dt = np.dtype(dtype)
        key = (dt.kind, dt.itemsize)
        table = {
            ("b", 1): DataType.BOOL,
            ("i", 1): DataType.INT8,
            ("i", 2): DataType.INT16,
            ("i", 4): DataType.INT32,
            ("i", 8): DataType.INT64,
            ("f", 4): DataType.FLOAT32,
            ("f", 8): DataType.FLOAT64,
        }
        if key not in table:
            raise TypeError(f"Unsupported data type {dt}")
        return table[key]


_DT_TO_NP = {
    DataType.BOOL: "bool",
    DataType.INT8: "int8",
    DataType.INT16: "int16",
    DataType.INT32: "int32",
    DataType.INT64: "int64",
    DataType.FLOAT32: "float32",
    DataType.FLOAT64: "float64",
}
_DT_TO_C = {
    DataType.BOOL: "bool",
    DataType.INT8: "int8_t",
    DataType.INT16: "int16_t",
    DataType.INT32: "int32_t",
    DataType.INT64: "int64_t",
    DataType.FLOAT32: "float",
    DataType.FLOAT64: "double",
}


class LoopOrder(enum.IntEnum):
    PARALLEL = 0
    FORWARD = 1
    BACKWARD = -1


class LevelMarker(enum.Enum):
    START = "start"
    END = "end"


# Operators -----------------------------------------------------------------------------

ARITH_OPS = ("+", "-", "*", "/")
COMPARE_OPS = (">", "<", ">=", "<=", "==", "!=")
LOGICAL_OPS = ("and", "or")
UNARY_OPS = ("+", "-", "not")

# NativeFunction names (gtc/common.py:150-191) -> arity
NATIVE_FUNCTIONS = {
    "abs": 1,
    "min": 2,
    "max": 2,
    "mod": 2,
    "sin": 1,
    "cos": 1,
    "tan": 1,
    "arcsin": 1,
    "arccos": 1,
    "arctan": 1,
    "sinh": 1,
    "cosh": 1,
    "tanh": 1,
    "arcsinh": 1,
    "arccosh": 1,
    "arctanh": 1,
    "sqrt": 1,
    "pow": 2,
    "exp": 1,
    "log": 1,
    "log10": 1,
    "gamma": 1,
    "cbrt": 1,
    "isfinite": 1,
    "isinf": 1,
    "isnan": 1,
    "floor": 1,
    "ceil": 1,
    "trunc": 1,
    "erf": 1,
    "erfc": 1,
    "round": 1,
    "round_away_from_zero": 1,
    "int32": 1,
    "int64": 1,
    "float32": 1,
    "float64": 1,
}


# Expressions ---------------------------------------------------------------------------


@dataclasses.dataclass(eq=True)
class Expr:
    pass


@dataclasses.dataclass(eq=True)
class Literal(Expr):
    value: Any  # python bool/int/float
    dtype: DataType


@dataclasses.dataclass(eq=True)
class FieldAccess(Expr):
    """Access to an API field or temporary at a relative offset (I, J, K).

    ``data_index``: one integer expression per data dimension of the field (``f[0, 0, 0][i]``,
    ``table.A[i, j]``; ``gtir.FieldAccess.data_index``). ``k_offset``: a run-time vertical offset
    added to ``offset[2]`` (``f[0, 0, lev]``; ``gtc/common.py:341-351`` VariableKOffset).
    """

    name: str
    offset: Tuple[int, int, int]
    dtype: DataType = DataType.AUTO
    data_index: List[Expr] = dataclasses.field(default_factory=list)
    k_offset: Optional[Expr] = None

    @property
    def is_direct(self) -> bool:
        """Needs an address computed at run time (cannot live in a register ring/window)."""
        return self.k_offset is not None


@dataclasses.dataclass(eq=True)
class ScalarAccess(Expr):
    """Access to a scalar stencil parameter."""

    name: str
    dtype: DataType = DataType.AUTO


@dataclasses.dataclass(eq=True)
class AxisIndex(Expr):
    """Current absolute index along an axis (relative to the compute-domain origin)."""

    axis: int
    dtype: DataType = DataType.INT64


@dataclasses.dataclass(eq=True)
class BinaryOp(Expr):
    op: str
    left: Expr
    right: Expr
    dtype: DataType = DataType.AUTO


@dataclasses.dataclass(eq=True)
class UnaryOp(Expr):
    op: str
    expr: Expr
    dtype: DataType = DataType.AUTO


@dataclasses.dataclass(eq=True)
class TernaryOp(Expr):
    cond: Expr
    true_expr: Expr
    false_expr: Expr
    dtype: DataType = DataType.AUTO


@dataclasses.dataclass(eq=True)
class NativeCall(Expr):
    func: str
    args: List[Expr]
    dtype: DataType = DataType.AUTO


@dataclasses.dataclass(eq=True)
class Cast(Expr):
    dtype: DataType
    expr: Expr


# Statements ----------------------------------------------------------------------------


@dataclasses.dataclass(eq=True)
class Stmt:
    pass


@dataclasses.dataclass(eq=True)
class Assign(Stmt):
    target: FieldAccess  # always zero offset
    value: Expr


@dataclasses.dataclass(eq=True)
class If(Stmt):
    cond: Expr
    body: List[Stmt]
    orelse: List[Stmt]


@dataclasses.dataclass(eq=True)
class While(Stmt):
    cond: Expr
    body: List[Stmt]


@dataclasses.dataclass(eq=True)
class AxisBound:
    """Horizontal region bound: ``I[0] + 2`` -> (START, 2); ``I[-1] - 2`` -> (END, -2)."""

    level: LevelMarker
    offset: int


@dataclasses.dataclass(eq=True)
class HorizontalInterval:
    start: Optional[AxisBound]  # None = unbounded
    end: Optional[AxisBound]


@dataclasses.dataclass(eq=True)
class HorizontalMask:
    i: HorizontalInterval
    j: HorizontalInterval


@dataclasses.dataclass(eq=True)
class HorizontalRegion(Stmt):
    """``with horizontal(region[...], ...)``: body applies where ANY of the masks holds."""

    masks: List[HorizontalMask]
    body: List[Stmt]


# Declarations & structure --------------------------------------------------------------


@dataclasses.dataclass(eq=True)
class FieldDecl:
    name: str
    dtype: DataType
    axes: Tuple[str, ...] = ("I", "J", "K")
    data_dims: Tuple[int, ...] = ()
    is_temporary: bool = False

    @property
    def mask(self) -> Tuple[bool, bool, bool]:
        return tuple(a in self.axes for a in ("I", "J", "K"))


@dataclasses.dataclass(eq=True)
class ScalarDecl:
    name: str
    dtype: DataType


@dataclasses.dataclass(eq=True)
class Interval:
    """K interval [start, end): bounds relative to START or END of the domain."""

    start: AxisBound
    end: AxisBound

    def resolve(self, nk: int) -> Tuple[int, int]:
        def r(b):
            return b.offset if b.level == LevelMarker.START else nk + b.offset

        return r(self.start), r(self.end)


@dataclasses.dataclass(eq=True)
class Section:
    interval: Interval
    body: List[Stmt]
    # position of the ``with interval`` block in the definition (-1: unknown); sections are
    # stored in sweep order, the parallel-model rules run in definition order (gtc/gtir.py:226)
    def_index: int = dataclasses.field(default=-1, compare=False)


@dataclasses.dataclass(eq=True)
class VerticalLoop:
    loop_order: LoopOrder
    sections: List[Section]


@dataclasses.dataclass(eq=True)
class Stencil:
    name: str
    api_signature: List[str]  # argument names in definition order
    params: List[Union[FieldDecl, ScalarDecl]]  # API params in definition order
    temporaries: List[FieldDecl]
    vertical_loops: List[VerticalLoop]
    externals: dict = dataclasses.field(default_factory=dict)
    docstring: str = ""

    def field_params(self) -> List[FieldDecl]:
        return [p for p in self.params if isinstance(p, FieldDecl)]

    def scalar_params(self) -> List[ScalarDecl]:
        return [p for p in self.params if isinstance(p, ScalarDecl)]

    def decl(self, name: str):
        for p in self.params:
            if p.name == name:
                return p
        for t in self.temporaries:
            if t.name == name:
                return t
        raise KeyError(name)


# Generic traversal ----------------------------------------------------------------------


def iter_children(node):
    if isinstance(node, list):
        for x in node:
            yield x
        return
    if not dataclasses.is_dataclass(node):
        return
    for f in dataclasses.fields(node):
        v = getattr(node, f.name)
        if isinstance(v, (Expr, Stmt)):
            yield v
        elif isinstance(v, list):
            for x in v:
                if isinstance(x, (Expr, Stmt, Section, VerticalLoop, HorizontalMask)):
                    yield x


def walk(node):
    """Pre-order walk over IR nodes (Exprs, Stmts, Sections, VerticalLoops)."""
    stack = [node]
    while stack:
        n = stack.pop()
        if isinstance(n, list):
            stack.extend(reversed(n))
            continue
        yield n
        if isinstance(n, Stencil):
            stack.extend(reversed(n.vertical_loops))
        elif isinstance(n, VerticalLoop):
            stack.extend(reversed(n.sections))
        elif isinstance(n, Section):
            stack.extend(reversed(n.body))
        else:
            stack.extend(reversed(list(iter_children(n))))


def map_expr(node, fn):
    """Rebuild ``node`` bottom-up applying ``fn`` to every Expr (fn returns a new Expr)."""
    if isinstance(node, list):
        return [map_expr(x, fn) for x in node]
    if isinstance(node, Expr):
        kwargs = {}
        for f in dataclasses.fields(node):
            v = getattr(node, f.name)
            if isinstance(v, Expr):
                v = map_expr(v, fn)
            elif isinstance(v, list) and v and isinstance(v[0], Expr):
                v = [map_expr(x, fn) for x in v]
            kwargs[f.name] = v
        return fn(type(node)(**kwargs))
    if isinstance(node, Assign):
        return Assign(map_expr(node.target, fn), map_expr(node.value, fn))
    if isinstance(node, If):
        return If(map_expr(node.cond, fn), map_expr(node.body, fn), map_expr(node.orelse, fn))
    if isinstance(node, While):
        return While(map_expr(node.cond, fn), map_expr(node.body, fn))
    if isinstance(node, HorizontalRegion):
        return HorizontalRegion(node.masks, map_expr(node.body, fn))
    if isinstance(node, Section):
        return Section(node.interval, map_expr(node.body, fn), node.def_index)
    if isinstance(node, VerticalLoop):
        return VerticalLoop(node.loop_order, [map_expr(s, fn) for s in node.sections])
    raise TypeError(type(node))
