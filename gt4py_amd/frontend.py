"""GTScript frontend: Python AST of a stencil definition -> ``gt4py_amd.ir.Stencil``.

A re-implementation (not a port) of the subset of the reference frontend that the
hot path needs (``src/gt4py/cartesian/frontend/gtscript_frontend.py``:
``GTScriptParser.run`` ``:2474-2549``, ``IRMaker`` ``:886``; ``defir_to_gtir.py:297``):

- signature -> API fields (``Field[...]`` annotations) and scalar parameters,
- ``with computation(ORDER), interval(...)`` blocks (also nested ``with interval`` sections),
- assignments / aug-assignments to API fields and temporaries, ``if``/``elif``/``else``,
  ``while``, ternaries, math builtins, casts, ``**`` and ``%`` (as NativeFunction POW/MOD,
  ``defir_to_gtir.py:482-487``),
- externals (``from __externals__ import X``) and compile-time ``if __INLINED(...)``,
- inlining of ``@gtscript.function`` subroutines (single or tuple returns),
- ``with horizontal(region[...])`` restrictions.

Literal precision follows ``literal_int_precision``/``literal_float_precision``
(``gtscript_frontend.py:913-990``).
"""

from __future__ import annotations

import ast
import warnings
import copy
import dataclasses
import builtins
import inspect
import itertools
import numbers
import sys
import textwrap
import types
from typing import Any, Dict, List, Optional, Tuple

import numpy as np

from gt4py_amd import ir
from gt4py_amd.gtscript import Axis
from gt4py_amd.definitions import GTSpecificationError, GTSyntaxError
from gt4py_amd.ir import DataType

_GTSCRIPT_FUNC_ATTR = "__gtscript_function__"


# the reference's frontend error hierarchy (``frontend/exceptions.py:15-100``): symbol and
# definition errors ARE syntax errors, assertion failures are specification errors
class GTScriptSyntaxError(GTSyntaxError):
    pass


class GTScriptSymbolError(GTScriptSyntaxError):
    pass


class GTScriptDefinitionError(GTScriptSyntaxError):
    pass


class GTScriptValueError(GTScriptDefinitionError):
    pass


class GTScriptDataTypeError(GTScriptSyntaxError):
    pass


class GTScriptAssertionError(GTSpecificationError):
    pass


def _valid_external(value) -> bool:
    """An external's value the reference accepts (``GTScriptParser.CONST_VALUE_TYPES``: numbers,
    bools, numpy scalars, functions, None, axis indices and axes)."""
    from gt4py_amd.gtscript import AxisIndex

    return value is None or isinstance(value, (bool, numbers.Number, np.generic, types.FunctionType, AxisIndex, Axis))


def annotate_function(func):
    """Mark a ``@gtscript.function`` (parse lazily at inlining time)."""
    if not isinstance(func, types.FunctionType):
        raise TypeError(f"gtscript.function expects a function, got {func!r}")
    setattr(func, _GTSCRIPT_FUNC_ATTR, True)
    return func


def is_gtscript_function(obj) -> bool:
    return isinstance(obj, types.FunctionType) and getattr(obj, _GTSCRIPT_FUNC_ATTR, False)


def _func_ast(func) -> ast.FunctionDef:
    src = textwrap.dedent(inspect.getsource(func))
    mod = ast.parse(src)
    for node in mod.body:
        if isinstance(node, ast.FunctionDef) and node.name == func.__name__:
            return node
    for node in ast.walk(mod):
        if isinstance(node, ast.FunctionDef):
            return node
    raise GTScriptSyntaxError(f"Could not find the definition of {func.__name__}")


def _func_namespace(func) -> Dict[str, Any]:
    ns = dict(func.__globals__)
    if func.__closure__:
        for name, cell in zip(func.__code__.co_freevars, func.__closure__):
            try:
                ns[name] = cell.cell_contents
            except ValueError:
                pass
    return ns


def _scalar_dtype(annotation, options) -> DataType:
    if annotation is float:
        return DataType.FLOAT64 if options.literal_float_precision == 64 else DataType.FLOAT32
    if annotation is int:
        return DataType.INT64 if options.literal_int_precision == 64 else DataType.INT32
    if annotation is bool:
        return DataType.BOOL
    try:
        return DataType.from_np(np.dtype(annotation))
    except TypeError as ex:
        raise GTScriptDefinitionError(f"Invalid scalar parameter annotation {annotation!r}") from ex


class _Scope:
    """Name resolution for one function body (stencil or inlined gtscript.function)."""

    def __init__(self, namespace: Dict[str, Any], externals: Dict[str, Any]):
        self.namespace = namespace
        self.externals = externals
        self.imported: Dict[str, Any] = {}  # names imported from __externals__
        self.aliases: Dict[str, Any] = {}  # function args -> ("field", name, offset) | ir.Expr
        self.locals: Dict[str, str] = {}  # local (user) name -> temporary name

    def lookup_external(self, name):
        if name in self.imported:
            return True, self.imported[name]
        if name in self.namespace:
            return True, self.namespace[name]
        if hasattr(builtins, name):
            return True, getattr(builtins, name)
        return False, None


class StencilParser:
    def __init__(self, definition, externals: Dict[str, Any], options, dtypes=None):
        self.definition = definition
        self.externals = dict(externals or {})
        # ``stencil(dtypes=...)``: names usable as types of annotated locals (gtscript_frontend.py:1835-1850)
        self.dtypes = dict(dtypes or {})
        self.options = options
        self.fields: Dict[str, ir.FieldDecl] = {}
        self.scalars: Dict[str, ir.ScalarDecl] = {}
        self.temporaries: Dict[str, ir.FieldDecl] = {}
        self.temp_declared_dtype: Dict[str, DataType] = {}
        self.api_order: List[str] = []
        self._uid = itertools.count()
        self.used_externals: Dict[str, Any] = {}
        # names assigned so far outside horizontal regions (reference IRMaker.written_vars,
        # gtscript_frontend.py:920, 1891-1892)
        self.written_vars: set = set()
        self._in_region = 0

    # ------------------------------------------------------------------ signature
    def _parse_signature(self):
        func = self.definition
        sig = inspect.signature(func)
        annotations = dict(getattr(func, "__annotations__", {}))
        ns = _func_namespace(func)
        from gt4py_amd.gtscript import _FieldDescriptor

        for name, param in sig.parameters.items():
            if param.kind in (param.VAR_POSITIONAL, param.VAR_KEYWORD):
                raise GTScriptDefinitionError("Variable arguments are not supported in stencil definitions")
            ann = annotations.get(name, param.annotation)
            if isinstance(ann, str):
                try:
                    ann = eval(ann, ns)  # noqa: S307 - annotation strings from user code
                except Exception as ex:
                    raise GTScriptDefinitionError(f"Cannot resolve annotation {ann!r} of '{name}'") from ex
            if ann is inspect.Parameter.empty:
                raise GTScriptDefinitionError(f"Missing type annotation for argument '{name}'")
            self.api_order.append(name)
            if isinstance(ann, _FieldDescriptor):
                if isinstance(ann.dtype, str):
                    raise GTScriptDefinitionError(f"Unresolved dtype '{ann.dtype}' for field '{name}'")
                axes = ann.axes_names
                self.fields[name] = ir.FieldDecl(
                    name=name,
                    dtype=DataType.from_np(ann.dtype),
                    axes=tuple(axes),
                    data_dims=tuple(ann.data_dims),
                )
            else:
                self.scalars[name] = ir.ScalarDecl(name=name, dtype=_scalar_dtype(ann, self.options))

    # ------------------------------------------------------------------ helpers
    def _new_temp_name(self, base: str) -> str:
        return f"{base}__{next(self._uid)}"

    def _literal(self, value) -> ir.Literal:
        if isinstance(value, (bool, np.bool_)):
            return ir.Literal(bool(value), DataType.BOOL)
        if isinstance(value, np.generic):
            return ir.Literal(value.item(), DataType.from_np(value.dtype))
        if isinstance(value, numbers.Integral):
            dt = DataType.INT64 if self.options.literal_int_precision == 64 else DataType.INT32
            return ir.Literal(int(value), dt)
        if isinstance(value, numbers.Real):
            dt = DataType.FLOAT64 if self.options.literal_float_precision == 64 else DataType.FLOAT32
            return ir.Literal(float(value), dt)
        raise GTScriptSyntaxError(f"Unsupported literal {value!r}")

    def _const_eval(self, node: ast.AST, scope: _Scope):
        """Evaluate a compile-time expression (externals, literals, simple ops)."""
        if isinstance(node, ast.Constant):
            return node.value
        if isinstance(node, ast.Name):
            found, val = scope.lookup_external(node.id)
            if not found:
                raise GTScriptSymbolError(f"Unknown compile-time symbol '{node.id}'")
            return val
        if isinstance(node, ast.Attribute):
            return getattr(self._const_eval(node.value, scope), node.attr)
        if isinstance(node, ast.UnaryOp):
            v = self._const_eval(node.operand, scope)
            return {ast.USub: lambda x: -x, ast.UAdd: lambda x: +x, ast.Not: lambda x: not x}[type(node.op)](v)
        if isinstance(node, ast.BoolOp):
            vals = [self._const_eval(v, scope) for v in node.values]
            if isinstance(node.op, ast.And):
                return all(vals)
            return any(vals)
        if isinstance(node, ast.BinOp):
            a, b = self._const_eval(node.left, scope), self._const_eval(node.right, scope)
            ops = {
                ast.Add: lambda x, y: x + y,
                ast.Sub: lambda x, y: x - y,
                ast.Mult: lambda x, y: x * y,
                ast.Div: lambda x, y: x / y,
                ast.FloorDiv: lambda x, y: x // y,
                ast.Mod: lambda x, y: x % y,
                ast.Pow: lambda x, y: x**y,
            }
            return ops[type(node.op)](a, b)
        if isinstance(node, ast.Compare):
            left = self._const_eval(node.left, scope)
            res = True
            for op, comp in zip(node.ops, node.comparators):
                right = self._const_eval(comp, scope)
                res = res and {
                    ast.Eq: lambda x, y: x == y,
                    ast.NotEq: lambda x, y: x != y,
                    ast.Lt: lambda x, y: x < y,
                    ast.LtE: lambda x, y: x <= y,
                    ast.Gt: lambda x, y: x > y,
                    ast.GtE: lambda x, y: x >= y,
                    ast.Is: lambda x, y: x is y,
                    ast.IsNot: lambda x, y: x is not y,
                }[type(op)](left, right)
                left = right
            return res
        if isinstance(node, ast.Tuple):
            return tuple(self._const_eval(e, scope) for e in node.elts)
        if isinstance(node, ast.Subscript):
            return self._const_eval(node.value, scope)[self._const_eval(node.slice, scope)]
        if isinstance(node, ast.Call):
            fn = self._const_eval(node.func, scope)
            args = [self._const_eval(a, scope) for a in node.args]
            return fn(*args)
        raise GTScriptSyntaxError(f"Not a compile-time expression: {ast.dump(node)}")

    def _parse_import(self, stmt, scope: _Scope):
        if isinstance(stmt, ast.ImportFrom) and stmt.module == "__externals__":
            for alias in stmt.names:
                if alias.name not in self.externals:
                    raise GTScriptDefinitionError(f"Missing value for external symbol '{alias.name}'")
                value = self.externals[alias.name]
                scope.imported[alias.asname or alias.name] = value
                self.used_externals[alias.name] = value
        elif isinstance(stmt, ast.ImportFrom) and stmt.module in ("__gtscript__", "gt4py.cartesian.gtscript"):
            return
        elif isinstance(stmt, ast.ImportFrom) and stmt.module and stmt.module.endswith("gtscript"):
            return
        else:
            raise GTScriptSyntaxError("Only 'from __externals__ import ...' and '__gtscript__' imports are allowed")

    # ------------------------------------------------------------------ computations
    def _call_name(self, node) -> Optional[str]:
        if isinstance(node, ast.Call):
            f = node.func
            if isinstance(f, ast.Name):
                return f.id
            if isinstance(f, ast.Attribute):
                return f.attr
        return None

    def _parse_order(self, node, scope) -> ir.LoopOrder:
        if len(node.args) != 1:
            raise GTScriptSyntaxError("computation() takes exactly one argument")
        arg = node.args[0]
        if isinstance(arg, ast.Name) and arg.id in ("PARALLEL", "FORWARD", "BACKWARD"):
            return ir.LoopOrder[arg.id]
        if isinstance(arg, ast.Attribute) and arg.attr in ("PARALLEL", "FORWARD", "BACKWARD"):
            return ir.LoopOrder[arg.attr]
        val = self._const_eval(arg, scope)
        return ir.LoopOrder(int(val))

    def _parse_interval(self, node, scope) -> ir.Interval:
        """``interval(start, end)`` with the reference's range checks (``gtscript_frontend.py:
        1105-1140``, ``IntervalParser``): no ``None`` start, no END-relative start with a
        START-relative end, and a non-empty range when both ends are relative to the same level."""
        itv = self._parse_interval_bounds(node, scope)
        where = f"at line {node.lineno} (column {node.col_offset + 1})"
        s_, e_ = itv.start, itv.end
        if (s_.level == ir.LevelMarker.END and e_.level == ir.LevelMarker.START) or (
                s_.level == e_.level and e_.offset <= s_.offset):
            raise GTScriptSyntaxError(f"Invalid interval range specification {where}")
        return itv

    def _parse_interval_bounds(self, node, scope) -> ir.Interval:
        args = node.args
        if len(args) == 1 and isinstance(args[0], ast.Constant) and args[0].value is Ellipsis:
            return ir.Interval(ir.AxisBound(ir.LevelMarker.START, 0), ir.AxisBound(ir.LevelMarker.END, 0))
        if len(args) == 1:
            # interval(k) == single level, or a slice-like K[...] expression
            raise GTScriptSyntaxError("interval() needs (start, end) or ...")
        if len(args) != 2:
            raise GTScriptSyntaxError("interval() takes '...' or (start, end)")

        def bound(a, is_start):
            if isinstance(a, ast.Constant) and a.value is None:
                if is_start:  # the reference's IntervalParser refuses a None start
                    raise GTScriptSyntaxError(
                        f"Invalid interval range specification at line {node.lineno} (column: {node.col_offset + 1})")
                return ir.AxisBound(ir.LevelMarker.END, 0)
            runtime = [
                n.id for n in ast.walk(a)
                if isinstance(n, ast.Name) and n.id not in scope.imported
                and (n.id in self.fields or n.id in self.scalars or self._temp_for_local(n.id, scope, create=False))
            ]
            if runtime:
                # RuntimeAxisBound: parsed by the reference frontend, then rejected by the numpy and
                # gt:* backends (gtc/numpy/oir_to_npir.py:91-94, gtc/gtcpp/oir_to_gtcpp.py:186-196)
                raise NotImplementedError(
                    "Runtime interval bounds (e.g. `with interval(0, field)`) is an experimental feature and "
                    f"not implemented for this backend ({', '.join(runtime)})."
                )
            v = self._const_eval(a, scope)
            from gt4py_amd.gtscript import AxisIndex

            if isinstance(v, AxisIndex):
                level = ir.LevelMarker.START if v.index >= 0 else ir.LevelMarker.END
                return ir.AxisBound(level, v.index + v.offset)
            if v is None:
                if is_start:
                    raise GTScriptSyntaxError(
                        f"Invalid interval range specification at line {node.lineno} (column: {node.col_offset + 1})")
                return ir.AxisBound(ir.LevelMarker.END, 0)
            v = int(v)
            if v < 0:
                return ir.AxisBound(ir.LevelMarker.END, v)
            if v == 0 and not is_start:
                # interval(x, 0) is empty by python slicing semantics; keep START 0
                return ir.AxisBound(ir.LevelMarker.START, 0)
            return ir.AxisBound(ir.LevelMarker.START, v)

        return ir.Interval(bound(args[0], True), bound(args[1], False))

    def _parse_computation(self, stmt: ast.With, scope: _Scope) -> List[ir.VerticalLoop]:
        items = stmt.items
        first = items[0].context_expr
        if self._call_name(first) != "computation":
            raise GTScriptSyntaxError("Expected 'with computation(...)'")
        order = self._parse_order(first, scope)
        self._loop_order = order
        sections: List[ir.Section] = []
        if len(items) == 2:
            second = items[1].context_expr
            if self._call_name(second) != "interval":
                raise GTScriptSyntaxError("Expected 'interval(...)' after 'computation(...)'")
            itv = self._parse_interval(second, scope)
            sections.append(ir.Section(itv, self._parse_block(stmt.body, scope), 0))
        elif len(items) == 1:
            for sub in stmt.body:
                if isinstance(sub, ast.Expr) and isinstance(sub.value, ast.Constant):
                    continue
                if not (isinstance(sub, ast.With) and self._call_name(sub.items[0].context_expr) == "interval"):
                    raise GTScriptSyntaxError("Inside 'with computation(...)' only 'with interval(...)' blocks")
                itv = self._parse_interval(sub.items[0].context_expr, scope)
                sections.append(ir.Section(itv, self._parse_block(sub.body, scope), len(sections)))
        else:
            raise GTScriptSyntaxError("Invalid 'with computation(...)' statement")

        def key(sec):
            b = sec.interval.start
            return (0 if b.level == ir.LevelMarker.START else 100000) + b.offset

        if len(items) == 1 and sections:
            # nested intervals: listed in execution order and disjoint (gtscript_frontend.py:
            # 1019-1079, 1996-2004)
            where = (f"Invalid 'with' statement in '{self.definition.__name__}' at line {stmt.lineno} "
                     f"(column {stmt.col_offset + 1})")
            if sorted(sections, key=key, reverse=(order == ir.LoopOrder.BACKWARD)) != sections:
                raise GTScriptSyntaxError(f"{where}: Intervals must be specified in order of execution.")

            def pos(b):
                return b.offset if b.level == ir.LevelMarker.START else sys.maxsize + b.offset

            for a, b in zip(sections, sections[1:]):
                a0, a1, b0, b1 = pos(a.interval.start), pos(a.interval.end), pos(b.interval.start), pos(b.interval.end)
                if (b0 <= a0 < b1) or (a0 <= b0 < a1):
                    raise GTScriptSyntaxError(f"{where}: Overlapping intervals detected.")
        sections.sort(key=key, reverse=(order == ir.LoopOrder.BACKWARD))
        # drop empty sections (e.g. everything inlined away)
        sections = [s for s in sections if s.body]
        if not sections:
            return []
        return [ir.VerticalLoop(order, sections)]

    # ------------------------------------------------------------------ statements
    def _parse_block(self, stmts, scope: _Scope) -> List[ir.Stmt]:
        out: List[ir.Stmt] = []
        for s in stmts:
            out.extend(self._parse_stmt(s, scope))
        return out

    def _is_inlined_call(self, node) -> bool:
        return self._call_name(node) == "__INLINED"

    def _parse_stmt(self, s, scope: _Scope) -> List[ir.Stmt]:
        if isinstance(s, ast.Expr):
            if isinstance(s.value, ast.Constant):
                return []
            if isinstance(s.value, ast.Call) and self._call_name(s.value) == "compile_assert":
                if not self._const_eval(s.value.args[0], scope):
                    raise GTScriptAssertionError(f"Assertion failed at line {s.lineno}, col {s.col_offset + 1}:\n"
                                                 f"{ast.unparse(s.value.args[0])}")
                return []
            raise GTScriptSyntaxError(f"Invalid expression statement (line {s.lineno})")
        if isinstance(s, ast.Pass):
            return []
        if isinstance(s, (ast.Import, ast.ImportFrom)):
            self._parse_import(s, scope)
            return []
        if isinstance(s, ast.Assign):
            if len(s.targets) != 1:
                raise GTScriptSyntaxError("Chained assignments are not supported")
            return self._parse_assign(s.targets[0], s.value, scope)
        if isinstance(s, ast.AnnAssign):
            if s.value is None:
                raise GTScriptSyntaxError("Annotated declaration without value")
            if isinstance(s.annotation, ast.Name) and s.annotation.id in self.dtypes:
                ann = self.dtypes[s.annotation.id]
            else:
                ann = self._const_eval(s.annotation, scope)
            if isinstance(s.target, ast.Name):
                from gt4py_amd.gtscript import _FieldDescriptor

                if isinstance(ann, _FieldDescriptor):
                    # typed temporary inside a computation: only IJ (2-D) fields
                    # (reference gtscript_frontend.py:1870-1900)
                    axes = tuple(ann.axes_names)
                    if axes != ("I", "J"):
                        raise GTScriptSyntaxError(
                            f"Typed temporaries must be IJ, temporaries for axes {''.join(axes)} is not yet available."
                        )
                    tname = self._temp_for_local(s.target.id, scope, create=True)
                    dt = DataType.from_np(ann.dtype)
                    self.temporaries[tname] = ir.FieldDecl(tname, dt, axes, tuple(ann.data_dims), is_temporary=True)
                    self.temp_declared_dtype[tname] = dt
                else:
                    tname = self._temp_for_local(s.target.id, scope, create=True)
                    self.temp_declared_dtype[tname] = _scalar_dtype(ann, self.options)
            return self._parse_assign(s.target, s.value, scope)
        if isinstance(s, ast.AugAssign):
            binop = ast.BinOp(left=_load_copy(s.target), op=s.op, right=s.value)
            ast.copy_location(binop, s)
            return self._parse_assign(s.target, binop, scope)
        if isinstance(s, ast.If):
            if self._is_inlined_call(s.test):
                cond = self._const_eval(s.test.args[0], scope)
                return self._parse_block(s.body if cond else s.orelse, scope)
            pre: List[ir.Stmt] = []
            cond = self._parse_expr(s.test, scope, pre)
            if pre or self._calls_gtscript_function(s.test, scope):  # gtscript_frontend.py:1607-1616
                raise GTScriptSyntaxError(
                    "Using function calls in the condition of an if is not allowed, the function needs to be "
                    f"assigned to a variable outside the condition (line {s.lineno})")
            body = self._parse_block(s.body, scope)
            orelse = self._parse_block(s.orelse, scope)
            return pre + [ir.If(cond, body, orelse)]
        if isinstance(s, ast.While):
            pre = []
            cond = self._parse_expr(s.test, scope, pre)
            if pre:
                raise GTScriptSyntaxError("Function calls in while conditions are not supported")
            return [ir.While(cond, self._parse_block(s.body, scope))]
        if isinstance(s, ast.With):
            name = self._call_name(s.items[0].context_expr)
            if name == "horizontal":
                where = (f"Invalid 'with' statement in '{self.definition.__name__}' at line {s.lineno} "
                         f"(column {s.col_offset + 1})")
                if any(isinstance(c, ast.With) for c in s.body):
                    raise GTScriptSyntaxError(f"{where}: Cannot nest `with` node inside a horizontal region.")
                masks = []
                for item in s.items:
                    for reg in item.context_expr.args:
                        masks.append(self._parse_region(reg, scope))
                self._in_region += 1
                try:
                    body = self._parse_block(s.body, scope)
                finally:
                    self._in_region -= 1
                # a value written earlier and read at an IJ offset inside a region: the reference
                # refuses it (gtscript_frontend.py:1952-1956)
                offs = {a.name for n in body for a in ir.walk(n)
                        if isinstance(a, ir.FieldAccess) and (a.offset[0] != 0 or a.offset[1] != 0)}
                bad = sorted(offs & self.written_vars)
                if bad:
                    raise GTScriptSyntaxError(
                        f"{where} The following variables are written before being referenced with an offset in "
                        f"a horizontal region: {', '.join(bad)}")
                # one region statement per mask, in order, as the reference emits one HorizontalIf
                # per region with the same body (gtscript_frontend.py:1957-1962): a point inside
                # two overlapping masks runs the body twice
                return [ir.HorizontalRegion([m], body if n == 0 else copy.deepcopy(body)) for n, m in enumerate(masks)]
            raise GTScriptSyntaxError(f"Invalid 'with' statement inside a computation (line {s.lineno})")
        if isinstance(s, ast.Return):
            # the reference refuses it while building its IR with a ValueError (not a GTScript error)
            raise ValueError("'return' is only allowed in gtscript functions")
        raise GTScriptSyntaxError(f"Unsupported statement {type(s).__name__} (line {getattr(s, 'lineno', '?')})")

    def _parse_region(self, node, scope) -> ir.HorizontalMask:
        # region[I[0]:I[0]+2, J[-1]-2:J[-1]]
        if not (isinstance(node, ast.Subscript)):
            raise GTScriptSyntaxError("Expected region[...]")
        sl = node.slice
        elts = sl.elts if isinstance(sl, ast.Tuple) else [sl]
        if len(elts) != 2:
            raise GTScriptSyntaxError("region[...] needs an I and a J slice")
        from gt4py_amd.gtscript import AxisIndex

        def bound(expr):
            if expr is None:
                return None
            v = self._const_eval(expr, scope)
            if isinstance(v, AxisIndex):
                level = ir.LevelMarker.START if v.index >= 0 else ir.LevelMarker.END
                return ir.AxisBound(level, v.index + v.offset)
            if isinstance(v, int):
                return ir.AxisBound(ir.LevelMarker.END if v < 0 else ir.LevelMarker.START, v)
            raise GTScriptSyntaxError("Region bounds must be axis indices like I[0] + n")

        res = []
        for e in elts:
            if isinstance(e, ast.Slice):
                res.append(ir.HorizontalInterval(bound(e.lower), bound(e.upper)))
            else:
                b = bound(e)
                res.append(ir.HorizontalInterval(b, ir.AxisBound(b.level, b.offset + 1)))
        return ir.HorizontalMask(res[0], res[1])

    def _declare_temporary(self, stmt: ast.AnnAssign, scope: _Scope) -> List[ir.VerticalLoop]:
        """Top-level ``tmp: Field[(dtype, (n, m))] = value``: an IJK temporary (optionally with data
        dimensions) initialised by a full-domain PARALLEL computation
        (reference ``gtscript_frontend.py:2183-2230``, ``_make_init_computations`` ``:791-830``)."""
        from gt4py_amd.gtscript import IJK, _FieldDescriptor

        desc = self._const_eval(stmt.annotation, scope)
        if not isinstance(desc, _FieldDescriptor):
            raise GTScriptSyntaxError("Top-level annotated assignments must declare Field temporaries")
        if tuple(desc.axes_names) != tuple(a.name for a in IJK):
            raise GTScriptSyntaxError(
                f"Found {''.join(desc.axes_names)}, but only IJK is currently supported for temporaries"
            )
        name = stmt.target.id
        dtype = DataType.from_np(desc.dtype)
        tname = self._temp_for_local(name, scope, create=True)
        self.temporaries[tname] = ir.FieldDecl(tname, dtype, ("I", "J", "K"), tuple(desc.data_dims), is_temporary=True)
        self.temp_declared_dtype[tname] = dtype
        if stmt.value is None:
            return []
        value = self._const_eval(stmt.value, scope)
        body = []
        for index in itertools.product(*(range(n) for n in desc.data_dims)):
            didx = [ir.Literal(i, DataType.INT32) for i in index]
            body.append(ir.Assign(ir.FieldAccess(tname, (0, 0, 0), data_index=didx), ir.Literal(value, dtype)))
        full = ir.Interval(ir.AxisBound(ir.LevelMarker.START, 0), ir.AxisBound(ir.LevelMarker.END, 0))
        return [ir.VerticalLoop(ir.LoopOrder.PARALLEL, [ir.Section(full, body)])]

    # ------------------------------------------------------------------ vector expressions
    def _vector_expr(self, node, scope: _Scope, pre):
        """Nested lists of component expressions for a data-dimension expression, or a scalar
        ``ir.Expr`` (reference ``defir_to_gtir.py:123-291``: UnrollVectorAssignments/Expressions)."""
        if isinstance(node, (ast.Name, ast.Subscript)):
            base = node
            offs = (0, 0, 0)
            if isinstance(node, ast.Subscript):
                base = node.value
            if isinstance(base, ast.Name):
                decl = self._decl_of(base.id, scope)
                if decl is not None and decl.data_dims:
                    if isinstance(node, ast.Subscript):
                        offs = self._parse_offset(node.slice, scope, pre)
                    dims = decl.data_dims
                    if len(dims) > 2:
                        raise GTScriptSyntaxError("Higher dimensional fields only supported for vectors and matrices.")

                    def comp(idx):
                        didx = [ir.Literal(i, DataType.INT32) for i in idx]
                        return self._resolve_name(base.id, scope, offs, didx)

                    if len(dims) == 1:
                        return [comp((a,)) for a in range(dims[0])]
                    return [[comp((a, b)) for b in range(dims[1])] for a in range(dims[0])]
        if isinstance(node, ast.Attribute) and node.attr == "T":
            m = self._vector_expr(node.value, scope, pre)
            if not (isinstance(m, list) and m and isinstance(m[0], list)):
                raise GTScriptSyntaxError("'.T' needs a matrix")
            return [list(r) for r in zip(*m)]
        if isinstance(node, ast.UnaryOp) and isinstance(node.op, (ast.USub, ast.UAdd)):
            v = self._vector_expr(node.operand, scope, pre)
            if isinstance(v, list):
                op = "-" if isinstance(node.op, ast.USub) else "+"
                return _vmap(lambda x: ir.UnaryOp(op, x), v)
        if isinstance(node, ast.BinOp):
            lhs = self._vector_expr(node.left, scope, pre)
            rhs = self._vector_expr(node.right, scope, pre)
            if isinstance(node.op, ast.MatMult):
                if not (isinstance(lhs, list) and isinstance(lhs[0], list) and isinstance(rhs, list)):
                    raise GTScriptSyntaxError("'@' needs a matrix and a vector")
                out = []
                for row in lhs:
                    acc = ir.BinaryOp("*", row[0], rhs[0])
                    for a, b in zip(row[1:], rhs[1:]):
                        acc = ir.BinaryOp("+", acc, ir.BinaryOp("*", a, b))
                    out.append(acc)
                return out
            if isinstance(lhs, list) or isinstance(rhs, list):
                op = {ast.Add: "+", ast.Sub: "-", ast.Mult: "*", ast.Div: "/"}.get(type(node.op))
                if op is None:
                    raise GTScriptSyntaxError(f"Unsupported vector operator {type(node.op).__name__}")
                return _vzip(lambda a, b: ir.BinaryOp(op, a, b), lhs, rhs)
        return self._parse_expr(node, scope, pre)

    def _temp_for_local(self, name: str, scope: _Scope, create: bool) -> Optional[str]:
        if name in scope.locals:
            return scope.locals[name]
        if not create:
            return None
        # stencil-level names keep their name, function locals get a unique suffix
        tname = name if scope is self._root_scope else self._new_temp_name(name)
        if tname in self.fields or tname in self.scalars:
            raise GTScriptDefinitionError(f"Cannot assign to parameter '{name}'")
        scope.locals[name] = tname
        return tname

    def _parse_assign(self, target, value, scope: _Scope) -> List[ir.Stmt]:
        pre: List[ir.Stmt] = []
        if isinstance(target, ast.Tuple):
            if not isinstance(value, ast.Call):
                raise GTScriptSyntaxError("Tuple assignment requires a gtscript function call")
            results = self._inline_call(value, scope, pre, n_results=len(target.elts))
            out = pre
            for t, r in zip(target.elts, results):
                out.extend(self._assign_to(t, r, scope))
            return out
        tdecl = None
        tbase = target.value if isinstance(target, ast.Subscript) else target
        if isinstance(tbase, ast.Name):
            tdecl = self._decl_of(tbase.id, scope)
        if tdecl is not None and tdecl.data_dims:
            # whole-field assignment to a data-dimension field: one assignment per component
            vec = self._vector_expr(value, scope, pre)
            out = pre
            for index in itertools.product(*(range(n) for n in tdecl.data_dims)):
                v = vec
                for i in index:
                    v = v[i] if isinstance(v, list) else v
                if isinstance(v, list):
                    raise GTScriptSyntaxError(f"Assignment dimension mismatch for '{tbase.id}'")
                sub = ast.Subscript(
                    value=target if isinstance(target, ast.Subscript) else ast.Subscript(
                        value=tbase, slice=ast.Tuple(elts=[ast.Constant(0)] * 3, ctx=ast.Load()), ctx=ast.Store()
                    ),
                    slice=ast.Tuple(elts=[ast.Constant(i) for i in index], ctx=ast.Load()),
                    ctx=ast.Store(),
                )
                out = out + self._assign_to(sub, v, scope)
            return out
        val = self._parse_expr(value, scope, pre)
        return pre + self._assign_to(target, val, scope)

    def _assign_to(self, target, val: ir.Expr, scope: _Scope) -> List[ir.Stmt]:
        pre: List[ir.Stmt] = []
        t_off = (0, 0, 0)
        t_didx = None
        if isinstance(target, ast.Subscript):
            base = target.value
            if isinstance(base, ast.Subscript) and isinstance(base.value, ast.Name):
                t_didx = self._parse_data_index(target.slice, scope, pre)
                target = base
                base = target.value
            if not isinstance(base, ast.Name):
                raise GTScriptSyntaxError("Invalid assignment target")
            offs = self._parse_offset(target.slice, scope, pre)
            if isinstance(offs, tuple) and len(offs) == 2 and offs[0] == "axes":
                offs = offs[1]
            decl = self._decl_of(base.id, scope)
            if decl is not None and base.id in self.fields and len(offs) == sum(decl.mask) and len(offs) != 3:
                it = iter(offs)
                offs = tuple(next(it) if m else 0 for m in decl.mask)
            if len(offs) == 3:
                if any(isinstance(o, ir.Expr) or o != 0 for o in offs[:2]):
                    raise GTScriptSyntaxError("Assignment to non-zero offsets is not supported in IJ.")
                if (isinstance(offs[2], ir.Expr) or offs[2] != 0) and getattr(self, "_loop_order", None) == ir.LoopOrder.PARALLEL:
                    raise GTScriptSyntaxError(
                        "Assignment to non-zero offsets in K is not available in PARALLEL. Choose FORWARD or BACKWARD."
                    )
            t_off = offs
            target = base
        if not isinstance(target, ast.Name):
            raise GTScriptSyntaxError("Invalid assignment target")
        name = target.id
        if name in scope.aliases:
            alias = scope.aliases[name]
            if isinstance(alias, tuple) and alias[0] == "field" and alias[2] == (0, 0, 0):
                name_res = alias[1]
            else:
                raise GTScriptSyntaxError(f"Cannot assign to function argument '{name}'")
        elif name in self.fields and scope is self._root_scope:
            name_res = name
        elif name in self.scalars and scope is self._root_scope:
            raise GTScriptDefinitionError(f"Cannot assign to scalar parameter '{name}'")
        else:
            name_res = self._temp_for_local(name, scope, create=True)
            if name_res not in self.temporaries:
                if t_didx:
                    raise GTScriptSyntaxError("Temporaries with data dimensions need to be declared explicitly.")
                self.temporaries[name_res] = ir.FieldDecl(name_res, DataType.AUTO, is_temporary=True)
        decl = self.fields.get(name_res) or self.temporaries.get(name_res)
        axes = tuple(getattr(decl, "axes", ("I", "J", "K")) or ("I", "J", "K"))
        need = ["I", "J"] + (["K"] if getattr(self, "_loop_order", None) == ir.LoopOrder.PARALLEL else [])
        if set(need) - set(axes):
            # a lower-dimensional field is written only by a sweep that covers its missing axes
            # (reference gtscript_frontend.py:1894-1902)
            raise GTScriptSyntaxError(
                f"Cannot assign to field '{name}' as all parallel axes '{need}' are not present.")
        if t_off != (0, 0, 0) or t_didx:
            tgt = self._field_access(name_res, t_off, scope, t_didx)
            if tgt.offset[2] != 0 or tgt.k_offset is not None:
                if name_res not in self.fields:
                    raise GTScriptSyntaxError("Assignment with a K offset is only supported for API fields")
        else:
            tgt = ir.FieldAccess(name_res, (0, 0, 0))
        if not self._in_region:
            self.written_vars.add(name_res)
        return pre + [ir.Assign(tgt, val)]

    # ------------------------------------------------------------------ expressions
    def _parse_offset(self, sl, scope, pre=None) -> Tuple:
        """Spatial index of a subscript: ints, or (K only) a run-time integer expression.

        Accepts ``[1, 0, -1]``, ``[0, 0, lev + 1]`` and the axis form ``[I - 1]`` / ``[K + 1]``
        (reference ``gtscript_frontend.py:1316-1390``); the axis form returns all three offsets.
        """
        elts = sl.elts if isinstance(sl, ast.Tuple) else [sl]
        axis_form = any(
            isinstance(n, ast.Name) and n.id in ("I", "J", "K") and isinstance(self._try_const(n, scope), Axis)
            for e in elts
            for n in ast.walk(e)
        )
        if axis_form:
            off = [0, 0, 0]
            last = -1  # axes in I, J, K order, each once (reference gtscript_frontend.py:1326-1339)
            for e in elts:
                shift = 0
                node = e
                if isinstance(e, ast.BinOp) and isinstance(e.op, (ast.Add, ast.Sub)):
                    shift = int(self._const_eval(e.right, scope)) * (1 if isinstance(e.op, ast.Add) else -1)
                    node = e.left
                ax = self._try_const(node, scope)
                if not isinstance(ax, Axis):
                    raise GTScriptSyntaxError("Invalid axis offset expression")
                idx = "IJK".index(ax.name)
                if idx < last:
                    raise GTScriptSyntaxError(f"Axis {ax.name} is specified out of order")
                if idx == last:
                    raise GTScriptSyntaxError(f"Duplicate axis found: {ax.name}")
                last = idx
                off[idx] = shift
            return ("axes", tuple(off))
        vals = []
        for e in elts:
            v = self._try_const(e, scope)
            if isinstance(v, (int, np.integer)) and not isinstance(v, (bool, np.bool_)):
                vals.append(int(v))
            elif pre is None:
                raise GTScriptSyntaxError("Run-time offsets are only allowed in expressions and assignment targets")
            else:
                vals.append(self._parse_expr(e, scope, pre))
        return tuple(vals)

    def _decl_of(self, name: str, scope: _Scope):
        """FieldDecl a (possibly aliased) name refers to, or None."""
        if name in scope.aliases:
            alias = scope.aliases[name]
            if isinstance(alias, tuple) and alias[0] == "field":
                name = alias[1]
            else:
                return None
        elif name in scope.locals:
            name = scope.locals[name]
        return self.fields.get(name) or self.temporaries.get(name)

    def _try_const(self, node, scope):
        try:
            return self._const_eval(node, scope)
        except Exception:  # noqa: BLE001 - not a compile-time value
            return None

    def _parse_data_index(self, sl, scope, pre) -> List[ir.Expr]:
        elts = sl.elts if isinstance(sl, ast.Tuple) else [sl]
        out = []
        for e in elts:
            v = self._try_const(e, scope)
            if isinstance(v, (int, np.integer)) and not isinstance(v, (bool, np.bool_)):
                out.append(ir.Literal(int(v), DataType.INT32))
            else:
                out.append(self._parse_expr(e, scope, pre))
        return out

    def _field_access(self, name: str, offset, scope, data_index=None) -> ir.FieldAccess:
        decl = self.fields.get(name) or self.temporaries.get(name)
        if isinstance(offset, tuple) and len(offset) == 2 and offset[0] == "axes":
            off = list(offset[1])
        else:
            off = list(offset)
            if decl is not None and name in self.fields:
                mask = decl.mask
                if len(off) == sum(mask) and len(off) != 3:
                    it = iter(off)
                    off = [next(it) if m else 0 for m in mask]
        if len(off) != 3:
            raise GTScriptSyntaxError(f"Invalid offset {tuple(offset)} for '{name}'")
        k_expr = None
        if isinstance(off[2], ir.Expr):
            k_expr, off[2] = off[2], 0
            if off[0] or off[1]:
                # as the reference: a run-time K offset becomes gtir.VariableKOffset(k=...) and the I/J
                # offsets written beside it are dropped (frontend/defir_to_gtir.py:626-639,
                # gtc/common.py:341-345 `to_dict` -> i = j = 0), so `f[1, 0, lev]` reads f[0, 0, lev]
                warnings.warn(
                    f"'{name}[{off[0]}, {off[1]}, <run-time K offset>]': the I/J offsets of a field read at a "
                    f"run-time K offset are ignored, as in the reference (it reads '{name}' at the centre column)",
                    stacklevel=2,
                )
                off[0] = off[1] = 0
        if any(isinstance(o, ir.Expr) for o in off[:2]):
            raise GTScriptSyntaxError(f"Run-time offsets are only supported along K ('{name}')")
        ndd = len(decl.data_dims) if decl is not None else 0
        data_index = list(data_index or [])
        if len(data_index) != ndd:
            raise GTScriptSyntaxError(
                f"Incorrect data index length {len(data_index)}. Invalid data dimension index. "
                f"Field {name} has {ndd} data dimensions."
            )
        for d, n in zip(data_index, decl.data_dims if decl is not None else ()):
            if isinstance(d, ir.Literal) and not (0 <= int(d.value) < n):
                raise GTScriptSyntaxError(f"Data index out of bounds for field {name}")
        return ir.FieldAccess(name, tuple(off), data_index=data_index, k_offset=k_expr)

    def _resolve_name(self, name: str, scope: _Scope, offset=(0, 0, 0), data_index=None) -> ir.Expr:
        if isinstance(offset, tuple) and len(offset) == 2 and offset[0] == "axes":
            offset = offset[1]
        if name in scope.aliases:
            alias = scope.aliases[name]
            if isinstance(alias, tuple) and alias[0] == "field":
                base_off = alias[2]
                off = tuple(
                    (a + b) if not isinstance(b, ir.Expr) else (b if a == 0 else ir.BinaryOp("+", b, ir.Literal(a, DataType.INT64)))
                    for a, b in zip(base_off, offset)
                )
                return self._field_access(alias[1], off, scope, data_index)
            if any(not isinstance(o, int) or o for o in offset):
                raise GTScriptSyntaxError(f"Offset access to non-field argument '{name}'")
            return alias
        if name in scope.locals:
            return self._field_access(scope.locals[name], tuple(offset), scope, data_index)
        if scope is self._root_scope:
            if name in self.fields:
                return self._field_access(name, offset, scope, data_index)
            if name in self.scalars:
                if any(offset):
                    raise GTScriptSyntaxError(f"Offset access to scalar '{name}'")
                return ir.ScalarAccess(name)
        if name in ("True", "False"):
            return ir.Literal(name == "True", DataType.BOOL)
        if name in ("I", "J", "K") and not any(offset):
            # iterator access (gtir.IteratorAccess): only K may be queried (gtscript_frontend.py:860-872)
            if name != "K":
                raise GTScriptSyntaxError(f"Parallel axis {name} can't be queried - only K")
            return ir.AxisIndex(2)
        found, val = scope.lookup_external(name)
        if found:
            if isinstance(val, (bool, np.bool_, numbers.Number, np.generic)):
                if any(offset):
                    raise GTScriptSyntaxError(f"Offset access to constant '{name}'")
                self.used_externals.setdefault(name, val)
                return self._literal(val)
            if name in scope.imported and not _valid_external(val):
                # the reference's GTScriptParser.eval_external (gtscript_frontend.py:2317-2334)
                raise GTScriptDefinitionError(f"Missing or invalid value for external symbol {name}")
        raise GTScriptSymbolError(f"Unknown symbol '{name}'")

    def _parse_expr(self, node, scope: _Scope, pre: List[ir.Stmt]) -> ir.Expr:
        if isinstance(node, ast.Constant):
            if node.value is None:
                raise GTScriptSyntaxError("None is not a valid expression")
            return self._literal(node.value)
        if isinstance(node, ast.Name):
            return self._resolve_name(node.id, scope)
        if isinstance(node, ast.Subscript):
            if isinstance(node.value, ast.Name):
                decl = self._decl_of(node.value.id, scope)
                if decl is not None and decl.data_dims and not any(decl.mask):
                    raise GTScriptSyntaxError(
                        f"Incorrect offset specification detected for {node.value.id}. "
                        f"Did you mean absolute indexing via .A[...]?"
                    )
                offs = self._parse_offset(node.slice, scope, pre)
                return self._resolve_name(node.value.id, scope, offs)
            if isinstance(node.value, ast.Subscript) and isinstance(node.value.value, ast.Name):
                # f[i, j, k][d0, d1, ...]: data-dimension index
                offs = self._parse_offset(node.value.slice, scope, pre)
                didx = self._parse_data_index(node.slice, scope, pre)
                return self._resolve_name(node.value.value.id, scope, offs, didx)
            if (
                isinstance(node.value, ast.Attribute)
                and node.value.attr == "A"
                and isinstance(node.value.value, ast.Name)
            ):
                # table.A[d0, ...]: absolute data index at the current point (GlobalTable)
                didx = self._parse_data_index(node.slice, scope, pre)
                return self._resolve_name(node.value.value.id, scope, (0, 0, 0), didx)
            raise GTScriptSyntaxError("Invalid subscript")
        if isinstance(node, ast.Attribute):
            v = self._const_eval(node, scope)
            return self._literal(v)
        if isinstance(node, ast.UnaryOp):
            operand = self._parse_expr(node.operand, scope, pre)
            op = {ast.USub: "-", ast.UAdd: "+", ast.Not: "not"}.get(type(node.op))
            if op is None:
                raise GTScriptSyntaxError(f"Unsupported unary operator {type(node.op).__name__}")
            return ir.UnaryOp(op, operand)
        if isinstance(node, ast.BinOp):
            left = self._parse_expr(node.left, scope, pre)
            right = self._parse_expr(node.right, scope, pre)
            if isinstance(node.op, ast.Pow):
                return ir.NativeCall("pow", [left, right])
            if isinstance(node.op, ast.Mod):
                return ir.NativeCall("mod", [left, right])
            op = {ast.Add: "+", ast.Sub: "-", ast.Mult: "*", ast.Div: "/"}.get(type(node.op))
            if op is None:
                raise GTScriptSyntaxError(f"Unsupported binary operator {type(node.op).__name__}")
            return ir.BinaryOp(op, left, right)
        if isinstance(node, ast.BoolOp):
            op = "and" if isinstance(node.op, ast.And) else "or"
            vals = [self._parse_expr(v, scope, pre) for v in node.values]
            res = vals[0]
            for v in vals[1:]:
                res = ir.BinaryOp(op, res, v)
            return res
        if isinstance(node, ast.Compare):
            ops = {ast.Gt: ">", ast.Lt: "<", ast.GtE: ">=", ast.LtE: "<=", ast.Eq: "==", ast.NotEq: "!="}
            left = self._parse_expr(node.left, scope, pre)
            res = None
            for op, comp in zip(node.ops, node.comparators):
                right = self._parse_expr(comp, scope, pre)
                if type(op) not in ops:
                    raise GTScriptSyntaxError(f"Unsupported comparison {type(op).__name__}")
                c = ir.BinaryOp(ops[type(op)], left, right)
                res = c if res is None else ir.BinaryOp("and", res, c)
                left = right
            return res
        if isinstance(node, ast.IfExp):
            cond = self._parse_expr(node.test, scope, pre)
            t = self._parse_expr(node.body, scope, pre)
            f = self._parse_expr(node.orelse, scope, pre)
            return ir.TernaryOp(cond, t, f)
        if isinstance(node, ast.Call):
            return self._parse_call(node, scope, pre)
        raise GTScriptSyntaxError(f"Unsupported expression {type(node).__name__}")

    def _absolute_k(self, node: ast.Call, scope: _Scope, pre) -> ir.Expr:
        """``field.at(K=expr[, ddim=[...]])``: the field at absolute level ``expr`` (relative to the
        field's origin) -- lowered to a run-time K offset ``expr - K`` of the current level
        (reference ``gtscript_frontend.py:1660-1711``, AbsoluteKIndex)."""
        kws = node.keywords
        if node.args or not kws or kws[0].arg != "K" or len(kws) > 2 or (len(kws) == 2 and kws[1].arg != "ddim"):
            raise GTScriptSyntaxError(
                "Absolute K index: Bad syntax. Must be of the form `.at(K=..., ddim=[...])` "
            )
        kval = self._parse_expr(kws[0].value, scope, pre)
        if isinstance(kval, ir.AxisIndex):
            raise GTScriptSyntaxError("Absolute K index: bad syntax, you cannot use an axis iterator in `.at(K=...)`")
        didx = None
        if len(kws) == 2:
            if not isinstance(kws[1].value, (ast.List, ast.Tuple)):
                raise GTScriptSyntaxError("Absolute K index: `ddim` must be a list of values")
            didx = self._parse_data_index(ast.Tuple(elts=kws[1].value.elts, ctx=ast.Load()), scope, pre)
        base = node.func.value
        if not isinstance(base, ast.Name) or self._decl_of(base.id, scope) is None:
            raise GTScriptSyntaxError("Absolute K index: `.at` needs a field")
        decl = self._decl_of(base.id, scope)
        if not decl.mask[2]:
            raise GTScriptSyntaxError("Tried accessing a field with no K-dimensions with an absolute K-index.")
        acc = self._resolve_name(base.id, scope, (0, 0, 0), didx)
        koff = ir.BinaryOp("-", ir.NativeCall("int64", [kval]), ir.AxisIndex(2))
        return dataclasses.replace(acc, k_offset=koff)

    def _parse_call(self, node: ast.Call, scope: _Scope, pre) -> ir.Expr:
        if isinstance(node.func, ast.Attribute) and node.func.attr == "at":
            return self._absolute_k(node, scope, pre)
        fname = self._call_name(node)
        func_obj = None
        if isinstance(node.func, ast.Name):
            if node.func.id in scope.aliases or node.func.id in scope.locals:
                raise GTScriptSyntaxError(f"'{node.func.id}' is not callable")
            found, func_obj = scope.lookup_external(node.func.id)
            if not found:
                raise GTScriptSymbolError(f"Unknown function '{node.func.id}'")
        elif isinstance(node.func, ast.Attribute):
            # a dotted callee is an external symbol to the reference (``np.sqrt``, ``gtscript.sqrt``):
            # its value must be a gtscript function (eval_external + resolve_external_symbols,
            # gtscript_frontend.py:2317-2354)
            dotted = ast.unparse(node.func)
            try:
                func_obj = self._const_eval(node.func, scope)
            except Exception as ex:  # noqa: BLE001
                raise GTScriptDefinitionError(f"Missing or invalid value for external symbol {dotted}") from ex
            if not is_gtscript_function(func_obj):
                if isinstance(func_obj, types.FunctionType):
                    raise TypeError(f"{func_obj.__name__} is not a gtscript function")
                raise GTScriptDefinitionError(f"Missing or invalid value for external symbol {dotted}")
        if is_gtscript_function(func_obj):
            (res,) = self._inline_call(node, scope, pre, n_results=1, func=func_obj)
            return res
        native = None
        builtin_name = getattr(func_obj, "_gtscript_builtin_", None)
        if builtin_name is not None:
            native = builtin_name
        elif func_obj in (builtins.abs, builtins.min, builtins.max, builtins.round):
            native = {builtins.abs: "abs", builtins.min: "min", builtins.max: "max", builtins.round: "round"}[func_obj]
        elif func_obj in (np.int32, np.int64, np.float32, np.float64, builtins.float, builtins.int):
            if func_obj is builtins.float:
                native = "float64" if self.options.literal_float_precision == 64 else "float32"
            elif func_obj is builtins.int:
                native = "int64" if self.options.literal_int_precision == 64 else "int32"
            else:
                native = np.dtype(func_obj).name
        elif fname in ir.NATIVE_FUNCTIONS:
            native = fname
        if native is None:
            raise GTScriptSyntaxError(f"Unsupported function call '{fname}'")
        if node.keywords:
            raise GTScriptSyntaxError(f"Keyword arguments are not supported for '{fname}'")
        args = [self._parse_expr(a, scope, pre) for a in node.args]
        if len(args) != ir.NATIVE_FUNCTIONS[native]:
            raise GTScriptSyntaxError(f"{native} accepts {ir.NATIVE_FUNCTIONS[native]} arguments, {len(args)} given")
        return ir.NativeCall(native, args)

    # ------------------------------------------------------------------ inlining
    def _calls_gtscript_function(self, expr: ast.AST, scope: _Scope) -> bool:
        """Whether ``expr`` calls a gtscript function (native functions excluded)."""
        for n in ast.walk(expr):
            if isinstance(n, ast.Call) and isinstance(n.func, ast.Name):
                found, func = scope.lookup_external(n.func.id)
                if found and is_gtscript_function(func):
                    return True
        return False

    def _inline_call(self, node: ast.Call, scope: _Scope, pre: List[ir.Stmt], n_results: int, func=None):
        if func is None:
            if isinstance(node.func, ast.Name):
                found, func = scope.lookup_external(node.func.id)
                if not found:
                    raise GTScriptSymbolError(f"Unknown function '{node.func.id}'")
            else:
                func = self._const_eval(node.func, scope)
        if not is_gtscript_function(func):
            raise GTScriptSyntaxError(f"'{getattr(func, '__name__', func)}' is not a gtscript function")
        fdef = _func_ast(func)
        sig = inspect.signature(func)
        # bind arguments
        bound_args: Dict[str, ast.AST] = {}
        names = list(sig.parameters)
        for i, a in enumerate(node.args):
            bound_args[names[i]] = a
        for kw in node.keywords:
            bound_args[kw.arg] = kw.value
        for pname, p in sig.parameters.items():
            if pname not in bound_args:
                if p.default is inspect.Parameter.empty:
                    raise GTScriptSyntaxError(f"Missing argument '{pname}' calling {func.__name__}")
                bound_args[pname] = ast.Constant(p.default)
        fscope = _Scope(_func_namespace(func), self.externals)
        fscope.imported = dict(scope.imported)
        for pname, arg in bound_args.items():
            alias = None
            if isinstance(arg, ast.Name) and (arg.id in scope.aliases or arg.id in scope.locals or (
                scope is self._root_scope and (arg.id in self.fields or arg.id in self.scalars)
            )):
                e = self._resolve_name(arg.id, scope)
                if isinstance(e, ir.FieldAccess):
                    alias = ("field", e.name, e.offset)
                else:
                    alias = e
            elif isinstance(arg, ast.Subscript) and isinstance(arg.value, ast.Name):
                e = self._parse_expr(arg, scope, pre)
                alias = ("field", e.name, e.offset) if isinstance(e, ir.FieldAccess) else e
            else:
                e = self._parse_expr(arg, scope, pre)
                if isinstance(e, ir.Literal):
                    alias = e
                else:
                    tname = self._new_temp_name(f"{func.__name__}_{pname}")
                    self.temporaries[tname] = ir.FieldDecl(tname, DataType.AUTO, is_temporary=True)
                    pre.append(ir.Assign(ir.FieldAccess(tname, (0, 0, 0)), e))
                    alias = ("field", tname, (0, 0, 0))
            fscope.aliases[pname] = alias
        results = None
        body = list(fdef.body)
        if body and isinstance(body[0], ast.Expr) and isinstance(body[0].value, ast.Constant):
            body = body[1:]
        for st in body:
            if isinstance(st, ast.Return):
                if results is not None:
                    raise GTScriptSyntaxError("Multiple return statements in gtscript function")
                vals = st.value.elts if isinstance(st.value, ast.Tuple) else [st.value]
                results = []
                for v in vals:
                    if isinstance(v, ast.Call) and is_gtscript_function(self._maybe_func(v, fscope)):
                        results.extend(self._inline_call(v, fscope, pre, n_results=1))
                    else:
                        results.append(self._parse_expr(v, fscope, pre))
            else:
                pre.extend(self._parse_stmt_in_function(st, fscope))
        if results is None:
            raise GTScriptSyntaxError(f"gtscript function {func.__name__} has no return statement")
        if len(results) != n_results:
            raise GTScriptSyntaxError(
                f"gtscript function {func.__name__} returns {len(results)} values, {n_results} expected"
            )
        return results

    def _maybe_func(self, call: ast.Call, scope):
        try:
            if isinstance(call.func, ast.Name):
                found, f = scope.lookup_external(call.func.id)
                return f if found else None
            return self._const_eval(call.func, scope)
        except Exception:
            return None

    def _parse_stmt_in_function(self, st, fscope):
        return self._parse_stmt(st, fscope)

    # ------------------------------------------------------------------ public
    def parse(self) -> ir.Stencil:
        func = self.definition
        self._parse_signature()
        fdef = _func_ast(func)
        scope = _Scope(_func_namespace(func), self.externals)
        self._root_scope = scope
        loops: List[ir.VerticalLoop] = []
        body = list(fdef.body)
        if body and isinstance(body[0], ast.Expr) and isinstance(getattr(body[0], "value", None), ast.Constant):
            body = body[1:]
        for stmt in body:
            if isinstance(stmt, (ast.Import, ast.ImportFrom)):
                self._parse_import(stmt, scope)
            elif isinstance(stmt, ast.With):
                loops.extend(self._parse_computation(stmt, scope))
            elif isinstance(stmt, ast.AnnAssign) and isinstance(stmt.target, ast.Name):
                loops.extend(self._declare_temporary(stmt, scope))
            elif isinstance(stmt, ast.Pass) or (
                isinstance(stmt, ast.Expr) and isinstance(getattr(stmt, "value", None), ast.Constant)
            ):
                continue
            else:
                raise GTScriptSyntaxError(
                    "Invalid stencil definition: only 'with computation(...)' blocks are allowed at the top "
                    f"level (line {getattr(stmt, 'lineno', '?')})"
                )
        params: List[Any] = [self.fields[n] if n in self.fields else self.scalars[n] for n in self.api_order]
        return ir.Stencil(
            # the stencil's build name (gtscript.stencil(name=...), last component) as the
            # reference's GTIR carries it, else the definition's
            name=(getattr(self.options, "name", "") or func.__name__),
            api_signature=list(self.api_order),
            params=params,
            temporaries=list(self.temporaries.values()),
            vertical_loops=loops,
            externals=dict(self.used_externals),
            docstring=inspect.getdoc(func) or "",
        )


def _vmap(fn, v):
    return [_vmap(fn, x) for x in v] if isinstance(v, list) else fn(v)


def _vzip(fn, a, b):
    if isinstance(a, list) and isinstance(b, list):
        if len(a) != len(b):
            raise GTScriptSyntaxError("Vector operands of different lengths")
        return [_vzip(fn, x, y) for x, y in zip(a, b)]
    if isinstance(a, list):
        return [_vzip(fn, x, b) for x in a]
    if isinstance(b, list):
        return [_vzip(fn, a, y) for y in b]
    return fn(a, b)


def _load_copy(target):
    """Turn an assignment target into an equivalent load expression."""
    if isinstance(target, ast.Name):
        return ast.Name(id=target.id, ctx=ast.Load())
    if isinstance(target, ast.Subscript):
        return ast.Subscript(value=_load_copy(target.value), slice=target.slice, ctx=ast.Load())
    raise GTScriptSyntaxError("Invalid augmented assignment target")


def parse_stencil(definition, externals, options, dtypes=None) -> ir.Stencil:
    parser = StencilParser(definition, externals, options, dtypes)
    stencil = parser.parse()
    stencil.temp_declared_dtype = dict(parser.temp_declared_dtype)
    return stencil
