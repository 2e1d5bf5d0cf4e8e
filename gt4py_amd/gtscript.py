"""GTScript DSL surface of gt4py_amd (mirrors ``gt4py.cartesian.gtscript``).

Same names and meaning as the reference module (``src/gt4py/cartesian/gtscript.py``):
``stencil`` (``:171-352``), ``function`` (``:160``), ``Field`` (``:702-745``), ``computation``/
``interval``/``horizontal``/``region`` (``:782-805``), ``PARALLEL/FORWARD/BACKWARD``
(``:647-653``), ``I/J/K`` (``:617-623``), math builtins (``:826-1004``). The stencil bodies are
never executed by Python: they are parsed by ``gt4py_amd.frontend``.
"""

from __future__ import annotations

import collections.abc
import inspect
import types
from typing import Any, Dict, Optional

import numpy as np

from gt4py_amd import definitions as gt_definitions

__all__ = [
    "IJK",
    "IJ",
    "IK",
    "JK",
    "I",
    "J",
    "K",
    "PARALLEL",
    "FORWARD",
    "BACKWARD",
    "Field",
    "GlobalTable",
    "computation",
    "interval",
    "horizontal",
    "region",
    "function",
    "stencil",
    "lazy_stencil",
    "mark_stencil",
]

# --------------------------------------------------------------------------------------
# Axes
# --------------------------------------------------------------------------------------


class AxisIndex:
    def __init__(self, axis: str, index: int, offset: int = 0):
        self.axis, self.index, self.offset = axis, index, offset

    def __add__(self, offset: int):
        if not isinstance(offset, int):
            raise TypeError(f"Can only add type int, got {type(offset)}")
        return AxisIndex(self.axis, self.index, self.offset + offset)

    def __sub__(self, offset: int):
        return self + (-offset)

    def __repr__(self):
        return f"{self.axis}[{self.index}] + {self.offset}"


class AxisInterval:
    def __init__(self, axis: str, start, stop):
        self.axis, self.start, self.stop = axis, start, stop


class Axis:
    def __init__(self, name: str):
        assert name
        self.name = name

    @property
    def __gt_axis_name__(self) -> str:
        return self.name

    def __repr__(self):
        return f"Axis(name={self.name})"

    def __str__(self):
        return self.name

    def __getitem__(self, index):
        if isinstance(index, slice):
            return AxisInterval(self.name, index.start, index.stop)
        if isinstance(index, int):
            return AxisIndex(self.name, index)
        raise TypeError("Unrecognized index type")


I = Axis("I")  # noqa: E741
J = Axis("J")
K = Axis("K")
IJ = (I, J)
IK = (I, K)
JK = (J, K)
IJK = (I, J, K)

# Iteration orders (gtscript.py:647-653)
FORWARD = +1
BACKWARD = -1
PARALLEL = 0

# --------------------------------------------------------------------------------------
# Field descriptors
# --------------------------------------------------------------------------------------

_VALID_DATA_TYPES = (
    np.dtype(np.bool_),
    np.dtype(np.int8),
    np.dtype(np.int16),
    np.dtype(np.int32),
    np.dtype(np.int64),
    np.dtype(np.float32),
    np.dtype(np.float64),
)


class _FieldDescriptor:
    def __init__(self, dtype, axes, data_dims=tuple()):
        if isinstance(dtype, str):
            self.dtype = dtype
        else:
            try:
                dtype = np.dtype(dtype)
                if dtype.shape:
                    assert not data_dims
                    data_dims = dtype.shape
                    dtype = dtype.base
                if dtype not in _VALID_DATA_TYPES:
                    raise ValueError("Invalid data type descriptor")
            except TypeError as ex:
                raise ValueError("Invalid data type descriptor") from ex
            self.dtype = np.dtype(dtype)
        self.axes = axes if isinstance(axes, collections.abc.Collection) else [axes]
        if data_dims:
            self.data_dims = (
                tuple(data_dims) if isinstance(data_dims, collections.abc.Collection) else (data_dims,)
            )
        else:
            self.data_dims = ()

    @property
    def axes_names(self):
        return tuple(a.name if isinstance(a, Axis) else str(a) for a in self.axes)

    def __repr__(self):
        return f"_FieldDescriptor(dtype={self.dtype!r}, axes={self.axes!r}, data_dims={self.data_dims!r})"

    def __str__(self):
        return f"Field<[{', '.join(str(a) for a in self.axes)}], ({self.dtype}, {self.data_dims})>"


class _FieldDescriptorMaker:
    @staticmethod
    def _is_axes_spec(spec) -> bool:
        return isinstance(spec, Axis) or (
            isinstance(spec, collections.abc.Collection) and all(isinstance(i, Axis) for i in spec)
        )

    def __getitem__(self, field_spec):
        axes = IJK
        data_dims = ()
        if isinstance(field_spec, str) or not isinstance(field_spec, collections.abc.Collection):
            dtype = field_spec
        elif _FieldDescriptorMaker._is_axes_spec(field_spec[0]):
            assert len(field_spec) == 2
            axes, dtype = field_spec
        elif len(field_spec) == 2 and not _FieldDescriptorMaker._is_axes_spec(field_spec[1]):
            dtype = field_spec
        else:
            raise ValueError("Invalid field type descriptor")
        if isinstance(dtype, collections.abc.Collection) and not isinstance(dtype, str):
            assert len(dtype) == 2
            dtype, data_dims = dtype
        return _FieldDescriptor(dtype, axes, data_dims)


Field = _FieldDescriptorMaker()


class _TableDescriptorMaker:
    """``GlobalTable[(dtype, (n0, n1, ...))]``: data dimensions only, read with ``table.A[...]``
    (reference ``gtscript.py:734-749``)."""

    def __getitem__(self, spec):
        if not isinstance(spec, collections.abc.Collection) or len(spec) != 2:
            raise ValueError("GlobalTable is defined by a tuple (type, [axes_size..])")
        dtype, data_dims = spec
        return _FieldDescriptor(dtype, [], data_dims)


GlobalTable = _TableDescriptorMaker()

# --------------------------------------------------------------------------------------
# Context managers / markers (bodies are parsed, never executed)
# --------------------------------------------------------------------------------------


class _ComputationContextManager:
    def __enter__(self):
        pass

    def __exit__(self, exc_type, exc_value, traceback):
        pass


def computation(order):
    """Define the computation (iteration order along K)."""
    return _ComputationContextManager()


def interval(*args):
    """Define the interval of computation in the K sequential axis."""
    return _ComputationContextManager()


def horizontal(*args):
    """Restrict a block of code to a set of regions in the parallel axes."""
    return _ComputationContextManager()


class _Region:
    def __getitem__(self, *args):
        pass


region = _Region()


def __INLINED(compile_if_expression):  # noqa: N802
    """Evaluate condition at compile time and inline statements from the selected branch."""


def compile_assert(expr):
    """Assert that expr evaluates to True at compile time."""


def externals(*args):
    return args


# Type casts
int32 = np.int32
int64 = np.int64
float32 = np.float32
float64 = np.float64

# --------------------------------------------------------------------------------------
# Math builtins: stubs (parsed by the frontend; names match gtscript.py:826-1004)
# --------------------------------------------------------------------------------------

MATH_BUILTINS = {
    "abs": "abs",
    "min": "min",
    "max": "max",
    "mod": "mod",
    "sin": "sin",
    "cos": "cos",
    "tan": "tan",
    "asin": "arcsin",
    "acos": "arccos",
    "atan": "arctan",
    "sinh": "sinh",
    "cosh": "cosh",
    "tanh": "tanh",
    "asinh": "arcsinh",
    "acosh": "arccosh",
    "atanh": "arctanh",
    "sqrt": "sqrt",
    "exp": "exp",
    "log": "log",
    "log10": "log10",
    "gamma": "gamma",
    "cbrt": "cbrt",
    "isfinite": "isfinite",
    "isinf": "isinf",
    "isnan": "isnan",
    "floor": "floor",
    "ceil": "ceil",
    "trunc": "trunc",
    "erf": "erf",
    "erfc": "erfc",
    "round": "round",
    "round_away_from_zero": "round_away_from_zero",
}


def _make_builtin(name):
    def _stub(*args):
        raise RuntimeError(f"GTScript builtin '{name}' can only be used inside a stencil definition")

    _stub.__name__ = name
    _stub._gtscript_builtin_ = MATH_BUILTINS[name]
    return _stub


for _n in MATH_BUILTINS:
    globals()[_n] = _make_builtin(_n)
    __all__.append(_n)
del _n

# --------------------------------------------------------------------------------------
# Functions and stencils
# --------------------------------------------------------------------------------------


def function(func):
    """Mark a GTScript function (inlined into stencils at parse time)."""
    from gt4py_amd import frontend

    frontend.annotate_function(func)
    return func


def _set_arg_dtypes(definition, dtypes: Dict[str, Any]):
    """Resolve string dtype annotations (``Field["dtype_name"]``) through ``dtypes``."""
    assert isinstance(definition, types.FunctionType)
    annotations = getattr(definition, "__annotations__", {})
    original = dict(annotations)
    for arg, value in list(annotations.items()):
        if isinstance(value, _FieldDescriptor) and isinstance(value.dtype, str):
            if value.dtype in dtypes:
                annotations[arg] = _FieldDescriptor(dtypes[value.dtype], value.axes, value.data_dims)
            else:
                raise ValueError(f"Missing '{value.dtype}' dtype definition for arg '{arg}'")
        elif isinstance(value, str):
            if value in dtypes:
                annotations[arg] = dtypes[value]
            else:
                # postponed annotation (``from __future__ import annotations``): evaluate it
                from gt4py_amd.frontend import _func_namespace

                try:
                    resolved = eval(value, _func_namespace(definition))  # noqa: S307 - user annotation
                except Exception as ex:
                    raise ValueError(f"Missing '{value}' dtype definition for arg '{arg}'") from ex
                if isinstance(resolved, _FieldDescriptor) and isinstance(resolved.dtype, str):
                    if resolved.dtype not in dtypes:
                        raise ValueError(f"Missing '{resolved.dtype}' dtype definition for arg '{arg}'")
                    resolved = _FieldDescriptor(dtypes[resolved.dtype], resolved.axes, resolved.data_dims)
                annotations[arg] = resolved
    return original


def stencil(
    backend,
    definition=None,
    *,
    build_info=None,
    dtypes=None,
    externals=None,
    format_source=True,
    name=None,
    rebuild=False,
    cache_settings=None,
    raise_if_not_cached=False,
    literal_int_precision=gt_definitions.LITERAL_INT_PRECISION,
    literal_float_precision=gt_definitions.LITERAL_FLOAT_PRECISION,
    **kwargs,
):
    """Generate an implementation of the stencil definition with the given backend.

    Same contract as ``gt4py.cartesian.gtscript.stencil`` (reference ``gtscript.py:171-352``):
    usable as ``@stencil(backend=...)`` decorator or called with ``definition``; returns the
    singleton instance of a generated :class:`gt4py_amd.stencil_object.StencilObject` subclass.
    """
    from gt4py_amd import loader

    if build_info is not None and not isinstance(build_info, dict):
        raise ValueError(f"Invalid 'build_info' dictionary ('{build_info}')")
    if dtypes is not None and not isinstance(dtypes, dict):
        raise ValueError(f"Invalid 'dtypes' dictionary ('{dtypes}')")
    if externals is not None and not isinstance(externals, dict):
        raise ValueError(f"Invalid 'externals' dictionary ('{externals}')")
    if not isinstance(format_source, bool):
        raise ValueError(f"Invalid 'format_source' bool value ('{name}')")
    if name is not None and not isinstance(name, str):
        raise ValueError(f"Invalid 'name' string ('{name}')")
    if not isinstance(rebuild, bool):
        raise ValueError(f"Invalid 'rebuild' bool value ('{rebuild}')")
    if not isinstance(raise_if_not_cached, bool):
        raise ValueError(f"Invalid 'raise_if_not_cached' bool value ('{raise_if_not_cached}')")
    if cache_settings is not None and not isinstance(cache_settings, dict):
        raise ValueError(f"Invalid 'cache_settings' dictionary ('{cache_settings}')")
    if literal_int_precision not in (32, 64):
        raise ValueError(f"Invalid 'literal_int_precision'. Got '{literal_int_precision}', expected 32 or 64.")
    if literal_float_precision not in (32, 64):
        raise ValueError(
            f"Invalid 'literal_float_precision'. Got '{literal_float_precision}', expected 32 or 64."
        )

    module = None
    if name:
        parts = name.split(".")
        name = parts[-1]
        module = ".".join(parts[:-1])
    name = name or ""
    module = module or inspect.currentframe().f_back.f_globals.get("__name__", "__main__")

    impl_opts = {k: v for k, v in kwargs.items() if k.startswith("_")}
    for k in impl_opts:
        kwargs.pop(k)

    if build_info is not None:
        build_info.update({k: 0.0 for k in ("parse_time", "module_time", "codegen_time", "build_time", "load_time")})

    build_options = gt_definitions.BuildOptions(
        name=name,
        module=module,
        format_source=format_source,
        rebuild=rebuild,
        raise_if_not_cached=raise_if_not_cached,
        backend_opts=kwargs,
        build_info=build_info,
        cache_settings=cache_settings or {},
        literal_int_precision=literal_int_precision,
        literal_float_precision=literal_float_precision,
        impl_opts=impl_opts,
    )

    def _decorator(definition_func):
        if not isinstance(definition_func, types.FunctionType):
            if hasattr(definition_func, "definition_func"):
                definition_func = definition_func.definition_func
            elif callable(definition_func):
                definition_func = definition_func.__call__
        original = _set_arg_dtypes(definition_func, dtypes or {})
        try:
            return loader.load_stencil(
                definition_func,
                backend=backend,
                build_options=build_options,
                externals=externals or {},
                dtypes=dtypes or {},
            )
        finally:
            definition_func.__annotations__ = original

    if definition is None:
        return _decorator
    return _decorator(definition)


def lazy_stencil(backend=None, definition=None, **kwargs):
    """Deferred build: returns a callable that builds on first use (``lazy_stencil.py``)."""

    def _decorator(func):
        holder = {}

        def _call(*args, **call_kwargs):
            if "stencil" not in holder:
                holder["stencil"] = stencil(backend, func, **kwargs)
            return holder["stencil"](*args, **call_kwargs)

        _call.definition_func = func
        return _call

    return _decorator if definition is None else _decorator(definition)


def mark_stencil(func):
    func._gtscript_stencil_ = True
    return func
