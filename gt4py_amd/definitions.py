"""Public info types of the stencil call contract.

Mirror ``src/gt4py/cartesian/definitions.py:45-141`` (``AccessKind``, ``DomainInfo``,
``FieldInfo``, ``ParameterInfo``, ``BuildOptions``) and the ``Boundary``/``Shape``/``Index``
helpers of ``gtc/definitions.py:457-560`` that ``StencilObject`` validation uses.
"""

from __future__ import annotations

import dataclasses
import enum
import functools
import hashlib
import os
import platform
from typing import Any, Dict, Optional, Tuple

import numpy as np

_ARCH_PRECISION = int(platform.architecture()[0][:2])
LITERAL_INT_PRECISION = int(os.environ.get("GT4PY_LITERAL_INT_PRECISION", default=_ARCH_PRECISION))
LITERAL_FLOAT_PRECISION = int(os.environ.get("GT4PY_LITERAL_FLOAT_PRECISION", default=_ARCH_PRECISION))

CARTESIAN_AXES = ("I", "J", "K")


class AccessKind(enum.IntFlag):
    NONE = 0
    READ = 1
    WRITE = 2
    READ_WRITE = READ | WRITE

    def __str__(self):
        return self.name


class Boundary(tuple):
    """Per-axis (lower, upper) halo: ``Boundary(((2, 2), (2, 2), (0, 0)))``."""

    def __new__(cls, pairs):
        return super().__new__(cls, tuple((int(a), int(b)) for a, b in pairs))

    @property
    def lower_indices(self) -> Tuple[int, ...]:
        return tuple(a for a, _ in self)

    @property
    def upper_indices(self) -> Tuple[int, ...]:
        return tuple(b for _, b in self)

    @property
    def ndim(self):
        return len(self)

    def __repr__(self):
        return f"Boundary({tuple(self)!r})"


@dataclasses.dataclass(frozen=True)
class DomainInfo:
    parallel_axes: Tuple[str, ...]
    sequential_axis: str
    min_sequential_axis_size: int
    ndim: int


@dataclasses.dataclass(frozen=True)
class FieldInfo:
    access: AccessKind
    boundary: Boundary
    axes: Tuple[str, ...]
    data_dims: Tuple[int, ...]
    dtype: np.dtype

    def __repr__(self):
        return (
            f"FieldInfo(access=AccessKind.{self.access.name}, boundary={self.boundary!r}, "
            f"axes={self.axes!r}, data_dims={self.data_dims!r}, dtype={self.dtype!r})"
        )

    @functools.cached_property
    def domain_mask(self) -> Tuple[bool, ...]:
        return tuple(axis in self.axes for axis in CARTESIAN_AXES)

    @functools.cached_property
    def domain_ndim(self) -> int:
        return len(self.axes)

    @functools.cached_property
    def mask(self):
        return (*self.domain_mask, *((True,) * len(self.data_dims)))

    @functools.cached_property
    def ndim(self) -> int:
        return len(self.axes) + len(self.data_dims)


@dataclasses.dataclass(frozen=True)
class ParameterInfo:
    access: AccessKind
    dtype: np.dtype

    def __repr__(self):
        return f"ParameterInfo(access=AccessKind.{self.access.name}, dtype={self.dtype!r})"


@dataclasses.dataclass
class BuildOptions:
    name: str
    module: str
    format_source: bool = True
    backend_opts: Dict[str, Any] = dataclasses.field(default_factory=dict)
    build_info: Optional[dict] = None
    rebuild: bool = False
    raise_if_not_cached: bool = False
    cache_settings: Dict[str, Any] = dataclasses.field(default_factory=dict)
    impl_opts: Dict[str, Any] = dataclasses.field(default_factory=dict)
    literal_int_precision: int = LITERAL_INT_PRECISION
    literal_float_precision: int = LITERAL_FLOAT_PRECISION

    @property
    def qualified_name(self) -> str:
        return ".".join(x for x in (self.module, self.name) if x)

    @property
    def shashed_id(self) -> str:
        items = (
            self.name,
            self.module,
            self.format_source,
            self.literal_int_precision,
            self.literal_float_precision,
            *sorted((k, repr(v)) for k, v in self.backend_opts.items()),
        )
        return hashlib.sha256(repr(items).encode()).hexdigest()[:12]


# --------------------------------------------------------------------------------------
# Small helpers with the semantics of gtc/definitions.py Index/Shape comparisons
# --------------------------------------------------------------------------------------


def all_le(a, b) -> bool:
    return all(x <= y for x, y in zip(a, b))


def all_lt(a, b) -> bool:
    return all(x < y for x, y in zip(a, b))


def filter_mask(seq, mask):
    return tuple(x for x, m in zip(seq, mask) if m)


def interpolate_mask(seq, mask, default):
    it = iter(seq)
    return tuple(next(it) if m else default for m in mask)


# Error hierarchy of the reference (``src/gt4py/cartesian/definitions.py:152-165``): frontend
# errors derive from these, so ``except GTError`` / ``except GTSyntaxError`` catch the same
# errors as with the reference.
class GTError(Exception):
    pass


class GTSyntaxError(GTError):
    pass


class GTSpecificationError(GTError):
    pass
