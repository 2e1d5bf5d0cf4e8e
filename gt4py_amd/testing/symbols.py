"""Symbol descriptors of a ``StencilTestSuite`` and the Hypothesis strategies behind them.

User-facing contract of ``gt4py.cartesian.testing.input_strategies`` (``field`` ``:83-98``,
``parameter`` ``:101-126``, ``global_name`` ``:44-80``, ``none`` ``:129-137``; scalar value
generation ``:140-156``): a suite's ``symbols`` mapping names every argument of the stencil
definition (and every external) with one of these descriptors. Here a descriptor is one frozen
``Symbol`` record that knows how to produce its own value strategy for a given dtype.
"""

from __future__ import annotations

import dataclasses
import enum
import math
import numbers
from typing import Any, Optional, Sequence, Tuple

import numpy as np


class SymbolKind(enum.Enum):
    NONE = 0
    GLOBAL_STRATEGY = 1  # external drawn from a range at build time
    GLOBAL_SET = 2  # external taking each of a set of values (one test per value)
    SINGLETON = 3  # external with one fixed value
    PARAMETER = 4  # scalar run-time argument
    FIELD = 5  # array argument


@dataclasses.dataclass(frozen=True)
class Symbol:
    kind: SymbolKind
    boundary: Optional[Tuple[Tuple[int, int], ...]] = None
    axes: Optional[str] = None
    data_dims: Tuple[int, ...] = ()
    values: Tuple[Any, ...] = ()
    value_range: Optional[Tuple[Any, Any]] = None

    def value_strategy(self, dtype):
        """Hypothesis strategy of one value of this symbol (an array element for fields)."""
        import hypothesis.strategies as st

        dtype = np.dtype(dtype)
        if self.kind == SymbolKind.NONE:
            return st.none()
        if self.value_range is not None:
            return scalar_strategy(dtype, *self.value_range)
        if not self.values:
            return st.just(None)
        return st.sampled_from(list(self.values)).map(dtype.type)


def scalar_strategy(dtype, lo, hi, allow_nan: bool = False):
    """Values of ``dtype`` in ``[lo, hi]``; infinities only when a bound is infinite."""
    import hypothesis.strategies as st

    dtype = np.dtype(dtype)
    if dtype.kind == "b":
        base = st.booleans()
    elif issubclass(dtype.type, numbers.Integral):
        base = st.integers(int(lo), int(hi))
    else:
        finite = math.isfinite(lo) and math.isfinite(hi)
        base = st.floats(lo, hi, allow_nan=allow_nan, allow_infinity=not finite, width=dtype.itemsize * 8)
    return base.map(dtype.type)


def global_name(*, singleton=None, symbol=None, one_of=None, in_range=None) -> Symbol:
    """An external: a fixed value, a set of values (one test each), or a drawn value."""
    given = [x is not None for x in (singleton, symbol, one_of, in_range)]
    if sum(given) != 1:
        raise AssertionError("global_name() takes exactly one of singleton / symbol / one_of / in_range")
    if singleton is not None:
        return Symbol(SymbolKind.SINGLETON, values=(singleton,))
    if symbol is not None:
        return Symbol(SymbolKind.GLOBAL_SET, values=(symbol,))
    if one_of is not None:
        assert isinstance(one_of, Sequence), "one_of must be a sequence"
        return Symbol(SymbolKind.GLOBAL_SET, values=tuple(one_of))
    assert len(in_range) == 2
    return Symbol(SymbolKind.GLOBAL_STRATEGY, value_range=tuple(in_range))


def field(*, in_range, boundary=None, axes=None, data_dims=None, extent=None) -> Symbol:
    """An array argument with values in ``in_range`` and a halo of ``boundary`` (or ``extent``)."""
    if boundary is None and extent is None:
        raise AssertionError("field() needs a boundary or an extent")
    assert len(in_range) == 2
    if boundary is None:
        boundary = [(abs(lo), abs(hi)) for lo, hi in extent]
    boundary = tuple((int(lo), int(hi)) for lo, hi in boundary)
    if extent is not None:
        assert all((-b[0], b[1]) == tuple(e) for b, e in zip(boundary, extent)), "boundary and extent disagree"
    assert all(lo >= 0 and hi >= 0 for lo, hi in boundary), "negative boundary"
    return Symbol(
        SymbolKind.FIELD, boundary=boundary, axes=axes, data_dims=tuple(data_dims or ()), value_range=tuple(in_range)
    )


def parameter(*, one_of=None, in_range=None) -> Symbol:
    """A scalar run-time argument drawn from ``one_of`` or ``in_range``."""
    if (one_of is None) == (in_range is None):
        raise AssertionError("parameter() takes exactly one of one_of / in_range")
    if one_of is not None:
        assert isinstance(one_of, Sequence), "one_of must be a sequence"
        return Symbol(SymbolKind.PARAMETER, values=tuple(one_of))
    assert len(in_range) == 2
    return Symbol(SymbolKind.PARAMETER, value_range=tuple(in_range))


def none() -> Symbol:
    """An argument passed as ``None``."""
    return Symbol(SymbolKind.NONE)
