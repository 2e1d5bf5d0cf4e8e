"""Stencil test suites (``gt4py.cartesian.testing`` API: ``testing/__init__.py``): Hypothesis-driven
parity checks of GTScript stencils against numpy validation functions, for any backend."""

from gt4py_amd.testing.suites import ATOL, EQUAL_NAN, RTOL, StencilTestSuite  # noqa: F401
from gt4py_amd.testing.symbols import Symbol, SymbolKind, field, global_name, none, parameter  # noqa: F401

__all__ = ["StencilTestSuite", "field", "global_name", "none", "parameter"]
