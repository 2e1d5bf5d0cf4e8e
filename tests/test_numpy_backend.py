"""Frontend + passes + numpy backend vs the reference golden vectors (CPU)."""

import numpy as np
import pytest

import golden_utils as gu
import stencil_cases as sc
from gt4py_amd import gtscript

CASE_NAMES = gu.available()


def build(case, backend):
    return gtscript.stencil(
        backend=backend,
        definition=case.definition,
        externals=case.externals,
        name=f"tests.{case.name}",
    )


def call_kwargs(case):
    kw = {}
    if case.origin is not None:
        kw["origin"] = case.origin
    if case.domain is not None:
        kw["domain"] = case.domain
    return kw


@pytest.mark.parametrize("name", CASE_NAMES)
def test_numpy_backend_matches_golden(name):
    case = sc.CASES[name]
    inputs, outputs, meta = gu.load(name)
    stencil = build(case, "numpy")
    arrays = {k: (None if v is None else v.copy()) for k, v in case.make_inputs().items()}
    stencil(**arrays, **case.params, **call_kwargs(case))
    for k, v in outputs.items():
        gu.assert_match(arrays[k], v, rtol=case.rtol, atol=case.atol, name=f"{name}:{k}")


@pytest.mark.parametrize("name", CASE_NAMES)
def test_field_info_matches_reference(name):
    case = sc.CASES[name]
    _, _, meta = gu.load(name)
    stencil = build(case, "numpy")
    for fname, ref in meta["field_info"].items():
        fi = stencil.field_info[fname]
        assert int(fi.access) == ref["access"], (fname, fi.access, ref["access"])
        assert [list(b) for b in fi.boundary] == ref["boundary"], (fname, fi.boundary, ref["boundary"])
        assert list(fi.axes) == ref["axes"]
        assert str(fi.dtype) == ref["dtype"]
    for pname, ref in meta["parameter_info"].items():
        pi = stencil.parameter_info[pname]
        assert int(pi.access) == ref["access"] and str(pi.dtype) == ref["dtype"], pname
    assert stencil.domain_info.min_sequential_axis_size == meta["domain_info"]["min_sequential_axis_size"]
