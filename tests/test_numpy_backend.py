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


def test_c1_copy_config_numpy_backend():
    """BASELINE.json configs[0]: copy_stencil 128x128x64 f64 through the CPU (numpy) path, bit-exact."""
    import time

    from gt4py_amd import gtscript, storage

    st = gtscript.stencil(backend="numpy", definition=sc.copy_stencil, name="c1.copy")
    a = storage.from_array(np.random.default_rng(0).random((128, 128, 64)), backend="numpy")
    b = storage.zeros((128, 128, 64), np.float64, backend="numpy")
    st(a, b, origin=(0, 0, 0), domain=(128, 128, 64))
    t0 = time.perf_counter()
    st(a, b, origin=(0, 0, 0), domain=(128, 128, 64), validate_args=False)
    dt = time.perf_counter() - t0
    assert np.array_equal(np.asarray(b), np.asarray(a))
    assert dt < 5.0
