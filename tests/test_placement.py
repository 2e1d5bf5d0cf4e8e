"""``gt4py_amd.storage.placement``: re-homing the written fields of a stencil call to the
fastest of several buffer sets (DESIGN.md §5 "HBM placement"). The tuner may only change WHERE
the fields live: results must stay bit-exact against the reference-generated golden outputs,
every field keeps its contents, layouts (strides, 2-MiB address residue) are preserved, and
aliasing arguments are refused."""

import numpy as np
import pytest

import golden_utils as gu
import stencil_cases as sc
from gt4py_amd import gtscript
from gt4py_amd.storage import placement


def test_written_fields_from_field_info():
    hd = gtscript.stencil(backend="numpy", definition=sc.CASES["hdiff_f64"].definition, name="placement.hdiff")
    assert placement.written_fields(hd) == ["out_field"]
    case = sc.CASES["tridiag"]
    td = gtscript.stencil(backend="numpy", definition=case.definition, externals=case.externals,
                          name="placement.tridiag")
    assert placement.written_fields(td) == ["sup", "rhs", "out"]


def test_like_keeps_layout_and_residue():
    import torch

    base = torch.empty(3 * (1 << 20) + 4096, dtype=torch.float64)
    t = torch.as_strided(base, size=(33, 17, 9), stride=(1, 40, 40 * 17), storage_offset=77)
    u = placement.like(t)
    assert tuple(u.shape) == tuple(t.shape) and u.stride() == t.stride() and u.dtype == t.dtype
    assert (u.data_ptr() - t.data_ptr()) % (2 << 20) == 0
    assert u.untyped_storage().nbytes() >= placement.like_bytes(t) - (2 << 20)


def test_rejects_host_arrays():
    import torch

    hd = gtscript.stencil(backend="numpy", definition=sc.CASES["hdiff_f64"].definition, name="placement.hdiff")
    arrays = {"in_field": torch.zeros(8, 8, 2, dtype=torch.float64), "out_field": torch.zeros(4, 4, 2, dtype=torch.float64),
              "coeff": torch.zeros(4, 4, 2, dtype=torch.float64)}
    with pytest.raises(TypeError, match="not a device tensor"):
        placement.tune_written_fields(hd, arrays, domain=(4, 4, 2))


GPU_CASES = ["hdiff_f64", "hdiff_f32", "tridiag", "vertical_advection_dycore", "mixed_precision",
             "staged_forward_ij_temp"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", GPU_CASES)
def test_tuned_placement_bit_exact(name):
    import test_gpu_parity as tg

    tg._torch()
    case = sc.CASES[name]
    _, outputs, _ = gu.load(name)
    res = tg.run_case_on_gpu(case, tune=2)
    for k, v in outputs.items():
        gu.assert_match(res[k], v, rtol=case.rtol, atol=case.atol, name=f"{name}:{k}")


@pytest.mark.gpu
def test_aliased_written_field_refused():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    case = sc.CASES["copy"]
    st = gtscript.stencil(backend="gt:mi355x", definition=case.definition, externals=case.externals,
                          name=f"gpu.{case.name}")
    a = storage.zeros((8, 8, 4), np.float64, backend="gt:mi355x")
    names = list(st.field_info)
    with pytest.raises(ValueError, match="shares memory"):
        placement.tune_written_fields(st, {names[0]: a, names[1]: a[:, :, :]}, domain=(8, 8, 4))


@pytest.mark.gpu
def test_invalid_domain_is_rejected_before_any_timed_launch():
    """The tuner validates the call once (the timed launches skip validation): a domain larger
    than the fields raises the ordinary ValueError and leaves the fields untouched."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    case = sc.CASES["copy"]
    st = gtscript.stencil(backend="gt:mi355x", definition=case.definition, externals=case.externals,
                          name=f"gpu.{case.name}")
    a = storage.from_array(np.arange(8 * 8 * 4, dtype=np.float64).reshape(8, 8, 4), backend="gt:mi355x")
    b = storage.zeros((8, 8, 4), np.float64, backend="gt:mi355x")
    names = list(st.field_info)
    with pytest.raises(ValueError):
        placement.tune_written_fields(st, {names[0]: a, names[1]: b}, origin=(0, 0, 0), domain=(9, 8, 4))
    assert float(b.abs().sum()) == 0.0
