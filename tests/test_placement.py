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
    assert placement.scope_fields(td, "written") == ["sup", "rhs", "out"]
    assert placement.scope_fields(td, "all") == list(td.field_info)
    with pytest.raises(ValueError, match="scope"):
        placement.scope_fields(td, "read")


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


def test_exclusive_storage_check():
    """The in-place form refuses a written field that other tensors view: they would keep the
    old pages. A gt4py_amd storage is a strided view of its own flat buffer, which is allowed."""
    import torch

    from gt4py_amd import storage

    t = torch.zeros(6, 5, 4, dtype=torch.float64)
    assert placement._exclusive(t)
    v = t[1:, :, :]
    assert not placement._exclusive(t) and not placement._exclusive(v)
    del v
    assert placement._exclusive(t)
    s = torch.from_numpy(storage.zeros((6, 5, 4), np.float64, backend="numpy"))
    assert placement._exclusive(s)
    buf = torch.zeros(200, dtype=torch.float64)
    w = torch.as_strided(buf, (3, 4), (1, 3), 5)
    assert not placement._exclusive(w)  # its flat buffer is still referenced by `buf`
    del buf
    assert placement._exclusive(w)


def _dev_case(name, st):
    from gt4py_amd import storage

    case = sc.CASES[name]
    host = case.make_inputs()
    dev = {k: storage.from_array(v, None, backend="gt:mi355x",
                                 aligned_index=tuple(case.origin.get(k, (0, 0, 0))) if isinstance(case.origin, dict)
                                 else (0, 0, 0))
           for k, v in host.items() if v is not None}
    kw = {}
    if case.origin is not None:
        kw["origin"] = case.origin
    if case.domain is not None:
        kw["domain"] = case.domain
    return case, host, dev, kw


@pytest.mark.gpu
@pytest.mark.parametrize("name,frozen,scope", [("hdiff_f64", False, "written"), ("hdiff_f64", True, "written"),
                                               ("tridiag", False, "written"), ("tridiag", True, "written"),
                                               ("tridiag", False, "all"), ("vertical_advection_dycore", True, "all")])
def test_tune_placement_in_place_drop_in(name, frozen, scope):
    """``StencilObject.tune_placement`` / ``FrozenStencil.tune_placement`` with the arguments of
    an ordinary call: the caller's tensors stay the same objects with the same contents, the
    written ones on the chosen buffers; a prepared launch made before tuning is dropped, and the
    next call is bit-exact against the reference golden."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    case = sc.CASES[name]
    st = gtscript.stencil(backend="gt:mi355x", definition=case.definition, externals=case.externals,
                          name=f"gpu.{case.name}")
    case, host, dev, kw = _dev_case(name, st)
    # a prepared launch on the first allocation (its result is discarded)
    scratch = {k: v.clone() for k, v in dev.items()}
    st(**scratch, **case.params, **kw)
    st(**scratch, **case.params, **kw)
    del scratch
    ids = {k: id(v) for k, v in dev.items()}
    ptrs = {k: v.data_ptr() for k, v in dev.items()}
    if frozen:
        org = kw.get("origin")
        org = {k: tuple(org.get(k, (0, 0, 0))) for k in st.field_info} if isinstance(org, dict) else \
            {k: tuple(org or (0, 0, 0)) for k in st.field_info}
        fz = st.freeze(origin=org, domain=kw["domain"] if "domain" in kw else tuple(dev[next(iter(dev))].shape))
        fz(**dev, **case.params)
        for k, v in host.items():
            dev[k].copy_(torch.from_numpy(np.ascontiguousarray(v)).to(dev[k].device))
        rep = fz.tune_placement(**dev, **case.params, candidates=2, reps=2, scope=scope)
    else:
        rep = st.tune_placement(**dev, **case.params, **kw, candidates=2, reps=2, scope=scope)
    assert rep["in_place"] and len(rep["candidates_ms"]) == 3 and rep["written"] == placement.written_fields(st)
    assert rep["scope"] == scope and rep["fields"] == placement.scope_fields(st, scope)
    for k, v in dev.items():
        assert id(v) == ids[k]
        gu.assert_match(storage.to_numpy(v), host[k], name=f"{name}:{k} contents kept")
        if k not in rep["fields"]:
            assert v.data_ptr() == ptrs[k]
    if rep["chosen"] != 0:
        assert all(dev[k].data_ptr() != ptrs[k] for k in rep["fields"])
    if frozen:
        fz(**dev, **case.params)
    else:
        st(**dev, **case.params, **kw)
    _, outputs, _ = gu.load(name)
    for k, v in outputs.items():
        gu.assert_match(storage.to_numpy(dev[k]), v, rtol=case.rtol, atol=case.atol, name=f"{name}:{k}")


@pytest.mark.gpu
def test_tune_placement_in_place_refusals():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import weakref

    from gt4py_amd import storage

    case = sc.CASES["copy"]
    st = gtscript.stencil(backend="gt:mi355x", definition=case.definition, externals=case.externals,
                          name=f"gpu.{case.name}")
    names = list(st.field_info)
    a = storage.from_array(np.arange(8 * 8 * 4, dtype=np.float64).reshape(8, 8, 4), backend="gt:mi355x")
    b = storage.zeros((8, 8, 4), np.float64, backend="gt:mi355x")
    view = b[:, :, 1:]
    with pytest.raises(ValueError, match="shares its storage"):
        st.tune_placement(**{names[0]: a, names[1]: b}, origin=(0, 0, 0), domain=(8, 8, 4), candidates=2, reps=1)
    del view
    ref = weakref.ref(b)
    ptr = b.data_ptr()
    from gt4py_amd.storage import placement

    def no_timing(*a_, **k_):
        raise AssertionError("refused only after timing (ADVICE r04)")

    saved = placement.tune_written_fields, placement.tune_fields
    placement.tune_written_fields = placement.tune_fields = no_timing
    try:
        with pytest.raises(RuntimeError, match="weakly referenced"):  # before anything is timed
            st.tune_placement(**{names[0]: a, names[1]: b}, origin=(0, 0, 0), domain=(8, 8, 4), candidates=2, reps=1)
    finally:
        placement.tune_written_fields, placement.tune_fields = saved
    assert ref() is b and b.data_ptr() == ptr
