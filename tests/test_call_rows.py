"""``StencilObject.call_rows``: one call over the rows [0, j_split) and [j_split + j_skip, nj)
(the two boundary strips of a J-strip rank after its halo exchange, distributed/halo.py).

Its definition is two ordinary calls -- domain (ni, j_split, nk) at the origin, and the remaining
rows at the origin advanced by j_split + j_skip along J -- so every test compares it with exactly
those two calls on the same backend, bit for bit over every array (the skipped rows must stay
untouched). On gt:mi355x plane-kernel stencils without scratch or regions take the one-launch
path (``gtmi_stencil_run_jsplit`` mapping the J chunks around the gap), the others the library's
two-pass fallback; both are covered here.
"""

import os

import numpy as np
import pytest

import stencil_cases as sc

# (golden case, expected gt:mi355x path)
CASES = [
    ("hdiff_f64", "native"),
    ("lap5", "native"),
    ("copy", "native"),
    ("hdiff_f32", "native"),
    ("horizontal_regions", "two-pass"),
    ("tridiag", "two-pass"),
    ("staged_forward_ij_temp", "two-pass"),
    ("multi_stage_temps", None),
]


def _org(case, name, axes):
    o = case.origin
    if isinstance(o, dict):
        return tuple(o.get(name, o.get("_all_", (0,) * len(axes))))[: len(axes)]
    if o is None:
        return (0,) * len(axes)
    return tuple(o["IJK".index(a)] for a in axes)


def _setup(case, stencil):
    host = case.make_inputs()
    origin = {k: _org(case, k, tuple(stencil.field_info[k].axes)) for k in host if stencil.field_info.get(k)}
    if case.domain is not None:
        domain = tuple(case.domain)
    else:  # the largest domain every field covers from its origin
        ext = []
        for ax in range(3):
            ext.append(min(host[k].shape[ax] - origin[k][ax] for k in origin if len(host[k].shape) > ax))
        domain = tuple(ext)
    return host, origin, domain


def _shift_j(stencil, origin, dj):
    out = {}
    for k, o in origin.items():
        axes = tuple(stencil.field_info[k].axes)
        out[k] = tuple(v + (dj if a == "J" else 0) for a, v in zip(axes, o))
    return out


def _splits(nj):
    js = max(1, min(2, nj // 3))
    return [(js, nj - 2 * js), (0, nj - 2), (nj - 1, 1), (1, 0)]


def _check(backend, name, to_dev, to_host):
    from gt4py_amd import gtscript

    case = sc.CASES[name]
    st = gtscript.stencil(backend=backend, definition=case.definition, externals=case.externals,
                          name=f"{'gpu.' if backend != 'numpy' else ''}{name}")
    host, origin, (ni, nj, nk) = _setup(case, st)
    for js, jk in _splits(nj):
        a = {k: to_dev(v, origin.get(k)) for k, v in host.items()}
        b = {k: to_dev(v, origin.get(k)) for k, v in host.items()}
        if js > 0:
            st(**a, **case.params, origin=origin, domain=(ni, js, nk))
        if nj - js - jk > 0:
            st(**a, **case.params, origin=_shift_j(st, origin, js + jk), domain=(ni, nj - js - jk, nk))
        st.call_rows(js, jk, domain=(ni, nj, nk), origin=origin, **b, **case.params)
        for k in host:
            if host[k] is None:
                continue
            x, y = to_host(a[k]), to_host(b[k])
            same = (x == y) | (np.isnan(x) & np.isnan(y)) if x.dtype.kind == "f" else (x == y)
            assert same.all(), f"{name} split ({js}, {jk}): field {k} differs at {np.argwhere(~same)[:3].tolist()}"
    return st


@pytest.mark.parametrize("name", [c for c, _ in CASES])
def test_call_rows_numpy_backend(name):
    _check("numpy", name, lambda v, o: None if v is None else v.copy(), np.asarray)


def test_call_rows_rejects_bad_split():
    from gt4py_amd import gtscript

    case = sc.CASES["copy"]
    st = gtscript.stencil(backend="numpy", definition=case.definition, name="copy")
    host, origin, (ni, nj, nk) = _setup(case, st)
    with pytest.raises(ValueError):
        st.call_rows(nj, 1, domain=(ni, nj, nk), origin=origin, **host)
    with pytest.raises(TypeError):
        st.call_rows(1, 1, domain=(ni, nj, nk), origin=origin, not_a_field=host["field_a"], **host)


@pytest.mark.parametrize("name,path", [c for c in CASES if c[1] is not None])
def test_jsplit_path_in_generated_library(name, path):
    """Which path ``gtmi_stencil_run_jsplit`` takes is decided at code generation (CPU only)."""
    from gt4py_amd import gtscript

    case = sc.CASES[name]
    st = gtscript.stencil(backend="gt:mi355x", definition=case.definition, externals=case.externals,
                          name=f"gpu.{name}")
    lib = type(st)._gt_run_impl_.compiled.lib_path
    src = open(os.path.join(os.path.dirname(lib), "stencil.hip")).read()
    native = "return gtmi_run_rows(domain, (int)j_split, (int)j_skip, f, sc, stream);" in src
    assert native == (path == "native"), (name, path)
    assert "gtmi_stencil_run_jsplit" in src


@pytest.mark.gpu
@pytest.mark.parametrize("name", [c for c, _ in CASES])
def test_call_rows_gpu(name):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    def to_dev(v, o):
        if v is None:
            return None
        return storage.from_array(v, v.dtype, backend="gt:mi355x", aligned_index=o if o is not None else (0,) * v.ndim)

    _check("gt:mi355x", name, to_dev, lambda t: storage.to_numpy(t))
    torch.cuda.synchronize()
