"""The cached-call fast path of ``StencilObject.__call__`` / ``FrozenStencil.__call__``
(gt4py_amd/stencil_object.py, ``StencilLauncher.bind``): a repeated call with the same arrays,
domain and origin skips argument extraction and packing. These tests pin that it never changes
results: scalar parameters are re-read on every call, swapped / re-allocated / re-pointed
(``set_``) / re-shaped arrays and changed domains or origins take the ordinary path, and
``exec_info`` calls keep their timestamps. Every case is checked against numpy, once with the
native prepared launch (``csrc/gtmi_fastcall.cpp``) and once with the launcher's ctypes closure.
"""

import numpy as np
import pytest

from gt4py_amd import gtscript
from gt4py_amd import storage as gt_storage
from gt4py_amd.gtscript import PARALLEL, Field, computation, interval

BK = "gt:mi355x"


@pytest.fixture(params=["native", "ctypes"])
def mode(request, monkeypatch):
    from gt4py_amd.runtime import fastcall

    if request.param == "ctypes":
        monkeypatch.setattr(fastcall, "_module", None)
        monkeypatch.setattr(fastcall, "_tried", True)
    elif fastcall.module() is None:
        pytest.skip("gt4py_amd._gtmi_fastcall not built")
    return request.param




def _need_gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")


def shift_axpy(a: Field[np.float64], b: Field[np.float64], *, w: np.float64):
    with computation(PARALLEL), interval(...):
        b = a[1, 0, 0] * w + a[0, 0, 0]


def _expect(a, w, domain, org_a=(0, 0, 0), org_b=(0, 0, 0), b_init=None):
    a = gt_storage.to_numpy(a)
    ni, nj, nk = domain
    out = np.array(b_init, copy=True)
    ia, ja, ka = org_a
    ib, jb, kb = org_b
    out[ib:ib + ni, jb:jb + nj, kb:kb + nk] = (a[ia + 1:ia + 1 + ni, ja:ja + nj, ka:ka + nk] * w
                                              + a[ia:ia + ni, ja:ja + nj, ka:ka + nk])
    return out


def _fields(seed, shape=(17, 9, 5)):
    rng = np.random.default_rng(seed)
    a = gt_storage.from_array(rng.uniform(-1, 1, (shape[0] + 1,) + shape[1:]), backend=BK, aligned_index=(0, 0, 0))
    b = gt_storage.zeros(shape, np.float64, backend=BK)
    return a, b


def _memo(st):
    return type(st)._gt_fast_memo_


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_repeated_calls_hit_and_reread_scalars():
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    a, b = _fields(1)
    dom = (17, 9, 5)
    for w in (0.5, 2.0, -3.25, 0.5):
        st(a, b, w=w, domain=dom, origin=(0, 0, 0))
        np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a, w, dom, b_init=np.zeros(dom)))
    assert len(_memo(st)) == 1


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_swapped_and_new_arrays():
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    dom = (16, 9, 5)
    rng = np.random.default_rng(7)
    x = gt_storage.from_array(rng.uniform(-1, 1, (17, 9, 5)), backend=BK, aligned_index=(0, 0, 0))
    y = gt_storage.from_array(rng.uniform(-1, 1, (17, 9, 5)), backend=BK, aligned_index=(0, 0, 0))
    for it in range(4):  # ping-pong: (x -> y), (y -> x), ... two memo entries
        src, dst = (x, y) if it % 2 == 0 else (y, x)
        want = _expect(src, 1.5, dom, b_init=gt_storage.to_numpy(dst))
        st(src, dst, w=1.5, domain=dom, origin=(0, 0, 0))
        np.testing.assert_array_equal(gt_storage.to_numpy(dst), want)
    assert len(_memo(st)) == 2
    for seed in range(3):  # fresh tensors every call (ids may be reused after a free)
        a, b = _fields(100 + seed)
        st(a, b, w=0.75, domain=(17, 9, 5), origin=(0, 0, 0))
        np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a, 0.75, (17, 9, 5), b_init=np.zeros((17, 9, 5))))
        del a, b


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_set_and_resize_take_the_ordinary_path():
    _need_gpu()
    import torch

    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    a, b = _fields(3)
    dom = (17, 9, 5)
    st(a, b, w=1.0, domain=dom, origin=(0, 0, 0))
    a2, _ = _fields(4)
    a.set_(a2.untyped_storage(), a2.storage_offset(), a2.shape, a2.stride())  # same object, new data
    st(a, b, w=1.0, domain=dom, origin=(0, 0, 0))
    np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a2, 1.0, dom, b_init=np.zeros(dom)))
    # same object re-shaped in place (smaller): the cached validation must not be reused
    b.resize_((4, 4, 4))
    with pytest.raises(ValueError):
        st(a, b, w=1.0, domain=dom, origin=(0, 0, 0))
    torch.cuda.synchronize()


def _square(seed, n=12, nk=4):
    rng = np.random.default_rng(seed)
    a = gt_storage.from_array(rng.uniform(-1, 1, (n, n, nk)), backend=BK, aligned_index=(0, 0, 0))
    b = gt_storage.from_array(rng.uniform(-1, 1, (n, n, nk)), backend=BK, aligned_index=(0, 0, 0))
    return a, b


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
@pytest.mark.parametrize("which", ["a", "b", "both"])
def test_restride_in_place_takes_the_ordinary_path(which):
    """``transpose_`` on a square-IJ field keeps the tensor's identity, data pointer and sizes but
    swaps its strides: a prepared launch with the strides packed at bind time would read (or
    write) the wrong cells, so the entry must miss and the ordinary path re-pack the field."""
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    a, b = _square(21)
    n, nk = a.shape[0], a.shape[2]
    dom = (n - 1, n, nk)
    st(a, b, w=1.25, domain=dom, origin=(0, 0, 0))
    st(a, b, w=1.25, domain=dom, origin=(0, 0, 0))  # prepared
    ptrs = (a.data_ptr(), b.data_ptr())
    for t in ((a,) if which == "a" else (b,) if which == "b" else (a, b)):
        t.transpose_(0, 1)
    assert (a.data_ptr(), b.data_ptr()) == ptrs and a.shape == b.shape == (n, n, nk)
    want = _expect(a, 1.25, dom, b_init=gt_storage.to_numpy(b))
    st(a, b, w=1.25, domain=dom, origin=(0, 0, 0))
    np.testing.assert_array_equal(gt_storage.to_numpy(b), want)
    want = _expect(a, -0.5, dom, b_init=gt_storage.to_numpy(b))
    st(a, b, w=-0.5, domain=dom, origin=(0, 0, 0))  # the re-made entry hits
    np.testing.assert_array_equal(gt_storage.to_numpy(b), want)


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_as_strided_in_place_takes_the_ordinary_path():
    """``as_strided_`` to a new I stride (every other row of a larger buffer) with the same
    sizes and storage offset, on the call and the frozen path."""
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    rng = np.random.default_rng(22)
    n, nj, nk = 9, 7, 3
    a = gt_storage.from_array(rng.uniform(-1, 1, (2 * n + 2, nj, nk)), backend=BK, aligned_index=(0, 0, 0))
    b = gt_storage.zeros((n, nj, nk), np.float64, backend=BK)
    dom = (n, nj, nk)
    a_big = gt_storage.to_numpy(a).copy()
    a.as_strided_((n + 1, nj, nk), a.stride(), a.storage_offset())
    fz = st.freeze(origin={"a": (0, 0, 0), "b": (0, 0, 0)}, domain=dom)
    for call in (lambda w: st(a, b, w=w, domain=dom, origin=(0, 0, 0)), lambda w: fz(a=a, b=b, w=w)):
        call(2.0)
        call(2.0)  # prepared
        np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a_big[:n + 1], 2.0, dom, b_init=np.zeros(dom)))
        s0, s1, s2 = a.stride()
        a.as_strided_((n + 1, nj, nk), (2 * s0, s1, s2), a.storage_offset())
        call(2.0)
        np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a_big[0::2], 2.0, dom, b_init=np.zeros(dom)))
        a.as_strided_((n + 1, nj, nk), (s0, s1, s2), a.storage_offset())
        b.zero_()


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_alternating_domains_keep_their_entries():
    """Two (domain, origin) signatures on the same arrays both stay prepared (advisor r03: a
    single entry per argument tuple re-bound on every alternation)."""
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    a, b = _fields(23)
    sigs = [((17, 4, 5), {"a": (0, 0, 0), "b": (0, 0, 0)}), ((17, 5, 5), {"a": (0, 4, 0), "b": (0, 4, 0)})]
    for it in range(6):
        dom, org = sigs[it % 2]
        b.zero_()
        st(a, b, w=0.5 + it, domain=dom, origin=org)
        np.testing.assert_array_equal(gt_storage.to_numpy(b),
                                      _expect(a, 0.5 + it, dom, org["a"], org["b"], b_init=np.zeros((17, 9, 5))))
    (entries,) = _memo(st).values()
    assert len(entries) == 2
    launches = [e[2] for e in entries]
    for it in range(4):
        dom, org = sigs[it % 2]
        st(a, b, w=1.0, domain=dom, origin=org)
    assert [e[2] for e in _memo(st)[next(iter(_memo(st)))]] in (launches, launches[::-1])


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_domain_and_origin_changes():
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    a, b = _fields(5)
    full = (17, 9, 5)
    st(a, b, w=2.0, domain=full, origin=(0, 0, 0))
    b.zero_()
    st(a, b, w=2.0, domain=(5, 4, 3), origin={"a": (1, 2, 1), "b": (3, 1, 2)})
    np.testing.assert_array_equal(gt_storage.to_numpy(b),
                                  _expect(a, 2.0, (5, 4, 3), (1, 2, 1), (3, 1, 2), b_init=np.zeros(full)))
    b.zero_()
    org = {"a": (1, 2, 1), "b": (3, 1, 2)}
    st(a, b, w=2.0, domain=(5, 4, 3), origin=org)
    org["b"] = (0, 0, 0)  # the caller mutates its origin dict: must not hit the stale entry
    b.zero_()
    st(a, b, w=2.0, domain=(5, 4, 3), origin=org)
    np.testing.assert_array_equal(gt_storage.to_numpy(b),
                                  _expect(a, 2.0, (5, 4, 3), (1, 2, 1), (0, 0, 0), b_init=np.zeros(full)))


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_exec_info_after_fast_calls():
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    a, b = _fields(6)
    for _ in range(3):
        st(a, b, w=1.0, domain=(17, 9, 5), origin=(0, 0, 0))
    info = {}
    st(a, b, w=1.0, domain=(17, 9, 5), origin=(0, 0, 0), exec_info=info)
    for k in ("call_start_time", "call_end_time", "run_start_time", "run_end_time", "run_cpp_start_time"):
        assert k in info


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_frozen_fast_path():
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    a, b = _fields(8)
    dom = (17, 9, 5)
    fz = st.freeze(origin={"a": (0, 0, 0), "b": (0, 0, 0)}, domain=dom)
    for w in (1.0, -2.0, 0.125):
        fz(a=a, b=b, w=w)
        np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a, w, dom, b_init=np.zeros(dom)))
    assert len(fz._memo) == 1
    a2, b2 = _fields(9)
    fz(a=a2, b=b2, w=3.0)
    np.testing.assert_array_equal(gt_storage.to_numpy(b2), _expect(a2, 3.0, dom, b_init=np.zeros(dom)))
    info = {}
    fz(a=a2, b=b2, w=3.0, exec_info=info)
    assert "call_run_start_time" in info and "run_cpp_start_time" in info


@pytest.mark.gpu
@pytest.mark.usefixtures("mode")
def test_parameter_types_and_entry_kind(mode):
    """Parameter types follow the reference: validation runs when the (shapes, origins,
    parameter names, domain) cache misses (stencil_object.py:578-591), so a float32 value for a
    float64 parameter raises TypeError on a fresh signature and is converted afterwards, as are
    numpy scalars, ints and bools in unvalidated calls. The memo entry is the native Prepared
    object when the extension is built."""
    _need_gpu()
    st = gtscript.stencil(backend=BK, definition=shift_axpy, name="fast_call.axpy")
    st.clean_call_args_cache()
    a, b = _fields(10)
    dom = (17, 9, 5)
    for bad in (np.float32(1.5), 2, True):
        with pytest.raises(TypeError):
            st(a, b, w=bad, domain=dom, origin=(0, 0, 0))
    st(a, b, w=0.5, domain=dom, origin=(0, 0, 0))
    (entries,) = _memo(st).values()
    (entry,) = entries
    assert (type(entry[2]).__name__ == "Prepared") == (mode == "native")
    for w in (np.float32(1.5), 2, np.float64(-0.25), np.int64(3), True, 0.125):
        st(a, b, w=w, domain=dom, origin=(0, 0, 0))
        np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a, float(w), dom, b_init=np.zeros(dom)))
        st(a, b, w=w * 2, domain=dom, origin=(0, 0, 0), validate_args=False)
        np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a, float(w * 2), dom, b_init=np.zeros(dom)))
    fz = st.freeze(origin={"a": (0, 0, 0), "b": (0, 0, 0)}, domain=dom)
    for w in (0.5, np.float32(2.5), 4):  # FrozenStencil never validates (reference :94-128)
        fz(a=a, b=b, w=w)
        np.testing.assert_array_equal(gt_storage.to_numpy(b), _expect(a, float(w), dom, b_init=np.zeros(dom)))


def test_native_prepared_rejects_other_arguments():
    """CPU: a Prepared launch returns False (no launch) for other tensors, a re-pointed tensor,
    another argument count or a wrong container -- every path that never reaches the library."""
    import ctypes

    import torch

    from gt4py_amd.runtime import fastcall, ffi

    m = fastcall.module()
    if m is None:
        pytest.skip("gt4py_amd._gtmi_fastcall not built")
    x, y = torch.zeros(4, 3, 2), torch.zeros(4, 3, 2)
    fields = (ffi.GtmiField * 2)()
    scal = (ffi.GtmiScalar * 1)()
    p = m.Prepared(0, 0, (4, 3, 2), ctypes.addressof(fields), 2, ctypes.addressof(scal), 1, [(0, 0, 0)], 1,
                   [x, y], 0, False, "t")
    assert p((y, x), (1.0,)) is False  # swapped
    assert p((x,), (1.0,)) is False  # too few fields
    assert p((x, y), ()) is False  # too few params
    assert p([x, y], (1.0,)) is False  # not a tuple
    x.as_strided_((4, 3, 2), (1, 4, 12))
    assert p((x, y), (1.0,)) is False  # same object, data pointer and sizes; new strides
    x.as_strided_((4, 3, 2), (6, 2, 1))
    y.set_(torch.zeros(4, 3, 2).untyped_storage())
    assert p((x, y), (1.0,)) is False  # same object, new data
    with pytest.raises(TypeError):
        p((x, y))  # params missing
    with pytest.raises(ValueError):
        m.Prepared(0, 0, (4, 3, 2), ctypes.addressof(fields), 2, ctypes.addressof(scal), 1, [(5, 0, 0)], 1,
                   [x, y], 0, False, "t")


def test_native_module_survives_a_moved_tree(tmp_path):
    """The built extension's stamp must not depend on where the tree lives: the GPU box runs the
    tree from another directory (round 4: an absolute path in the digest made every box see a
    'stale' module and fall back to the ctypes launch)."""
    import os
    import shutil
    import subprocess
    import sys

    from gt4py_amd.runtime import fastcall

    if not fastcall.up_to_date():
        pytest.skip("gt4py_amd._gtmi_fastcall not built")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(fastcall.__file__)))
    repo = os.path.dirname(repo)
    shutil.copytree(os.path.join(repo, "gt4py_amd"), tmp_path / "gt4py_amd",
                    ignore=shutil.ignore_patterns("__pycache__"))
    shutil.copytree(os.path.join(repo, "include"), tmp_path / "include")
    code = ("import warnings; warnings.simplefilter('error'); from gt4py_amd.runtime import fastcall; "
            "assert fastcall.up_to_date(); assert fastcall.module() is not None")
    res = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, capture_output=True, text=True,
                         env={k: v for k, v in os.environ.items() if k != "PYTHONPATH"})
    assert res.returncode == 0, res.stderr[-2000:]
