"""Call-interface fidelity, after the reference's
``integration_tests/feature_tests/test_call_interface.py`` and ``test_exec_info.py``:
origin/domain selection and precedence (``__gt_origin__`` wrappers, ``"_all_"``), defaults and
optional fields, halo checks, numpy integer types, exec_info timings, axes / data-dimension
mismatch errors, permuted axes (``__gt_dims__``), origin dicts left unchanged.

Every test runs on the ``numpy`` backend (CPU) and, marked ``gpu``, on ``gt:mi355x``.
"""

import copy

import numpy as np
import pytest

from gt4py_amd import gtscript
from gt4py_amd import storage as gt_storage
from gt4py_amd.frontend import GTScriptSyntaxError
from gt4py_amd.gtscript import FORWARD, PARALLEL, Field, K, computation, interval

BACKENDS = ["numpy", pytest.param("gt:mi355x", marks=pytest.mark.gpu)]


def _skip_without_gpu(backend):
    if backend == "gt:mi355x":
        import torch

        if not torch.cuda.is_available():
            pytest.skip("no ROCm device")


def _host(a):
    return gt_storage.to_numpy(a) if not isinstance(a, np.ndarray) else a


class OriginWrapper:
    """An array carrying its default origin (``__gt_origin__``), like the reference test utils."""

    def __init__(self, array, origin):
        self.array = array
        self.__gt_origin__ = tuple(origin)

    @property
    def __array_interface__(self):
        return self.array.__array_interface__

    @property
    def __cuda_array_interface__(self):
        return self.array.__cuda_array_interface__


class DimensionsWrapper:
    def __init__(self, array, dimensions):
        self.array = array
        self.__gt_dims__ = tuple(dimensions)

    @property
    def __array_interface__(self):
        return self.array.__array_interface__

    @property
    def __cuda_array_interface__(self):
        return self.array.__cuda_array_interface__


def base_stencil(field1: Field[np.float64], field2: Field[np.float64], field3: Field[np.float32], *, param: np.float64):
    with computation(PARALLEL), interval(...):
        field1 = field2 + field3 * param
        field2 = field1 + field3 * param
        field3 = param * field2


def avg_stencil(in_field: Field[np.float64], out_field: Field[np.float64]):
    with computation(PARALLEL), interval(...):
        out_field = 0.25 * (+in_field[0, 1, 0] + in_field[0, -1, 0] + in_field[1, 0, 0] + in_field[-1, 0, 0])


def _abc(backend):
    a = gt_storage.ones((3, 3, 3), np.float64, backend=backend, aligned_index=(0, 0, 0))
    b = gt_storage.ones((3, 3, 3), np.float64, backend=backend, aligned_index=(2, 2, 2))
    c = gt_storage.ones((3, 3, 3), np.float32, backend=backend, aligned_index=(0, 1, 0))
    return a, b, c


@pytest.mark.parametrize("backend", BACKENDS)
def test_origin_selection(backend):
    _skip_without_gpu(backend)
    st = gtscript.stencil(definition=base_stencil, backend=backend)
    # explicit origin overrides the wrappers' __gt_origin__
    A, B, C = _abc(backend)
    st(OriginWrapper(A, (0, 0, 0)), OriginWrapper(B, (2, 2, 2)), OriginWrapper(C, (0, 1, 0)), param=3.0,
       origin=(1, 1, 1), domain=(1, 1, 1))
    A, B, C = _host(A), _host(B), _host(C)
    assert A[1, 1, 1] == 4 and B[1, 1, 1] == 7 and C[1, 1, 1] == 21
    assert (np.sum(A), np.sum(B), np.sum(C)) == (30, 33, 47)
    # per-field entries beat "_all_"
    A, B, C = _abc(backend)
    st(OriginWrapper(A, (0, 0, 0)), OriginWrapper(B, (2, 2, 2)), OriginWrapper(C, (0, 1, 0)), param=3.0,
       origin={"_all_": (1, 1, 1), "field1": (2, 2, 2)}, domain=(1, 1, 1))
    A, B, C = _host(A), _host(B), _host(C)
    assert A[2, 2, 2] == 4 and B[1, 1, 1] == 7 and C[1, 1, 1] == 21
    # fields without an entry fall back to their __gt_origin__
    A, B, C = _abc(backend)
    st(OriginWrapper(A, (0, 0, 0)), OriginWrapper(B, (2, 2, 2)), OriginWrapper(C, (0, 1, 0)), param=3.0,
       origin={"field1": (2, 2, 2)}, domain=(1, 1, 1))
    A, B, C = _host(A), _host(B), _host(C)
    assert A[2, 2, 2] == 4 and B[2, 2, 2] == 7 and C[0, 1, 0] == 21
    assert (np.sum(A), np.sum(B), np.sum(C)) == (30, 33, 47)


@pytest.mark.parametrize("backend", BACKENDS)
def test_domain_selection(backend):
    _skip_without_gpu(backend)
    st = gtscript.stencil(definition=base_stencil, backend=backend)
    A, B, C = _abc(backend)
    st(A, B, C, param=3.0, origin=(1, 1, 1), domain=(1, 1, 1))
    A, B, C = _host(A), _host(B), _host(C)
    assert A[1, 1, 1] == 4 and B[1, 1, 1] == 7 and C[1, 1, 1] == 21
    assert (np.sum(A), np.sum(B), np.sum(C)) == (30, 33, 47)
    # default domain: the largest that fits every field from its origin
    A, B, C = _abc(backend)
    st(A, B, C, param=3.0, origin=(0, 0, 0))
    A, B, C = _host(A), _host(B), _host(C)
    assert (A == 4).all() and (B == 7).all() and (C == 21).all()


def a_stencil(arg1: Field[np.float64], arg2: Field[np.float64], arg3: Field[np.float64] = None, *, par1: np.float64,
              par2: np.float64 = 7.0, par3: np.float64 = None):
    from __externals__ import BRANCH

    with computation(PARALLEL), interval(...):
        if __INLINED(BRANCH):  # noqa: F821
            arg1 = arg1 * par1 * par2
        else:
            arg1 = arg2 + arg3 * par1 * par2 * par3


@pytest.mark.parametrize("backend", BACKENDS)
def test_default_arguments(backend):
    _skip_without_gpu(backend)
    t = gtscript.stencil(backend=backend, definition=a_stencil, externals={"BRANCH": True}, rebuild=True)
    f = gtscript.stencil(backend=backend, definition=a_stencil, externals={"BRANCH": False}, rebuild=True)

    def fresh():
        a1 = gt_storage.ones((3, 3, 3), np.float64, backend=backend, aligned_index=(0, 0, 0))
        a2 = gt_storage.zeros((3, 3, 3), np.float64, backend=backend, aligned_index=(0, 0, 0))
        a3 = gt_storage.full((3, 3, 3), 2.0, np.float64, backend=backend, aligned_index=(0, 0, 0))
        return a1, a2, a3

    a1, a2, a3 = fresh()
    t(a1, None, a3, par1=2.0)
    assert (_host(a1) == 14).all()
    t(a1, None, par1=2.0)
    assert (_host(a1) == 196).all()
    f(a1, a2, a3, par1=2.0, par3=2.0)
    assert (_host(a1) == 56).all()
    with pytest.raises((ValueError, AssertionError)):
        f(a1, a2, par1=2.0, par3=2.0)  # the optional field is used by this branch
    a1, a2, a3 = fresh()
    t(a1, arg2=None, par1=2.0, par2=5.0, par3=3.0)
    assert (_host(a1) == 10).all()
    t(a1, arg2=None, par1=2.0, par2=5.0)
    assert (_host(a1) == 100).all()
    f(a1, a2, a3, par1=2.0, par2=5.0, par3=3.0)
    assert (_host(a1) == 60).all()
    with pytest.raises((TypeError, AssertionError)):
        f(a1, a2, a3, par1=2.0, par2=5.0)  # par3=None where a float is required


@pytest.mark.parametrize("backend", BACKENDS)
def test_halo_checks(backend):
    _skip_without_gpu(backend)
    st = gtscript.stencil(definition=avg_stencil, backend=backend)

    def pair(n):
        i = gt_storage.ones((n, n, 10), np.float64, backend=backend, aligned_index=(1, 1, 0))
        o = gt_storage.zeros((n, n, 10), np.float64, backend=backend, aligned_index=(1, 1, 0))
        return OriginWrapper(i, (1, 1, 0)), OriginWrapper(o, (1, 1, 0))

    i, o = pair(22)
    st(in_field=i, out_field=o)
    assert (_host(o.array)[1:-1, 1:-1, :] == 1).all()
    i, o = pair(22)
    st(in_field=i, out_field=o, origin=(2, 2, 0), domain=(10, 10, 10))
    assert (_host(o.array)[2:12, 2:12, :] == 1).all()
    assert (_host(o.array)[12:, :, :] == 0).all()
    i, o = pair(22)
    with pytest.raises(ValueError):
        st(in_field=i, out_field=o, origin=(2, 2, 0), domain=(20, 20, 10))
    i, o = pair(23)  # 2*origin + domain fits: must not raise
    st(in_field=i, out_field=o, origin=(2, 2, 0), domain=(20, 20, 10))


@pytest.mark.parametrize("backend", BACKENDS)
def test_np_int_types(backend):
    _skip_without_gpu(backend)
    st = gtscript.stencil(definition=avg_stencil, backend=backend)
    shape = (np.int8(23), np.int16(23), np.int32(10))
    i = gt_storage.ones(shape, np.float64, backend=backend, aligned_index=(np.int64(1), int(1), 0))
    o = gt_storage.zeros(shape, np.float64, backend=backend, aligned_index=(np.int64(1), int(1), 0))
    st(in_field=i, out_field=o, origin=(np.int8(2), np.int16(2), np.int32(0)), domain=(np.int64(20), int(20), 10))
    assert (_host(o)[2:22, 2:22] == 1).all()


@pytest.mark.parametrize("backend", BACKENDS)
def test_exec_info(backend):
    _skip_without_gpu(backend)
    st = gtscript.stencil(definition=avg_stencil, backend=backend)
    exec_info = {}
    i = gt_storage.ones((23, 23, 10), np.float64, backend=backend, aligned_index=(1, 1, 0))
    o = gt_storage.zeros((23, 23, 10), np.float64, backend=backend, aligned_index=(1, 1, 0))
    st(in_field=i, out_field=o, origin=(2, 2, 0), domain=(20, 20, 10), exec_info=exec_info)
    for k in ("call", "call_run", "run"):
        assert exec_info[k + "_end_time"] > exec_info[k + "_start_time"], k
    if backend.startswith("gt:"):
        assert exec_info["run_cpp_end_time"] > exec_info["run_cpp_start_time"]
    # aggregated per-stencil statistics (test_exec_info.py)
    exec_info["__aggregate_data"] = True
    for _ in range(3):
        st(in_field=i, out_field=o, origin=(2, 2, 0), domain=(20, 20, 10), exec_info=exec_info)
    stats = exec_info[st.__class__.__name__]
    assert stats["ncalls"] == 3
    assert stats["total_call_time"] > stats["call_time"] > stats["run_time"] > 0
    assert stats["total_run_time"] > stats["run_time"]
    assert stats["call_start_time"] == exec_info["call_start_time"]
    if backend.startswith("gt:"):
        assert stats["run_time"] > stats["run_cpp_time"] > 0


@pytest.mark.parametrize("backend", BACKENDS)
def test_axes_mismatch(backend):
    _skip_without_gpu(backend)

    @gtscript.stencil(backend=backend)
    def st(field_out: gtscript.Field[gtscript.IJ, np.float64]):
        with computation(FORWARD), interval(...):
            field_out = 1.0

    with pytest.raises(ValueError, match="Storage for '.*' has 3 dimensions but the API signature expects 2 .*"):
        st(field_out=gt_storage.empty((3, 3, 3), np.float64, backend=backend, aligned_index=(0, 0, 0)))
    with pytest.raises(Exception, match="Storage for '.*' has dimensions '.*' but the API signature expects '\\[I, J\\]'"):
        st(field_out=DimensionsWrapper(
            gt_storage.empty((3, 3), np.float64, backend=backend, aligned_index=(0, 0), dimensions=["I", "K"]),
            ("I", "K")))


@pytest.mark.parametrize("backend", BACKENDS)
def test_data_dimensions(backend):
    _skip_without_gpu(backend)

    @gtscript.stencil(backend=backend)
    def st(field_out: gtscript.Field[gtscript.IJK, (np.float64, (2,))]):
        with computation(FORWARD), interval(...):
            field_out[0, 0, 0][0] = 0.0
            field_out[0, 0, 0][1] = 1.0

    @gtscript.stencil(backend=backend)
    def one(field_out: gtscript.Field[gtscript.IJ, (np.float64, (1,))]):
        with computation(FORWARD), interval(...):
            field_out[0, 0][0] = 42.0

    with pytest.raises(ValueError, match="Field '.*' expects data dimensions \\(2,\\) but got \\(3,\\)"):
        st(field_out=gt_storage.empty((3, 3, 1), (np.float64, (3,)), backend=backend, aligned_index=(0, 0, 0)))
    f = gt_storage.full((3, 3, 1), 5.0, (np.float64, (2,)), backend=backend, aligned_index=(0, 0, 0))
    st(field_out=f)
    h = _host(f)
    assert (h[..., 0] == 0).all() and (h[..., 1] == 1).all()

    ones = gt_storage.ones((2, 3), (np.float64, (1,)), backend=backend, aligned_index=(0, 0), dimensions=["I", "J"])
    one(ones)
    assert (_host(ones) == 42.0).all()

    with pytest.raises(GTScriptSyntaxError, match="Data index out of bounds"):

        @gtscript.stencil(backend=backend)
        def bad(field_out: gtscript.Field[gtscript.IJ, (np.float64, (1,))]):
            with computation(FORWARD), interval(...):
                field_out[0, 0][1] = 42.0


@pytest.mark.parametrize("backend", BACKENDS)
def test_origin_unchanged(backend):
    _skip_without_gpu(backend)

    @gtscript.stencil(backend=backend)
    def calc_damp(outp: Field[float], inp: Field[K, float]):
        with computation(FORWARD), interval(...):
            outp = inp

    outp = gt_storage.ones((4, 4, 4), float, backend=backend, aligned_index=(1, 1, 1), dimensions="IJK")
    inp = gt_storage.ones((4,), float, backend=backend, aligned_index=(1,), dimensions="K")
    origin = {"_all_": (1, 1, 1), "inp": (1,)}
    ref = copy.deepcopy(origin)
    calc_damp(outp, inp, origin=origin, domain=(3, 3, 3))
    assert all(origin.get(k) == v for k, v in ref.items())


def test_permute_axes():
    @gtscript.stencil(backend="numpy")
    def calc_damp(outp: Field[float], inp: Field[K, float]):
        with computation(FORWARD), interval(...):
            outp = inp

    outp = gt_storage.ones((4, 4, 4), float, backend="numpy", aligned_index=(1, 1, 1), dimensions="KJI")
    inp = gt_storage.from_array(np.arange(4), backend="numpy", aligned_index=(1,), dtype=float, dimensions="K")
    calc_damp(DimensionsWrapper(outp, "KJI"), inp)
    for i in range(4):
        np.testing.assert_equal(outp[i, :, :], i)
