"""Known-answer and smoke tests of the reference's ``multi_feature_tests/test_code_generation.py``
and ``test_math_functions.py``, on the ``numpy`` backend (CPU) and on ``gt:mi355x`` (GPU).

The reference pins absolute values in these tests (e.g. the BACKWARD sweep 5/4/3/2, the halo'ed
temporary 4-inside/0-outside); each test here restates one of them with the same inputs and
the same expected values, and runs it through the public API (storages, ``gtscript.stencil``,
``origin``/``domain``) of both backends.
"""

import math

import numpy as np
import pytest

from gt4py_amd import gtscript, storage
from gt4py_amd.gtscript import (
    BACKWARD, FORWARD, PARALLEL, Field, GlobalTable, I, J, computation, erf, erfc, horizontal, interval, region,
    round, round_away_from_zero, sin,
)

import stencil_cases as sc

BACKENDS = [pytest.param("numpy", id="numpy"), pytest.param("gt:mi355x", id="gt:mi355x", marks=pytest.mark.gpu)]


@pytest.fixture(params=BACKENDS)
def backend(request):
    if storage.from_name(request.param)["device"] == "gpu":
        import torch

        if not torch.cuda.is_available():
            pytest.skip("no ROCm device")
    return request.param


def cpu(x):
    return storage.to_numpy(x)


def ones(shape, backend, dtype=np.float64, aligned_index=None):
    return storage.ones(shape, dtype, backend=backend, aligned_index=aligned_index or (0,) * len(shape))


def zeros(shape, backend, dtype=np.float64, aligned_index=None):
    return storage.zeros(shape, dtype, backend=backend, aligned_index=aligned_index or (0,) * len(shape))


# ------------------------------------------------------------------------------ smoke over the registry
# the 28 programs registered in the reference's stencil_definitions.py -> their stencil_cases names
REGISTRY = {
    "copy_stencil": "copy", "arithmetic_ops": "arithmetic_ops", "scalar_inputs": "scalar_inputs",
    "unary_operation": "unary_operation", "temporary_stencil": "temporary_stencil", "data_types": "data_types",
    "native_functions": "native_functions", "while_stencil": "while_stencil",
    "copy_stencil_plus_one": "copy_stencil_plus_one", "runtime_if": "runtime_if",
    "simple_horizontal_diffusion": "simple_horizontal_diffusion", "tridiagonal_solver": "tridiag",
    "vertical_advection_dycore": "vertical_advection_dycore", "horizontal_diffusion": "hdiff_f64",
    "large_k_interval": "large_k_interval", "single_level_with_offset": "single_level_with_offset",
    "form_land_mask": "form_land_mask", "set_inner_as_kord": "set_inner_as_kord",
    "local_var_inside_nested_conditional": "local_var_inside_nested_conditional",
    "multibranch_param_conditional": "multibranch_param_conditional_pos",
    "allow_empty_computation": "allow_empty_computation", "unused_optional_field": "optional_field_unused",
    "required_optional_field": "optional_field_used", "two_optional_fields_00": "two_optional_fields_00",
    "two_optional_fields_01": "two_optional_fields_01", "two_optional_fields_11": "two_optional_fields_11",
    "horizontal_regions": "horizontal_regions",
    "horizontal_region_with_conditional": "horizontal_region_with_conditional",
}


def _smoke_run(be, case, tag):
    st = gtscript.stencil(be, case.definition, externals=case.externals, name=f"smoke.{tag}")
    args = {}
    for pname, info in st.field_info.items():
        if info is None:
            args[pname] = None
            continue
        dt = (np.dtype(info.dtype), info.data_dims) if info.data_dims else info.dtype
        args[pname] = storage.ones((23,) * len(info.axes), dt, backend=be, dimensions=info.axes,
                                   aligned_index=(10,) * len(info.axes))
    for pname, info in st.parameter_info.items():
        args[pname] = None if info is None else np.dtype(info.dtype).type(1.5)
    st(**args, origin=(10, 10, 5), domain=(3, 3, 17))
    return {k: cpu(v) for k, v in args.items() if k in st.field_info and v is not None}


@pytest.mark.parametrize("ref_name", sorted(REGISTRY))
def test_generation_smoke(ref_name, backend):
    """test_code_generation.py:44-63: every registered program on ones storages of 23 per axis,
    aligned at 10, origin (10, 10, 5), domain (3, 3, 17). gt:mi355x must in addition reproduce the
    numpy backend on these inputs bit for bit (the reference test checks no values)."""
    case = sc.CASES[REGISTRY[ref_name]]
    got = _smoke_run(backend, case, f"{backend.replace(':', '_')}.{ref_name}")
    if backend != "numpy":
        ref = _smoke_run("numpy", case, f"numpy.{ref_name}")
        for k, r in ref.items():
            assert np.array_equal(got[k], r, equal_nan=True), f"{ref_name}: field '{k}' differs from numpy"


# ------------------------------------------------------------------------------ builds
def test_temporary_field_declared_in_if(backend):
    @gtscript.stencil(backend=backend)
    def definition(field_a: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            if field_a < 0:
                field_b = -field_a
            else:
                field_b = field_a
            field_a = field_b

    a = storage.from_array(np.arange(-4, 4, dtype=np.float64).reshape(2, 2, 2), backend=backend)
    definition(a)
    assert np.array_equal(cpu(a), np.abs(np.arange(-4, 4, dtype=np.float64)).reshape(2, 2, 2))


def test_stage_without_effect(backend):
    @gtscript.stencil(backend=backend)
    def definition(field_a: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            field_c = 0.0  # noqa: F841

    definition(ones((3, 3, 3), backend))


def test_stencil_without_effect(backend):
    def definition1(field_in: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            tmp = 0.0  # noqa: F841

    def definition2(f_in: Field[np.float64]):
        from __externals__ import flag

        with computation(PARALLEL), interval(...):
            if __INLINED(flag):  # noqa: F821
                B = f_in  # noqa: F841

    s1 = gtscript.stencil(backend, definition1)
    s2 = gtscript.stencil(backend, definition2, externals={"flag": False})
    f = ones((23, 23, 23), backend)
    s1(f, domain=(3, 3, 3))
    s2(f, domain=(3, 3, 3))
    s1(f)


def test_lazy_stencil(backend):
    @gtscript.lazy_stencil(backend=backend)
    def definition(field_a: Field[np.float64], field_b: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            field_a[0, 0, 0] = field_b

    a, b = zeros((3, 3, 3), backend), ones((3, 3, 3), backend)
    definition(a, b)
    assert (cpu(a) == 1).all()


def test_ignore_np_errstate():
    def run(**kwargs):
        a = zeros((3, 3, 1), "numpy")

        @gtscript.stencil(backend="numpy", **kwargs)
        def divide_by_zero(field_a: Field[np.float64]):
            with computation(PARALLEL), interval(...):
                field_a = 1.0 / field_a

        divide_by_zero(a)

    run()
    with pytest.warns(RuntimeWarning, match="divide by zero encountered"):
        run(ignore_np_errstate=False)


# ------------------------------------------------------------------------------ known answers
def test_stage_merger_induced_interval_block_reordering(backend):
    fin, fout = ones((23, 23, 23), backend), zeros((23, 23, 23), backend)

    @gtscript.stencil(backend=backend)
    def stencil(field_in: Field[np.float64], field_out: Field[np.float64]):
        with computation(BACKWARD):
            with interval(-2, -1):
                field_out = field_in
            with interval(0, -2):
                field_out = field_in
        with computation(BACKWARD):
            with interval(-1, None):
                field_out = 2 * field_in
            with interval(0, -1):
                field_out[0, 0, 0] = 3 * field_in

    stencil(fin, fout)
    out = cpu(fout)
    assert (out[:, :, :-1] == 3).all() and (out[:, :, -1] == 2).all()


def test_nested_while_loop(backend):
    @gtscript.stencil(backend=backend)
    def stencil(field_a: Field[np.float64], field_b: Field[np.int_]):
        with computation(PARALLEL), interval(...):
            while field_a < 1:
                add = 0
                while field_a + field_b < 1:
                    add += 1
                field_a += add

    # the reference only builds this stencil; run it on inputs for which both loops terminate
    # (field_a >= 1 skips the outer loop; the loops never end for field_a < 1 <= field_a + field_b)
    b = storage.from_array(np.full((2, 2, 2), 1, dtype=np.int_), np.int_, backend=backend)
    a = storage.from_array(np.full((2, 2, 2), 2.0), backend=backend)
    stencil(a, b)
    assert (cpu(a) == 2.0).all()


def test_mask_with_offset_written_in_conditional(backend):
    @gtscript.stencil(backend)
    def stencil(outp: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            cond = True
            if cond[0, -1, 0] or cond[0, 0, 0]:
                outp = 1.0
            else:
                outp[0, 0, 0] = 0.0

    outp = zeros((10, 10, 10), backend)
    stencil(outp)
    assert np.allclose(cpu(outp), 1.0)


def test_write_data_dim_indirect_addressing(backend):
    V2 = (np.int32, (2,))

    def definition(input_field: Field[gtscript.IJK, np.int32], output_field: Field[gtscript.IJK, V2], index: int):
        with computation(PARALLEL), interval(...):
            output_field[0, 0, 0][index] = input_field

    inp = ones((1, 1, 2), backend, np.int32)
    out = zeros((1, 1, 2), backend, V2)
    gtscript.stencil(definition=definition, backend=backend)(inp, out, 1)
    assert cpu(out)[0, 0, 0, 1] == 1 and cpu(out)[0, 0, 0, 0] == 0


def test_read_data_dim_indirect_addressing(backend):
    V2 = (np.int32, (2,))

    def definition(input_field: Field[gtscript.IJK, V2], output_field: Field[gtscript.IJK, np.int32], index: int):
        with computation(PARALLEL), interval(...):
            output_field[0, 0, 0] = input_field[0, 0, 0][index]

    inp = ones((1, 1, 2), backend, V2)
    out = zeros((1, 1, 2), backend, np.int32)
    gtscript.stencil(definition=definition, backend=backend)(inp, out, 1)
    assert cpu(out)[0, 0, 0] == 1


def test_negative_origin_i(backend):
    @gtscript.stencil(backend=backend)
    def stencil_i(input_field: Field[gtscript.IJK, np.int32], output_field: Field[gtscript.IJK, np.int32]):
        with computation(PARALLEL), interval(...):
            output_field[0, 0, 0] = input_field[1, 0, 0]

    inp, out = ones((1, 1, 1), backend, np.int32), zeros((1, 1, 1), backend, np.int32)
    stencil_i(inp, out, origin={"input_field": (-1, 0, 0)})
    assert cpu(out)[0, 0, 0] == 1


def test_negative_origin_k(backend):
    @gtscript.stencil(backend=backend)
    def stencil_k(input_field: Field[gtscript.IJK, np.int32], output_field: Field[gtscript.IJK, np.int32]):
        with computation(PARALLEL), interval(...):
            output_field[0, 0, 0] = input_field[0, 0, 1]

    inp, out = ones((1, 1, 1), backend, np.int32), zeros((1, 1, 1), backend, np.int32)
    stencil_k(inp, out, origin={"input_field": (0, 0, -1)})
    assert cpu(out)[0, 0, 0] == 1


def test_origin_k_fields(backend):
    @gtscript.stencil(backend=backend, rebuild=True)
    def k_to_ijk(outp: Field[np.float64], inp: Field[gtscript.K, np.float64]):
        with computation(PARALLEL), interval(...):
            outp[0, 0, 0] = inp

    data = np.arange(10, dtype=np.float64)
    inp = storage.from_array(data, np.float64, backend=backend, aligned_index=(0,), dimensions="K")
    outp = zeros((2, 2, 10), backend)
    k_to_ijk(outp, inp, origin={"outp": (0, 0, 1), "inp": (2,)}, domain=(2, 2, 8))
    out = cpu(outp)
    assert np.array_equal(cpu(inp), data)
    assert np.array_equal(out[:, :, 1:-1], np.broadcast_to(data[2:], (2, 2, 8)))
    assert (out[:, :, 0] == 0).all() and (out[:, :, -1] == 0).all()


def test_tmp_stencil(backend):
    fin, fout = ones((6, 6, 6), backend), zeros((6, 6, 6), backend)

    @gtscript.stencil(backend=backend)
    def stencil(field_in: Field[np.float64], field_out: Field[np.float64]):
        with computation(PARALLEL):
            with interval(...):
                tmp = field_in + 1
        with computation(PARALLEL):
            with interval(...):
                field_out[0, 0, 0] = tmp[-1, 0, 0] + tmp[1, 0, 0]

    stencil(fin, fout, origin=(1, 1, 0), domain=(4, 4, 6))
    out = cpu(fout)
    assert (out[1:-1, 1:-1] == 4).all()
    ring = np.ones_like(out, dtype=bool)
    ring[1:-1, 1:-1] = False
    assert (out[ring] == 0).all()


def test_backward_stencil(backend):
    fin, fout = ones((4, 4, 4), backend), zeros((4, 4, 4), backend)

    @gtscript.stencil(backend=backend)
    def stencil(field_in: Field[np.float64], field_out: Field[np.float64]):
        with computation(BACKWARD):
            with interval(-1, None):
                field_in = 2
                field_out = field_in
            with interval(0, -1):
                field_in = field_in[0, 0, 1] + 1
                field_out[0, 0, 0] = field_in

    stencil(fin, fout)
    out = cpu(fout)
    for k, expected in enumerate((5, 4, 3, 2)):
        assert (out[:, :, k] == expected).all()


def test_while_stencil(backend):
    fin, fout = ones((6, 6, 6), backend), zeros((6, 6, 6), backend)

    @gtscript.stencil(backend=backend)
    def stencil(field_in: Field[np.float64], field_out: Field[np.float64]):
        with computation(PARALLEL):
            with interval(...):
                while field_in < 10:
                    field_in += 1
                field_out[0, 0, 0] = field_in

    stencil(fin, fout)
    assert (cpu(fout) == 10).all()


@pytest.mark.parametrize("scalar_index", [False, True])
def test_higher_dim_literal_and_scalar_index(backend, scalar_index):
    V4 = (np.float64, (4,))
    fin, fout = ones((6, 6, 6), backend, V4), zeros((6, 6, 6), backend)
    fin[:, :, :, 2] = 5

    if scalar_index:
        @gtscript.stencil(backend=backend)
        def stencil(vec_field: Field[V4], out_field: Field[np.float64], scalar_argument: int):
            with computation(PARALLEL), interval(...):
                out_field[0, 0, 0] = vec_field[0, 0, 0][scalar_argument]

        stencil(fin, fout, 2)
    else:
        @gtscript.stencil(backend=backend)
        def stencil(vec_field: Field[V4], out_field: Field[np.float64]):
            with computation(PARALLEL), interval(...):
                out_field[0, 0, 0] = vec_field[0, 0, 0][2]

        stencil(fin, fout)
    assert (cpu(fout) == 5).all()


def test_native_function_call_stencil(backend):
    fin, fout = ones((4, 4, 4), backend), zeros((4, 4, 4), backend)

    @gtscript.stencil(backend=backend)
    def stencil(in_field: Field[np.float64], out_field: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            out_field[0, 0, 0] = in_field[0, 0, 0] + sin(0.848062)

    stencil(fin, fout)
    np.testing.assert_allclose(cpu(fout), 1.75)


def test_unary_operator_stencil(backend):
    fin, fout = ones((4, 4, 4), backend), zeros((4, 4, 4), backend)

    @gtscript.stencil(backend=backend)
    def stencil(in_field: Field[np.float64], out_field: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            out_field[0, 0, 0] = -in_field[0, 0, 0]

    stencil(fin, fout)
    assert (cpu(fout) == -1).all()


def test_ternary_operator_stencil(backend):
    fin, fout = ones((4, 4, 4), backend), zeros((4, 4, 4), backend)
    fin[0, 0, 1] = 20

    @gtscript.stencil(backend=backend)
    def stencil(in_field: Field[np.float64], out_field: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            out_field[0, 0, 0] = in_field[0, 0, 0] if in_field > 10 else in_field[0, 0, 0] + 1

    stencil(fin, fout)
    out = cpu(fout)
    assert out[0, 0, 1] == 20 and (out[1:, 1:, 1] == 2).all()


def test_mask_stencil(backend):
    fin, fout = ones((4, 4, 4), backend), zeros((4, 4, 4), backend)
    fin[0, 0, 1] = -20

    @gtscript.stencil(backend=backend)
    def stencil(in_field: Field[np.float64], out_field: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            if in_field[0, 0, 0] > 0:
                out_field[0, 0, 0] = in_field
            else:
                out_field[0, 0, 0] = 1

    stencil(fin, fout)
    assert (cpu(fout) > 0).all()


def test_k_offset_stencil(backend):
    fin, fout = ones((4, 4, 4), backend), zeros((4, 4, 4), backend)
    fin[:, :, 0] *= 10

    @gtscript.stencil(backend=backend)
    def stencil(in_field: Field[np.float64], out_field: Field[np.float64], scalar_value: int):
        with computation(PARALLEL), interval(1, None):
            out_field[0, 0, 0] = in_field[0, 0, scalar_value]

    stencil(fin, fout, -1)
    assert (cpu(fout)[:, :, 1] == 10).all()


def test_k_offset_field_stencil(backend):
    fin, fout = ones((4, 4, 4), backend), zeros((4, 4, 4), backend)
    idx = ones((4, 4), backend, np.int64)
    fin[:, :, 0] *= 10
    idx[:, :] *= -2

    @gtscript.stencil(backend=backend)
    def stencil(in_field: Field[np.float64], out_field: Field[np.float64], idx_field: Field[gtscript.IJ, np.int64]):
        with computation(PARALLEL), interval(1, None):
            out_field[0, 0, 0] = in_field[0, 0, idx_field + 1]

    stencil(fin, fout, idx)
    assert (cpu(fout)[:, :, 1] == 10).all()


def test_k_only_access_stencil(backend):
    fin = storage.from_array(np.array([2, 3, 4, 5]), np.float64, backend=backend, aligned_index=(0,))
    fout = zeros((4, 4, 4), backend)

    @gtscript.stencil(backend=backend)
    def stencil(in_field: Field[gtscript.K, np.float64], out_field: Field[np.float64]):
        with computation(PARALLEL):
            with interval(0, 1):
                out_field[0, 0, 0] = in_field[1]
            with interval(1, None):
                out_field[0, 0, 0] = in_field[-1]

    stencil(fin, fout)
    assert list(cpu(fout)[1, 1, :]) == [3, 2, 3, 4]


def test_table_access_stencil(backend):
    table = storage.from_array(np.array([2, 3, 4, 5]), np.float64, backend=backend, aligned_index=(0,))
    fout = zeros((4, 4, 4), backend)

    @gtscript.stencil(backend=backend)
    def stencil(table_view: GlobalTable[(np.float64, (4))], out_field: Field[np.float64]):
        with computation(PARALLEL):
            with interval(0, 1):
                out_field[0, 0, 0] = table_view.A[1]
            with interval(1, None):
                out_field[0, 0, 0] = table_view.A[2]

    stencil(table, fout)
    assert list(cpu(fout)[1, 1, :]) == [3, 4, 4, 4]


def test_pruned_args_match(backend):
    @gtscript.stencil(backend=backend)
    def stencil(out: Field[np.float64], inp: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            out = 0.0
            with horizontal(region[I[0] - 1, J[0] - 1]):
                out[0, 0, 0] = inp

    inp = zeros((2, 2, 2), backend)
    out = storage.empty((2, 2, 2), np.float64, backend=backend, aligned_index=(0, 0, 0))
    stencil(out, inp)
    assert (cpu(out) == 0).all()


def test_k_offset_write_forward(backend):
    """test_code_generation.py:966-995: a FORWARD sweep writing A one level below while B reads A."""
    kv = np.arange(40, 44, dtype=np.float64)

    @gtscript.stencil(backend=backend)
    def forward(A: Field[np.float64], B: Field[np.float64], scalar: np.float64):
        with computation(FORWARD), interval(1, None):
            A[0, 0, -1] = scalar
            B[0, 0, 0] = A

    a = storage.from_array(kv.reshape(1, 1, 4), backend=backend)
    b = zeros((1, 1, 4), backend)
    forward(a, b, 2.0)
    ah, bh = cpu(a)[0, 0], cpu(b)[0, 0]
    assert (ah[:3] == 2.0).all() and ah[3] == kv[3]
    assert bh[0] == 0 and (bh[1:] == kv[1:]).all()


# ------------------------------------------------------------------------------ math functions
@pytest.mark.parametrize("which", ["erf", "erfc"])
def test_erf_erfc(backend, which):
    if which == "erf":
        @gtscript.stencil(backend=backend)
        def st(field_a: Field[np.float32], field_b: Field[np.float32]):
            with computation(PARALLEL), interval(...):
                field_b = erf(field_a)
    else:
        @gtscript.stencil(backend=backend)
        def st(field_a: Field[np.float32], field_b: Field[np.float32]):
            with computation(PARALLEL), interval(...):
                field_b = erfc(field_a)
    ref = getattr(math, which)
    init = np.array([[[-1, 0, 1, 2]]], dtype=np.float32)
    a = storage.from_array(init, np.float32, backend=backend)
    b = storage.full(init.shape, 42.0, np.float32, backend=backend)
    st(a, b)
    assert (cpu(a) == init).all()
    # device libm differs from glibc in the last bits (the reference's comment says the same of gt:gpu)
    np.testing.assert_allclose(cpu(b)[0, 0], np.array([ref(v) for v in init[0, 0]], dtype=np.float32), rtol=1e-6)


@pytest.mark.parametrize("away", [False, True])
def test_round(backend, away):
    init = np.array([[[-1.5, -0.5, 0.3, 0.5, 0.8, 1.2, 1.5]]], dtype=np.float32)
    if away:
        @gtscript.stencil(backend=backend)
        def st(field_a: Field[np.float32], field_b: Field[np.float32]):
            with computation(PARALLEL), interval(...):
                field_b = round_away_from_zero(field_a)

        expected = [-2.0, -1.0, 0.0, 1.0, 1.0, 1.0, 2.0]
    else:
        @gtscript.stencil(backend=backend)
        def st(field_a: Field[np.float32], field_b: Field[np.float32]):
            with computation(PARALLEL), interval(...):
                field_b = round(field_a)

        expected = [-2.0, 0.0, 0.0, 0.0, 1.0, 1.0, 2.0]
    a = storage.from_array(init, np.float32, backend=backend)
    b = storage.full(init.shape, -1.0, np.float32, backend=backend)
    st(a, b)
    assert (cpu(a) == init).all()
    assert list(cpu(b)[0, 0]) == expected
