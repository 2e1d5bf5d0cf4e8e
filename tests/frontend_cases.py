"""GTScript programs for accept / reject parity with the reference frontend.

Each case is a stencil definition (written against ``gt4py_amd.gtscript``; the verdict generator
aliases that module to the reference ``gt4py.cartesian.gtscript``, as ``golden/make_golden.py``
does) plus externals. ``tests/golden/make_frontend_verdicts.py`` builds every case with the
reference (numpy backend) in the build container and records whether it was accepted and, if
not, the exception class and message (``tests/golden/frontend_verdicts.json``);
``tests/test_frontend_verdicts.py`` requires gt4py_amd to accept and refuse the same programs,
with the same exception class. The categories follow the reference's frontend unit tests
(``tests/cartesian_tests/unit_tests/frontend_tests/test_gtscript_frontend.py``) and its
parallel-model validators (``src/gt4py/cartesian/gtc/gtir.py``); the programs are our own.
"""

import numpy as np

from gt4py_amd import gtscript
from gt4py_amd.gtscript import (
    BACKWARD,
    FORWARD,
    IJ,
    PARALLEL,
    Field,
    I,
    J,
    K,
    compile_assert,
    computation,
    horizontal,
    interval,
    asin,
    cos,
    float32,
    float64,
    isfinite,
    region,
    sin,
)

F64 = Field[np.float64]
CASES = {}  # name -> (definition, externals)


def case(name=None, externals=None):
    def deco(func):
        CASES[name or func.__name__] = (func, dict(externals or {}))
        return func

    return deco


# ----------------------------------------------------------------------------- externals


@case(externals={"SCALE": 2.0})
def ext_ok(a: F64, b: F64):
    from __externals__ import SCALE

    with computation(PARALLEL), interval(...):
        b = a * SCALE


@case()
def ext_missing(a: F64, b: F64):
    from __externals__ import NOT_GIVEN  # noqa: F401

    with computation(PARALLEL), interval(...):
        b = a * NOT_GIVEN  # noqa: F821


@case(externals={"BAD": {"x": 1}})
def ext_wrong_type(a: F64, b: F64):
    from __externals__ import BAD

    with computation(PARALLEL), interval(...):
        b = a * BAD


@case()
def unknown_symbol(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a * UNDEFINED_NAME  # noqa: F821


# ----------------------------------------------------------------------------- functions


@gtscript.function
def _twice(x):
    return 2.0 * x


@gtscript.function
def _pair(x):
    return x, x + 1.0


@gtscript.function
def _noret(x):
    y = x + 1.0  # noqa: F841


@case()
def func_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = _twice(a) + _twice(_twice(a))


@case()
def func_tuple_ok(a: F64, b: F64, c: F64):
    with computation(PARALLEL), interval(...):
        b, c = _pair(a)


@case()
def func_tuple_in_expr(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = _pair(a) + 1.0


@case()
def func_no_return(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = _noret(a)


@case()
def func_not_gtscript(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = np.sqrt(a)


# ----------------------------------------------------------------------------- axis syntax


@case()
def axis_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a[I + 1] + a[J - 1] + a[I - 1, J + 1]


@case()
def axis_dup(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a[I + 1, I - 1]


@case()
def axis_out_of_order(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a[J + 1, I]


# ----------------------------------------------------------------------------- intervals


@case()
def interval_ok(a: F64, b: F64):
    with computation(PARALLEL):
        with interval(0, 1):
            b = a
        with interval(1, -1):
            b = a * 2.0
        with interval(-1, None):
            b = a * 3.0


@case()
def interval_overlap(a: F64, b: F64):
    with computation(PARALLEL):
        with interval(0, 3):
            b = a
        with interval(2, None):
            b = a * 2.0


@case()
def interval_reversed(a: F64, b: F64):
    with computation(PARALLEL), interval(3, 1):
        b = a


@case()
def interval_none_none(a: F64, b: F64):
    with computation(PARALLEL), interval(None, None):
        b = a


@case()
def forward_k_offset_ok(a: F64, b: F64):
    with computation(FORWARD):
        with interval(0, 1):
            b = a
        with interval(1, None):
            b = b[0, 0, -1] + a


# ----------------------------------------------------------------------------- regions


@case()
def region_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a
        with horizontal(region[I[0], :], region[:, J[-1]]):
            b = a + 1.0


@case()
def region_nested_with(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        with horizontal(region[I[0], :]):
            with horizontal(region[:, J[0]]):
                b = a


@case()
def region_written_then_offset(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        t = a * 2.0
        b = t
        with horizontal(region[I[0], :]):
            b = t[1, 0, 0]


@case()
def region_offset_read_of_input_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a
        with horizontal(region[I[-1], :]):
            b = a[-1, 0, 0]


# ----------------------------------------------------------------------------- assignments


@case()
def assign_ij_offset(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b[1, 0, 0] = a


@case()
def assign_k_offset_parallel(a: F64, b: F64):
    with computation(PARALLEL), interval(0, -1):
        b[0, 0, 1] = a


@case()
def assign_k_offset_forward_ok(a: F64, b: F64):
    with computation(FORWARD), interval(0, -1):
        b[0, 0, 1] = a


@case()
def assign_to_scalar(a: F64, b: F64, *, s: float):
    with computation(PARALLEL), interval(...):
        s = a  # noqa: F841
        b = a


@case()
def augmented_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b += a
        b *= 2.0


# ----------------------------------------------------------------------------- parallel model


@case()
def api_write_read_offset(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a
        a = b[1, 0, 0]


@case()
def temp_write_read_offset_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        t = a * 2.0
        b = t[1, 0, 0] + t[-1, 0, 0]


@case()
def while_write_read_offset(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        t = a
        while t < 10.0:
            t = t[1, 0, 0] + 1.0
        b = t


@case()
def parallel_self_k_offset(a: F64, b: F64):
    with computation(PARALLEL), interval(1, None):
        b = b[0, 0, -1] + a


@case()
def temp_read_before_write(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = t + a  # noqa: F821
        t = a  # noqa: F841


# ----------------------------------------------------------------------------- misc


@case(externals={"FLAG": False})
def compile_assert_fails(a: F64, b: F64):
    from __externals__ import FLAG

    with computation(PARALLEL), interval(...):
        compile_assert(FLAG)
        b = a


@case(externals={"FLAG": True})
def compile_assert_ok(a: F64, b: F64):
    from __externals__ import FLAG

    with computation(PARALLEL), interval(...):
        compile_assert(FLAG)
        b = a


@case()
def lowdim_ok(a: Field[IJ, np.float64], b: F64):
    with computation(PARALLEL), interval(...):
        b = a + 1.0


@case()
def lowdim_write_from_parallel(a: F64, b: Field[IJ, np.float64]):
    with computation(PARALLEL), interval(...):
        b = a


@case()
def lowdim_write_forward_ok(a: F64, b: Field[IJ, np.float64]):
    with computation(FORWARD), interval(...):
        b = a


@case()
def datadim_ok(a: Field[(np.float64, (3,))], b: F64):
    with computation(PARALLEL), interval(...):
        b = a[0, 0, 0][0] + a[0, 0, 0][2]


@case()
def datadim_out_of_bounds(a: Field[(np.float64, (3,))], b: F64):
    with computation(PARALLEL), interval(...):
        b = a[0, 0, 0][3]


@case()
def datadim_missing_index(a: Field[(np.float64, (3,))], b: F64):
    with computation(PARALLEL), interval(...):
        b = a


@case()
def k_axis_field_ok(a: Field[gtscript.K, np.float64], b: F64):
    with computation(PARALLEL), interval(...):
        b = a + 1.0


@case()
def ternary_and_math_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = gtscript.sqrt(a * a) if a > 0.0 else gtscript.abs(a)


@case()
def backward_ok(a: F64, b: F64):
    with computation(BACKWARD):
        with interval(-1, None):
            b = a
        with interval(0, -1):
            b = b[0, 0, 1] * 0.5 + a


@case()
def bad_statement_return(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a
        return b  # noqa: B901


@case()
def bad_with_outside(a: F64, b: F64):
    b = a  # noqa: F841


@case()
def k_index_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a[K - 1] + a[K + 1]


@case()
def interval_blocks_out_of_order(a: F64, b: F64):
    with computation(FORWARD):
        with interval(1, None):
            b = a
        with interval(0, 1):
            b = a * 2.0


@case()
def interval_blocks_backward_ok(a: F64, b: F64):
    with computation(BACKWARD):
        with interval(1, None):
            b = a
        with interval(0, 1):
            b = a * 2.0


@case()
def interval_none_start(a: F64, b: F64):
    with computation(PARALLEL), interval(None, 5):
        b = a


@case()
def interval_end_before_start(a: F64, b: F64):
    with computation(PARALLEL), interval(-1, 1):
        b = a


@case()
def interval_mixed_levels_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(3, -2):
        b = a


@case()
def axis_dup_k(a: F64, b: F64):
    with computation(PARALLEL), interval(1, -1):
        b = a[K + 1, K - 1]


@case(externals={"NS": np})
def ext_module_value(a: F64, b: F64):
    from __externals__ import NS

    with computation(PARALLEL), interval(...):
        b = a * NS


@case()
def lowdim_k_write(a: F64, b: Field[gtscript.K, np.float64]):
    with computation(FORWARD), interval(...):
        b = a


# ----------------------------------------------------------------------------- native functions,
# absolute K indexing, casts, typed temporaries, the K iterator (cf. the reference's
# TestNativeFunctions, TestFunctionIfError, TestAbsoluteIndex, TestLiteralCasts,
# TestTemporaryTypes, TestNumpyTypedConstants, TestIteratorAccess)

NP_F32_CONST = np.float32(42.0)


@gtscript.function
def _boolean_return(x):
    return x == 1.0


@gtscript.function
def _sinus(x):
    return sin(x)


@case()
def native_offset_arg_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = sin(a[1, 0, 0]) + cos(a)


@case()
def native_nested_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = min(abs(sin(a)), -0.5)  # the Python builtins' names, as the reference's own test


@case()
def native_in_function_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = _sinus(a) + 1.0


@case()
def native_not_isfinite_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = not isfinite(a)


@case()
def native_ternary_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = asin(a) + 1 if 1 < a else sin(a)


@case()
def native_dotted(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = gtscript.sin(a)


@case()
def native_wrong_arity(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = sin(a, a)


@case()
def function_call_in_if(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = 0.0
        if _boolean_return(a):
            b = 1.0


@case()
def abs_k_positional(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a.at(2)


@case()
def abs_k_with_i(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a.at(I=1, K=0)


@case()
def abs_k_iterator(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a.at(K=K)


@case()
def literal_casts_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(0, 1):
        b = float(0) + int(3) + a


@case()
def typed_temporaries_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        t32: float32 = 12.12
        t64: float64 = 34.34
        ti: int = 12
        b = t32 + t64 + ti + a


@case()
def numpy_typed_constant_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a + NP_F32_CONST


@case()
def k_iterator_read_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a + K


@case()
def k_iterator_condition_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a
        if K == 2:
            b = 42.0


@case()
def i_iterator_condition(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a
        if I == 2:
            b = 42.0


@case()
def while_loop_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        t = a
        while t < 10.0:
            t = t + 1.0
        b = t


@case()
def if_elif_else_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        if a > 1.0:
            b = 1.0
        elif a > 0.0:
            b = 2.0
        else:
            b = 3.0


@case()
def bool_ops_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = 1.0 if (a > 0.0 and a < 1.0) or not (a == 2.0) else 0.0


@case()
def power_ok(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = a**2 + a**0.5


@case()
def unsupported_lambda(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = (lambda x: x)(a)


@case()
def unsupported_list(a: F64, b: F64):
    with computation(PARALLEL), interval(...):
        b = [a, a][0]
