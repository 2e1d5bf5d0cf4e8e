"""More of the reference's ``multi_feature_tests/test_code_generation.py``, restated.

Each test follows the reference test of the same name (file:line in its docstring) with the
same stencil, inputs and expected values, on the ``numpy`` backend (CPU) and on ``gt:mi355x``
(GPU). Build-time errors are checked on both backends without a GPU: they are raised while the
stencil is generated, before any device work.
"""

import numpy as np
import pytest

from gt4py_amd import gtscript, storage
from gt4py_amd.gtscript import FORWARD, IJ, PARALLEL, Field, I, J, K, computation, interval

REF = "tests/cartesian_tests/integration_tests/multi_feature_tests/test_code_generation.py"
BACKENDS = [pytest.param("numpy", id="numpy"), pytest.param("gt:mi355x", id="gt:mi355x", marks=pytest.mark.gpu)]
BUILD_BACKENDS = ["numpy", "gt:mi355x"]


@pytest.fixture(params=BACKENDS)
def backend(request):
    if storage.from_name(request.param)["device"] == "gpu":
        import torch

        if not torch.cuda.is_available():
            pytest.skip("no ROCm device")
    return request.param


def cpu(x):
    return storage.to_numpy(x)


def test_input_order(backend):
    """REF:364-383 -- a scalar parameter between two fields keeps its position."""

    @gtscript.stencil(backend=backend)
    def stencil(in_field: Field[np.float64], parameter: np.float64, out_field: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            out_field[0, 0, 0] = in_field * parameter

    field_in = storage.ones((23, 23, 23), np.float64, backend=backend, aligned_index=(0, 0, 0))
    field_out = storage.zeros((23, 23, 23), np.float64, backend=backend, aligned_index=(0, 0, 0))
    stencil(field_in, 3.1415, field_out)
    np.testing.assert_allclose(cpu(field_out), 3.1415)


def test_function_inline_in_while(backend):
    """REF:1112-1133 -- a gtscript.function inlined in a while loop body."""

    @gtscript.function
    def add_42(v):
        return v + 42

    @gtscript.stencil(backend=backend)
    def test(in_field: Field[np.float64], out_field: Field[np.float64]):
        with computation(PARALLEL), interval(...):
            count = 1
            while count < 10:
                sa = add_42(out_field)
                out_field = in_field + sa
                count = count + 1

    domain = (5, 5, 2)
    in_arr = storage.ones(domain, np.float64, backend=backend)
    out_arr = storage.ones(domain, np.float64, backend=backend)
    test(in_arr, out_arr)
    assert (cpu(out_arr) == 388.0).all()


def test_upcasting_both_sides_of_assignment(backend):
    """REF:1604-1619 -- int32 index field in a written K offset (FORWARD)."""
    domain = (5, 5, 5)
    inp = storage.ones(domain, np.float64, backend=backend)
    output = storage.zeros(domain, np.float64, backend=backend)
    index_array = storage.ones((domain[0], domain[1]), np.int32, backend=backend)

    @gtscript.stencil(backend=backend)
    def test_upcasting_stencil(in_field: Field[np.float64], index_field: Field[IJ, np.int32],
                               out_field: Field[np.float64]) -> None:
        with computation(FORWARD), interval(...):
            out_field[0, 0, index_field - 1] = in_field

    test_upcasting_stencil(inp, index_array, output)
    assert (cpu(inp) == cpu(output)).all()


def test_upcasting_leave_integer_power_arguments_alone(backend):
    """REF:1623-1639 -- ``float32 ** int32`` keeps the integer exponent (the reference runs it on
    ``debug`` only and checks that it builds and runs); here the values are checked too."""
    domain = (5, 5, 5)
    inp = storage.full(domain, 3.0, np.float32, backend=backend)
    output = storage.zeros(domain, np.float32, backend=backend)
    squared = storage.full((domain[0], domain[1]), 2, np.int32, backend=backend)

    @gtscript.stencil(backend=backend)
    def test_upcasting_stencil(in_field: Field[np.float32], squared: Field[IJ, np.int32],
                               out_field: Field[np.float32]) -> None:
        with computation(FORWARD), interval(...):
            out_field = in_field**squared

    test_upcasting_stencil(inp, squared, output)
    assert (cpu(output) == 9.0).all()


def test_reset_mask_2d(backend):
    """REF:1737-1755 -- an IJ field written in a one-level FORWARD interval."""
    domain = (5, 5, 5)
    inp = storage.ones(domain, np.float64, backend=backend)
    output = storage.zeros(domain, np.float64, backend=backend)
    mask_2d = storage.ones((domain[0], domain[1]), np.int32, backend=backend)

    @gtscript.stencil(backend=backend)
    def test_set_2d_mask(dp1: Field[np.float64], pe1: Field[np.float64], lev: Field[IJ, np.int32]) -> None:
        with computation(PARALLEL), interval(0, -1):
            dp1 = pe1[0, 0, 1] - pe1
        with computation(FORWARD), interval(0, 1):
            lev = 0

    test_set_2d_mask(output, inp, mask_2d)
    assert (cpu(mask_2d) == 0).all()
    assert (cpu(output)[:, :, :-1] == 0).all()


def test_2d_temporaries(backend):
    """REF:1536-1578 -- IJ temporaries, declared with a field type or through ``dtypes``."""
    domain = (5, 5, 3)
    in_arr = storage.ones(domain, np.float64, backend=backend)
    out_arr = storage.zeros(domain, np.float64, backend=backend)

    @gtscript.stencil(backend=backend)
    def test_with_plain_gt4py(in_field: Field[np.float64], out_field: Field[np.float64]) -> None:
        with computation(FORWARD), interval(0, 1):
            tmp_2D: Field[IJ, np.float64] = 0
        with computation(FORWARD), interval(...):
            tmp_2D = tmp_2D + in_field
        with computation(FORWARD), interval(...):
            out_field = tmp_2D

    @gtscript.stencil(backend=backend, dtypes={"MyFancySymbol": Field[IJ, np.float64]})
    def test_with_user_dtype(in_field: Field[np.float64], out_field: Field[np.float64]) -> None:
        with computation(FORWARD), interval(0, 1):
            tmp_2D: MyFancySymbol = 0  # noqa: F821
        with computation(FORWARD), interval(...):
            out_field = tmp_2D

    test_with_plain_gt4py(in_arr, out_arr)
    assert (cpu(out_arr) == domain[2]).all()

    out_arr = storage.full(domain, 9.0, np.float64, backend=backend)
    test_with_user_dtype(in_arr, out_arr)
    assert (cpu(out_arr) == 0).all()


@pytest.mark.parametrize("backend", BUILD_BACKENDS)
def test_typed_temporaries_must_be_ij(backend):
    """REF:1566-1578 -- a typed temporary on K only is a syntax error."""
    from gt4py_amd.frontend import GTScriptSyntaxError

    with pytest.raises(GTScriptSyntaxError, match="Typed temporaries must be IJ,"):

        @gtscript.stencil(backend=backend)
        def test_failing_on_non_IJ(in_field: Field[np.float64], out_field: Field[np.float64]) -> None:
            with computation(FORWARD), interval(0, 1):
                tmp_2D: Field[K, np.float64] = 0
            with computation(FORWARD), interval(...):
                out_field = tmp_2D


@pytest.mark.parametrize("backend", BUILD_BACKENDS)
def test_runtime_interval_raises(backend):
    """REF:1455-1524 -- run-time interval bounds (scalar, IJ field, IJ temporary) are not
    implemented by numpy / gt:* (``NotImplementedError``)."""
    with pytest.raises(NotImplementedError):

        @gtscript.stencil(backend=backend)
        def test_stencil(out_field: Field[np.float64], input_data: Field[np.float64],
                         index_data: Field[IJ, np.int64], scalar_arg: int):
            with computation(FORWARD), interval(0, 1):
                temporary: Field[IJ, np.float64] = 7
            with computation(PARALLEL), interval(0, scalar_arg):
                out_field = input_data
            with computation(PARALLEL), interval(0, index_data):
                out_field = input_data[0, 0, 0]
            with computation(PARALLEL), interval(0, temporary):
                out_field[0, 0, 0] = input_data[0, 0, 0]


@pytest.mark.parametrize("backend", BUILD_BACKENDS)
def test_no_write_and_read_with_horizontal_offset(backend):
    """REF:1642-1657."""
    with pytest.raises(ValueError, match="Self-assignment with offset in I or J is illegal."):

        @gtscript.stencil(backend=backend)
        def self_assign_offset(field: Field[np.float64]) -> None:
            with computation(PARALLEL), interval(...):
                field = (field[I - 1] + field[I + 1]) / 2

    with pytest.raises(ValueError, match="Illegal write and read with horizontal offset"):

        @gtscript.stencil(backend=backend)
        def self_assign_offset2(field: Field[np.float64]) -> None:
            with computation(PARALLEL), interval(...):
                tmp = (field[J - 1] + field[J + 1]) / 2
                field = tmp * 2


@pytest.mark.parametrize("backend", BUILD_BACKENDS)
def test_temporary_declared_in_definition_order(backend):
    """A temporary belongs to the interval block that assigns it FIRST IN THE DEFINITION
    (gtc/gtir.py:226-240: each block is a GTIR VerticalLoop with its own ``temporaries``),
    whatever the statements of a later block do: here ``tmp`` is declared by the lower block, so
    the upper block, defined later, writes it and reads it at an I offset -- rejected (checked
    against the reference itself; blocks must also be listed in execution order, which the
    reference enforces first, tests/frontend_cases.py)."""
    with pytest.raises(ValueError, match="Illegal write and read with horizontal offset"):

        @gtscript.stencil(backend=backend)
        def declared_later(a: Field[np.float64], b: Field[np.float64]) -> None:
            with computation(PARALLEL):
                with interval(0, 1):
                    tmp = a
                    b = tmp
                with interval(1, None):
                    tmp = a * 2
                    b = tmp[1, 0, 0]

    # defined the other way round the lower block declares tmp and may read it at an offset
    @gtscript.stencil(backend=backend)
    def declared_first(a: Field[np.float64], b: Field[np.float64]) -> None:
        with computation(PARALLEL):
            with interval(0, 1):
                tmp = a
                b = tmp[1, 0, 0]
            with interval(1, None):
                tmp = a * 2
                b = tmp


@pytest.mark.parametrize("backend", BUILD_BACKENDS)
def test_k_offsets_in_parallel_loops(backend):
    """REF:1660-1720 -- writes and K-offset reads of one field in a PARALLEL loop."""
    with pytest.raises(ValueError, match="write and read with k-offsets in PARALLEL"):

        @gtscript.stencil(backend=backend)
        def self_assign_offset_parallel(field: Field[np.int32]) -> None:
            with computation(PARALLEL), interval(1, None):
                field = field[K - 1] * 2

    with pytest.raises(ValueError, match="write and read with k-offsets in PARALLEL"):

        @gtscript.stencil(backend=backend)
        def self_assign_offset_parallel_temp(field: Field[np.int32]) -> None:
            with computation(PARALLEL), interval(1, None):
                tmp = field[K - 1]
                field = tmp * 2

    with pytest.raises(ValueError, match="write and read with `VariableKOffset` and/or `AbsoluteKIndex`"):

        @gtscript.stencil(backend=backend)
        def mixed_read_write(field: Field[np.int32]):
            with computation(PARALLEL), interval(...):
                level = field.at(K=1)
                field = 2 * level

    with pytest.raises(ValueError, match="write and read with `VariableKOffset` and/or `AbsoluteKIndex`"):

        @gtscript.stencil(backend=backend)
        def mixed_read_write2(field: Field[np.int32], offset: int = -1):
            with computation(PARALLEL), interval(1, None):
                bottom = field[0, 0, offset]
                field = field + 2 * bottom

    # allowed: center reads and writes, no mixing, static one-level intervals
    @gtscript.stencil(backend=backend)
    def self_assignment_center_read_parallel(field: Field[np.int32]) -> None:
        with computation(PARALLEL), interval(...):
            field = field[0, 0, 0] * 2

    @gtscript.stencil(backend=backend)
    def self_assignment_center_write_parallel(field: Field[np.int32]) -> None:
        with computation(PARALLEL), interval(...):
            field[0, 0, 0] = field * 2

    @gtscript.stencil(backend=backend)
    def self_assignment_center_parallel(field: Field[np.float32], index: Field[np.int32]) -> None:
        with computation(PARALLEL), interval(1, None):
            field = index + index[K - 1] * 2

    @gtscript.stencil(backend=backend)
    def the_stencil(field: Field[np.bool_]) -> None:
        with computation(PARALLEL):
            with interval(0, 1):
                field = field[K + 1]
            with interval(-1, None):
                field = field[K - 1]


def test_self_assignment_in_forward(backend):
    """REF:1722-1733 -- K-offset self reads are fine in a FORWARD loop (the reference only builds
    them; here they also run: field[k] = 2 * field[k-1])."""

    @gtscript.stencil(backend=backend)
    def self_assignment_parallel(field: Field[np.int32]) -> None:
        with computation(FORWARD), interval(1, None):
            field = field[K - 1] * 2

    @gtscript.stencil(backend=backend)
    def self_assignment_2_parallel(field: Field[np.int32]) -> None:
        with computation(FORWARD), interval(1, None):
            tmp = field[K - 1]
            field = tmp * 2

    for st in (self_assignment_parallel, self_assignment_2_parallel):
        f = storage.ones((3, 2, 6), np.int32, backend=backend)
        st(f)
        assert (cpu(f) == 2 ** np.arange(6)[None, None, :]).all()


def test_size_one_parallel_k_offsets(backend):
    """REF:1711-1718 builds ``the_stencil``; here it runs: one-level PARALLEL intervals read the
    field they write at a K offset (levels 0 and nk-1 only are written). The expected columns
    ([1, 1] for nk=2, [1, 1, 2, 3, 3] for nk=5) are what the reference numpy backend returns."""

    @gtscript.stencil(backend=backend)
    def the_stencil(field: Field[np.float64]) -> None:
        with computation(PARALLEL):
            with interval(0, 1):
                field = field[K + 1]
            with interval(-1, None):
                field = field[K - 1]

    for nk in (2, 5):
        f = storage.from_array(np.broadcast_to(np.arange(nk, dtype=np.float64), (4, 3, nk)).copy(), backend=backend)
        the_stencil(f)
        want = np.arange(nk, dtype=np.float64)
        want[0] = 1.0
        want[-1] = 1.0 if nk == 2 else nk - 2.0  # sections run in order: nk=2 reads the new level 0
        assert (cpu(f) == want[None, None, :]).all(), (nk, cpu(f)[0, 0])
