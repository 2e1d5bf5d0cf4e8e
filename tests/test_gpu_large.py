"""Fields beyond 2**31 elements on MI355X (288 GB HBM): every address computation of the plane
and column kernels is 64-bit (the reference's storage path overflows int32 at >= 2 GiB,
SURVEY.md §6). Checked on the device against exact references (integer-valued data: the f64
results are exact, so bit-equality is the test)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from gt4py_amd.gtscript import FORWARD, PARALLEL, Field, computation, interval

SHAPE = (2048, 1024, 1040)  # 2.18e9 elements, 17.4 GB per f64 field


def copy_big(a: Field[np.float64], b: Field[np.float64]):
    with computation(PARALLEL), interval(...):
        b = a[0, 0, 0]


def prefix_sum(a: Field[np.float64], s: Field[np.float64]):
    with computation(FORWARD):
        with interval(0, 1):
            s = a[0, 0, 0]
        with interval(1, None):
            s = s[0, 0, -1] + a[0, 0, 0]


def _torch():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    return torch


def _pattern(torch, shape):
    from gt4py_amd import storage

    a = storage.empty(shape, np.float64, backend="gt:mi355x")
    ni, nj, nk = shape
    i = torch.arange(ni, device="cuda", dtype=torch.float64).view(ni, 1)
    j = torch.arange(nj, device="cuda", dtype=torch.float64).view(1, nj)
    for k in range(nk):  # plane by plane: no field-sized temporaries
        a[:, :, k] = torch.remainder(i + 3 * j + 7 * k, 11.0)
    return a


def test_plane_copy_beyond_int32():
    torch = _torch()
    from gt4py_amd import gtscript, storage

    assert SHAPE[0] * SHAPE[1] * SHAPE[2] > 2**31
    st = gtscript.stencil(backend="gt:mi355x", definition=copy_big, name="large.copy")
    a = _pattern(torch, SHAPE)
    b = storage.zeros(SHAPE, np.float64, backend="gt:mi355x")
    st(a, b)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    del a, b
    torch.cuda.empty_cache()


def test_column_sweep_beyond_int32():
    torch = _torch()
    from gt4py_amd import gtscript, storage

    st = gtscript.stencil(backend="gt:mi355x", definition=prefix_sum, name="large.prefix_sum")
    a = _pattern(torch, SHAPE)
    s = storage.zeros(SHAPE, np.float64, backend="gt:mi355x")
    st(a, s)
    torch.cuda.synchronize()
    # integer partial sums < 2**53: exact in any order, so torch.cumsum is an exact reference
    ok = True
    carry = torch.zeros(SHAPE[:2], device="cuda", dtype=torch.float64)
    for k0 in range(0, SHAPE[2], 128):  # compare in K slabs (bounded temporaries)
        k1 = min(SHAPE[2], k0 + 128)
        ref = torch.cumsum(a[:, :, k0:k1], dim=2) + carry[:, :, None]
        ok = ok and torch.equal(ref, s[:, :, k0:k1])
        carry = ref[:, :, -1].clone()
        del ref
    assert ok
    del a, s
    torch.cuda.empty_cache()
