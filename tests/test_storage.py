"""Storage allocator contract (reference ``tests/storage_tests/unit_tests/test_interface.py``):
layout/alignment/aligned-index properties of the raw allocators, spec normalisation errors,
constructors per backend (numpy arrays on the host, torch tensors on the ROCm device)."""

import random

import hypothesis as hyp
import hypothesis.strategies as st
import numpy as np
import pytest

from gt4py_amd import gtscript, storage
from gt4py_amd.backend import REGISTRY

CPU_BACKENDS = [n for n, b in REGISTRY.items() if b.storage_info["device"] == "cpu"]
GPU_BACKENDS = [pytest.param(n, marks=pytest.mark.gpu) for n, b in REGISTRY.items()
                if b.storage_info["device"] == "gpu"]
ALL_DTYPES = [np.int8, np.int16, np.int32, np.int64, np.uint8, np.uint16, np.uint32, np.uint64,
              np.float16, np.float32, np.float64]
# torch on ROCm implements element writes for these (uint16/32/64 tensors are storage-only there)
GPU_DTYPES = [np.int8, np.int16, np.int32, np.int64, np.uint8, np.float16, np.float32, np.float64]
SETTINGS = hyp.settings(max_examples=60, deadline=None, suppress_health_check=list(hyp.HealthCheck))


def _alloc_case(dtypes):
    @st.composite
    def strat(draw):
        dtype = np.dtype(draw(st.sampled_from(dtypes)))
        ndim = draw(st.integers(1, 4))
        shape = tuple(draw(st.integers(1, 64)) for _ in range(ndim))
        aligned = tuple(draw(st.integers(0, min(32, n - 1))) for n in shape)
        return dict(
            dtype=dtype, alignment=draw(st.integers(1, 64)) * dtype.itemsize, shape=shape, aligned_index=aligned,
            layout=tuple(draw(st.permutations(range(ndim)))),
        )

    return strat()


def _check_layout_properties(arr, case, addr_of, write):
    shape, aligned, layout = case["shape"], case["aligned_index"], case["layout"]
    fastest = int(np.argmax(layout))
    rnd = random.Random(0)
    # the first compute point of every "column" along the contiguous dimension is aligned
    for _ in range(100):
        sl = tuple(slice(aligned[d], None) if d == fastest else slice(rnd.randint(0, shape[d] - 1), None)
                   for d in range(len(shape)))
        assert addr_of(arr[sl]) % case["alignment"] == 0
    for idx in ((0,) * len(shape), aligned, tuple(n - 1 for n in shape)):
        write(arr, idx)
    with pytest.raises(IndexError):
        write(arr, tuple(shape))
    assert tuple(arr.shape) == shape


@SETTINGS
@hyp.given(case=_alloc_case(ALL_DTYPES))
def test_allocate_cpu(case):
    raw, arr = storage.allocate_cpu(case["shape"], case["layout"], case["dtype"], case["alignment"],
                                    case["aligned_index"])
    lo, hi = np.lib.array_utils.byte_bounds(arr)
    rlo, rhi = np.lib.array_utils.byte_bounds(raw)
    assert rlo <= lo and hi <= rhi

    def write(a, idx):
        a[idx] = 1

    _check_layout_properties(arr, case, lambda a: a.ctypes.data, write)


@pytest.mark.gpu
@SETTINGS
@hyp.given(case=_alloc_case(GPU_DTYPES))
def test_allocate_gpu(case):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    buf, arr = storage.allocate_gpu(case["shape"], case["layout"], case["dtype"], case["alignment"],
                                    case["aligned_index"])
    assert arr.is_cuda and arr.untyped_storage().data_ptr() == buf.untyped_storage().data_ptr()
    last = tuple(n - 1 for n in case["shape"])
    end = buf.data_ptr() + buf.numel() * buf.element_size()
    assert arr.data_ptr() >= buf.data_ptr() and arr[last].data_ptr() + arr.element_size() <= end

    def write(a, idx):
        if any(i >= n for i, n in zip(idx, a.shape)):
            raise IndexError(idx)  # torch raises IndexError too; checked explicitly to stay on the host
        a[idx] = 1

    _check_layout_properties(arr, case, lambda a: a.data_ptr(), write)
    with pytest.raises(IndexError):
        arr[tuple(case["shape"])] = 1


class TestNormalizeStorageSpec:
    def test_normal(self):
        out = storage.normalize_storage_spec((0, 0, 0), (10, 10, 10), np.float64, ("I", "J", "K"))
        assert out == ((0, 0, 0), (10, 10, 10), np.dtype(np.float64), ("I", "J", "K"))

    def test_aligned_index(self):
        shape, dims = (10, 10, 10), ("I", "J", "K")
        assert storage.normalize_storage_spec((1, 1, 1), shape, np.float64, dims)[0] == (1, 1, 1)
        assert storage.normalize_storage_spec(None, shape, np.float64, dims)[0] == (0, 0, 0)
        with pytest.raises(TypeError, match="aligned_index"):
            storage.normalize_storage_spec(("1", "1", "1"), shape, np.float64, dims)
        with pytest.raises(ValueError, match="aligned_index"):
            storage.normalize_storage_spec((1, 1, 1, 1), shape, np.float64, dims)
        with pytest.raises(ValueError, match="aligned_index"):
            storage.normalize_storage_spec((-1, -1, -1), shape, np.float64, dims)

    def test_shape(self):
        out = storage.normalize_storage_spec((0, 0), (10, 10), np.float64, ("I", "J"))
        assert out == ((0, 0), (10, 10), np.dtype(np.float64), ("I", "J"))
        with pytest.raises(ValueError, match="non-matching"):
            storage.normalize_storage_spec((0, 0), (10, 20), np.float64, ("J",))
        with pytest.raises(TypeError, match="shape"):
            storage.normalize_storage_spec((0, 0), "(10,10)", np.float64, ("I", "J", "K"))
        with pytest.raises(TypeError, match="shape"):
            storage.normalize_storage_spec((0, 0), None, np.float64, ("I", "J", "K"))
        with pytest.raises(ValueError, match="shape"):
            storage.normalize_storage_spec((0, 0, 0), (10, 10, 0), np.float64, ("I", "J", "K"))

    def test_dimensions(self):
        assert storage.normalize_storage_spec((0, 0), (10, 10), np.float64, "IJ")[3] == ("I", "J")
        assert storage.normalize_storage_spec((0, 0), (10, 10), np.float64, gtscript.IJ)[3] == ("I", "J")
        assert storage.normalize_storage_spec((0, 0, 0), (10, 10, 10), np.float64, gtscript.IJK)[3] == (
            "I", "J", "K")
        assert storage.normalize_storage_spec(None, (4, 4, 4, 2), np.float64, None)[3] == ("I", "J", "K", "0")
        with pytest.raises(ValueError, match="imensions"):
            storage.normalize_storage_spec((0, 0), (10, 10), np.float64, ())
        with pytest.raises(ValueError, match="dimensions"):
            storage.normalize_storage_spec((0, 0), (10, 10), np.float64, ("I", "X"))

    def test_dtype(self):
        out = storage.normalize_storage_spec((0, 0, 0), (10, 10, 10), (np.float64, (2,)), ("I", "J", "K"))
        assert out == ((0, 0, 0, 0), (10, 10, 10, 2), np.dtype(np.float64), ("I", "J", "K", "0"))


def _full7(*, dtype, aligned_index, shape, backend):
    return storage.full(shape, 7, dtype, backend=backend, aligned_index=aligned_index)


def _from_array7(*, dtype, aligned_index, shape, backend):
    return storage.from_array(np.full(shape, 7, dtype=dtype), dtype, backend=backend, aligned_index=aligned_index)


CONSTRUCTORS = [storage.empty, storage.ones, storage.zeros, _full7, _from_array7]


def _is_device_tensor(x):
    import torch

    return isinstance(x, torch.Tensor) and x.is_cuda


@pytest.mark.parametrize("ctor", CONSTRUCTORS)
@pytest.mark.parametrize("backend", CPU_BACKENDS)
def test_cpu_constructor(ctor, backend):
    s = ctor(dtype=np.float64, aligned_index=(1, 2, 3), shape=(2, 4, 6), backend=backend)
    assert s.shape == (2, 4, 6) and isinstance(s, np.ndarray)
    s0 = ctor(shape=(), dtype=np.float64, backend=backend, aligned_index=())
    assert s0.shape == () and isinstance(s0, np.ndarray)


@pytest.mark.parametrize("ctor", CONSTRUCTORS)
@pytest.mark.parametrize("backend", GPU_BACKENDS)
def test_gpu_constructor(ctor, backend):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    s = ctor(dtype=np.float64, aligned_index=(1, 2, 3), shape=(2, 4, 6), backend=backend)
    assert tuple(s.shape) == (2, 4, 6) and _is_device_tensor(s)
    if ctor in (_full7, _from_array7):
        assert bool((s == 7).all())
    # I-first layout, the aligned index on a 256-B boundary
    assert s.stride(0) == 1 and (s[1:, 2:, 3:].data_ptr() % 256) == 0
    s0 = ctor(shape=(), dtype=np.float64, backend=backend, aligned_index=())
    assert tuple(s0.shape) == () and _is_device_tensor(s0)


@pytest.mark.gpu
@SETTINGS
@hyp.given(data=st.data())
def test_masked_storage_gpu(data):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    ndim = data.draw(st.integers(1, 6))
    shape = tuple(data.draw(st.integers(1, 32)) for _ in range(ndim))
    aligned = tuple(data.draw(st.integers(0, min(32, n - 1))) for n in shape)
    mask = data.draw(st.one_of(st.just(None), st.permutations([True] * ndim + [False] * max(0, 3 - ndim))))
    dims = None
    if mask is not None:
        names = ["I", "J", "K"] + [str(d) for d in range(max(0, ndim - 3))]
        dims = [d for m, d in zip(mask, names) if m]
    a = storage.empty(shape, np.float64, backend="gt:mi355x", aligned_index=aligned, dimensions=dims)
    assert _is_device_tensor(a) and a.ndim == ndim


def test_masked_storage_asserts():
    with pytest.raises(ValueError):
        storage.empty((2, 2, 2), np.float64, backend="numpy", aligned_index=(1, 1, 1), dimensions=())


def test_non_existing_backend():
    with pytest.raises(RuntimeError, match="backend"):
        storage.empty([10, 10, 10], (np.float64, (3,)), backend="non_existing_backend", aligned_index=[0, 0, 0])


@pytest.mark.parametrize("backend", CPU_BACKENDS)
def test_from_array_data_dims(backend):
    host = np.arange(4 * 3 * 2 * 2, dtype=np.float64).reshape(4, 3, 2, 2)
    s = storage.from_array(host, (np.float64, (2,)), backend=backend)
    assert s.shape == (4, 3, 2, 2) and np.array_equal(s, host)
    with pytest.raises(ValueError, match="Incompatible"):
        storage.from_array(host, (np.float64, (3,)), backend=backend)
    assert storage.from_array(np.arange(6).reshape(1, 2, 3), backend=backend).dtype == np.float64
    assert storage.from_array(np.arange(6).reshape(1, 2, 3), None, backend=backend).dtype == np.arange(1).dtype


def test_hbm_stagger_policy_cpu():
    """Large device allocations alternate their 1 MiB residue; small ones are left alone."""
    from gt4py_amd import storage as gs

    start = gs._stagger_count
    assert gs.hbm_stagger_residue(1 << 20) is None
    rs = [gs.hbm_stagger_residue(gs.HBM_STAGGER_MIN_BYTES) for _ in range(4)]
    assert rs == [((start + q) % 2) * gs.HBM_STAGGER_QUANTUM for q in range(4)]


@pytest.mark.gpu
def test_hbm_stagger_device_addresses():
    """The aligned elements of consecutive large gt:mi355x storages alternate address bit 20
     and stay aligned; the data round-trips."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage as gs

    shape = (1030, 1024, 16)  # > 64 MiB in f64 with the I padding
    arrs = [gs.empty(shape, np.float64, backend="gt:mi355x", aligned_index=(2, 2, 0)) for _ in range(4)]
    addrs = [a[2:, 2:, :].data_ptr() for a in arrs]
    bits = [(p >> 20) & 1 for p in addrs]
    assert all(p % 256 == 0 for p in addrs)
    assert all(bits[q] != bits[q + 1] for q in range(3)), [hex(p) for p in addrs]
    host = np.random.default_rng(0).uniform(size=shape)
    a = gs.from_array(host, backend="gt:mi355x", aligned_index=(2, 2, 0))
    assert np.array_equal(gs.to_numpy(a), host)
