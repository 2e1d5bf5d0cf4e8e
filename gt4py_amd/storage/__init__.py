"""Backend-aware storage allocation (mirrors ``gt4py.storage``).

Reference: ``src/gt4py/storage/cartesian/interface.py:40-327`` (``empty/zeros/ones/full/
from_array``), ``layout_registry.py:13-122`` (per-backend ``LayoutInfo``),
``allocators.py:189-275`` (padding + aligned index). Differences, by design:

- device storages are **torch tensors on the ROCm device** (no CuPy), built with
  ``torch.as_strided`` over one flat allocation so the layout map and the aligned index hold;
- every size is a Python int (64-bit): the reference's ``allocators.py:215,223-225`` builds
  ``padded_shape`` from ``np.int32`` and overflows for >= 2 GiB.
"""

from __future__ import annotations

import math
import os
import numbers
from typing import Any, Callable, Dict, Optional, Sequence, Tuple

import numpy as np

from gt4py_amd.storage.layout import (
    LayoutInfo,
    check_layout,
    layout_checker_factory,
    layout_maker_factory,
    make_strides,
)

REGISTRY: Dict[str, LayoutInfo] = {}


def register(name: str, info: LayoutInfo) -> None:
    REGISTRY[name] = info


def from_name(name: str) -> Optional[LayoutInfo]:
    return REGISTRY.get(name)


def _error_on_invalid_preset(backend):
    if backend not in REGISTRY:
        raise RuntimeError(f"Storage preset '{backend}' is not registered.")


def normalize_storage_spec(aligned_index, shape, dtype, dimensions):
    """Homogeneous ``(aligned_index, shape, dtype, dimensions)``; the checks, their order and the
    error types of ``storage/cartesian/utils.py:84-167``. A subarray dtype appends its shape as
    trailing data dimensions (aligned index 0 there)."""
    if shape is None or isinstance(shape, (str, bytes)) or not isinstance(shape, Sequence):
        raise TypeError("shape must be an iterable of ints.")
    if dimensions is None:
        dimensions = ("I", "J", "K")[: min(3, len(shape))] + tuple(str(d) for d in range(len(shape) - 3))
    dimensions = tuple(getattr(d, "__gt_axis_name__", d) for d in dimensions)
    if not all(isinstance(d, str) and (d.isdigit() or d in ("I", "J", "K")) for d in dimensions):
        raise ValueError(f"Invalid dimensions definition: '{dimensions}'")
    if not all(isinstance(x, numbers.Integral) for x in shape):
        raise TypeError("shape must be an iterable of ints.")
    if len(shape) != len(dimensions):
        raise ValueError(
            f"Dimensions ({dimensions}) and shape ({tuple(shape)}) have non-matching sizes: "
            f"len(shape)={len(shape)} must equal len(dimensions)={len(dimensions)}."
        )
    shape = tuple(int(x) for x in shape)
    if any(x <= 0 for x in shape):
        raise ValueError(f"shape ({shape}) contains non-positive value.")
    if aligned_index is None:
        aligned_index = (0,) * len(shape)
    if (isinstance(aligned_index, (str, bytes)) or not isinstance(aligned_index, Sequence)
            or not all(isinstance(a, numbers.Integral) for a in aligned_index)):
        raise TypeError("aligned_index must be an iterable of ints.")
    if len(aligned_index) != len(shape):
        raise ValueError(
            f"Shape ({shape}) and aligned_index ({tuple(aligned_index)}) have non-matching sizes."
        )
    aligned_index = tuple(int(a) for a in aligned_index)
    if any(a < 0 for a in aligned_index):
        raise ValueError(f"aligned_index ({aligned_index}) contains negative value.")
    dtype = np.dtype(dtype)
    if dtype.shape:
        sub = tuple(dtype.shape)
        shape = shape + sub
        aligned_index = aligned_index + (0,) * len(sub)
        dimensions = dimensions + tuple(str(d) for d in range(len(sub)))
        dtype = dtype.base
    return aligned_index, shape, dtype, tuple(str(d) for d in dimensions)


_normalize_spec = normalize_storage_spec


def _allocation_plan(shape, layout_map, itemsize, alignment_bytes, aligned_index):
    """Padded element strides, element offset of the first element (so that ``aligned_index``
    lands on an ``alignment_bytes`` boundary when the buffer base does), total elements.
    64-bit Python ints throughout."""
    if alignment_bytes % itemsize:
        raise ValueError("alignment must be a multiple of the item size")
    align_el = max(1, alignment_bytes // itemsize)
    ndim = len(shape)
    if ndim == 0:
        return (), 0, 1, align_el
    fastest = max(range(ndim), key=lambda d: layout_map[d])
    padded = list(shape)
    padded[fastest] = int(math.ceil(max(shape[fastest], 1) / align_el) * align_el)
    strides = make_strides(padded, layout_map)
    ai_off = sum(a * st for a, st in zip(aligned_index, strides))
    shift = (-ai_off) % align_el
    total = shift + sum((n - 1) * st for n, st in zip(padded, strides)) + 1
    return tuple(strides), shift, total, align_el


def allocate_cpu(shape, layout_map, dtype, alignment_bytes, aligned_index):
    """``(raw byte buffer, ndarray view)``: ``layout_map`` orders the strides (highest rank
    contiguous), the contiguous dimension is padded to the alignment and ``aligned_index`` sits on
    an ``alignment_bytes`` boundary (``storage/cartesian/utils.py:232-248``)."""
    dtype = np.dtype(dtype)
    shape = tuple(int(x) for x in shape)
    aligned_index = tuple(aligned_index) if aligned_index is not None else (0,) * len(shape)
    strides, shift, total, _ = _allocation_plan(shape, layout_map, dtype.itemsize, alignment_bytes, aligned_index)
    raw = np.empty(total * dtype.itemsize + alignment_bytes, dtype=np.uint8)
    base = (-raw.ctypes.data) % alignment_bytes
    flat = raw[base : base + total * dtype.itemsize].view(dtype)
    arr = np.lib.stride_tricks.as_strided(
        flat[shift:], shape=shape, strides=tuple(st * dtype.itemsize for st in strides)
    )
    return raw, arr


# HBM placement of large fields: hipMalloc hands out 2 MiB-aligned blocks, so every
# large field starts at the same address residue modulo 2 MiB, and the K sweeps of the column
# kernels, which stream all their fields level by level, then collide on the same HBM channels
# (measured: tridiag 1.97 ms with equal residues, 1.86-1.89 ms when consecutive fields alternate
# bit 20 of the address; the plane kernels are insensitive). Large allocations therefore place
# their aligned element at (n mod 2) MiB modulo 2 MiB, n counting large allocations.
HBM_STAGGER_MIN_BYTES = 64 << 20
HBM_STAGGER_QUANTUM = 1 << 20
_stagger_count = 0


def hbm_stagger_residue(nbytes: int) -> Optional[int]:
    """Target address residue (modulo 2 quanta) of the next large device allocation, or None for
    small ones (and when ``GTMI_HBM_STAGGER=0``)."""
    global _stagger_count
    if nbytes < HBM_STAGGER_MIN_BYTES or os.environ.get("GTMI_HBM_STAGGER", "1") == "0":
        return None
    r = (_stagger_count % 2) * HBM_STAGGER_QUANTUM
    _stagger_count += 1
    return r


def staggered_device_buffer(n_elements: int, dtype, device):
    """A flat device tensor of ``n_elements`` whose first element follows the HBM stagger policy
    (scratch fields of the generated kernels)."""
    import torch

    dtype = np.dtype(dtype)
    residue = hbm_stagger_residue(n_elements * dtype.itemsize)
    if residue is None:
        return torch.empty(n_elements, dtype=torch_dtype(dtype), device=device)
    buf = torch.empty(n_elements + (2 * HBM_STAGGER_QUANTUM) // dtype.itemsize, dtype=torch_dtype(dtype), device=device)
    off = ((residue - buf.data_ptr()) % (2 * HBM_STAGGER_QUANTUM)) // dtype.itemsize
    return buf[off:off + n_elements]


def allocate_gpu(shape, layout_map, dtype, alignment_bytes, aligned_index):
    """``(flat device buffer, strided tensor view)`` on the current ROCm device, same layout rules
    as :func:`allocate_cpu` (the reference's CuPy ``allocate_gpu``, ``utils.py:251-316``); large
    fields are staggered in HBM (``hbm_stagger_residue``)."""
    import torch

    from gt4py_amd.runtime import device as dev

    dtype = np.dtype(dtype)
    shape = tuple(int(x) for x in shape)
    aligned_index = tuple(aligned_index) if aligned_index is not None else (0,) * len(shape)
    strides, shift, total, align_el = _allocation_plan(
        shape, layout_map, dtype.itemsize, alignment_bytes, aligned_index
    )
    # the stagger keeps the alignment only when the alignment divides its 2-quantum period (every
    # backend's 256 B does; an arbitrary alignment such as 152 B gets plain alignment)
    residue = hbm_stagger_residue(total * dtype.itemsize) if (2 * HBM_STAGGER_QUANTUM) % alignment_bytes == 0 else None
    extra = align_el if residue is None else (2 * HBM_STAGGER_QUANTUM) // dtype.itemsize + align_el
    buf = torch.empty(int(total + extra), dtype=torch_dtype(dtype), device=dev.current_device())
    if residue is None:
        base = ((-buf.data_ptr()) % alignment_bytes) // dtype.itemsize
    else:
        # the aligned element (flat index shift + ai_off, a multiple of the alignment) lands on an
        # address == residue (mod 2 quanta); the quantum is a multiple of the alignment
        ai_off = sum(int(a) * st for a, st in zip(aligned_index, strides))
        target = (residue - (buf.data_ptr() + (shift + ai_off) * dtype.itemsize)) % (2 * HBM_STAGGER_QUANTUM)
        base = target // dtype.itemsize
    arr = torch.as_strided(buf, size=shape, stride=strides, storage_offset=int(base + shift))
    return buf, arr


def _device_of(info: LayoutInfo) -> str:
    return info["device"]


def empty(
    shape: Sequence[int],
    dtype=np.float64,
    *,
    backend: str,
    aligned_index: Optional[Sequence[int]] = None,
    dimensions: Optional[Sequence[str]] = None,
):
    """Allocate uninitialized storage with the backend's optimal layout and alignment."""
    _error_on_invalid_preset(backend)
    info = REGISTRY[backend]
    aligned_index, shape, dtype, dimensions = normalize_storage_spec(aligned_index, shape, dtype, dimensions)
    layout_map = info["layout_map"](dimensions)
    alloc = allocate_gpu if _device_of(info) == "gpu" else allocate_cpu
    _, arr = alloc(shape, layout_map, dtype, info["alignment"] * dtype.itemsize, aligned_index)
    return arr


def zeros(shape, dtype=np.float64, *, backend, aligned_index=None, dimensions=None):
    arr = empty(shape, dtype, backend=backend, aligned_index=aligned_index, dimensions=dimensions)
    _fill(arr, 0)
    return arr


def ones(shape, dtype=np.float64, *, backend, aligned_index=None, dimensions=None):
    arr = empty(shape, dtype, backend=backend, aligned_index=aligned_index, dimensions=dimensions)
    _fill(arr, 1)
    return arr


def full(shape, fill_value, dtype=np.float64, *, backend, aligned_index=None, dimensions=None):
    arr = empty(shape, dtype, backend=backend, aligned_index=aligned_index, dimensions=dimensions)
    _fill(arr, fill_value)
    return arr


def from_array(data, dtype=np.float64, *, backend, aligned_index=None, dimensions=None):
    """Allocate with the backend's layout and copy ``data`` (numpy / torch / array-like) in.

    As ``storage/cartesian/interface.py:263-327``: ``dtype`` defaults to float64 (``None`` keeps
    the data's dtype); a subarray dtype ``(base, dims)`` takes its data dimensions from the
    trailing axes of ``data``, which must match ``dims``.
    """
    if hasattr(data, "detach") and hasattr(data, "cpu"):
        host = data.detach().cpu().numpy()
    else:
        host = np.asarray(data)
    dtype = np.dtype(host.dtype if dtype is None else dtype)
    shape = host.shape
    if dtype.shape:
        if tuple(shape[-dtype.ndim:]) != tuple(dtype.shape):
            raise ValueError(f"Incompatible data shape {shape} with dtype of shape {dtype.shape}.")
        shape = shape[: -dtype.ndim]
    arr = empty(shape, dtype, backend=backend, aligned_index=aligned_index, dimensions=dimensions)
    _copy_in(arr, host.astype(dtype.base, copy=False))
    return arr


def _fill(arr, value):
    if isinstance(arr, np.ndarray):
        arr[...] = value
    else:
        arr.fill_(value)


def _copy_in(arr, host: np.ndarray):
    if isinstance(arr, np.ndarray):
        arr[...] = host
    else:
        import torch

        arr.copy_(torch.from_numpy(np.array(host, order="C")))  # keeps 0-d shapes


def to_numpy(arr) -> np.ndarray:
    """Copy any storage (numpy / torch, host or device) into a numpy array."""
    if isinstance(arr, np.ndarray):
        return arr.copy()
    if hasattr(arr, "detach"):
        return arr.detach().cpu().numpy()
    return np.asarray(arr)


cpu_copy = to_numpy  # storage/cartesian/utils.py:170-175


_TORCH_DTYPES: Dict[np.dtype, Any] = {}


def torch_dtype(dtype):
    import torch

    dtype = np.dtype(dtype)
    table = {
        np.dtype(np.bool_): torch.bool,
        np.dtype(np.uint8): torch.uint8,
        np.dtype(np.uint16): torch.uint16,
        np.dtype(np.uint32): torch.uint32,
        np.dtype(np.uint64): torch.uint64,
        np.dtype(np.float16): torch.float16,
        np.dtype(np.int8): torch.int8,
        np.dtype(np.int16): torch.int16,
        np.dtype(np.int32): torch.int32,
        np.dtype(np.int64): torch.int64,
        np.dtype(np.float32): torch.float32,
        np.dtype(np.float64): torch.float64,
    }
    return table[dtype]


def numpy_dtype_of(arr) -> np.dtype:
    dt = arr.dtype
    if isinstance(dt, np.dtype):
        return dt
    import torch

    table = {
        torch.bool: np.bool_,
        torch.uint8: np.uint8,
        torch.uint16: np.uint16,
        torch.uint32: np.uint32,
        torch.uint64: np.uint64,
        torch.float16: np.float16,
        torch.int8: np.int8,
        torch.int16: np.int16,
        torch.int32: np.int32,
        torch.int64: np.int64,
        torch.float32: np.float32,
        torch.float64: np.float64,
    }
    return np.dtype(table[dt])


def array_info(obj) -> Tuple[Any, Optional[Tuple[str, ...]], Optional[Tuple[int, ...]]]:
    """(array, __gt_dims__, __gt_origin__) for a stencil argument (``storage/cartesian/utils.py:176-215``)."""
    dims = getattr(obj, "__gt_dims__", None)
    origin = getattr(obj, "__gt_origin__", None)
    array = obj
    if not isinstance(obj, np.ndarray) and not _is_torch(obj):
        if hasattr(obj, "__cuda_array_interface__"):
            import torch

            array = torch.as_tensor(obj, device="cuda")
        elif hasattr(obj, "__array_interface__") or hasattr(obj, "__array__"):
            array = np.asarray(obj)
        else:
            raise TypeError(f"Unsupported field argument of type {type(obj)}")
    if dims is not None:
        dims = tuple(str(d) for d in dims)
    if origin is not None:
        origin = tuple(int(o) for o in origin)
    return array, dims, origin


def _is_torch(obj) -> bool:
    mod = type(obj).__module__
    return mod.startswith("torch")


__all__ = [
    "REGISTRY",
    "register",
    "from_name",
    "empty",
    "zeros",
    "ones",
    "full",
    "from_array",
    "to_numpy",
    "cpu_copy",
    "normalize_storage_spec",
    "allocate_cpu",
    "allocate_gpu",
    "array_info",
    "layout_maker_factory",
    "layout_checker_factory",
    "check_layout",
]
