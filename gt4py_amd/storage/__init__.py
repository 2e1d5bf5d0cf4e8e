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


def _normalize_spec(aligned_index, shape, dtype, dimensions):
    """Validate the spec; a subarray dtype appends its shape as trailing data dimensions
    (aligned index 0 there), as ``storage/cartesian/utils.py:84-170`` does."""
    if not isinstance(shape, (tuple, list)) or not all(isinstance(s, numbers.Integral) for s in shape):
        raise TypeError("shape must be a sequence of integers")
    shape = tuple(int(s) for s in shape)
    if dimensions is None:
        dimensions = ("I", "J", "K")[: min(3, len(shape))] + tuple(str(d) for d in range(len(shape) - 3))
    dimensions = tuple(str(getattr(d, "__gt_axis_name__", d)) for d in dimensions)
    if not all(d.isdigit() or d in ("I", "J", "K") for d in dimensions):
        raise ValueError(f"Invalid dimensions definition: '{dimensions}'")
    if len(dimensions) != len(shape):
        raise ValueError(f"dimensions {dimensions} do not match shape {shape}")
    if any(s <= 0 for s in shape):
        raise ValueError(f"shape ({shape}) contains non-positive value.")
    if aligned_index is None:
        aligned_index = (0,) * len(shape)
    aligned_index = tuple(int(a) for a in aligned_index)
    if len(aligned_index) != len(shape):
        raise ValueError("aligned_index must have one entry per dimension")
    if any(a < 0 for a in aligned_index):
        raise ValueError("aligned_index must be non-negative")
    dtype = np.dtype(dtype)
    if dtype.shape:
        sub = tuple(dtype.shape)
        shape = shape + sub
        aligned_index = aligned_index + (0,) * len(sub)
        dimensions = dimensions + tuple(str(d) for d in range(len(sub)))
        dtype = dtype.base
    return aligned_index, shape, dtype, dimensions


def _allocation_plan(shape, layout_map, itemsize, alignment_bytes, aligned_index):
    """Padded strides (elements) and element offset of the aligned index (int64-safe)."""
    if alignment_bytes % itemsize:
        raise ValueError("alignment must be a multiple of the item size")
    align_el = max(1, alignment_bytes // itemsize)
    ndim = len(shape)
    if ndim == 0:
        return (), 0, 1, align_el
    order = sorted(range(ndim), key=lambda d: layout_map[d])  # slowest .. fastest
    fastest = order[-1]
    padded = list(shape)
    padded[fastest] = int(math.ceil(max(shape[fastest], 1) / align_el) * align_el)
    strides = make_strides(padded, layout_map)
    # shift so that aligned_index lands on an aligned address
    ai_off = sum(a * s for a, s in zip(aligned_index, strides))
    shift = (-ai_off) % align_el
    total = shift + sum((s - 1) * st for s, st in zip(padded, strides)) + 1 if all(padded) else shift + 1
    return tuple(strides), shift, total, align_el


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
    aligned_index, shape, dtype, dimensions = _normalize_spec(aligned_index, shape, dtype, dimensions)
    layout_map = info["layout_map"](dimensions)
    strides, shift, total, _ = _allocation_plan(
        shape, layout_map, dtype.itemsize, info["alignment"] * dtype.itemsize, aligned_index
    )
    if _device_of(info) == "gpu":
        import torch

        from gt4py_amd.runtime import device as dev

        tdtype = torch_dtype(dtype)
        buf = torch.empty(int(total), dtype=tdtype, device=dev.current_device())
        arr = torch.as_strided(buf, size=shape, stride=strides, storage_offset=int(shift))
    else:
        nbytes = int(total) * dtype.itemsize
        raw = np.empty(nbytes + 256, dtype=np.uint8)
        base_off = (-raw.ctypes.data) % 256
        flat = raw[base_off : base_off + nbytes].view(dtype)
        arr = np.lib.stride_tricks.as_strided(
            flat[shift:], shape=shape, strides=tuple(s * dtype.itemsize for s in strides)
        )
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

        arr.copy_(torch.from_numpy(np.ascontiguousarray(host)))


def to_numpy(arr) -> np.ndarray:
    """Copy any storage (numpy / torch, host or device) into a numpy array."""
    if isinstance(arr, np.ndarray):
        return arr.copy()
    if hasattr(arr, "detach"):
        return arr.detach().cpu().numpy()
    return np.asarray(arr)


_TORCH_DTYPES: Dict[np.dtype, Any] = {}


def torch_dtype(dtype):
    import torch

    dtype = np.dtype(dtype)
    table = {
        np.dtype(np.bool_): torch.bool,
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
    "array_info",
    "layout_maker_factory",
    "layout_checker_factory",
    "check_layout",
]
