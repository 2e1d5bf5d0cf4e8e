"""Batched halo pack/unpack on the device (``include/gtmi_halo.h``, ``csrc/gtmi_halo.hip``).

One ``gtmi_halo_copy`` launch moves every face of an exchange phase between the strided fields
and the contiguous RCCL message buffers. Built once with hipcc into the in-tree cache like the
stencil libraries (``runtime/jit.py``); loaded through ctypes after torch (same HIP runtime).
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import List, Optional, Sequence, Tuple

from gt4py_amd.runtime import jit

_SRC = os.path.join(jit.CSRC_DIR, "gtmi_halo.hip")
_lock = threading.Lock()
_lib = None

MAX_BOXES = 64  # GTMI_HALO_MAX_BOXES


class GtmiBox(ctypes.Structure):
    _fields_ = [
        ("field", ctypes.c_void_p),
        ("strides", ctypes.c_int64 * 3),
        ("start", ctypes.c_int64 * 3),
        ("extent", ctypes.c_int64 * 3),
        ("buffer", ctypes.c_void_p),
        ("itemsize", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


def library_path() -> str:
    with open(_SRC) as f:
        return jit.compile_source(f.read())


def _library():
    global _lib
    with _lock:
        if _lib is None:
            import torch  # noqa: F401  (bind to torch's HIP runtime first)

            lib = ctypes.CDLL(library_path(), mode=ctypes.RTLD_LOCAL)
            lib.gtmi_halo_copy.restype = ctypes.c_int
            lib.gtmi_halo_copy.argtypes = [ctypes.POINTER(GtmiBox), ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p]
            lib.gtmi_halo_last_error.restype = ctypes.c_char_p
            lib.gtmi_halo_abi_version.restype = ctypes.c_int
            if lib.gtmi_halo_abi_version() != 1:
                raise RuntimeError("gtmi_halo ABI mismatch")
            _lib = lib
        return _lib


Box = Tuple[object, Tuple[int, int, int], Tuple[int, int, int], object]  # (field, start, extent, buffer)


class BatchedCopy:
    """Packs the ctypes descriptors of a fixed list of boxes once; ``run`` enqueues one launch per
    ``MAX_BOXES`` boxes (one launch for every exchange phase up to 64 faces, i.e. 8 fields with the
    diagonal scheme's 8 faces; more fields take further launches on the same stream)."""

    def __init__(self, boxes: Sequence[Box]):
        self.n = len(boxes)
        self.parts = []
        for c0 in range(0, self.n, MAX_BOXES):
            chunk = boxes[c0:c0 + MAX_BOXES]
            arr = (GtmiBox * len(chunk))()
            for b, (t, start, extent, buf) in zip(arr, chunk):
                if t.dim() != 3 or not buf.is_contiguous() or buf.numel() < extent[0] * extent[1] * extent[2]:
                    raise ValueError("halo boxes need 3-D fields and large-enough contiguous buffers")
                if buf.dtype != t.dtype:
                    raise TypeError("halo buffer dtype differs from the field's")
                b.field = t.data_ptr()
                b.strides[:] = t.stride()
                b.start[:] = start
                b.extent[:] = extent
                b.buffer = buf.data_ptr()
                b.itemsize = t.element_size()
            self.parts.append((arr, len(chunk)))

    def run(self, direction: int, stream=None) -> None:
        import torch

        if self.n == 0:
            return
        s = stream if stream is not None else torch.cuda.current_stream()
        for arr, n in self.parts:
            rc = _library().gtmi_halo_copy(arr, n, direction, ctypes.c_void_p(s.cuda_stream))
            if rc != 0:
                raise RuntimeError(f"gtmi_halo_copy failed: {_library().gtmi_halo_last_error().decode()}")


def slice_box(sl: Tuple[slice, slice], nk: int) -> Tuple[Tuple[int, int, int], Tuple[int, int, int]]:
    (si, sj) = sl
    return (si.start, sj.start, 0), (si.stop - si.start, sj.stop - sj.start, nk)


__all__: List[str] = ["BatchedCopy", "GtmiBox", "library_path", "slice_box"]
del Optional
