"""ctypes binding of the C ABI in ``include/gtmi.h`` (no pybind11, no CuPy).

``load_library`` always imports torch first so that the generated library binds to the
same HIP runtime instance as torch (both resolve the SONAME ``libamdhip64.so.7``); the
stream handle passed to ``gtmi_stencil_run`` is then valid in both.
"""

from __future__ import annotations

import ctypes
import json
import threading
from typing import Dict

GTMI_ABI_VERSION = 3

DTYPE_IDS = {
    "bool": 10,
    "int8": 11,
    "int16": 12,
    "int32": 14,
    "int64": 18,
    "float32": 104,
    "float64": 108,
}


MAX_DATA_DIMS = 4  # GTMI_MAX_DATA_DIMS


class GtmiField(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("strides", ctypes.c_int64 * 3),
        ("origin", ctypes.c_int64 * 3),
        ("shape", ctypes.c_int64 * 3),
        ("dtype", ctypes.c_int32),
        ("ndim", ctypes.c_int32),
        ("n_data_dims", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
        ("data_strides", ctypes.c_int64 * MAX_DATA_DIMS),
        ("data_shape", ctypes.c_int64 * MAX_DATA_DIMS),
    ]


class GtmiScalar(ctypes.Union):
    _fields_ = [
        ("f64", ctypes.c_double),
        ("f32", ctypes.c_float),
        ("i64", ctypes.c_int64),
        ("i32", ctypes.c_int32),
        ("i16", ctypes.c_int16),
        ("i8", ctypes.c_int8),
        ("b", ctypes.c_uint8),
    ]


EXPORTED_SYMBOLS = ("gtmi_stencil_run", "gtmi_stencil_run_jsplit", "gtmi_stencil_signature", "gtmi_last_error",
                    "gtmi_abi_version")

_libs: Dict[str, "StencilLibrary"] = {}
_lock = threading.Lock()


class StencilLibrary:
    def __init__(self, path: str):
        import torch  # noqa: F401  (bind to torch's HIP runtime first, see module docstring)

        self.path = path
        self.lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        self.run = self.lib.gtmi_stencil_run
        self.run.restype = ctypes.c_int
        self.run.argtypes = [
            ctypes.POINTER(ctypes.c_int64),
            ctypes.POINTER(GtmiField),
            ctypes.c_int32,
            ctypes.POINTER(GtmiScalar),
            ctypes.c_int32,
            ctypes.c_void_p,
        ]
        self.run_jsplit = self.lib.gtmi_stencil_run_jsplit
        self.run_jsplit.restype = ctypes.c_int
        self.run_jsplit.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.c_int64, ctypes.c_int64] + self.run.argtypes[1:]
        self.lib.gtmi_last_error.restype = ctypes.c_char_p
        self.lib.gtmi_stencil_signature.restype = ctypes.c_char_p
        self.lib.gtmi_abi_version.restype = ctypes.c_int
        abi = self.lib.gtmi_abi_version()
        if abi != GTMI_ABI_VERSION:
            raise RuntimeError(f"{path}: ABI version {abi}, expected {GTMI_ABI_VERSION}")
        self.signature = json.loads(self.lib.gtmi_stencil_signature().decode())

    def last_error(self) -> str:
        return self.lib.gtmi_last_error().decode()


def load_library(path: str) -> StencilLibrary:
    with _lock:
        if path not in _libs:
            _libs[path] = StencilLibrary(path)
        return _libs[path]


def _to_bool(v) -> int:
    return 1 if v else 0


# dtype name -> (GtmiScalar member, Python conversion): the launcher's prepared scalar setters
SCALAR_SLOTS = {
    "float64": ("f64", float),
    "float32": ("f32", float),
    "int64": ("i64", int),
    "int32": ("i32", int),
    "int16": ("i16", int),
    "int8": ("i8", int),
    "bool": ("b", _to_bool),
}


def set_scalar(slot: GtmiScalar, dtype_name: str, value) -> None:
    if dtype_name == "float64":
        slot.f64 = float(value)
    elif dtype_name == "float32":
        slot.f32 = float(value)
    elif dtype_name == "int64":
        slot.i64 = int(value)
    elif dtype_name == "int32":
        slot.i32 = int(value)
    elif dtype_name == "int16":
        slot.i16 = int(value)
    elif dtype_name == "int8":
        slot.i8 = int(value)
    elif dtype_name == "bool":
        slot.b = 1 if value else 0
    else:
        raise TypeError(dtype_name)
