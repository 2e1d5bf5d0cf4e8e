"""ctypes binding of ``oracle/cpu_stencils.c`` (TEST INFRASTRUCTURE ONLY).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg use this.
Arrays are numpy arrays of any strides; origins/domain follow the StencilObject convention.
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_cpu.so")


class OField(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("stride", ctypes.c_int64 * 3), ("origin", ctypes.c_int64 * 3)]


_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def _of(arr: np.ndarray, origin) -> OField:
    assert arr.ndim == 3
    f = OField()
    f.data = arr.ctypes.data
    for d in range(3):
        f.stride[d] = arr.strides[d] // arr.itemsize
        f.origin[d] = int(origin[d])
    return f


def _call(fn, arrays, origins, domain, nthreads):
    structs = [_of(a, o) for a, o in zip(arrays, origins)]
    args = [ctypes.byref(s) for s in structs]
    ni, nj, nk = (int(x) for x in domain)
    rc = fn(*args, ctypes.c_int64(ni), ctypes.c_int64(nj), ctypes.c_int64(nk), ctypes.c_int(nthreads))
    if rc != 0:
        raise RuntimeError(f"oracle call failed rc={rc}")


def copy_stencil(field_a, field_b, origin, domain, nthreads=0):
    _call(lib().oracle_copy_f64, [field_a, field_b], [origin["field_a"], origin["field_b"]], domain, nthreads)


def lap5(in_field, out_field, origin, domain, nthreads=0):
    _call(lib().oracle_lap5_f64, [in_field, out_field], [origin["in_field"], origin["out_field"]], domain, nthreads)


def horizontal_diffusion(in_field, out_field, coeff, origin, domain, nthreads=0):
    fn = lib().oracle_hdiff_f64 if in_field.dtype == np.float64 else lib().oracle_hdiff_f32
    assert in_field.dtype == out_field.dtype == coeff.dtype
    _call(fn, [in_field, out_field, coeff], [origin["in_field"], origin["out_field"], origin["coeff"]], domain, nthreads)


def tridiagonal_solver(inf, diag, sup, rhs, out, origin, domain, nthreads=0):
    names = ("inf", "diag", "sup", "rhs", "out")
    _call(lib().oracle_tridiag_f64, [inf, diag, sup, rhs, out], [origin[n] for n in names], domain, nthreads)


STENCILS = {
    "copy_stencil": (copy_stencil, ("field_a", "field_b")),
    "lap5": (lap5, ("in_field", "out_field")),
    "horizontal_diffusion": (horizontal_diffusion, ("in_field", "out_field", "coeff")),
    "tridiagonal_solver": (tridiagonal_solver, ("inf", "diag", "sup", "rhs", "out")),
}
