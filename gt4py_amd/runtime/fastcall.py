"""Native prepared launches for the call fast path (``csrc/gtmi_fastcall.cpp``).

``build()`` compiles the CPython extension ``gt4py_amd/_gtmi_fastcall*.so`` in-tree with the host
compiler against torch's headers and libraries (c10 for the current HIP stream and device,
torch_python to read a tensor's data pointer and sizes without a Python call); ``__graft_entry__.
build()`` runs it, and the built module travels with the tree like the stencil libraries.
``module()`` returns the imported extension, or None when it was not built: the launcher then
uses its ctypes closure (same semantics, about 1 us more per call). Either way the kernels are
the HIP ones -- the extension only replaces Python-side argument handling.
"""

from __future__ import annotations

import hashlib
import os
import subprocess
import sysconfig
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
_SRC = os.path.join(_PKG, "csrc", "gtmi_fastcall.cpp")
_INCLUDE = os.path.join(os.path.dirname(_PKG), "include")
_NAME = "_gtmi_fastcall"

ABI = 2  # PyModule_AddIntConstant(m, "ABI", ...) in csrc/gtmi_fastcall.cpp

_module = None
_tried = False


def target_path() -> str:
    return os.path.join(_PKG, _NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def _command(out: str):
    import torch
    from torch.utils.cpp_extension import include_paths, library_paths

    tlib = library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-fPIC", "-shared", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-D__HIP_PLATFORM_AMD__", f"-I{sysconfig.get_paths()['include']}"]
    cmd += [f"-I{p}" for p in include_paths()]
    cmd += ["-I/opt/rocm/include", f"-I{_INCLUDE}", "-o", out, _SRC, f"-L{tlib}", "-lc10", "-lc10_hip",
            "-ltorch_python", "-lamdhip64", f"-Wl,-rpath,{tlib}"]
    return cmd


def _digest() -> str:
    """Sources + torch version + the compile command: a binary built against another torch (its
    at::Tensor / THPVariable layout) or with other flags is never reused."""
    import torch

    h = hashlib.sha256()
    for p in (_SRC, os.path.join(_INCLUDE, "gtmi.h")):
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(torch.__version__.encode())
    # the command (flags, C++ ABI) with every installation prefix replaced by its role: the tree
    # is built here and run from another directory on the GPU box, whose torch and Python may
    # live under other prefixes
    prefixes = [(os.path.dirname(_PKG), "<repo>"), (os.path.dirname(os.path.abspath(torch.__file__)), "<torch>"),
                (sysconfig.get_paths()["include"], "<python-include>"), ("/opt/rocm", "<rocm>")]
    cmd = []
    for c in _command(target_path()):
        for pre, role in prefixes:
            c = c.replace(pre, role)
        cmd.append(c)
    h.update(" ".join(cmd).encode())
    return h.hexdigest()[:24]


def up_to_date() -> bool:
    out = target_path()
    stamp = out + ".sha"
    if not (os.path.exists(out) and os.path.exists(stamp)):
        return False
    with open(stamp) as f:
        return f.read().strip() == _digest()


def build(verbose: bool = False) -> str:
    """Compile the extension if its sources changed since the last build; returns its path."""
    out = target_path()
    stamp = out + ".sha"
    if up_to_date():
        return out
    digest = _digest()
    cmd = _command(out)
    cmd[cmd.index(out)] = out + ".tmp"
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True, capture_output=not verbose)
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(digest + "\n")
    return out


def module():
    """The extension module, or None if it is not built, is stale (built from other sources, for
    another torch or with other flags) or fails to import -- the launcher then uses its ctypes
    closure, with a warning for the last two cases. Stale under ``GTMI_NO_COMPILE`` raises."""
    global _module, _tried
    if not _tried:
        _tried = True
        if os.environ.get("GTMI_FASTCALL", "1") != "0" and os.path.exists(target_path()):
            import importlib
            import warnings

            import torch  # noqa: F401  (its libraries first)

            if not up_to_date():
                if os.environ.get("GTMI_NO_COMPILE"):
                    # a run that may not compile must not quietly measure the slower ctypes path
                    _tried = False
                    raise RuntimeError(f"{target_path()} is stale and GTMI_NO_COMPILE is set: rebuild it with "
                                       "gt4py_amd.runtime.fastcall.build() (or set GTMI_FASTCALL=0)")
                warnings.warn(f"{target_path()} is stale (rebuild with gt4py_amd.runtime.fastcall.build()); "
                              "using the ctypes launch path", RuntimeWarning, stacklevel=2)
                return None
            try:
                m = importlib.import_module(f"gt4py_amd.{_NAME}")
            except ImportError as e:
                warnings.warn(f"cannot import {target_path()} ({e}); using the ctypes launch path",
                              RuntimeWarning, stacklevel=2)
                return None
            if getattr(m, "ABI", None) != ABI:
                warnings.warn(f"{target_path()} has ABI {getattr(m, 'ABI', None)}, expected {ABI}; "
                              "using the ctypes launch path", RuntimeWarning, stacklevel=2)
                return None
            _module = m
    return _module


def loaded() -> Optional[str]:
    m = module()
    return getattr(m, "__file__", None) if m is not None else None
