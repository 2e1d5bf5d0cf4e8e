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

_module = None
_tried = False


def target_path() -> str:
    return os.path.join(_PKG, _NAME + sysconfig.get_config_var("EXT_SUFFIX"))


def _digest() -> str:
    h = hashlib.sha256()
    for p in (_SRC, os.path.join(_INCLUDE, "gtmi.h")):
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:24]


def build(verbose: bool = False) -> str:
    """Compile the extension if its sources changed since the last build; returns its path."""
    import torch
    from torch.utils.cpp_extension import include_paths, library_paths

    out = target_path()
    stamp = out + ".sha"
    digest = _digest()
    if os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return out
    tlib = library_paths()[0]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cmd = ["g++", "-O2", "-fPIC", "-shared", "-std=c++17", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
           "-D__HIP_PLATFORM_AMD__", f"-I{sysconfig.get_paths()['include']}"]
    cmd += [f"-I{p}" for p in include_paths()]
    cmd += ["-I/opt/rocm/include", f"-I{_INCLUDE}", "-o", out + ".tmp", _SRC, f"-L{tlib}", "-lc10", "-lc10_hip",
            "-ltorch_python", "-lamdhip64", f"-Wl,-rpath,{tlib}"]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True, capture_output=not verbose)
    os.replace(out + ".tmp", out)
    with open(stamp, "w") as f:
        f.write(digest + "\n")
    return out


def module():
    """The extension module, or None if it is not built (or fails to import)."""
    global _module, _tried
    if not _tried:
        _tried = True
        if os.environ.get("GTMI_FASTCALL", "1") != "0" and os.path.exists(target_path()):
            import importlib

            import torch  # noqa: F401  (its libraries first)

            _module = importlib.import_module(f"gt4py_amd.{_NAME}")
    return _module


def loaded() -> Optional[str]:
    m = module()
    return getattr(m, "__file__", None) if m is not None else None
