"""hipcc JIT with a content-addressed, in-tree cache (the analogue of the reference's
``backend/pyext_builder.py:190-309`` + ``caching.py:198-265``, without setuptools/pybind11).

The cache key is a hash of the generated source, the device/ABI headers and the compiler
flags, so a library built in the build container is found again on the GPU box (the repo is
copied there, ``.gt_cache`` included). Builds are atomic (temp file + rename) and serialised
by a file lock so that several ranks building the same stencil do not race.
"""

from __future__ import annotations

import fcntl
import hashlib
import os
import shutil
import subprocess
import tempfile
from typing import List, Optional

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPO_ROOT = os.path.dirname(PKG_DIR)
CSRC_DIR = os.path.join(PKG_DIR, "csrc")
INCLUDE_DIR = os.path.join(REPO_ROOT, "include")

OFFLOAD_ARCH = os.environ.get("GTMI_OFFLOAD_ARCH", "gfx950")

BASE_FLAGS = [
    f"--offload-arch={OFFLOAD_ARCH}",
    "-O3",
    "-std=c++17",
    "-fPIC",
    "-shared",
    # numerics contract with the reference numpy backend:
    "-ffp-contract=off",  # no FMA contraction
    "-fno-fast-math",
    "-fno-gpu-flush-denormals-to-zero",
    "-fhip-fp32-correctly-rounded-divide-sqrt",
    # keep every DPP wave rotate a separate v_mov_b32_dpp: folded into its consumer
    # (v_subrev_u32_dpp ... wave_rol:1) it gave wrong lanes on gfx950 (scripts/lab/dpp_combine_lab.hip,
    # DESIGN.md §3 K1 "I offsets"); tests/test_dpp_fold.py checks the generated code for it
    "-mllvm",
    "-amdgpu-dpp-combine=false",
    "-Wno-unused-variable",
    "-Wno-unused-but-set-variable",
]

# ROCTX ranges around every stencil call (csrc/gtmi_roctx.h): only when this ROCm install has
# rocprofiler-sdk-roctx; otherwise the ranges compile to nothing and nothing extra is linked
_ROCTX_LIB = "/opt/rocm/lib/librocprofiler-sdk-roctx.so"
if os.path.exists(_ROCTX_LIB) and os.environ.get("GTMI_BUILD_ROCTX", "1") != "0":
    BASE_FLAGS += ["-DGTMI_ROCTX=1", "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-Wl,-rpath,/opt/rocm/lib"]
else:
    BASE_FLAGS += ["-DGTMI_ROCTX=0"]


def hipcc_path() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC)")


def cache_root() -> str:
    # in-tree by default so that libraries built in the build container travel with the repo
    root = os.environ.get("GTMI_CACHE_ROOT", REPO_ROOT)
    name = os.environ.get("GTMI_CACHE_DIR_NAME", ".gt_cache")
    return os.path.join(root, name, "gt_mi355x")


def _headers_digest() -> str:
    h = hashlib.sha256()
    for path in (os.path.join(CSRC_DIR, "gtmi_device.h"), os.path.join(CSRC_DIR, "gtmi_roctx.h"),
                 os.path.join(INCLUDE_DIR, "gtmi.h"), os.path.join(INCLUDE_DIR, "gtmi_halo.h")):
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def build_key(source: str, extra_flags: Optional[List[str]] = None) -> str:
    h = hashlib.sha256()
    h.update(source.encode())
    h.update(" ".join(BASE_FLAGS + list(extra_flags or [])).encode())
    h.update(_headers_digest().encode())
    return h.hexdigest()[:24]


def library_path(source: str, extra_flags=None) -> str:
    key = build_key(source, extra_flags)
    return os.path.join(cache_root(), key, "stencil.so")


def compile_source(source: str, extra_flags: Optional[List[str]] = None, verbose: bool = False) -> str:
    """Return the path of the shared library for ``source``, compiling it if needed."""
    key = build_key(source, extra_flags)
    d = os.path.join(cache_root(), key)
    so = os.path.join(d, "stencil.so")
    log = os.environ.get("GTMI_CACHE_LOG")
    if log:  # scripts/prune_cache.py: which entries a build still uses
        with open(log, "a") as f:
            f.write(key + "\n")
    if os.path.exists(so):
        return so
    if os.environ.get("GTMI_NO_COMPILE"):
        # set on the GPU box to prove that every library a run needs was prebuilt by build()
        raise RuntimeError(f"GTMI_NO_COMPILE is set and {so} is not prebuilt")
    os.makedirs(d, exist_ok=True)
    lock_path = os.path.join(d, ".lock")
    with open(lock_path, "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        try:
            if os.path.exists(so):
                return so
            src_path = os.path.join(d, "stencil.hip")
            with open(src_path, "w") as f:
                f.write(source)
            fd, tmp_so = tempfile.mkstemp(suffix=".so", dir=d)
            os.close(fd)
            cmd = [hipcc_path()] + BASE_FLAGS + list(extra_flags or [])
            cmd += [f"-I{CSRC_DIR}", f"-I{INCLUDE_DIR}", "-o", tmp_so, src_path]
            if verbose:
                print(" ".join(cmd))
            res = subprocess.run(cmd, capture_output=True, text=True)
            if res.returncode != 0:
                os.unlink(tmp_so)
                raise RuntimeError(
                    f"hipcc failed ({res.returncode}) for {src_path}:\n{res.stderr[-8000:]}"
                )
            os.replace(tmp_so, so)
        finally:
            fcntl.flock(lock, fcntl.LOCK_UN)
    return so
