"""I-neighbour moves stay separate DPP moves (regression for the mixed-precision fuzz seed 9130).

The plane kernel moves a lane's I neighbour with a DPP wave rotate (``gtmi::shfl_c<±1>`` ->
``v_mov_b32_dpp wave_rol:1 / wave_ror:1``). LLVM's DPP combiner folds such a move into the VALU
instruction that consumes it; for ``|m[0,0,0] - m[1,0,0]|`` on int32 that gave
``v_subrev_u32_dpp ... wave_rol:1`` and wrong values in the odd elements of 2-element lanes on the
MI355X (``scripts/lab/dpp_combine_lab.hip``). The JIT compiles with ``-amdgpu-dpp-combine=false``
(``runtime/jit.py``): the CPU test checks the gfx950 code of such stencils for folded DPP
instructions, the GPU test their results against the numpy backend.
"""

import os
import re
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

from gt4py_amd import gtscript, storage
from gt4py_amd.gtscript import PARALLEL, Field, computation, interval

LLVM = "/opt/rocm/lib/llvm/bin"


def i32_absdiff(m: Field[np.int32], out: Field[np.float64]):
    with computation(PARALLEL), interval(...):
        out = abs(m[0, 0, 0] - m[1, 0, 0]) + abs(m[0, 0, 0] - m[-1, 0, 0]) + out


def f32_neighbours(a: Field[np.float32], out: Field[np.float32]):
    with computation(PARALLEL), interval(...):
        out = (a[1, 0, 0] - a[0, 0, 0]) + (a[-1, 0, 0] + a[0, 0, 0]) * a[1, 0, 0]


def i32_mixed(m: Field[np.int32], a: Field[np.float32], out: Field[np.float64]):
    with computation(PARALLEL), interval(...):
        out = (m[1, 0, 0] - a[0, 0, 0]) * (m[-1, 0, 0] + m[0, 0, 0]) + max(m[1, 0, 0] - m[0, 0, 0], 0)


CASES = [i32_absdiff, f32_neighbours, i32_mixed]
DTYPES = {
    "i32_absdiff": {"m": np.int32, "out": np.float64},
    "f32_neighbours": {"a": np.float32, "out": np.float32},
    "i32_mixed": {"m": np.int32, "a": np.float32, "out": np.float64},
}


def _gfx950_disassembly(lib_path):
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    if not all(os.path.exists(t) for t in tools):
        pytest.skip("ROCm LLVM tools not installed")
    objcopy, bundler, objdump = tools
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat"), os.path.join(d, "co")
        subprocess.run([objcopy, f"--dump-section=.hip_fatbin={fat}", lib_path, os.path.join(d, "stripped")],
                       check=True, capture_output=True)
        listing = subprocess.run([bundler, "--list", "--type=o", f"--input={fat}"], check=True,
                                 capture_output=True, text=True).stdout.split()
        target = next(t for t in listing if "gfx950" in t)
        subprocess.run([bundler, "--unbundle", "--type=o", f"--input={fat}", f"--targets={target}", f"--output={co}"],
                       check=True, capture_output=True)
        return subprocess.run([objdump, "-d", "--mcpu=gfx950", co], check=True, capture_output=True, text=True).stdout


@pytest.mark.parametrize("defn", CASES, ids=lambda f: f.__name__)
def test_no_folded_dpp_in_generated_code(defn):
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not installed")
    st = gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"dppfold.{defn.__name__}")
    asm = _gfx950_disassembly(st._gt_run_impl_.compiled.lib_path)
    dpp = re.findall(r"^\s*(v_\w+_dpp)\b", asm, flags=re.M)
    assert dpp, "the I-offset reads should use DPP wave rotates"
    folded = sorted(set(x for x in dpp if x != "v_mov_b32_dpp"))
    assert not folded, f"DPP moves folded into VALU instructions: {folded}"


@pytest.mark.gpu
@pytest.mark.parametrize("defn", CASES, ids=lambda f: f.__name__)
def test_i_neighbour_moves_match_numpy(defn):
    import torch

    st = gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"dppfold.{defn.__name__}")
    ref_st = gtscript.stencil(backend="numpy", definition=defn, name=f"dppfold.np.{defn.__name__}")
    assert torch.cuda.is_available(), "gt:mi355x needs a ROCm device"
    rng = np.random.default_rng(11)
    # several strips and both kernel variants' lane layouts: 300 wide, an odd J count
    ni, nj, nk = 300, 7, 3
    args, origin = {}, {}
    for name, dt in DTYPES[defn.__name__].items():
        dt = np.dtype(dt)
        if name == "out":
            args[name] = rng.uniform(-1, 1, (ni, nj, nk)).astype(dt)
            origin[name] = (0, 0, 0)
        elif dt.kind == "i":
            args[name] = rng.integers(-5, 6, (ni + 2, nj, nk)).astype(dt)
            origin[name] = (1, 0, 0)
        else:
            args[name] = rng.uniform(-4, 4, (ni + 2, nj, nk)).astype(dt)
            origin[name] = (1, 0, 0)
    ref = {k: v.copy() for k, v in args.items()}
    ref_st(**ref, origin=origin, domain=(ni, nj, nk))
    dev = {k: storage.from_array(v, dtype=v.dtype, backend="gt:mi355x", aligned_index=origin[k]) for k, v in args.items()}
    st(**dev, origin=origin, domain=(ni, nj, nk))
    got = storage.to_numpy(dev["out"])
    bad = int((got != ref["out"]).sum())
    assert bad == 0, f"{defn.__name__}: {bad} cells differ from the numpy backend"
