"""gt:mi355x code generation + hipcc cross-compilation for every case (CPU, no GPU needed).

Also checks that each generated library exports exactly the C ABI of include/gtmi.h.
Building here fills the in-tree JIT cache (.gt_cache) that travels to the GPU box.
"""

import os
import re
import subprocess

import pytest

import golden_utils as gu
import stencil_cases as sc
from gt4py_amd import gtscript
from gt4py_amd.runtime import ffi

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "gtmi.h")


def header_symbols():
    with open(HEADER) as f:
        text = f.read()
    decl = re.compile(r"^(?:int|const char\*|void)\s+(gtmi_\w+)\s*\(", re.M)
    return sorted(set(decl.findall(text)))


def test_header_declares_ffi_symbols():
    assert header_symbols() == sorted(ffi.EXPORTED_SYMBOLS)


@pytest.mark.parametrize("name", gu.available())
def test_case_compiles(name):
    case = sc.CASES[name]
    stencil = gtscript.stencil(backend="gt:mi355x", definition=case.definition, externals=case.externals,
                               name=f"gpu.{name}")
    compiled = type(stencil).run  # noqa: F841
    from gt4py_amd.backend.base import BaseBackend  # noqa: F401

    path = _lib_path(stencil)
    assert os.path.exists(path)
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for sym in header_symbols():
        assert sym in exported, (sym, path)


def _lib_path(stencil):
    import gc

    for obj in gc.get_referrers(type(stencil).run):
        pass
    run = type(stencil).run
    cell_fns = [c.cell_contents for c in (run.__closure__ or ())]
    for fn in cell_fns:
        comp = getattr(fn, "compiled", None)
        if comp is not None:
            return comp.lib_path
    raise AssertionError("no compiled library attached")


def test_jmirror_variants_build():
    """Odd J chunks of a plane kernel with J offsets stream top-down unless jmirror=0 (also builds
    the libraries tests/test_gpu_parity.py::test_hdiff_ragged_j_chunks_vs_c_oracle runs)."""
    from test_gpu_parity import RAGGED_CHUNK_OPTS, ragged_chunk_stencil

    for opts in RAGGED_CHUNK_OPTS:
        src = open(os.path.join(os.path.dirname(_lib_path(ragged_chunk_stencil(opts))), "stencil.hip")).read()
        assert ("if ((chunk & 1) == 0) {" in src) == bool(opts["jmirror"])
        assert ("jb + jce - 1 - (" in src) == bool(opts["jmirror"])
        u = opts.get("row_unroll", 0)
        assert src.count("// row copy ") == (u * (2 if opts["jmirror"] else 1) * 2 if u > 1 else 0)
    # no J offsets (copy): nothing to mirror
    copy = gtscript.stencil(backend="gt:mi355x", definition=sc.copy_stencil, name="gpu.copy_mirror_check",
                            pointwise_plane=1)
    src = open(os.path.join(os.path.dirname(_lib_path(copy)), "stencil.hip")).read()
    assert "chunk & 1" not in src


@pytest.mark.parametrize("name", ["hdiff_f64", "tridiag", "higher_dimensional_fields", "staged_forward_ij_temp"])
def test_library_loads_and_describes_itself(name):
    """The C-ABI library dlopens on a host without a GPU (no compute call is made), reports the
    ABI version of include/gtmi.h and a signature that matches the stencil's API."""
    case = sc.CASES[name]
    stencil = gtscript.stencil(backend="gt:mi355x", definition=case.definition, externals=case.externals,
                               name=f"gpu.{name}")
    lib = ffi.load_library(_lib_path(stencil))
    assert lib.lib.gtmi_abi_version() == ffi.GTMI_ABI_VERSION == 3
    sig = lib.signature
    assert sig["abi"] == 3
    assert [f["name"] for f in sig["fields"]] == list(stencil.field_info.keys())
    for f in sig["fields"]:
        fi = stencil.field_info[f["name"]]
        assert tuple(f["axes"]) == tuple(fi.axes) and tuple(f["data_dims"]) == tuple(fi.data_dims)
    assert [s["name"] for s in sig["scalars"]] == list(stencil.parameter_info.keys())
    assert lib.last_error() == ""
    with open(HEADER) as fh:
        hdr = fh.read()
    assert f"#define GTMI_ABI_VERSION {ffi.GTMI_ABI_VERSION}" in hdr
    # the header documents the signature the libraries emit: its version and its keys
    doc = hdr[hdr.index("JSON self-description"):hdr.index("gtmi_stencil_signature(void)")]
    assert f'{{"abi": {sig["abi"]},' in doc
    for key in sig:
        assert f'"{key}"' in doc, key
    for group in ("fields", "scratch", "scalars"):
        for entry in sig[group]:
            for key in entry:
                assert f'"{key}"' in doc, (group, key)


def test_halo_library_exports_its_header():
    """The halo pack/unpack library builds for gfx950 and exports exactly include/gtmi_halo.h."""
    from gt4py_amd.distributed import halo_copy

    path = halo_copy.library_path()
    hdr = os.path.join(os.path.dirname(HEADER), "gtmi_halo.h")
    with open(hdr) as f:
        declared = sorted(set(re.findall(r"^(?:int|const char\*|void)\s+(gtmi_\w+)\s*\(", f.read(), re.M)))
    assert declared == ["gtmi_halo_abi_version", "gtmi_halo_copy", "gtmi_halo_last_error"]
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(declared) <= exported


def test_row_unroll_auto_rule():
    """Auto row unroll (plane.py): 4 copies for small register state (lap5), 2 for 4 cells per
    lane (hdiff f32), none for hdiff f64; the 1-wide fallback variant always stays rolled.
    The buffer-load strip body (bufld, auto for 4 cells per lane) unrolls by its slot-ring
    length instead, marked "slot copy"."""
    cases = [(sc.lap5, "gpu.unroll_auto_lap5", 4, False), (sc.hdiff_f32, "gpu.unroll_auto_f32", 2, True),
             (sc.hdiff_f64, "gpu.unroll_auto_f64", 0, False)]
    for definition, name, u, slots in cases:
        st = gtscript.stencil(backend="gt:mi355x", definition=definition, name=name)
        src = open(os.path.join(os.path.dirname(_lib_path(st)), "stencil.hip")).read()
        v1 = src[src.index("k0_plane_v1("):src.index("__global__", src.index("k0_plane_v1("))]
        assert "// row copy" not in v1 and "// slot copy" not in v1
        copies = set(int(m) for m in re.findall(r"// row copy (\d+)", src))
        assert copies == (set(range(u)) if u else set()), (name, copies)
        assert ("// slot copy 0" in src) == slots, name


@pytest.mark.parametrize("opts", [{}, {"kreg": 48, "kreg_pf": 6}, {"kreg": 40, "kreg_pf": 50}])
@pytest.mark.parametrize("name", ["band_ij_accumulator", "band_ij_accumulator_reader"])
def test_register_band_never_prefetches_written_ij_fields(name, opts):
    """A field a loop both reads and writes that has no K axis (an IJ accumulator) is one address
    for every level: the register band must load it at its level, never levels ahead (ADVICE r04,
    high). Fields with a K axis, and IJ fields the loop only reads, may still be prefetched."""
    case = sc.CASES[name]
    st = gtscript.stencil(backend="gt:mi355x", definition=case.definition, name=f"gpu.{name}", **opts)
    src = st._gt_run_impl_.compiled.source
    assert "regband" in src
    prefetched = set(re.findall(r"\bbp\d+_w(\d+)_(\w+?)_p0_p0_", src))
    assert ("1", "s") not in prefetched and ("0", "lev") not in prefetched, prefetched
    assert {n for _, n in prefetched} >= {"a", "b"}


def test_sweep_cache_end_auto_rule():
    """ktail_head auto: cached API outputs (tridiag's sup/rhs, re-read anyway) keep the FIRST
    forward levels on chip, so the re-read ones come from the Infinity Cache; write-free scratch
    (vadv's ccol/dcol, whose 96-level register band would stay live through both memory sweeps)
    keeps the last ones. The writer's LDS band then sits at [rbase, rbase + tlen) or just below
    nk - rbase."""
    import bench

    srcs = {}
    for cfg in ("tridiag", "vadv"):
        sname, dtype, *_ = bench.CONFIGS[cfg]
        st = gtscript.stencil(backend="gt:mi355x", definition=bench.stencil_defs()[(sname, dtype)],
                              name=f"bench.{cfg}", device_sync=False, externals=bench.EXTERNALS.get(sname, {}))
        srcs[cfg] = st._gt_run_impl_.compiled.source
    assert "const int tc0 = rbase, tc1 = rbase + tlen;" in srcs["tridiag"]
    assert "if (ks < rbase) ks = rbase;" in srcs["tridiag"]
    assert "const int tc1 = nk - rbase, tc0 = tc1 - tlen;" in srcs["vadv"]
    assert "the reader's band: prefetched here" in srcs["vadv"] and "the reader's band" not in srcs["tridiag"]


def test_exact_products_render_as_fma():
    """An f64 add/sub of power-of-two literal x value widened from f32 renders as one fma (the
    product is exact, so one rounding equals the separate add's): the f32 hdiff cast tree's
    ``4.0 * f64(u) - f64(sum)``. f64 operands (the product may overflow) and other literals keep
    the separate multiply; ``exact_fma=0`` turns it off. Bit-exactness on the GPU: the f32 hdiff
    and mixed-precision goldens and the full-size C5 tile vs the C oracle (test_gpu_parity.py)."""
    from gt4py_amd.codegen.common import ExprRenderer
    from gt4py_amd.ir import BinaryOp, Cast, DataType, Literal, ScalarAccess

    f32 = ScalarAccess("u", DataType.FLOAT32)
    f64 = ScalarAccess("v", DataType.FLOAT64)
    wide = Cast(DataType.FLOAT64, f32)
    rend = ExprRenderer(lambda a: "?", lambda n: n)

    def expr(lit, x, op, c):
        p = BinaryOp("*", Literal(lit, DataType.FLOAT64), x, DataType.FLOAT64)
        return BinaryOp(op, p, c, DataType.FLOAT64)

    assert rend(expr(4.0, wide, "-", f64)).startswith("__builtin_fma(")
    assert rend(BinaryOp("-", f64, BinaryOp("*", wide, Literal(0.25, DataType.FLOAT64), DataType.FLOAT64),
                         DataType.FLOAT64)).startswith("__builtin_fma(((double)(-0x1")
    assert "__builtin_fma" not in rend(expr(4.0, f64, "-", f64))  # f64 factor: 4x may overflow
    assert "__builtin_fma" not in rend(expr(3.0, wide, "+", f64))  # not a power of two
    rend.exact_fma = False
    assert "__builtin_fma" not in rend(expr(4.0, wide, "-", f64))
    c = sc.CASES["hdiff_f32"]
    src = gtscript.stencil(backend="gt:mi355x", definition=c.definition, name="gpu.hdiff_f32")._gt_run_impl_.compiled.source
    assert "__builtin_fma" in src
    c = sc.CASES["hdiff_f64"]
    src = gtscript.stencil(backend="gt:mi355x", definition=c.definition, name="gpu.hdiff_f64")._gt_run_impl_.compiled.source
    assert "__builtin_fma" not in src
