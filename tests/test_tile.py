"""Tile kernels (column kernels in tile mode, codegen/column.py + plan.make_plan(tile=True)):
sequential sweeps that read their own products across columns, after
``lowering.fuse_sequential_loops``. The reference keeps such temporaries in IJ caches
(``gtc/passes/oir_optimizations/caches.py:44-90``); gt:mi355x exchanges them through an LDS plane
per level on overlapping 2-D tiles instead of the staged lowering's scratch round trips.

CPU tests check the plans (which stencils take the tile path, which fusions are refused);
GPU tests compare every program with the reference numpy backend's own outputs (goldens
``tile_<program>_d70`` / ``_d131`` and ``fuzz_tile_<seed>``, tests/stencil_cases.py, made by
tests/golden/make_golden.py) under every tile geometry, bit for bit, on ragged domains that
leave partial tiles on both axes, and with the numpy backend at a tiny domain.
"""

import numpy as np
import pytest

from gt4py_amd import gtscript
from gt4py_amd.gtscript import BACKWARD, FORWARD, PARALLEL, Field, computation, interval

F64 = Field[np.float64]
F32 = Field[np.float32]


from stencil_cases import (  # noqa: E402  (the programs live with their reference goldens)
    FUZZ_GOLDEN,
    TILE_GOLDEN,
    TILE_PROGRAMS,
    bwd_recurrence_ij_temp,
    tile_conditional,
    tile_f32,
    tile_scratch_product,
    tile_with_k_window,
    two_phase_chain,
)
from stencil_cases import staged_forward_ij_temp as fwd_recurrence_ij_temp  # noqa: E402

# (tile_by, tile_ti, tile_bx[, tile_lblock]): block rows, tile width in I and block lanes in I (0:
# defaults, the aligned tile width and 64 or 128 lanes by cell size), levels per LDS barrier
# (default 2 when a loop can be blocked)
GEOMS = [(8, 0, 0), (4, 0, 0), (16, 0, 0), (8, 60, 64), (16, 13, 0), (4, 0, 128), (8, 100, 128),
         (8, 0, 0, 1), (4, 0, 0, 4), (16, 0, 0, 1), (8, 60, 64, 4),
         # (tile_by, tile_ti, tile_bx, tile_lblock, tile_rows): two rows per thread
         (8, 0, 128, 2, 2), (4, 0, 0, 1, 2), (8, 60, 64, 4, 2),
         # row counts that are not powers of two
         (12, 0, 0, 2, 2), (11, 0, 0)]

# name: (definition, {field: (halo_i_lo, halo_i_hi, halo_j_lo, halo_j_hi)}, dtype)
CASES = {name: (defn, halos, np.dtype(dt).type) for name, (defn, halos, dt) in TILE_PROGRAMS.items()}


def _stencil(name, backend, **opts):
    defn = CASES[name][0]
    return gtscript.stencil(backend=backend, definition=defn, name=f"tile.{name}", **opts)


@pytest.mark.parametrize("name", sorted(CASES))
def test_tile_plan(name):
    """Each case fuses into one sweep and runs as a tile kernel (no scratch, except
    tile_scratch_product, whose tile-kernel product t2 a later kernel reads at IJ offsets)."""
    st = _stencil(name, "gt:mi355x")
    plan = st._gt_run_impl_.compiled.plan
    assert any(getattr(k, "tile", False) for k in plan.kernels), plan
    assert plan.scratch == (["t2"] if name == "tile_scratch_product" else []), plan


@pytest.mark.parametrize("name", FUZZ_GOLDEN)
def test_fuzz_golden_programs_take_the_tile_path(name):
    import stencil_cases as sc

    case = sc.CASES[name]
    st = gtscript.stencil(backend="gt:mi355x", definition=case.definition, name=f"golden.{name}")
    assert any(getattr(k, "tile", False) for k in st._gt_run_impl_.compiled.plan.kernels)


def test_scratch_stores_of_tile_kernels_are_tile_local():
    """Only lanes on which the stored temporary is valid store it (the owned tile grown by the
    statement's extent), so overlapping tiles never race on a scratch column."""
    st = _stencil("tile_scratch_product", "gt:mi355x")
    src = st._gt_run_impl_.compiled.source
    store = [ln for ln in src.splitlines() if "if (alive" in ln and "tx <" in ln]
    assert store, "no tile-local guard in the tile kernel"


@pytest.mark.parametrize("name,block", [("fwd_recurrence_ij_temp", "dim3(64, 16)"), ("tile_with_k_window", "dim3(64, 16)"),
                                        ("two_phase_chain", "dim3(64, 8)"), ("bwd_recurrence_ij_temp", "dim3(64, 8)"),
                                        ("tile_f32", "dim3(128, 8)")])
def test_tile_rows_auto_rule(name, block):
    """tile_by auto: 16 rows for a one-row J halo on 8-byte cells, else 8 (column.py TILE_BY)."""
    src = _stencil(name, "gt:mi355x")._gt_run_impl_.compiled.source
    assert block in src
    assert _stencil(name, "gt:mi355x", tile_by=8)._gt_run_impl_.compiled.source.count("dim3(64, 16)") == 0


def tile_many_planes(a: F64, out: F64):
    """Six temporaries read across columns: six LDS planes per level (column.py
    ``_fit_tile_lds``)."""
    with computation(FORWARD), interval(...):
        t0 = a * 1.5
        t1 = a * 2.5 + 1.0
        t2 = a - 0.5
        t3 = a * a
        t4 = a + 2.0
        t5 = a * 0.25
        out = t0[1, 0, 0] + t1[0, 1, 0] - t2[1, 0, 0] + t3[0, 1, 0] * t4[1, 0, 0] - t5[1, 0, 0] + t5


def tile_eleven_planes(a: F64, out: F64):
    with computation(FORWARD), interval(...):
        t0 = a * 1.5
        t1 = a * 2.5
        t2 = a - 0.5
        t3 = a * a
        t4 = a + 2.0
        t5 = a * 0.25
        t6 = a + 3.0
        t7 = a * 4.0
        t8 = a - 5.0
        t9 = a * 6.0
        t10 = a + 7.0
        out = (t0[1, 0, 0] + t1[1, 0, 0] + t2[1, 0, 0] + t3[1, 0, 0] + t4[1, 0, 0] + t5[1, 0, 0]
               + t6[0, 1, 0] + t7[0, 1, 0] + t8[0, 1, 0] + t9[0, 1, 0] + t10[0, 1, 0])


def _gen(defn, **opts):
    st = gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"tile.{defn.__name__}", **opts)
    return st._gt_run_impl_.compiled


def _lds_planes(src):
    import re

    return [tuple(int(x) for x in m) for m in re.findall(r"__shared__ double lds_\w+\[(\d+)\]\[(\d+)\]\[(\d+)\]", src)]


def test_tile_lds_planes_fit_the_cu():
    """The tile kernel's LDS planes stay within 160 KB: six f64 planes on 16-row
    blocks need 192 KB at two levels per barrier, so the kernel drops to one level per barrier
    (96 KB); eleven planes also drop to 8-row blocks when the rows are the automatic choice, and
    go to the staged lowering when 16 rows are asked for explicitly."""
    c = _gen(tile_many_planes)
    planes = _lds_planes(c.source)
    assert len(planes) == 6 and all(p == (2, 16, 64) for p in planes), planes
    assert sum(8 * a * b * d for a, b, d in planes) <= 160 * 1024
    c = _gen(tile_many_planes, tile_lblock=4)
    assert all(p == (2, 16, 64) for p in _lds_planes(c.source))
    c = _gen(tile_eleven_planes)
    planes = _lds_planes(c.source)
    assert len(planes) == 11 and all(p == (2, 8, 64) for p in planes), planes
    c = _gen(tile_eleven_planes, tile_by=16)
    assert not any(getattr(k, "tile", False) for k in c.plan.kernels), c.plan
    assert c.plan.scratch  # the staged lowering's phases


def test_tile_rows_two_rows_per_thread():
    """``tile_rows=2``: the block's threads cover twice ``tile_by`` rows (LDS planes and the launch
    grid sized for it), each thread carrying a second column's state under ``_r1`` names; other
    values are refused; the LDS budget counts both rows."""
    c = _gen(fwd_recurrence_ij_temp, tile_rows=2, tile_bx=128, tile_by=8)
    assert all(p[1:] == (16, 128) for p in _lds_planes(c.source)), _lds_planes(c.source)
    assert "const int ty_r1 = ty + 8, j_r1 = j + 8;" in c.source
    assert "dim3(128, 8)" in c.source and "(nj + 14) / 15" in c.source
    assert "one LDS barrier" in c.source  # still blocked
    with pytest.raises(ValueError, match="tile_rows"):
        _gen(fwd_recurrence_ij_temp, tile_rows=3)
    planes = _lds_planes(_gen(tile_many_planes, tile_rows=2, tile_by=8).source)
    assert sum(8 * a * b * d for a, b, d in planes) <= 160 * 1024, planes


def test_tile_levels_blocked_only_without_memory_raw():
    """A loop whose API output, stored after the barrier one level ahead, is read back before the
    next level's barrier keeps one level per barrier; the other tile programs are blocked
    (golden ``tile_kwrite_raw_*`` runs it under every geometry)."""
    import stencil_cases as sc

    for lb in (2, 4):
        assert "one LDS barrier" not in _gen(sc.tile_kwrite_raw, tile_lblock=lb).source
        assert "one LDS barrier" in _gen(fwd_recurrence_ij_temp, tile_lblock=lb).source


def test_tile_off_uses_staged_lowering():
    st = _stencil("fwd_recurrence_ij_temp", "gt:mi355x", tile=0)
    plan = st._gt_run_impl_.compiled.plan
    assert not any(getattr(k, "tile", False) for k in plan.kernels)
    assert set(plan.scratch) == {"s", "t"}


def test_sequential_fusion_refusals():
    """Fusion must not reorder: a later computation reading a level the sweep has not produced
    yet, or writing what the earlier one reads, keeps the computations apart."""
    from gt4py_amd.codegen.lowering import _seq_fusable
    from gt4py_amd.definitions import BuildOptions
    from gt4py_amd.frontend import parse_stencil
    from gt4py_amd.passes import run_pipeline

    def ahead(a: F64, out: F64):
        with computation(FORWARD), interval(...):
            s = a + 1.0
        with computation(FORWARD), interval(0, -1):
            out = s[0, 0, 1]

    def writes_back(a: F64, out: F64):
        with computation(FORWARD), interval(...):
            out = a + 1.0
        with computation(FORWARD), interval(...):
            a = out * 2.0

    def ok(a: F64, out: F64):
        with computation(FORWARD), interval(...):
            s = a + 1.0
        with computation(FORWARD), interval(...):
            out = s[1, 0, 0]

    def verdict(defn):
        st = run_pipeline(parse_stencil(defn, {}, BuildOptions(name=defn.__name__, module="t"))).stencil
        vls = st.vertical_loops
        return _seq_fusable(vls[0], vls[1], {p.name for p in st.field_params()})

    assert not verdict(ahead)
    assert not verdict(writes_back)
    assert verdict(ok)


# ------------------------------------------------------------------------------------ GPU


def _inputs(name, domain, seed):
    _, halos, dtype = CASES[name]
    ni, nj, nk = domain
    rng = np.random.default_rng(seed)
    arrays, origins = {}, {}
    for f, (ilo, ihi, jlo, jhi) in halos.items():
        arrays[f] = rng.uniform(0.5, 2.0, (ni + ilo + ihi, nj + jlo + jhi, nk)).astype(dtype)
        origins[f] = (ilo, jlo, 0)
    arrays["out"] = np.zeros((ni, nj, nk), dtype=dtype)
    origins["out"] = (0, 0, 0)
    return arrays, origins


# every geometry on the ragged 131 x 23 x 13 domain of each program and on four fuzz programs
# (every golden also runs with the default geometry in test_gpu_parity.py::test_golden_case)
GEOM_GOLDEN = [n for n in TILE_GOLDEN if n.endswith("_d131")] + FUZZ_GOLDEN[:4]


def geom_opts(geom):
    tile_by, tile_ti, tile_bx = geom[:3]
    opts = {"tile_by": tile_by, "tile_ti": tile_ti, "tile_bx": tile_bx}
    if len(geom) > 3:
        opts["tile_lblock"] = geom[3]
    if len(geom) > 4:
        opts["tile_rows"] = geom[4]
    return opts


@pytest.mark.gpu
@pytest.mark.parametrize("name", GEOM_GOLDEN)
@pytest.mark.parametrize("geom", GEOMS)
def test_tile_geometries_vs_reference_golden(name, geom):
    """Tile geometries on reference-generated tile goldens."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    import golden_utils as gu
    import stencil_cases as sc
    from test_gpu_parity import run_case_on_gpu

    case = sc.CASES[name]
    _, outputs, _ = gu.load(name)
    res = run_case_on_gpu(case, geom_opts(geom))
    for k, v in outputs.items():
        gu.assert_match(res[k], v, name=f"{name}{geom}:{k}")


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("geom", GEOMS)
def test_tile_vs_numpy_backend(name, geom):
    domain = (5, 3, 4)  # smaller than one tile; the ragged domains are the goldens above
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    arrays, origins = _inputs(name, domain, seed=sum(domain))
    ref = {k: v.copy() for k, v in arrays.items()}
    _stencil(name, "numpy")(**ref, origin=origins, domain=domain)
    st = _stencil(name, "gt:mi355x", **geom_opts(geom))
    dev = {k: storage.from_array(v, v.dtype, backend="gt:mi355x", aligned_index=origins[k]) for k, v in arrays.items()}
    st(**dev, origin=origins, domain=domain)
    got = storage.to_numpy(dev["out"])
    np.testing.assert_array_equal(got, ref["out"])


@pytest.mark.gpu
@pytest.mark.parametrize("defn", [tile_many_planes, tile_eleven_planes])
def test_tile_many_planes_vs_numpy_backend(defn):
    """The LDS-budget fallbacks (one level per barrier, 8-row blocks) against the numpy backend
    on a ragged domain."""
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    ni, nj, nk = 131, 23, 13
    rng = np.random.default_rng(11)
    arrays = {"a": rng.uniform(0.5, 2.0, (ni + 1, nj + 1, nk)), "out": np.zeros((ni, nj, nk))}
    origins = {"a": (0, 0, 0), "out": (0, 0, 0)}
    ref = {k: v.copy() for k, v in arrays.items()}
    gtscript.stencil(backend="numpy", definition=defn, name=f"tile.np.{defn.__name__}")(
        **ref, origin=origins, domain=(ni, nj, nk))
    st = gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"tile.{defn.__name__}")
    dev = {k: storage.from_array(v, v.dtype, backend="gt:mi355x", aligned_index=origins[k]) for k, v in arrays.items()}
    st(**dev, origin=origins, domain=(ni, nj, nk))
    np.testing.assert_array_equal(storage.to_numpy(dev["out"]), ref["out"])
