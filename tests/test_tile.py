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
         (8, 0, 0, 1), (4, 0, 0, 4), (16, 0, 0, 1), (8, 60, 64, 4)]

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
