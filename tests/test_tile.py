"""Tile kernels (column kernels in tile mode, codegen/column.py + plan.make_plan(tile=True)):
sequential sweeps that read their own products across columns, after
``lowering.fuse_sequential_loops``. The reference keeps such temporaries in IJ caches
(``gtc/passes/oir_optimizations/caches.py:44-90``); gt:mi355x exchanges them through an LDS plane
per level on overlapping 2-D tiles instead of the staged lowering's scratch round trips.

CPU tests check the plans (which stencils take the tile path, which fusions are refused);
GPU tests compare every stencil with the numpy backend (itself pinned to the reference's
fixtures), bit for bit, on ragged domains that leave partial tiles on both axes.
"""

import numpy as np
import pytest

from gt4py_amd import gtscript
from gt4py_amd.gtscript import BACKWARD, FORWARD, PARALLEL, Field, computation, interval

F64 = Field[np.float64]
F32 = Field[np.float32]


def fwd_recurrence_ij_temp(a: F64, out: F64):
    with computation(FORWARD):
        with interval(0, 1):
            s = a
        with interval(1, None):
            s = s[0, 0, -1] * 0.5 + a
    with computation(FORWARD), interval(...):
        t = s * 2.0 + a
        out = t[1, 0, 0] - t[-1, 0, 0] + t[0, 1, 0] * s


def bwd_recurrence_ij_temp(a: F64, b: F64, out: F64):
    with computation(BACKWARD):
        with interval(-1, None):
            s = a
        with interval(0, -1):
            s = s[0, 0, 1] * 0.25 + a - b
    with computation(BACKWARD), interval(...):
        t = s * b
        out = t[0, -1, 0] + t[0, 1, 0] - 2.0 * t[-2, 0, 0] + t[2, 0, 0]


def two_phase_chain(a: F64, c: F64, out: F64):
    with computation(FORWARD), interval(...):
        t1 = a * c + 1.0
        t2 = t1[1, 0, 0] + t1[-1, 0, 0] - t1
        out = t2[0, 1, 0] - t2[0, -1, 0] + c


def tile_with_k_window(a: F64, w: F64, out: F64):
    with computation(FORWARD):
        with interval(0, 1):
            acc = a
        with interval(1, None):
            acc = acc[0, 0, -1] + a * w
    with computation(FORWARD):
        with interval(0, 1):
            t0 = acc * w
            out = t0[1, 0, 0] - t0[0, -1, 0]
        with interval(1, None):
            t1 = acc + w * acc[0, 0, -1]
            out = t1[1, 0, 0] - t1[0, -1, 0] + out[0, 0, -1] * 0.5


def tile_conditional(a: F64, out: F64):
    with computation(FORWARD):
        with interval(0, 1):
            m = a
        with interval(1, None):
            m = m[0, 0, -1] if m[0, 0, -1] > a else a
    with computation(FORWARD), interval(...):
        d = m - a
        if d[1, 0, 0] > d[-1, 0, 0]:
            out = d[1, 0, 0] + d[0, 1, 0]
        else:
            out = d[-1, 0, 0] - d[0, -1, 0]


def tile_f32(a: F32, out: F32):
    with computation(FORWARD):
        with interval(0, 1):
            s = a
        with interval(1, None):
            s = s[0, 0, -1] * 0.5 + a
    with computation(FORWARD), interval(...):
        t = s * 3.0
        out = t[1, 1, 0] - t[-1, -1, 0]


# (tile_by, tile_ti, tile_bx): block rows, tile width in I and block lanes in I (0: defaults,
# the aligned tile width and 64 or 128 lanes by cell size)
GEOMS = [(8, 0, 0), (4, 0, 0), (16, 0, 0), (8, 60, 64), (16, 13, 0), (4, 0, 128), (8, 100, 128)]

# name: (definition, {field: (halo_i_lo, halo_i_hi, halo_j_lo, halo_j_hi)}, dtype)
CASES = {
    "fwd_recurrence_ij_temp": (fwd_recurrence_ij_temp, {"a": (1, 1, 0, 1)}, np.float64),
    "bwd_recurrence_ij_temp": (bwd_recurrence_ij_temp, {"a": (2, 2, 1, 1), "b": (2, 2, 1, 1)}, np.float64),
    "two_phase_chain": (two_phase_chain, {"a": (1, 1, 1, 1), "c": (1, 1, 1, 1)}, np.float64),
    "tile_with_k_window": (tile_with_k_window, {"a": (0, 1, 1, 0), "w": (0, 1, 1, 0)}, np.float64),
    "tile_conditional": (tile_conditional, {"a": (1, 1, 1, 1)}, np.float64),
    "tile_f32": (tile_f32, {"a": (1, 1, 1, 1)}, np.float32),
}


def _stencil(name, backend, **opts):
    defn = CASES[name][0]
    return gtscript.stencil(backend=backend, definition=defn, name=f"tile.{name}", **opts)


@pytest.mark.parametrize("name", sorted(CASES))
def test_tile_plan(name):
    """Each case fuses into one sweep and runs as a tile kernel (no scratch)."""
    st = _stencil(name, "gt:mi355x")
    plan = st._gt_run_impl_.compiled.plan
    assert any(getattr(k, "tile", False) for k in plan.kernels), plan
    assert not plan.scratch, plan


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


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("domain", [(5, 3, 4), (70, 9, 6), (131, 23, 13)])
@pytest.mark.parametrize("geom", GEOMS)
def test_tile_vs_numpy_backend(name, domain, geom):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import storage

    arrays, origins = _inputs(name, domain, seed=sum(domain))
    ref = {k: v.copy() for k, v in arrays.items()}
    _stencil(name, "numpy")(**ref, origin=origins, domain=domain)
    tile_by, tile_ti, tile_bx = geom
    st = _stencil(name, "gt:mi355x", tile_by=tile_by, tile_ti=tile_ti, tile_bx=tile_bx)
    dev = {k: storage.from_array(v, v.dtype, backend="gt:mi355x", aligned_index=origins[k]) for k, v in arrays.items()}
    st(**dev, origin=origins, domain=domain)
    got = storage.to_numpy(dev["out"])
    np.testing.assert_array_equal(got, ref["out"])
