"""Fusion of adjacent PARALLEL computations (``codegen/lowering.py:fuse_parallel_loops``).

CPU: which multi-block stencils fuse into one plane kernel (no scratch) and which must not
(K-offset reads of the other block's values, a block reading what a later block writes; API
fields written and read at IJ offsets are rejected by the parallel-model validation anyway). GPU: the fused launch reproduces the numpy backend (itself
pinned bit-for-bit to the reference's numpy backend by the golden fixtures) and, for hdiff
written as three blocks, the C oracle's single-block hdiff, bit for bit.
"""

import numpy as np
import pytest

from gt4py_amd.gtscript import PARALLEL, Field, computation, horizontal, interval, region, I, J

F = Field[np.float64]


def hdiff_blocks(in_field: F, out_field: F, coeff: F):
    with computation(PARALLEL), interval(...):
        lap = 4.0 * in_field[0, 0, 0] - (in_field[1, 0, 0] + in_field[-1, 0, 0] + in_field[0, 1, 0] + in_field[0, -1, 0])
    with computation(PARALLEL), interval(...):
        res = lap[1, 0, 0] - lap[0, 0, 0]
        flx = 0 if (res * (in_field[1, 0, 0] - in_field[0, 0, 0])) > 0 else res
        res2 = lap[0, 1, 0] - lap[0, 0, 0]
        fly = 0 if (res2 * (in_field[0, 1, 0] - in_field[0, 0, 0])) > 0 else res2
    with computation(PARALLEL), interval(...):
        out_field = in_field[0, 0, 0] - coeff[0, 0, 0] * (flx[0, 0, 0] - flx[-1, 0, 0] + fly[0, 0, 0] - fly[0, -1, 0])


def sections_blocks(a: F, b: F):
    """Both blocks with the same two sections: fused section by section."""
    with computation(PARALLEL):
        with interval(0, 1):
            t = a[1, 0, 0] + a[0, 1, 0]
        with interval(1, None):
            t = a[-1, 0, 0] - a[0, -1, 0]
    with computation(PARALLEL):
        with interval(0, 1):
            b = t[1, 1, 0] * 2.0
        with interval(1, None):
            b = t[-1, 0, 0] + t[0, 1, 0]


def region_blocks(a: F, b: F):
    with computation(PARALLEL), interval(...):
        t = a[1, 0, 0] - a[-1, 0, 0]
        with horizontal(region[I[0], :]):
            t = 0.0
    with computation(PARALLEL), interval(...):
        b = t[1, 0, 0] + t[-1, 0, 0] + t[0, 0, 0]


def k_offset_blocks(a: F, b: F):
    """Not fusable: the second block reads the first block's temporary at a K offset."""
    with computation(PARALLEL), interval(...):
        t = a[1, 0, 0] + a[-1, 0, 0]
    with computation(PARALLEL), interval(1, None):
        b = t[0, 0, -1]


def war_blocks(a: F, b: F, c: F):
    """The first pair fuses, the third block overwrites the temporary the fused pair reads (not
    fusable with it), the fourth fuses with the third."""
    with computation(PARALLEL), interval(...):
        t = c[0, 0, 0] * 3.0
    with computation(PARALLEL), interval(...):
        b = t[1, 0, 0] + t[-1, 0, 0]
    with computation(PARALLEL), interval(...):
        t = c[0, 0, 0] + 1.0
    with computation(PARALLEL), interval(...):
        a = t[0, 1, 0]


CASES = {
    # name: (definition, fused loop count, halo of the first field, domain)
    "hdiff_blocks": (hdiff_blocks, 1, 2, (48, 40, 6)),
    "sections_blocks": (sections_blocks, 1, 2, (40, 36, 5)),
    "region_blocks": (region_blocks, 1, 2, (40, 36, 4)),
    "k_offset_blocks": (k_offset_blocks, 2, 1, (40, 36, 5)),
    "war_blocks": (war_blocks, 2, 1, (40, 36, 4)),
}


def _analysis(defn):
    from gt4py_amd import frontend, passes
    from gt4py_amd.definitions import BuildOptions

    return passes.run_pipeline(frontend.parse_stencil(defn, {}, BuildOptions(name=defn.__name__, module="t"), {}))


@pytest.mark.parametrize("name", sorted(CASES))
def test_fusion_plan(name):
    from gt4py_amd.backend.mi355x_backend import generate_source
    from gt4py_amd.codegen.lowering import fuse_parallel_loops, lower_data_dims

    defn, n_loops, _, _ = CASES[name]
    low, _ = lower_data_dims(_analysis(defn))
    fused = fuse_parallel_loops(low)
    assert len(fused.stencil.vertical_loops) == n_loops
    plan, source, signature = generate_source(_analysis(defn), {})
    if n_loops == 1:
        assert signature["kernels"] == ["PlaneKernel"] * len(fused.stencil.vertical_loops[0].sections)
        assert signature["scratch"] == []  # every temporary stays in registers


def test_unfused_option_keeps_blocks():
    from gt4py_amd.backend.mi355x_backend import generate_source

    plan, _, signature = generate_source(_analysis(hdiff_blocks), {"fuse": 0})
    assert len(signature["kernels"]) == 3 and len(signature["scratch"]) == 3


def _inputs(name, rng):
    defn, _, h, (ni, nj, nk) = CASES[name]
    if name == "hdiff_blocks":
        arrays = {"in_field": rng.uniform(-10, 10, (ni + 2 * h, nj + 2 * h, nk)),
                  "out_field": np.zeros((ni, nj, nk)), "coeff": rng.uniform(0, 0.5, (ni, nj, nk))}
        origin = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    else:
        import inspect

        names = list(inspect.signature(defn).parameters)
        arrays = {n: rng.uniform(-10, 10, (ni + 2 * h, nj + 2 * h, nk)) for n in names}
        origin = {n: (h, h, 0) for n in names}
    return arrays, origin, (ni, nj, nk)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_fused_gpu_matches_numpy(name):
    import torch

    from gt4py_amd import gtscript, storage

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    defn = CASES[name][0]
    rng = np.random.default_rng(11)
    arrays, origin, domain = _inputs(name, rng)
    ref_st = gtscript.stencil(backend="numpy", definition=defn, name=f"fusion.np.{name}")
    ref = {k: storage.from_array(v, backend="numpy", aligned_index=origin[k]) for k, v in arrays.items()}
    ref_st(**ref, origin=origin, domain=domain)
    st = gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"fusion.gpu.{name}")
    dev = {k: storage.from_array(v, backend="gt:mi355x", aligned_index=origin[k]) for k, v in arrays.items()}
    st(**dev, origin=origin, domain=domain)
    for k in arrays:
        got = storage.to_numpy(dev[k])
        want = np.asarray(ref[k])
        assert np.array_equal(got, want, equal_nan=True), f"{name}:{k}: {int((got != want).sum())} cells differ"


@pytest.mark.gpu
def test_hdiff_blocks_full_size_vs_c_oracle():
    """hdiff written as three computations, at the C3 size: one launch, bit-exact vs the oracle."""
    import torch

    from gt4py_amd import gtscript, storage
    from oracle import c_oracle

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    ni, nj, nk, h = 2048, 2048, 160, 2
    rng = np.random.default_rng(5)
    in_h = rng.uniform(-10, 10, (ni + 2 * h, nj + 2 * h, nk))
    co_h = rng.uniform(0, 0.5, (ni, nj, nk))
    st = gtscript.stencil(backend="gt:mi355x", definition=hdiff_blocks, name="fusion.hdiff_blocks.full")
    org = {"in_field": (h, h, 0), "out_field": (0, 0, 0), "coeff": (0, 0, 0)}
    in_d = storage.from_array(in_h, backend="gt:mi355x", aligned_index=(h, h, 0))
    co_d = storage.from_array(co_h, backend="gt:mi355x")
    out_d = storage.zeros((ni, nj, nk), np.float64, backend="gt:mi355x")
    st(in_d, out_d, co_d, origin=org, domain=(ni, nj, nk))
    ref = np.zeros((ni, nj, nk), order="F")
    c_oracle.horizontal_diffusion(np.asfortranarray(in_h), ref, np.asfortranarray(co_h), org, (ni, nj, nk))
    got = storage.to_numpy(out_d)
    assert np.array_equal(got, ref), f"{int((got != ref).sum())} cells differ"
