"""Differential fuzzing: random GTScript programs (tests/fuzz_stencils.py) through gt:mi355x
must reproduce the numpy backend bit for bit. The CPU part checks that every program parses,
runs on numpy and builds for gfx950; the GPU part compares results."""

import importlib.util
import json
import os
import sys

import numpy as np
import pytest

import fuzz_stencils

HEADER = """import numpy as np
from gt4py_amd.gtscript import BACKWARD, FORWARD, IJ, PARALLEL, Field, I, J, K, computation, horizontal, interval, region
from gt4py_amd.gtscript import (ceil, float32, float64, floor, function, int32, int64, isfinite, isnan, round,
                               round_away_from_zero, sqrt, trunc)

"""
SEEDS = list(range(60)) + list(range(1000, 1060))
# stress runs: GTMI_FUZZ_EXTRA=N adds N more programs (seeds 5000...), GTMI_FUZZ_V3=N adds N of
# the sweep-pair / tile templates (seeds 7000...)
SEEDS += list(range(5000, 5000 + int(os.environ.get("GTMI_FUZZ_EXTRA", "0"))))
SEEDS += list(range(7000, 7000 + int(os.environ.get("GTMI_FUZZ_V3", "24"))))
# mixed-precision programs (f32/f64/int32 fields; also pinned to the reference at small domains,
# tests/test_fuzz_reference.py)
SEEDS += list(range(fuzz_stencils.MIXED_BASE, fuzz_stencils.MIXED_BASE + int(os.environ.get("GTMI_FUZZ_MIXED", "160"))))
# K-offset programs (PARALLEL temporaries read at K offsets by a three-interval sweep)
SEEDS += list(range(fuzz_stencils.KOFF_BASE, fuzz_stencils.KOFF_BASE + int(os.environ.get("GTMI_FUZZ_KOFF", "80"))))
# lower-dimensional fields (IJ and K inputs, an IJ output of a FORWARD sweep)
SEEDS += list(range(fuzz_stencils.LOWDIM_BASE, fuzz_stencils.LOWDIM_BASE + int(os.environ.get("GTMI_FUZZ_LOWDIM", "60"))))
# operator programs (mod, ** 2, sqrt, floor/ceil/trunc/round, casts, if/elif/else with and/or/not)
SEEDS += list(range(fuzz_stencils.OPS_BASE, fuzz_stencils.OPS_BASE + int(os.environ.get("GTMI_FUZZ_OPS", "100"))))
# bounded while loops and horizontal regions in PARALLEL and sequential computations
SEEDS += list(range(fuzz_stencils.CTRL_BASE, fuzz_stencils.CTRL_BASE + int(os.environ.get("GTMI_FUZZ_CTRL", "100"))))
# tile-kernel shape with mixed precision and a vector field
SEEDS += list(range(fuzz_stencils.TILE_BASE, fuzz_stencils.TILE_BASE + int(os.environ.get("GTMI_FUZZ_TILE", "60"))))
# gtscript functions (nested calls, if/else inside) and a vector output written per component
SEEDS += list(range(fuzz_stencils.FUNC_BASE, fuzz_stencils.FUNC_BASE + int(os.environ.get("GTMI_FUZZ_FUNC", "60"))))
# run-time K offsets computed from an int32 field
SEEDS += list(range(fuzz_stencils.VK_BASE, fuzz_stencils.VK_BASE + int(os.environ.get("GTMI_FUZZ_VK", "60"))))
# K partitions with absolute/relative interval bounds and gaps
SEEDS += list(range(fuzz_stencils.IVL_BASE, fuzz_stencils.IVL_BASE + int(os.environ.get("GTMI_FUZZ_IVL", "60"))))
# absolute K indexing (field.at(K=...)), f64
SEEDS += list(range(fuzz_stencils.ABSK_BASE, fuzz_stencils.ABSK_BASE + int(os.environ.get("GTMI_FUZZ_ABSK", "40"))))


def _shape(seed):
    # odd seeds: several 128-wide plane strips, several J chunks, a partial last chunk;
    # GTMI_FUZZ_NK (stress runs) overrides the level count, e.g. 120 so that register bands,
    # head/tail sweep caches and blocked tile levels are reached
    nk = int(os.environ.get("GTMI_FUZZ_NK", "0"))
    ni, nj, nk0 = (13, 11, 8) if seed % 2 == 0 else (300, 45, 6)
    if seed >= fuzz_stencils.IVL_BASE:
        nk0 = 8  # interval bounds up to 3 and -3 / absolute levels up to 5: at least 7 levels
    return ni, nj, nk or nk0


def _opts(seed):
    # stress runs: GTMI_FUZZ_OPTS (JSON) adds backend options to every program, e.g.
    # '{"tile_rows": 2, "tile_bx": 128, "tile_by": 8}' for the two-row tile geometry
    extra = json.loads(os.environ.get("GTMI_FUZZ_OPTS") or "{}")
    return {**[{}, {"jchunk": 3}, {"jchunk": 8, "prefetch": 1}][seed % 3], **extra}


def _load(seed, tmpdir):
    src, name = fuzz_stencils.generate(seed)
    path = os.path.join(tmpdir, f"fuzz_mod_{seed}.py")
    with open(path, "w") as f:
        f.write(HEADER + src)
    spec = importlib.util.spec_from_file_location(f"fuzz_mod_{seed}", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return getattr(mod, name), src


def _inputs(seed):
    if seed >= fuzz_stencils.MIXED_BASE:
        fields, origin = fuzz_stencils.make_inputs(seed, _shape(seed))
        return ({k: v for k, v in fields.items() if not k.startswith("out")},
                {k: v for k, v in fields.items() if k.startswith("out")}, origin)
    rng = np.random.default_rng(1000 + seed)
    ni, nj, nk = _shape(seed)
    ins = {n: rng.uniform(-4, 4, (ni + 4, nj + 4, nk)) for n in ("a", "b", "c")}
    outs = {n: rng.uniform(-1, 1, (ni, nj, nk)) for n in ("out1", "out2")}
    origin = {"a": (2, 2, 0), "b": (2, 2, 0), "c": (2, 2, 0), "out1": (0, 0, 0), "out2": (0, 0, 0)}
    return ins, outs, origin


def to_device(fields, origin, seed):
    """gt:mi355x storages of the program's fields, aligned at their origins, with their axes."""
    from gt4py_amd import storage

    axes, dd = fuzz_stencils.field_axes(seed), fuzz_stencils.data_dims(seed)
    return {k: storage.from_array(v, dtype=np.dtype((v.dtype, dd[k])) if k in dd else v.dtype, backend="gt:mi355x",
                                  aligned_index=origin[k], dimensions=tuple(axes[k])) for k, v in fields.items()}


def _run_numpy(defn, seed):
    from gt4py_amd import gtscript

    st = gtscript.stencil(backend="numpy", definition=defn, name=f"fuzz.np.{seed}")
    ins, outs, origin = _inputs(seed)
    arrays = {**{k: v.copy() for k, v in ins.items()}, **{k: v.copy() for k, v in outs.items()}}
    st(**arrays, s=0.75, origin=origin, domain=_shape(seed))
    return arrays


@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_program_builds(seed, tmp_path):
    from gt4py_amd import gtscript

    defn, src = _load(seed, str(tmp_path))
    _run_numpy(defn, seed)
    gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"fuzz.hip.{seed}", **_opts(seed))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", SEEDS)
def test_fuzz_program_matches_numpy(seed, tmp_path):
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    from gt4py_amd import gtscript, storage

    defn, src = _load(seed, str(tmp_path))
    ref = _run_numpy(defn, seed)
    st = gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"fuzz.hip.{seed}", **_opts(seed))
    ins, outs, origin = _inputs(seed)
    dev = to_device({**ins, **outs}, origin, seed)
    st(**dev, s=0.75, origin=origin, domain=_shape(seed))
    for k in sorted(k for k in ref if k.startswith("out")):
        got = storage.to_numpy(dev[k])
        assert np.array_equal(got, ref[k]), f"seed {seed} field {k}:\n{src}"
