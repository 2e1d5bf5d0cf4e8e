"""Differential-fuzz programs pinned to the REFERENCE: for every case of ``fuzz_pinned.CASES``,
the output arrays of the reference numpy backend (``tests/golden/fuzz_reference.json``, SHA-256 of
the bytes, made by ``tests/golden/make_fuzz_golden.py``) must be reproduced bit for bit -- by our
numpy backend on the CPU and by gt:mi355x on the GPU. The f64 programs are the default fuzz seeds
(tests/test_fuzz.py compares gt:mi355x with our numpy backend on larger domains); the
mixed-precision programs (f32/f64/int32 fields, f64 and int literals) pin the upcasting and
cast-on-assignment rules of the frontend (``gtir_upcaster.py:80-143``), which both of our
backends share and which the fuzz against our own numpy backend alone cannot check."""

import hashlib
import importlib.util
import json
import os
import sys

import pytest

import fuzz_stencils
from fuzz_pinned import CASES, case_key, case_shape

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = """import numpy as np
from gt4py_amd.gtscript import BACKWARD, FORWARD, IJ, PARALLEL, Field, I, J, K, computation, horizontal, interval, region
from gt4py_amd.gtscript import (ceil, float32, float64, floor, function, int32, int64, isfinite, isnan, round,
                               round_away_from_zero, sqrt, trunc)

"""

with open(os.path.join(HERE, "golden", "fuzz_reference.json")) as _f:
    GOLDEN = json.load(_f)


def _load(seed, tmpdir):
    src, name = fuzz_stencils.generate(seed)
    path = os.path.join(tmpdir, f"fuzz_pin_{seed}.py")
    with open(path, "w") as f:
        f.write(HEADER + src)
    spec = importlib.util.spec_from_file_location(f"fuzz_pin_{seed}", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return getattr(mod, name), src


def _golden(seed, deep, src):
    rec = GOLDEN.get(case_key(seed, deep))
    assert rec is not None, f"seed {seed} has no reference record: run tests/golden/make_fuzz_golden.py"
    assert rec["source_sha256"] == hashlib.sha256(src.encode()).hexdigest(), (
        f"seed {seed}: the generator now writes a different program than the one pinned")
    assert "refused" not in rec, f"seed {seed}: the reference refused the program ({rec['refused']})"
    return rec


def _check(seed, src, rec, arrays):
    for k, exp in rec["outputs"].items():
        got = arrays[k]
        assert str(got.dtype) == exp["dtype"], f"seed {seed} {k}: dtype {got.dtype}, reference {exp['dtype']}"
        assert hashlib.sha256(got.tobytes()).hexdigest() == exp["sha256"], (
            f"seed {seed} field {k} differs from the reference numpy backend:\n{src}")


def _id(case):
    return case_key(*case)


def test_every_pinned_seed_has_a_reference_record():
    assert sorted(GOLDEN) == sorted(case_key(*c) for c in CASES)
    assert not [s for s, r in GOLDEN.items() if "refused" in r]


@pytest.mark.parametrize("case", CASES, ids=_id)
def test_numpy_backend_matches_reference(case, tmp_path):
    from gt4py_amd import gtscript

    seed, deep = case
    defn, src = _load(seed, str(tmp_path))
    rec = _golden(seed, deep, src)
    st = gtscript.stencil(backend="numpy", definition=defn, name=f"fuzzpin.np.{seed}")
    fields, origin = fuzz_stencils.make_inputs(seed, case_shape(seed, deep))
    st(**fields, s=0.75, origin=origin, domain=case_shape(seed, deep))
    _check(seed, src, rec, fields)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=_id)
def test_mi355x_matches_reference(case, tmp_path):
    import torch

    from gt4py_amd import gtscript, storage
    import test_fuzz

    seed, deep = case
    defn, src = _load(seed, str(tmp_path))
    rec = _golden(seed, deep, src)
    # the library of tests/test_fuzz.py (same program, same options): prebuilt by build()
    st = gtscript.stencil(backend="gt:mi355x", definition=defn, name=f"fuzz.hip.{seed}", **test_fuzz._opts(seed))
    assert torch.cuda.is_available(), "gt:mi355x needs a ROCm device"
    fields, origin = fuzz_stencils.make_inputs(seed, case_shape(seed, deep))
    dev = test_fuzz.to_device(fields, origin, seed)
    st(**dev, s=0.75, origin=origin, domain=case_shape(seed, deep))
    _check(seed, src, rec, {k: storage.to_numpy(v) for k, v in dev.items()})
