"""Pin the differential-fuzz programs to the REFERENCE numpy backend (build container only).

Usage (in the build container, where /root/reference and its offline import shim exist, see
tests/golden/make_golden.py)::

    PYTHONPATH=/tmp/gtoracle:/root/reference/src:/root/repo GT_CACHE_ROOT=/tmp/gtcache \
        python3 -W ignore tests/golden/make_fuzz_golden.py

For every case of ``tests/fuzz_pinned.py::CASES`` (each pinned seed at a small domain, the
sweep programs of ``DEEP`` again at >= 120 levels) this script generates the program with
``tests/fuzz_stencils.generate``, parses and builds it with the reference frontend and its numpy
backend (``src/gt4py/cartesian/backend/numpy_backend.py``), runs it on
``fuzz_stencils.make_inputs(seed, shape)`` and records, per output field, the SHA-256 of the
output array's bytes (the whole array: cells outside the domain must keep their initial values).
A program the reference refuses is recorded with the exception type. The program text's SHA-256
is kept too, so a change of the generator cannot silently re-pin a seed.

Output: ``tests/golden/fuzz_reference.json`` (plain data; nothing here runs on the GPU box).
"""

from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys
import tempfile
import types

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
HEADER = """import numpy as np
from gt4py_amd.gtscript import BACKWARD, FORWARD, IJ, PARALLEL, Field, I, J, K, computation, horizontal, interval, region
from gt4py_amd.gtscript import (ceil, float32, float64, floor, function, int32, int64, isfinite, isnan, round,
                               round_away_from_zero, sqrt, trunc)

"""


def _alias_reference():
    import gt4py.cartesian.gtscript as ref_gtscript

    pkg = types.ModuleType("gt4py_amd")
    pkg.__path__ = []
    pkg.gtscript = ref_gtscript
    sys.modules["gt4py_amd"] = pkg
    sys.modules["gt4py_amd.gtscript"] = ref_gtscript
    return ref_gtscript


def _load(src, name, tmpdir, seed):
    path = os.path.join(tmpdir, f"fuzzref_{seed}.py")
    with open(path, "w") as f:
        f.write(HEADER + src)
    spec = importlib.util.spec_from_file_location(f"fuzzref_{seed}", path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = mod
    spec.loader.exec_module(mod)
    return getattr(mod, name)


def main():
    ref_gtscript = _alias_reference()
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import fuzz_stencils as fs
    from fuzz_pinned import CASES, case_key, case_shape

    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for seed, deep in CASES:
            src, name = fs.generate(seed)
            shape = case_shape(seed, deep)
            rec = {"source_sha256": hashlib.sha256(src.encode()).hexdigest(), "shape": list(shape)}
            try:
                defn = _load(src, name, tmp, seed)
                # absolute K indexing: the reference's numpy backend raises for it, its debug backend
                # is the oracle (as for the golden fixtures, tests/golden/make_golden.py)
                backend = "debug" if seed >= fs.ABSK_BASE else "numpy"
                if backend != "numpy":
                    rec["backend"] = backend
                st = ref_gtscript.stencil(backend=backend, definition=defn, name=f"fuzzref.s{seed}", rebuild=False)
                fields, origin = fs.make_inputs(seed, shape)
                st(**fields, s=0.75, origin=origin, domain=shape)
            except Exception as ex:  # the reference refuses the program: record it
                rec["refused"] = type(ex).__name__
                print(f"[refused] {seed}: {type(ex).__name__}: {str(ex).splitlines()[0][:120]}")
            else:
                rec["outputs"] = {k: {"dtype": str(fields[k].dtype), "sha256": hashlib.sha256(fields[k].tobytes()).hexdigest()}
                                  for k in sorted(fields) if k.startswith("out")}
            out[case_key(seed, deep)] = rec
    with open(os.path.join(HERE, "fuzz_reference.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"{len(out)} programs, {sum('refused' in r for r in out.values())} refused")


if __name__ == "__main__":
    main()
