"""Generate the golden fixtures from the REFERENCE numpy backend (build container only).

Usage (in the build container, where /root/reference and its offline import shim exist)::

    PYTHONPATH=/tmp/gtoracle:/root/reference/src:/root/repo GT_CACHE_ROOT=/tmp/gtcache \
        python3 -W ignore tests/golden/make_golden.py

For every case in ``tests/stencil_cases.py`` this script
1. aliases ``gt4py_amd.gtscript`` to the reference ``gt4py.cartesian.gtscript`` so the
   case's GTScript definition is parsed by the reference frontend,
2. builds it with ``backend="numpy"`` (the reference oracle backend,
   ``src/gt4py/cartesian/backend/numpy_backend.py``),
3. calls it on the case's deterministic inputs with the case's origin/domain, and
4. writes ``tests/golden/<case>.npz`` holding ``in__<field>``/``out__<field>`` arrays and
   ``field_info``/``domain_info`` (as JSON) for the host-logic tests.

Nothing here runs on the GPU box; the fixtures are plain data.
"""

from __future__ import annotations

import json
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def _alias_reference():
    import gt4py.cartesian.gtscript as ref_gtscript

    pkg = types.ModuleType("gt4py_amd")
    pkg.__path__ = []  # mark as package
    pkg.gtscript = ref_gtscript
    sys.modules["gt4py_amd"] = pkg
    sys.modules["gt4py_amd.gtscript"] = ref_gtscript
    return ref_gtscript


def main(selected=None):
    ref_gtscript = _alias_reference()
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import stencil_cases as sc  # noqa: E402

    manifest = {}
    mpath = os.path.join(HERE, "manifest.json")
    if selected and os.path.exists(mpath):
        with open(mpath) as f:
            manifest = json.load(f)
    for name, case in sc.CASES.items():
        if selected and name not in selected:
            continue
        try:
            stencil = ref_gtscript.stencil(
                # the reference numpy backend raises for a few features (absolute K indexing):
                # their fixtures come from the reference's pure-Python debug backend
                backend="debug" if "golden_debug" in case.features else "numpy",
                definition=case.definition,
                externals=case.externals,
                name=f"golden.{name}",
                rebuild=False,
            )
        except Exception as ex:  # pragma: no cover - report and continue
            print(f"[skip] {name}: build failed: {type(ex).__name__}: {ex}")
            continue
        inputs = case.make_inputs()
        arrays = {k: (None if v is None else v.copy()) for k, v in inputs.items()}
        kwargs = dict(arrays)
        kwargs.update(case.params)
        call_kw = {}
        if case.origin is not None:
            call_kw["origin"] = case.origin
        if case.domain is not None:
            call_kw["domain"] = case.domain
        try:
            stencil(**kwargs, **call_kw)
        except Exception as ex:  # pragma: no cover
            print(f"[skip] {name}: call failed: {type(ex).__name__}: {ex}")
            continue
        payload = {}
        for k, v in inputs.items():
            if v is None:
                continue
            payload[f"in__{k}"] = v
            payload[f"out__{k}"] = arrays[k]
        finfo = {
            k: {
                "access": int(fi.access),
                "boundary": [list(b) for b in fi.boundary],
                "axes": list(fi.axes),
                "dtype": str(fi.dtype),
            }
            for k, fi in stencil.field_info.items()
        }
        dinfo = {
            "parallel_axes": list(stencil.domain_info.parallel_axes),
            "sequential_axis": stencil.domain_info.sequential_axis,
            "min_sequential_axis_size": int(stencil.domain_info.min_sequential_axis_size),
            "ndim": int(stencil.domain_info.ndim),
        }
        pinfo = {k: {"access": int(pi.access), "dtype": str(pi.dtype)} for k, pi in stencil.parameter_info.items()}
        meta = {"field_info": finfo, "domain_info": dinfo, "parameter_info": pinfo}
        payload["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **payload)
        manifest[name] = {"seed": case.seed, **meta}
        print(f"[ok]   {name}")
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main(set(sys.argv[1:]) or None)
