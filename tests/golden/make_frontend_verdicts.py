"""Record the reference frontend's verdict on every program of ``tests/frontend_cases.py``
(build container only; same offline shim and invocation as ``make_golden.py``)::

    PYTHONPATH=/tmp/gtoracle:/root/reference/src:/root/repo GT_CACHE_ROOT=/tmp/gtcache \\
        python3 -W ignore tests/golden/make_frontend_verdicts.py

Writes ``tests/golden/frontend/verdicts.json``: per case ``{"accepted": bool, "error": class
name, "error_mro": [class names], "message": str}``, and for every accepted case the reference's
results on seeded inputs, ``tests/golden/frontend/outputs.npz`` (keys ``<case>__in__<field>``,
``<case>__out__<field>``, ``<case>__org__<field>``, ``<case>__par__<param>``; domain
``DOMAIN``). Plain data; nothing here runs on the GPU box.
"""

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from make_golden import _alias_reference  # noqa: E402

DOMAIN = (6, 5, 8)
HALO = {"I": 3, "J": 3, "K": 2}  # every axis gets this much room on both sides


def _run_case(obj, seed):
    """Seeded inputs sized from the stencil's own field/parameter info; returns the npz entries."""
    rng = np.random.default_rng(seed)
    arrays, origin, params, out = {}, {}, {}, {}
    for name, info in obj.field_info.items():
        if info is None:
            continue
        axes = list(info.axes)
        shape = [DOMAIN["IJK".index(a)] + 2 * HALO[a] for a in axes] + list(info.data_dims)
        arr = rng.uniform(0.5, 2.0, size=shape)
        arrays[name] = arr.astype(info.dtype)
        origin[name] = tuple(HALO[a] for a in axes)
    for name, info in obj.parameter_info.items():
        if info is not None:
            params[name] = info.dtype.type(1.25)
    for k, v in arrays.items():
        out[f"in__{k}"] = v.copy()
        out[f"org__{k}"] = np.array(origin[k], dtype=np.int64)
    for k, v in params.items():
        out[f"par__{k}"] = np.array(v)
    obj(**arrays, **params, origin=origin, domain=DOMAIN)
    for k, v in arrays.items():
        if not np.array_equal(v, out[f"in__{k}"], equal_nan=True):  # unchanged fields: no entry
            out[f"out__{k}"] = v
    return out


def main():
    ref_gtscript = _alias_reference()
    import frontend_cases as fc

    out = {}
    npz = {}
    for seed, (name, (defn, externals)) in enumerate(fc.CASES.items()):
        try:
            obj = ref_gtscript.stencil(backend="numpy", definition=defn, externals=externals, name=f"verdict.{name}",
                                       rebuild=False)
            out[name] = {"accepted": True}
            npz.update({f"{name}__{k}": v for k, v in _run_case(obj, 4000 + seed).items()})
        except Exception as e:  # noqa: BLE001 - the verdict is the data
            out[name] = {"accepted": False, "error": type(e).__name__,
                         "error_mro": [c.__name__ for c in type(e).__mro__], "message": str(e)[:400]}
        print(f"{name:34s} {'ok' if out[name]['accepted'] else out[name]['error']}")
    with open(os.path.join(HERE, "frontend", "verdicts.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    np.savez_compressed(os.path.join(HERE, "frontend", "outputs.npz"), **npz)


if __name__ == "__main__":
    main()
