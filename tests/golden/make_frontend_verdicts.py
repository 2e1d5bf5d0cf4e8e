"""Record the reference frontend's verdict on every program of ``tests/frontend_cases.py``
(build container only; same offline shim and invocation as ``make_golden.py``)::

    PYTHONPATH=/tmp/gtoracle:/root/reference/src:/root/repo GT_CACHE_ROOT=/tmp/gtcache \\
        python3 -W ignore tests/golden/make_frontend_verdicts.py

Writes ``tests/golden/frontend_verdicts.json``: per case ``{"accepted": bool, "error": class
name, "error_mro": [class names], "message": str}``. Plain data; nothing here runs on the GPU box.
"""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from make_golden import _alias_reference  # noqa: E402


def main():
    ref_gtscript = _alias_reference()
    import frontend_cases as fc

    out = {}
    for name, (defn, externals) in fc.CASES.items():
        try:
            ref_gtscript.stencil(backend="numpy", definition=defn, externals=externals, name=f"verdict.{name}",
                                 rebuild=False)
            out[name] = {"accepted": True}
        except Exception as e:  # noqa: BLE001 - the verdict is the data
            out[name] = {"accepted": False, "error": type(e).__name__,
                         "error_mro": [c.__name__ for c in type(e).__mro__], "message": str(e)[:400]}
        print(f"{name:34s} {'ok' if out[name]['accepted'] else out[name]['error']}")
    with open(os.path.join(HERE, "frontend_verdicts.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
