"""gt:mi355x registered inside the REFERENCE gt4py (only where the reference is importable).

Runs tests/helpers/gt4py_plugin_check.py in a subprocess with the reference sources and the
offline import shim of SURVEY.md Appendix B on PYTHONPATH; skipped where they are absent
(e.g. on the GPU box, where the reference never travels).
"""

import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SRC = "/root/reference/src"
SHIM = "/tmp/gtoracle"


def _available():
    if not (os.path.isdir(REF_SRC) and os.path.isdir(SHIM)):
        return False
    env = dict(os.environ, PYTHONPATH=f"{SHIM}:{REF_SRC}")
    r = subprocess.run([sys.executable, "-W", "ignore", "-c", "import gt4py.cartesian.gtscript"], env=env,
                       capture_output=True, timeout=300)
    return r.returncode == 0


@pytest.mark.skipif(not _available(), reason="reference gt4py not importable here")
def test_plugin_in_reference_registry(tmp_path):
    env = dict(os.environ, PYTHONPATH=f"{SHIM}:{REF_SRC}", GT_CACHE_ROOT=str(tmp_path))
    env.pop("GT_CACHE_DIR_NAME", None)
    # the JIT cache of gt:mi355x stays in-tree (it shares libraries with the native frontend)
    env["GTMI_CACHE_ROOT"] = REPO
    r = subprocess.run([sys.executable, "-W", "ignore", os.path.join(REPO, "tests", "helpers", "gt4py_plugin_check.py")],
                       env=env, capture_output=True, text=True, timeout=1200)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0
    assert "OK" in r.stdout
