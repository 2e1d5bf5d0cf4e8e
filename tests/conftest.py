import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


if os.environ.get("GTMI_PREBUILD_TESTS"):
    # build-container prebuild of the GPU tests' libraries (__graft_entry__.build): every GPU test
    # runs up to its first device allocation, so the gt:mi355x stencils it constructs before that
    # are compiled into the in-tree cache the GPU box then loads; the tests themselves fail here
    import torch

    import gt4py_amd.storage as _gt_storage

    from gt4py_amd.runtime import launcher as _gt_launcher

    torch.cuda.is_available = lambda: True
    _gt_storage._device_of = lambda info: "cpu"  # tests that allocate first reach their stencils
    # the full-size tests allocate GBs per field on the host stand-in; eight workers at once ran
    # the container out of memory (a worker was killed, its test left unrecorded). A stencil is
    # built before its fields, so stop such a test at its first large allocation instead
    _gt_empty = _gt_storage.empty

    def _bounded_empty(shape, *args, **kwargs):
        import numpy as _np

        if int(_np.prod(shape)) > (64 << 20):
            raise MemoryError("GTMI_PREBUILD_TESTS: full-size field not allocated on the host stand-in")
        return _gt_empty(shape, *args, **kwargs)

    _gt_storage.empty = _bounded_empty

    def _no_launch(self, *args, **kwargs):
        raise RuntimeError("GTMI_PREBUILD_TESTS: built, not launched")

    _gt_launcher.StencilLauncher.__call__ = _no_launch

    _REPORT = os.environ.get("GTMI_PREBUILD_REPORT")

    @pytest.hookimpl(hookwrapper=True)
    def pytest_runtest_makereport(item, call):
        outcome = yield
        rep = outcome.get_result()
        # the call's outcome, or a set-up that did not pass (a fixture touching the device first:
        # the test body, and the stencils it constructs, never ran)
        if _REPORT and (rep.when == "call" or (rep.when == "setup" and not rep.passed)):
            import json

            err = None
            if call.excinfo is not None:
                err = [call.excinfo.type.__name__, str(call.excinfo.value).splitlines()[0][:300] if str(call.excinfo.value) else ""]
            with open(_REPORT, "a") as f:
                f.write(json.dumps({"test": item.nodeid, "when": rep.when, "outcome": rep.outcome, "error": err}) + "\n")

    def pytest_collection_modifyitems(session, config, items):
        """The gpu-marked tests collected (tests/test_prebuild.py checks each has a record)."""
        if not _REPORT:
            return
        import json

        ids = sorted(it.nodeid for it in items if it.get_closest_marker("gpu") is not None)
        tmp = f"{_REPORT}.collected.{os.getpid()}"
        with open(tmp, "w") as f:
            json.dump(ids, f)
        os.replace(tmp, _REPORT + ".collected")
