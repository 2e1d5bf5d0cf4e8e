#!/bin/bash
# What the driver runs at round end: pytest -m gpu, smoke(), bench.py. With STRICT=1 a library
# missing from the prebuilt in-tree cache is an error instead of a compile on the box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
[ -n "$STRICT" ] && export GTMI_NO_COMPILE=1  # STRICT=1: fail instead of compiling a missing library on the box
timeout -k 10 900 python -u -m pytest tests -m gpu ${PYX--x} -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
