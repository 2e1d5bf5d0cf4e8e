#!/bin/bash
# GPU parity tests (one pytest process, per-test time limit), then smoke.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
# every library key the run requests (tests/gpu_build_keys.txt is made from it; tests/test_prebuild.py)
export GTMI_CACHE_LOG=${GTMI_CACHE_LOG:-$PWD/gpurun_out/build_keys.log}
timeout -k 10 ${TEST_TIMEOUT:-900} python -u -m pytest tests/ ${PYTEST_SEL:-} -x -v -m gpu --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -5
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" gpurun_out/pytest_gpu.log | head -120; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
exit $rc
