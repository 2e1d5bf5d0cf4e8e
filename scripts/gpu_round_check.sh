#!/bin/bash
# GPU tests (optionally filtered by K=...) followed by the rocprof profile of every bench config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
CONFIGS="${CONFIGS:-hdiff hdiff_f32 lap5 tridiag copy vadv}" TAG=${TAG:-r01g} timeout -k 10 900 bash scripts/profile.sh \
  > gpurun_out/profile.log 2>&1 || { tail -30 gpurun_out/profile.log; exit 1; }
echo profile done
