#!/bin/bash
# Round 4: GPU suite on the span-prefetch default, then kernel trace + FETCH/WRITE passes of the
# two column libraries that changed (vadv, tridiag).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
CONFIGS="vadv tridiag" TAG=r04o timeout -k 10 900 bash scripts/profile.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
grep '^{"metric"' $O/profile.log | cut -c1-300
