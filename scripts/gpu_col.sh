#!/bin/bash
# Column-kernel check: GPU parity tests, then the column configs through bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in ${CONFIGS:-tridiag vadv}; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-extra > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err || { tail -20 gpurun_out/bench_$cfg.err; exit 1; }
  cat gpurun_out/bench_$cfg.json
done
