#!/bin/bash
# GPU round check: smoke -> parity tests -> bench. Every GPU step has its own time limit;
# a crash/timeout (rc >= 2 for pytest, != 0 otherwise) stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
echo "== pytest -m gpu"
timeout -k 10 900 python -m pytest tests/ -q -m gpu -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
echo "== bench"
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 --cpu-budget ${CPU_BUDGET:-5} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $rc
