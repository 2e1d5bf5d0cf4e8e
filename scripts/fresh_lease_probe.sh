#!/bin/bash
# The driver's condition reproduced: bench workload as the FIRST GPU process of a lease, with a
# timeline of step time and clock/power state (scripts/clock_probe.py), then the plain bench line,
# then (FULL=1) the GPU test suite and the same probe + bench line again.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fresh
mkdir -p $O
(amd-smi static --json > $O/amdsmi_static.json 2>&1; amd-smi metric --json > $O/amdsmi_metric_before.json 2>&1) || true
rocm-smi --showclocks --showpower --showmaxpower --showperflevel --showtemp --json > $O/rocmsmi_before.json 2>&1 || true
timeout -k 10 150 python3 -u scripts/clock_probe.py --seconds ${FIRST_S:-45} --tag first > $O/probe_first.jsonl 2> $O/probe_first.err || exit $?
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench_second.json 2> $O/bench_second.err || exit $?
cat $O/bench_second.json
timeout -k 10 100 python3 -u scripts/clock_probe.py --seconds 15 --tag third > $O/probe_third.jsonl 2> $O/probe_third.err || exit $?
amd-smi metric --json > $O/amdsmi_metric_mid.json 2>&1 || true
if [ "${FULL:-0}" = 1 ]; then
  bash scripts/gpu_tests.sh || exit $?
  timeout -k 10 100 python3 -u scripts/clock_probe.py --seconds 15 --tag after_tests > $O/probe_after_tests.jsonl 2> $O/probe_after.err || exit $?
  timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench_after_tests.json 2> $O/bench_after.err || exit $?
  cat $O/bench_after_tests.json
fi
echo done
