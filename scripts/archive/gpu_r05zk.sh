#!/bin/bash
# Round 5: more candidate sets for the all-field-tuned column configs (5 vs 9), default bench
# lines alternating in separate processes on one box.
# (--placement-candidates-all was a trial option of bench.py, removed again after this call)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05zk}
mkdir -p $O
for i in 1 2; do
  for n in 5 9; do
    GTMI_NO_COMPILE=1 timeout -k 10 400 python3 bench.py --no-cpu-baseline --placement-candidates-all $n > $O/bench_${n}_$i.json 2> $O/err.log || { tail -30 $O/err.log; exit 1; }
    python3 -c "
import json; b=json.load(open('$O/bench_${n}_$i.json'))
for k in ('tridiag','vadv'): c=b['extra_configs'][k]; print('$n', k, c['kernel_ms'], c['frac'], c.get('placement',{}).get('candidates_ms'))"
  done
done
