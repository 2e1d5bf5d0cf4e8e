#!/bin/bash
# Round 5: why does scripts/sweep.py time tridiag/vadv ~12 % slower than bench.py does on the same
# library? The bench config alone (first allocation, no tuning), then the sweep with one variant
# under a kernel trace (per-dispatch durations in call order).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05t}
mkdir -p $O
for cfg in tridiag vadv; do
  timeout -k 10 300 python3 bench.py --config $cfg --no-extra --no-cpu-baseline --placement-candidates 0 --steps 20 --warmup 3 \
    > $O/bench_$cfg.json 2> $O/bench_$cfg.err || { tail -20 $O/bench_$cfg.err; exit 1; }
  cut -c1-200 $O/bench_$cfg.json
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_sweep_$cfg -o kt -- \
    python3 scripts/sweep.py --config $cfg --rounds 7 --variants "kreg=-1" > $O/sweep_$cfg.log 2>&1 || { tail -20 $O/sweep_$cfg.log; exit 1; }
  grep -v Warn $O/sweep_$cfg.log
done
