#!/bin/bash
# rocprofv3 evidence for the roofline: kernel-trace stats (durations) and PMC passes
# (FETCH_SIZE / WRITE_SIZE in separate passes, as MI355X_MICROARCH.md prescribes).
# Usage: CONFIGS="hdiff copy" TAG=r01 bash scripts/profile.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
for cfg in ${CONFIGS:-hdiff}; do
  # the bench line and the kernel-trace stats come from the SAME run, so rocprof's average kernel
  # duration and the bench's HIP-event kernel time describe the same launches
  cpu=--no-cpu-baseline
  [ "$cfg" = hdiff ] && cpu=
  echo "== $cfg: bench under kernel trace"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$cfg -o kt -- python3 bench.py --config $cfg --steps 20 --warmup 3 --no-extra $cpu > $OUT/kt_$cfg.log 2>&1 || exit $?
  grep '^{"metric"' $OUT/kt_$cfg.log > $OUT/bench_$cfg.json || exit $?
  cat $OUT/bench_$cfg.json
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "== $cfg: pmc $c"
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/pmc_${cfg}_$c -o pmc -- python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline --no-extra --placement-candidates 0 --sustain 0 > $OUT/pmc_${cfg}_$c.log 2>&1 || exit $?
  done
done
find $OUT -name "*.csv" | head -50
