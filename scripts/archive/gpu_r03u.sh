#!/bin/bash
# HBM bytes of slow vs fast placements: per-set HIP-event times, then FETCH_SIZE and WRITE_SIZE
# passes (each its own rocprofv3 run) of the same program, grouped by set.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
D=gpurun_out/r03u
mkdir -p $D
timeout -k 10 200 python3 scripts/placement_pmc.py --sets 6 2>> $D/err.log | tee $D/times.jsonl || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $D/pmc_$c -o p -- python3 scripts/placement_pmc.py --sets 6 > $D/pmc_$c.log 2>&1 || { tail -20 $D/pmc_$c.log; exit 1; }
  grep ms_by_set $D/pmc_$c.log
done
python3 scripts/placement_pmc.py --summarize $D/pmc_FETCH_SIZE $D/pmc_WRITE_SIZE --sets 6 | tee $D/summary.json
