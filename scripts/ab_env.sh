#!/bin/bash
# Process-separated A/B of an environment switch: ENVVAR=0/1 alternating, REPS times per config.
# Usage: ENVVAR=GTMI_HBM_STAGGER CONFIGS="tridiag vadv" REPS=3 bash scripts/ab_env.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${REPS:-3}); do for c in ${CONFIGS:-tridiag}; do for v in 0 1; do
  env $ENVVAR=$v timeout -k 10 200 python3 bench.py --config $c --no-extra --no-cpu-baseline --steps 30 2>/dev/null > gpurun_out/ab_one.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$c', '$ENVVAR=$v', d['roofline']['kernel_ms'])" | tee -a gpurun_out/ab_env.log
done; done; done
