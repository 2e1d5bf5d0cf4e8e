#!/bin/bash
# Process-separated A/B of bench arguments: A="..." B="..." alternating, REPS times per config.
# Usage: A="" B="--opt kreg=32" CONFIGS="tridiag vadv" REPS=3 bash scripts/ab_args.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in $(seq ${REPS:-3}); do for c in ${CONFIGS:-tridiag}; do for side in A B; do
  args=${!side}
  timeout -k 10 200 python3 bench.py --config $c --no-extra --no-cpu-baseline --steps 30 $args 2>/dev/null > gpurun_out/ab_one.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_one.json')); print('$c', '$side', '$args', d['roofline']['kernel_ms'])" | tee -a gpurun_out/ab_args.log
done; done; done
