#!/bin/bash
# Round 4: vadv band prefetch distance, each variant twice, interleaved (8/10/12 levels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "kreg_pf=8;kreg_pf=10;kreg_pf=12;kreg_pf=8;kreg_pf=10;kreg_pf=12" \
    --rounds 6 > $O/sweep_vadv_pf_$rep.log 2>&1 || { tail -30 $O/sweep_vadv_pf_$rep.log; exit 1; }
  grep variant $O/sweep_vadv_pf_$rep.log
done
