#!/bin/bash
# Round 4: GPU suite after the frontend parity work, then the vadv band prefetch distance sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "kreg_pf=8;kreg_pf=10;kreg_pf=12;kreg_pf=8;kreg_pf=10;kreg_pf=12" \
    --rounds 6 > $O/sweep_vadv_pf_$rep.log 2>&1 || { tail -30 $O/sweep_vadv_pf_$rep.log; exit 1; }
  grep variant $O/sweep_vadv_pf_$rep.log
done
