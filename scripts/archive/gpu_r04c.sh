#!/bin/bash
# Round 4: full GPU suite + smoke, then the register-band sweep of the column kernels (vadv,
# tridiag): kreg = levels of the sweep-to-sweep cache held in registers (VGPR + AGPR) on top of
# the 40 LDS levels, at the occupancy the LDS tail already fixes (one 256-thread block per CU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  bash scripts/gpu_tests.sh || exit $?
fi
timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "kreg=0;kreg=32;kreg=64;kreg=96;kreg=112;kreg=64,kreg_pf=0;kreg=96,kreg_pf=4" \
  --rounds 6 > gpurun_out/r04c_sweep_vadv_kreg.log 2>&1 || { tail -30 gpurun_out/r04c_sweep_vadv_kreg.log; exit 1; }
cat gpurun_out/r04c_sweep_vadv_kreg.log
timeout -k 10 300 python -u scripts/sweep.py --config tridiag --variants "kreg=0;kreg=32;kreg=64;kreg=96;kreg=112;kreg=64,kreg_pf=0;kreg=96,kreg_pf=4" \
  --rounds 6 > gpurun_out/r04c_sweep_tridiag_kreg.log 2>&1 || { tail -30 gpurun_out/r04c_sweep_tridiag_kreg.log; exit 1; }
cat gpurun_out/r04c_sweep_tridiag_kreg.log
