#!/bin/bash
# Round 4: band size / prefetch fine sweep around the new defaults (tridiag 48/6, vadv 96/12),
# and the N>1 headline path (hdiff + C5 leg) rehearsed with 2 ranks on one GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 300 python -u scripts/sweep.py --config tridiag --variants "kreg=48,kreg_pf=6;kreg=40,kreg_pf=6;kreg=56,kreg_pf=6;kreg=48,kreg_pf=4;kreg=48,kreg_pf=8;kreg=64,kreg_pf=4;kreg=0" \
  --rounds 6 > $O/sweep_tridiag_band2.log 2>&1 || { tail -30 $O/sweep_tridiag_band2.log; exit 1; }
grep variant $O/sweep_tridiag_band2.log
timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "kreg=96;kreg=88;kreg=80,kreg_pf=12;kreg=96,kreg_pf=10;kreg=96,kreg_pf=14;kreg=0" \
  --rounds 6 > $O/sweep_vadv_band2.log 2>&1 || { tail -30 $O/sweep_vadv_band2.log; exit 1; }
grep variant $O/sweep_vadv_band2.log
CONFIG=hdiff bash scripts/dist_rehearsal.sh > $O/dist_rehearsal_hdiff.log 2>&1 || { tail -30 $O/dist_rehearsal_hdiff.log; exit 1; }
cp gpurun_out/dist_*.json $O/
tail -4 $O/dist_rehearsal_hdiff.log | cut -c1-300
