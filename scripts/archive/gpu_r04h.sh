#!/bin/bash
# Round 4: host cost per call (stride/dtype checks added to the prepared launch), a 420-program
# differential-fuzz stress (tile kernels, regions, new generator) and the tridiag register-band sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 300 python3 scripts/call_overhead.py > $O/call_overhead.log 2>&1 || { tail -20 $O/call_overhead.log; exit 1; }
cat $O/call_overhead.log | grep '^{'
GTMI_FUZZ_EXTRA=300 timeout -k 10 900 python -u -m pytest tests/test_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/fuzz_stress_420.log 2>&1 || { tail -30 $O/fuzz_stress_420.log; exit 1; }
tail -1 $O/fuzz_stress_420.log
timeout -k 10 300 python -u scripts/sweep.py --config tridiag --variants "kreg=0;kreg=16;kreg=24,kreg_pf=8;kreg=32,kreg_pf=4;kreg=32;kreg=48,kreg_pf=6;kreg=0" \
  --rounds 6 > $O/sweep_tridiag_band.log 2>&1 || { tail -30 $O/sweep_tridiag_band.log; exit 1; }
cat $O/sweep_tridiag_band.log | grep variant
