#!/bin/bash
# Round 5: tridiag head placement -- band size, band prefetch and load ring around the defaults.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05k}
mkdir -p $O
timeout -k 10 400 python3 scripts/sweep.py --config tridiag --rounds 7 --variants \
  "kreg=48;kreg=40;kreg=56;kreg_pf=4;kreg_pf=8;kring=6;kring=10" > $O/sweep_tridiag.log 2>&1 || { tail -20 $O/sweep_tridiag.log; exit 1; }
grep -v Warn $O/sweep_tridiag.log
