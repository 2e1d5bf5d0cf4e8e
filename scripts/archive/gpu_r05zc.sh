#!/bin/bash
# Round 5: load-ring depth and register-band prefetch distance re-checked in both placement modes
# (the r05k sweeps that set them ran in the slow mode only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05zc}
mkdir -p $O
timeout -k 10 400 python3 scripts/column_placement_probe.py --config tridiag --sets 4 --reps 5 --rounds 3 \
  --variants "kreg=-1;kring=6;kring=10;kring=12;kreg_pf=4;kreg_pf=8;kreg_pf=10" > $O/matrix_tridiag.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
cut -c1-200 $O/matrix_tridiag.jsonl
timeout -k 10 400 python3 scripts/column_placement_probe.py --config vadv --sets 4 --reps 5 --rounds 3 \
  --variants "kreg=-1;kring=6;kring=10;kreg_pf=6;kreg_pf=12" > $O/matrix_vadv.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
cut -c1-200 $O/matrix_vadv.jsonl
