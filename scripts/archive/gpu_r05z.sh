#!/bin/bash
# Round 5: the column-kernel schedules were chosen by sweeps that all ran in the slow placement mode
# (a fresh process's first allocation). Variant x placement-set matrices for tridiag and vadv
# (scripts/column_placement_probe.py --variants): which schedule wins in the fast mode?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05z}
mkdir -p $O
timeout -k 10 400 python3 scripts/column_placement_probe.py --config tridiag --sets 5 --reps 5 --rounds 3 \
  --variants "kreg=-1;kreg=32;kreg=40;kreg=56;kreg=64;ktail_head=0" > $O/matrix_tridiag.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
cat $O/matrix_tridiag.jsonl | cut -c1-200
timeout -k 10 400 python3 scripts/column_placement_probe.py --config vadv --sets 5 --reps 5 --rounds 3 \
  --variants "kreg=-1;kreg=64;kreg=80;kreg=48;ktail_head=1,kreg=64" > $O/matrix_vadv.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
cat $O/matrix_vadv.jsonl | cut -c1-200
