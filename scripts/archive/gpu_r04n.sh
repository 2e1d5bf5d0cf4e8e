#!/bin/bash
# Round 4: register band prefetch and loop boundaries (kreg_pf_span, writer->reader), position 0 a throwaway, vadv and tridiag, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "kreg_pf=8;kreg_pf=10;kreg_pf_span=1,kreg_pf=10;kreg_pf=12;kreg_pf_span=1,kreg_pf=8;kreg_pf=10;kreg_pf_span=1,kreg_pf=10;kreg_pf_span=1,kreg_pf=12" --rounds 6 > $O/sweep_vadv_span_$rep.log 2>&1 || { tail -30 $O/sweep_vadv_span_$rep.log; exit 1; }
  grep variant $O/sweep_vadv_span_$rep.log
  timeout -k 10 300 python -u scripts/sweep.py --config tridiag --variants "kreg_pf_span=0;kreg_pf_span=1;kreg_pf_span=0;kreg_pf_span=1" --rounds 6 > $O/sweep_tridiag_span_$rep.log 2>&1 || { tail -30 $O/sweep_tridiag_span_$rep.log; exit 1; }
  grep variant $O/sweep_tridiag_span_$rep.log
done
