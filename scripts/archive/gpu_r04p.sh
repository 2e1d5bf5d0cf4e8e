#!/bin/bash
# Round 4: deeper prefetch for light streams (kpf_adapt: vadv's backward sweep), vadv and tridiag,
# twice; then the GPU suite and the profiles of the changed column libraries (gpu_r04o.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "kpf_adapt=0;kpf_adapt=1;kpf_adapt=1,kring=8;kpf_adapt=0;kpf_adapt=1;kpf_adapt=1,kring=8" --rounds 6 > $O/sweep_vadv_adapt_$rep.log 2>&1 || { tail -30 $O/sweep_vadv_adapt_$rep.log; exit 1; }
  grep variant $O/sweep_vadv_adapt_$rep.log
  timeout -k 10 300 python -u scripts/sweep.py --config tridiag --variants "kpf_adapt=0;kpf_adapt=1;kpf_adapt=0;kpf_adapt=1" --rounds 6 > $O/sweep_tridiag_adapt_$rep.log 2>&1 || { tail -30 $O/sweep_tridiag_adapt_$rep.log; exit 1; }
  grep variant $O/sweep_tridiag_adapt_$rep.log
done
bash scripts/gpu_r04o.sh
