#!/bin/bash
# Round 4: I-neighbour lane shifts (nbr_shfl): parity first, then vadv A/B in one process, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "neighbour or column_options or vadv" --timeout 120 --timeout-method thread > $O/pytest_nbr.log 2>&1 \
  || { tail -40 $O/pytest_nbr.log; exit 1; }
tail -2 $O/pytest_nbr.log
for rep in 1 2; do
  timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "nbr_shfl=0;nbr_shfl=2;nbr_shfl=0;nbr_shfl=2;nbr_shfl=0;nbr_shfl=2" --rounds 6 > $O/sweep_vadv_nbr_$rep.log 2>&1 || { tail -30 $O/sweep_vadv_nbr_$rep.log; exit 1; }
  grep variant $O/sweep_vadv_nbr_$rep.log
done
