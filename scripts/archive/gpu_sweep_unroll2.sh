#!/bin/bash
# lap5 / copy: row_unroll repeat (11 interleaved rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --config lap5 --rounds 11 --variants "jchunk=0;row_unroll=4;row_unroll=3;row_unroll=8;row_unroll=4,prefetch=6" > gpurun_out/sweep_unroll2_lap5.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll2_lap5.log
timeout -k 10 300 python scripts/sweep.py --config copy --rounds 11 --variants "jchunk=0;row_unroll=4" > gpurun_out/sweep_unroll2_copy.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll2_copy.log
