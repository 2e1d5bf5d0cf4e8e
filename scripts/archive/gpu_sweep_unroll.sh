#!/bin/bash
# plane kernels: manual row unroll (row_unroll=U copies of the row step per trip) vs default
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --config hdiff_f32 --rounds 7 --variants "jchunk=0;row_unroll=2;row_unroll=6;prefetch=1,row_unroll=6;prefetch=1" > gpurun_out/sweep_unroll_f32.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll_f32.log
timeout -k 10 300 python scripts/sweep.py --config hdiff --rounds 7 --variants "jchunk=0;row_unroll=6" > gpurun_out/sweep_unroll_hdiff.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll_hdiff.log
timeout -k 10 300 python scripts/sweep.py --config lap5 --rounds 7 --variants "jchunk=0;row_unroll=2;row_unroll=4" > gpurun_out/sweep_unroll_lap5.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll_lap5.log
