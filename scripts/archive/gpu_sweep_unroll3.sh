#!/bin/bash
# hdiff f64 / f32: row_unroll 2 and 3; lap5: auto unroll (default) vs prefetch=6 vs rolled
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --config hdiff --rounds 9 --variants "jchunk=0;row_unroll=2;row_unroll=3" > gpurun_out/sweep_unroll3_hdiff.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll3_hdiff.log
timeout -k 10 300 python scripts/sweep.py --config hdiff_f32 --rounds 9 --variants "jchunk=0;row_unroll=2;row_unroll=3" > gpurun_out/sweep_unroll3_f32.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll3_f32.log
timeout -k 10 300 python scripts/sweep.py --config lap5 --rounds 11 --variants "jchunk=0;prefetch=6;row_unroll=0" > gpurun_out/sweep_unroll3_lap5.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll3_lap5.log
