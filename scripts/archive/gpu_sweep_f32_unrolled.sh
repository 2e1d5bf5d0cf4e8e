#!/bin/bash
# hdiff f32 with the 2x row unroll: prefetch depth, J chunk, non-temporal loads (9 interleaved rounds)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python scripts/sweep.py --config hdiff_f32 --rounds 9 --variants "jchunk=0;prefetch=3;prefetch=1;jchunk=16;jchunk=8;nt_load=0" > gpurun_out/sweep_f32_unrolled.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_f32_unrolled.log
