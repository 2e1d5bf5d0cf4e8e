#!/bin/bash
# plane kernels: output-strip alignment (strip_align elements) vs the 128-B default, f32 and f64 hdiff
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --config hdiff_f32 --rounds 7 --variants "jchunk=0;strip_align=8;strip_align=16;strip_align=8,row_unroll=2" > gpurun_out/sweep_align_f32.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_align_f32.log
timeout -k 10 300 python scripts/sweep.py --config hdiff --rounds 7 --variants "jchunk=0;strip_align=4;strip_align=8" > gpurun_out/sweep_align_hdiff.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_align_hdiff.log
