#!/bin/bash
# hdiff f32: auto unroll (default, 2x) vs rolled, 11 interleaved rounds
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --config hdiff_f32 --rounds 11 --variants "jchunk=0;row_unroll=0" > gpurun_out/sweep_unroll4_f32.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_unroll4_f32.log
