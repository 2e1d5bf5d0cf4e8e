#!/bin/bash
# hdiff_f32 occupancy sweep: min_blocks (launch-bounds register cap, spills) x prefetch depth
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --config hdiff_f32 --rounds 7 --variants "jchunk=0;min_blocks=5;prefetch=1,min_blocks=5;prefetch=1;prefetch=1,min_blocks=6;min_blocks=6" > gpurun_out/sweep_occ.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_occ.log
