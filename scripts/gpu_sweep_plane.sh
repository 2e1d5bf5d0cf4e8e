#!/bin/bash
# plane-kernel sweep: prefetch depth / occupancy / load policy (interleaved A/B per config)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VH=${VH:-"jmirror=1;nt_load=2;prefetch=1;prefetch=2;prefetch=0;prefetch=2,min_blocks=6"}
for c in ${CONFIGS:-hdiff hdiff_f32 lap5}; do
  timeout -k 10 300 python scripts/sweep.py --config $c --rounds 7 --variants "$VH" > gpurun_out/sweep_$c.log 2>&1 || exit $?
  grep '^{' gpurun_out/sweep_$c.log
done
