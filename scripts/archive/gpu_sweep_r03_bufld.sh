#!/bin/bash
# round 3: bufld on the f64 plane configs (interleaved A/B in one process per config, bit-exact check)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 200 python3 -u scripts/sweep.py --config lap5 --variants "bufld=0;bufld=1;bufld=1,prefetch=2;bufld=1,prefetch=6" > gpurun_out/sweep_bufld_lap5.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/sweep.py --config copy --variants "bufld=0;bufld=1;bufld=1,prefetch=2" > gpurun_out/sweep_bufld_copy.log 2>&1 || exit 1
timeout -k 10 200 python3 -u scripts/sweep.py --config hdiff_blocks --variants "bufld=0;bufld=1" > gpurun_out/sweep_bufld_blocks.log 2>&1 || exit 1
grep -h variant gpurun_out/sweep_bufld_*.log
