#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03q
for c in vadv; do
  timeout -k 10 240 python3 scripts/scratch_placement_probe.py --config $c --sets 8 2>> gpurun_out/r03q/err.log | tee -a gpurun_out/r03q/scratch.jsonl || exit 1
done
