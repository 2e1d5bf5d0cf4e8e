#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s
for c in hdiff hdiff hdiff_f32 vadv tridiag; do
  timeout -k 10 240 python3 scripts/placement_two_stage.py --config $c 2>> gpurun_out/r03s/err.log | tee -a gpurun_out/r03s/two_stage.jsonl || exit 1
done
