#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03aa
CONFIG=hdiff bash scripts/dist_rehearsal.sh || exit 1
cp gpurun_out/dist_jstrips.json gpurun_out/dist_2d.json gpurun_out/r03aa/
