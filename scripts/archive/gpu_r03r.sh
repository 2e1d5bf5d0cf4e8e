#!/bin/bash
# N>1 rehearsal with placement tuning on one GPU (2 ranks over gloo), then the RCCL self-exchange
# line (world 1, the rank its own periodic neighbour through RCCL).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03r
CONFIG=hdiff_f32 bash scripts/dist_rehearsal.sh || exit 1
cp gpurun_out/dist_jstrips.json gpurun_out/dist_2d.json gpurun_out/r03r/
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29534
timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm > gpurun_out/r03r/selfcomm.json 2> gpurun_out/r03r/selfcomm.err || { tail -20 gpurun_out/r03r/selfcomm.err; exit 1; }
cat gpurun_out/r03r/selfcomm.json
