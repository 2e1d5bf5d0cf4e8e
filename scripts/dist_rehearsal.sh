#!/bin/bash
# Rehearse the N>1 bench path on ONE GPU: 2 ranks over gloo (RCCL needs one GPU per rank).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for decomp in jstrips 2d; do
  echo "== 2-rank gloo rehearsal, $decomp"
  GTMI_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --config ${CONFIG:-hdiff_f32} --decomp $decomp \
    --steps 3 --warmup 1 > gpurun_out/dist_$decomp.json 2> gpurun_out/dist_$decomp.err || { tail -20 gpurun_out/dist_$decomp.err; exit 1; }
  cat gpurun_out/dist_$decomp.json
done
