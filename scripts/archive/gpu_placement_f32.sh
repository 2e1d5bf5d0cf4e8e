#!/bin/bash
# hdiff f32 tile (C5 per-GPU workload): HBM channel aliasing -- base residues, I-pitch and K-stride paddings
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/placement_residue.py --config hdiff_f32 > gpurun_out/pl_f32_res.log 2>&1 || { tail -20 gpurun_out/pl_f32_res.log; exit 1; }
cat gpurun_out/pl_f32_res.log
timeout -k 10 300 python scripts/placement_residue.py --config hdiff_f32 --ipad 0,8,32,64,96 > gpurun_out/pl_f32_ipad.log 2>&1 || { tail -20 gpurun_out/pl_f32_ipad.log; exit 1; }
cat gpurun_out/pl_f32_ipad.log
timeout -k 10 300 python scripts/placement_residue.py --config hdiff_f32 --kpad 0,256,4096,65536 > gpurun_out/pl_f32_kpad.log 2>&1 || { tail -20 gpurun_out/pl_f32_kpad.log; exit 1; }
cat gpurun_out/pl_f32_kpad.log
