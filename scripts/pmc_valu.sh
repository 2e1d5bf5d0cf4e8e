#!/bin/bash
# VALU activity of the bench kernels (one --pmc pass per config; SQ/GRBM counters only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_valu
for cfg in ${CONFIGS:-hdiff hdiff_f32 tridiag vadv}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --output-format csv -d gpurun_out/pmc_valu/$cfg -o pmc -- python3 bench.py --config $cfg --steps 3 --warmup 1 \
    --no-cpu-baseline --no-extra > gpurun_out/pmc_valu/$cfg.log 2>&1 || { tail -5 gpurun_out/pmc_valu/$cfg.log; exit 1; }
done
find gpurun_out/pmc_valu -name "*counter_collection.csv"
