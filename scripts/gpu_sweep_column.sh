#!/bin/bash
# column-kernel occupancy x K-prefetch sweep (tridiag, vadv) + HBM traffic of the candidates
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
VT="kprefetch=0;col_occupancy=1,kprefetch=8;col_occupancy=1,kprefetch=16;col_occupancy=2,kprefetch=8;col_occupancy=2,kprefetch=4;kprefetch=4"
timeout -k 10 300 python scripts/sweep.py --config tridiag --rounds 7 --variants "$VT" > gpurun_out/sweep_tridiag.log 2>&1 &&
timeout -k 10 300 python scripts/sweep.py --config vadv --rounds 7 --variants "$VT" > gpurun_out/sweep_vadv.log 2>&1 &&
CONFIG=tridiag VARIANTS="kprefetch=0;col_occupancy=1,kprefetch=16;col_occupancy=2,kprefetch=8" timeout -k 10 600 bash scripts/variant_pmc.sh > gpurun_out/vpmc_tridiag.log 2>&1 &&
CONFIG=hdiff VARIANTS="jmirror=0;jmirror=1" timeout -k 10 600 bash scripts/variant_pmc.sh > gpurun_out/vpmc_hdiff.log 2>&1
echo "rc=$?"
