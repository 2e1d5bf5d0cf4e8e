#!/bin/bash
# Round 4: GPU suite + smoke, the default bench line (vadv now with the auto register band), the
# tile-height sweep of the staged config, and a kernel trace of the 2-D halo step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  bash scripts/gpu_tests.sh || exit $?
fi
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -u scripts/sweep.py --config staged --variants "tile_by=8;tile_by=16;tile_by=16,tile_ti=48;tile_by=8,tile_ti=48" \
  --rounds 6 > $O/sweep_staged_tile_by.log 2>&1 || { tail -30 $O/sweep_staged_tile_by.log; exit 1; }
cat $O/sweep_staged_tile_by.log
timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "kreg=96;kreg=104;kreg=112,kring=6;kreg=120,kring=4;kreg=96,kring=6;kreg=96,kreg_pf=12" \
  --rounds 6 > $O/sweep_vadv_band_size.log 2>&1 || { tail -30 $O/sweep_vadv_band_size.log; exit 1; }
cat $O/sweep_vadv_band_size.log
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_halo2d -o kt -- python3 bench.py --no-extra --no-cpu-baseline --steps 20 --halo-selfcomm --decomp 2d --placement-candidates 0 > $O/kt_halo2d.log 2>&1 || { tail -30 $O/kt_halo2d.log; exit 1; }
grep '^{"metric"' $O/kt_halo2d.log | cut -c1-200
