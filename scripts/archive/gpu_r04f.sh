#!/bin/bash
# Round 4: traffic of the new vadv library (kernel trace + FETCH/WRITE passes), and confirmation
# sweeps of the band prefetch distance (vadv) and the tile height (staged).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
CONFIGS="vadv" TAG=r04f timeout -k 10 600 bash scripts/profile.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
tail -3 $O/profile.log
timeout -k 10 300 python -u scripts/sweep.py --config vadv --variants "kreg=96;kreg=96,kreg_pf=12;kreg=96,kreg_pf=16;kreg=96,kring=6,kreg_pf=12;kreg=96,kreg_pf=24" \
  --rounds 8 > $O/sweep_vadv_band_pf.log 2>&1 || { tail -30 $O/sweep_vadv_band_pf.log; exit 1; }
cat $O/sweep_vadv_band_pf.log
timeout -k 10 300 python -u scripts/sweep.py --config staged --variants "tile_by=8;tile_by=16;tile_by=8;tile_by=16" \
  --rounds 8 > $O/sweep_staged_tile_by.log 2>&1 || { tail -30 $O/sweep_staged_tile_by.log; exit 1; }
cat $O/sweep_staged_tile_by.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "halo" tests/test_gpu_halo.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_halo.log 2>&1 || { tail -30 $O/pytest_halo.log; exit 1; }
tail -1 $O/pytest_halo.log
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
for d in 2d jstrips 2d; do
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm --decomp $d --placement-candidates 0 2>> $O/halo.err >> $O/halo.log || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_halo2d -o kt -- python3 bench.py --no-extra --no-cpu-baseline --steps 20 --halo-selfcomm --decomp 2d --placement-candidates 0 > $O/kt_halo2d.log 2>&1 || { tail -30 $O/kt_halo2d.log; exit 1; }
echo done
