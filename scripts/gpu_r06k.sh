#!/bin/bash
# Round 6 (k): staged tile geometry -- block-count quantisation (blocks per CU round) against
# the J-halo share: tile_ti 56/62, two-row tiles of 20-32 rows, 12-row tiles; timing + traffic.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
GTMI_NO_COMPILE=1 timeout -k 10 600 python -u -m pytest tests/test_tile.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "geom14 or geom15" > gpurun_out/r06k_pytest.log 2>&1 || { tail -30 gpurun_out/r06k_pytest.log; exit 1; }
tail -1 gpurun_out/r06k_pytest.log
CONFIG=staged VARIANTS="tile_order=0;tile_ti=56;tile_ti=62;tile_rows=2;tile_rows=2,tile_by=12;tile_rows=2,tile_by=10;tile_rows=2,tile_by=11;tile_by=12" bash scripts/variant_pmc.sh || exit $?
mkdir -p gpurun_out/r06k && cp -r gpurun_out/vpmc_staged gpurun_out/r06k/
