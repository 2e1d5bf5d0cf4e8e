#!/bin/bash
# Round 6 (i): tile_rows=2 (two J rows per thread) -- tile goldens under the two-row geometries,
# then timing + HBM traffic for the staged and hdiff_f32 tile configs against the defaults.
# (PMC passes build their single-variant libraries on the box: no GTMI_NO_COMPILE there.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06i
if [ -z "$SKIP_TESTS" ]; then
GTMI_NO_COMPILE=1 timeout -k 10 600 python -u -m pytest tests/test_tile.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "geom11 or geom12 or geom13" > gpurun_out/r06i/pytest_tile_rows.log 2>&1 || { tail -30 gpurun_out/r06i/pytest_tile_rows.log; exit 1; }
tail -2 gpurun_out/r06i/pytest_tile_rows.log
fi
CONFIG=hdiff_f32 VARIANTS="tile_order=0;tile_rows=2,tile_bx=128,tile_by=8;tile_rows=2,tile_bx=64,tile_by=8;tile_rows=2,tile_bx=128,tile_by=4" \
  bash scripts/variant_pmc.sh || exit $?
CONFIG=staged VARIANTS="tile_order=0;tile_rows=2,tile_bx=128,tile_by=8" bash scripts/variant_pmc.sh || exit $?
cp -r gpurun_out/vpmc_staged gpurun_out/vpmc_hdiff_f32 gpurun_out/r06i/ 2>/dev/null
