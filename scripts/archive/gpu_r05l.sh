#!/bin/bash
# Round 5: several levels per LDS barrier in tile kernels (tile_lblock): tile tests under every
# geometry, then staged and every tile program timed (plus a timing-only run without barriers).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05l}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_tile.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_tile.log 2>&1 || { tail -40 $O/pytest_tile.log; exit 1; }
tail -1 $O/pytest_tile.log
timeout -k 10 300 python3 scripts/sweep.py --config staged --rounds 9 --variants \
  "tile=1;tile_lblock=2;tile_lblock=4;tile_by=16;tile_by=16,tile_lblock=2;probe_nobar=1" > $O/sweep_staged.log 2>&1 || { tail -20 $O/sweep_staged.log; exit 1; }
grep -v Warn $O/sweep_staged.log
timeout -k 10 500 python3 scripts/tile_probe.py --variants "tile_by=8;tile_lblock=2;tile_lblock=4;tile_by=16,tile_lblock=2" \
  > $O/tile_probe.log 2>&1 || { tail -20 $O/tile_probe.log; exit 1; }
grep -v Warn $O/tile_probe.log
