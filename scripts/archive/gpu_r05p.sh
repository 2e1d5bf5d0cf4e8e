#!/bin/bash
# Round 5: tile_by auto (16 rows for a one-row J halo on 8-byte cells). GPU suite + smoke on
# prebuilt libraries, then staged and every tile program timed at 8 rows against the auto rule,
# then the PMC record of the new staged library and the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05p}
mkdir -p $O
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
timeout -k 10 300 python3 scripts/sweep.py --config staged --rounds 9 --variants "tile_by=8;tile_by=-1" \
  > $O/sweep_staged.log 2>&1 || { tail -20 $O/sweep_staged.log; exit 1; }
grep -v Warn $O/sweep_staged.log
timeout -k 10 500 python3 scripts/tile_probe.py --variants "tile_by=8;tile_by=-1" \
  > $O/tile_probe.log 2>&1 || { tail -20 $O/tile_probe.log; exit 1; }
grep -v Warn $O/tile_probe.log
GTMI_NO_COMPILE=1 CONFIGS="staged" TAG=${TAG:-r05p} timeout -k 10 600 bash scripts/profile.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
