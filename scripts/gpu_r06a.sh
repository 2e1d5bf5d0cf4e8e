#!/bin/bash
# Round 6 (a): GPU suite + smoke on the prebuilt libraries (key log), the default bench line under
# rocprofv3 kernel-trace stats, then two questions asked with counters:
#   staged: where does the tile kernel's 1.105x traffic come from (J halo rows or I halo lines)?
#           FETCH/WRITE per tile order / geometry (scripts/variant_pmc.sh)
#   C5 tile: where do hdiff f32's wave cycles go next to hdiff f64's (scripts/pmc_waits.sh A-D)?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06a}
mkdir -p $O
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $O/kt_bench -o kt -- python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
grep '^{"metric"' $O/bench.json | cut -c1-300
[ -n "$SKIP_STAGED" ] || CONFIG=staged VARIANTS="tile_order=0;tile_order=1;tile_order=2;tile_by=8;tile_by=8,tile_bx=128,tile_ti=112" \
  bash scripts/variant_pmc.sh > $O/staged_variants.log 2>&1 || { tail -30 $O/staged_variants.log; exit 1; }
cat $O/staged_variants.log | grep -v "^built"
[ -n "$SKIP_WAITS" ] || CONFIGS="hdiff_f32 hdiff" TAG=${TAG:-r06a} PASSES="A B C D" bash scripts/pmc_waits.sh > $O/waits.log 2>&1 || { tail -30 $O/waits.log; exit 1; }
tail -40 $O/waits.log
# the LDS-DMA prefetch ring against the register ring at one wave per SIMD
if [ -z "$SKIP_LAB" ]; then
  (cd scripts/lab && timeout -k 10 180 ./ldsring_lab 20) > $O/ldsring_lab.log 2>&1 || { tail -20 $O/ldsring_lab.log; exit 1; }
  cat $O/ldsring_lab.log
fi
