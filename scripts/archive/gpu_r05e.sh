#!/bin/bash
# Round 5: tile height across every tile program (tile_by 8 vs 16), and whether the column
# kernels' issue stalls are the memory pipe pushing back (TA FIFO-full counters, VMEM in flight).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05e}
mkdir -p $O
timeout -k 10 400 python3 scripts/tile_probe.py --variants "tile_by=8;tile_by=16" > $O/tile_probe.log 2>&1 \
  || { tail -20 $O/tile_probe.log; exit 1; }
grep -v Warn $O/tile_probe.log
CONFIGS="vadv copy" TAG=${TAG:-r05e}_kb0 PASSES="D" timeout -k 10 300 bash scripts/pmc_waits.sh > $O/waits_kb0.log 2>&1 \
  || { tail -30 $O/waits_kb0.log; exit 1; }
CONFIGS="vadv" TAG=${TAG:-r05e}_kb1 PASSES="D" BENCH_OPTS="--opt kbuf=1" timeout -k 10 300 bash scripts/pmc_waits.sh > $O/waits_kb1.log 2>&1 \
  || { tail -30 $O/waits_kb1.log; exit 1; }
cp gpurun_out/waits_${TAG:-r05e}_kb0/summary.json $O/waits_D_kb0.json; cp gpurun_out/waits_${TAG:-r05e}_kb1/summary.json $O/waits_D_kb1.json
cat $O/waits_D_kb0.json $O/waits_D_kb1.json | grep -v dispatches
