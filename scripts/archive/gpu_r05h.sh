#!/bin/bash
# Round 5: PMC record of the new tridiag library (head placement) + kernel trace, and the
# memory-pipe counters (pass D) of the staged tile kernel at tile_by 8 and 16.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05h}
mkdir -p $O
CONFIGS="tridiag" TAG=${TAG:-r05h} timeout -k 10 600 bash scripts/profile.sh > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
grep '^{"metric"' $O/profile.log | cut -c1-200
CONFIGS="staged" TAG=${TAG:-r05h}_by8 PASSES="A D" timeout -k 10 300 bash scripts/pmc_waits.sh > $O/waits_by8.log 2>&1 || { tail -30 $O/waits_by8.log; exit 1; }
CONFIGS="staged" TAG=${TAG:-r05h}_by16 PASSES="A D" BENCH_OPTS="--opt tile_by=16" timeout -k 10 300 bash scripts/pmc_waits.sh > $O/waits_by16.log 2>&1 || { tail -30 $O/waits_by16.log; exit 1; }
for t in by8 by16; do cp gpurun_out/waits_${TAG:-r05h}_$t/summary.json $O/waits_staged_$t.json; done
python3 -c "
import json
for t in ('by8','by16'):
    d=json.load(open('$O/waits_staged_%s.json' % t))['staged']
    print(t, {k: v for k, v in d.items() if 'dispatches' not in k})"
