#!/bin/bash
# Round 5: spread of vadv / staged / hdiff times over placements of ALL their fields (one process
# each, scripts/column_placement_probe.py), to see whether re-homing read fields could pay.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05y}
mkdir -p $O
for c in vadv vadv staged hdiff; do
  timeout -k 10 240 python3 scripts/column_placement_probe.py --config $c --sets 8 --reps 6 >> $O/plain_$c.jsonl 2>> $O/plain.err || { tail -20 $O/plain.err; exit 1; }
  python3 -c "import json; d=[json.loads(l) for l in open('$O/plain_$c.jsonl')][-1]; print('$c', [s['ms'] for s in d['sets']])"
done
