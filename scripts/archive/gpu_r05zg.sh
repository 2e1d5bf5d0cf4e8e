#!/bin/bash
# Round 5: the default bench line with the column configs tuned over all their fields
# (--placement-scope auto), twice in separate processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05zg}
mkdir -p $O
for i in 1 2; do
  GTMI_NO_COMPILE=1 timeout -k 10 400 python3 bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -30 $O/bench_$i.err; exit 1; }
  python3 -c "
import json; b=json.load(open('$O/bench_$i.json')); r=b['roofline']; print('hdiff', r['kernel_ms'], r['frac'])
for k,c in b['extra_configs'].items(): print(k, c['kernel_ms'], c['frac'], c.get('placement',{}).get('scope'), c.get('placement',{}).get('candidates_ms'))"
done
