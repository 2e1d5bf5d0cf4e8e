#!/bin/bash
# Round 5: does the written-fields placement tuner reach the fast mode in a fresh process for
# vadv (1 of its 5 fields written) and staged, as it does for tridiag (r05h)?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05ze}
mkdir -p $O
for c in vadv vadv staged tridiag; do
  timeout -k 10 300 python3 bench.py --config $c --no-extra --no-cpu-baseline --steps 20 --warmup 3 >> $O/bench_$c.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  tail -1 $O/bench_$c.jsonl | python3 -c "import json,sys; b=json.loads(sys.stdin.read()); r=b['roofline']; print('$c', r['kernel_ms_untuned'], r['kernel_ms'], b['placement'].get('candidates_ms'))"
done
