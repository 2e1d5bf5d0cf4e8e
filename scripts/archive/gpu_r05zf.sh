#!/bin/bash
# Round 5: placement tuning over ALL fields (scope="all"). Placement tests (incl. the new scope
# cases) on prebuilt libraries, then vadv / staged / tridiag in fresh processes tuned with the
# written fields only and with every field.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05zf}
mkdir -p $O
GTMI_NO_COMPILE=1 timeout -k 10 300 python -u -m pytest tests/test_placement.py -x -v -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_placement.log 2>&1 || { tail -40 $O/pytest_placement.log; exit 1; }
tail -1 $O/pytest_placement.log
for c in vadv staged tridiag vadv; do
  for sc in written all; do
    GTMI_NO_COMPILE=1 timeout -k 10 300 python3 bench.py --config $c --no-extra --no-cpu-baseline --steps 20 --warmup 3 \
      --placement-scope $sc >> $O/bench_${c}_$sc.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
    tail -1 $O/bench_${c}_$sc.jsonl | python3 -c "import json,sys; b=json.loads(sys.stdin.read()); r=b['roofline']; print('$c $sc', r['kernel_ms_untuned'], r['kernel_ms'], b['placement'].get('candidates_ms'))"
  done
done
