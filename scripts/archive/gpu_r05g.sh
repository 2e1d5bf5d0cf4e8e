#!/bin/bash
# Round 5: head vs tail placement of the sweep-to-sweep cache (ktail_head): the column goldens
# under every schedule and the full-size tridiag vs the C oracle, then interleaved A/B sweeps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "column_options or golden_case or full_size" \
  --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_head.log 2>&1 || { tail -40 $O/pytest_head.log; exit 1; }
tail -1 $O/pytest_head.log
timeout -k 10 300 python3 scripts/sweep.py --config tridiag --rounds 7 --variants \
  "ktail_head=0;ktail_head=1;ktail_head=1,kreg=32;ktail_head=1,kreg=64;ktail_head=1,kreg=80;ktail_head=1,kreg=0" \
  > $O/sweep_tridiag_head.log 2>&1 || { tail -20 $O/sweep_tridiag_head.log; exit 1; }
grep -v Warn $O/sweep_tridiag_head.log
timeout -k 10 300 python3 scripts/sweep.py --config vadv --rounds 7 --variants \
  "ktail_head=0;ktail_head=1,kreg=64;ktail_head=1,kreg=48;ktail_head=1,kreg=80" \
  > $O/sweep_vadv_head.log 2>&1 || { tail -20 $O/sweep_vadv_head.log; exit 1; }
grep -v Warn $O/sweep_vadv_head.log
