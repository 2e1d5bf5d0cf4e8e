#!/bin/bash
# Round 5: differential fuzz stress of the new column/tile schedules: 120 base programs + 200
# sweep-pair / tile programs (seeds 7000+) against the numpy backend, at the default level counts
# and at nk = 120 (register bands, head/tail caches, blocked tile levels all reached).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05n}
mkdir -p $O
GTMI_FUZZ_V3=200 timeout -k 10 500 python -u -m pytest tests/test_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/fuzz_default_nk.log 2>&1 || { tail -40 $O/fuzz_default_nk.log; exit 1; }
tail -1 $O/fuzz_default_nk.log
GTMI_FUZZ_V3=200 GTMI_FUZZ_NK=120 timeout -k 10 600 python -u -m pytest tests/test_fuzz.py -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $O/fuzz_nk120.log 2>&1 || { tail -40 $O/fuzz_nk120.log; exit 1; }
tail -1 $O/fuzz_nk120.log
