#!/bin/bash
# Round 6 (g): differential-fuzz stress after this round's codegen changes (tile blocking rule,
# LDS budget, exact-product fma): 444 random programs (120 default + 150 extra + 174 of the
# sweep-pair / tile templates) on the GPU, each bit-exact against the numpy backend.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06g}
mkdir -p $O
GTMI_NO_COMPILE=1 GTMI_FUZZ_OPTS="$FUZZ_OPTS" GTMI_FUZZ_NK=${FUZZ_NK:-0} GTMI_FUZZ_EXTRA=150 GTMI_FUZZ_V3=174 timeout -k 10 900 python -u -m pytest tests/test_fuzz.py -q -m gpu \
  --timeout 120 --timeout-method thread -p no:cacheprovider > $O/fuzz_stress_nk${FUZZ_NK:-0}.log 2>&1
rc=$?; tail -3 $O/fuzz_stress_nk${FUZZ_NK:-0}.log; exit $rc
