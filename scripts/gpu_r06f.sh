#!/bin/bash
# Round 6 closing evidence: GPU suite + smoke on prebuilt libraries (key log), then the default
# bench command under rocprofv3 kernel-trace stats (the line and the per-kernel averages from the
# same run).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06f}
mkdir -p $O
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $O/kt_bench -o kt -- python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
grep '^{"metric"' $O/bench.json | cut -c1-300
