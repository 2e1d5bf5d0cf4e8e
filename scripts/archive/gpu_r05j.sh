#!/bin/bash
# Round 5 checkpoint: GPU suite + smoke with every library prebuilt (GTMI_NO_COMPILE=1, key log
# -> tests/gpu_build_keys.txt), then the default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05j}
mkdir -p $O
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
