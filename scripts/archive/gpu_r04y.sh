#!/bin/bash
# Round 4 final check: GPU suite + smoke with every library prebuilt (GTMI_NO_COMPILE=1), then the
# default bench line (traffic fields must come from the PMC records of the libraries that ran).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
GTMI_NO_COMPILE=1 bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
GTMI_NO_COMPILE=1 timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
