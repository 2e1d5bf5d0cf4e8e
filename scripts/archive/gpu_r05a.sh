#!/bin/bash
# Round 5, first call: GPU suite + smoke on prebuilt libraries (records every library key the run
# loads -> tests/gpu_build_keys.txt), the lap5/copy launch-size probe, and the wave-cycle split
# (SQ wait/active, L2 hit) of the column and plane kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
GTMI_NO_COMPILE=1 timeout -k 10 180 python3 scripts/shape_probe.py > $O/shape_probe.log 2>&1 || { tail -20 $O/shape_probe.log; exit 1; }
cat $O/shape_probe.log
GTMI_NO_COMPILE=1 CONFIGS="vadv copy tridiag lap5 lap5_k160" TAG=r05a timeout -k 10 900 bash scripts/pmc_waits.sh > $O/waits.log 2>&1 || { tail -30 $O/waits.log; exit 1; }
cp gpurun_out/waits_r05a/summary.json $O/waits_summary.json
python3 -c "import json; d=json.load(open('$O/waits_summary.json')); [print(k, {x: d[k].get(x) for x in ('parked','stalled','active','L2_hit','issue_share_VMEM','issue_share_VALU')}) for k in d]"
