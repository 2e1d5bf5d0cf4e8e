#!/bin/bash
# Round 5: wave-cycle split of the plane kernels (hdiff f64, the C5 f32 tile) and the staged tile
# kernel, first allocation (no placement tuning).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05f}
mkdir -p $O
CONFIGS="hdiff hdiff_f32 staged" TAG=${TAG:-r05f} PASSES="A C" timeout -k 10 600 bash scripts/pmc_waits.sh > $O/waits.log 2>&1 \
  || { tail -30 $O/waits.log; exit 1; }
cp gpurun_out/waits_${TAG:-r05f}/summary.json $O/waits_summary.json
python3 -c "import json; d=json.load(open('$O/waits_summary.json')); [print(k, {x: d[k].get(x) for x in ('parked','stalled','active','issue_share_SCA','issue_share_VALU','issue_share_LDS')}) for k in d]"
