#!/bin/bash
# Round 4 closing measurements: GPU suite + smoke, then the default bench line, the vadv traffic
# of its final library (kernel trace + FETCH/WRITE passes) and the hdiff kernel-trace stats of
# the bench command itself.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUT_TAG:-r04g}
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  bash scripts/gpu_tests.sh || exit $?
fi
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json | cut -c1-400
CONFIGS="${PROF_CONFIGS:-vadv}" TAG=${PROF_TAG:-r04g} timeout -k 10 600 bash scripts/profile.sh > $O/profile_vadv.log 2>&1 || { tail -30 $O/profile_vadv.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_hdiff -o kt -- python3 bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline > $O/kt_hdiff.log 2>&1 || { tail -30 $O/kt_hdiff.log; exit 1; }
grep '^{"metric"' $O/kt_hdiff.log | cut -c1-300
