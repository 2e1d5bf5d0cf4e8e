#!/bin/bash
# Round 3, placement tuner: bench line (default flags) + the same command under rocprofv3 kernel
# trace, for the headline and the C5 tile. Every GPU step has its own limit; first failure ends it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03p
timeout -k 10 600 python3 bench.py > gpurun_out/r03p/bench.json 2> gpurun_out/r03p/bench.err || { tail -20 gpurun_out/r03p/bench.err; exit 1; }
cat gpurun_out/r03p/bench.json
for cfg in hdiff hdiff_f32; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03p/kt_$cfg -o kt -- \
    python3 bench.py --config $cfg --steps 20 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/r03p/kt_$cfg.log 2>&1 || exit $?
  grep '^{"metric"' gpurun_out/r03p/kt_$cfg.log
done
