#!/bin/bash
# f32 tile: register cap of 4 blocks per CU (131 -> 127 VGPRs, 3 -> 4 waves per SIMD) against the
# default, alternating processes; each line has placement-tuned buffers.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03t
for r in 1 2 3; do
  for o in "" "--opt min_blocks=4"; do
    timeout -k 10 200 python3 bench.py --config hdiff_f32 --no-extra --no-cpu-baseline --sustain 0 $o > gpurun_out/r03t/line.json 2>> gpurun_out/r03t/err.log || exit 1
    python3 -c "
import json,sys
r=json.loads(open('gpurun_out/r03t/line.json').read().strip().splitlines()[-1])
print(json.dumps({'opt': '$o', 'kernel_ms': r['roofline']['kernel_ms'], 'frac': r['roofline']['frac'], 'sets': r['placement']['candidates_ms']}))" | tee -a gpurun_out/r03t/ab.jsonl
  done
done
