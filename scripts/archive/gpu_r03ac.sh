#!/bin/bash
# How many candidate buffer sets does the tuner need? 12 sets for hdiff's out_field, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03ac
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --sustain 0 --placement-candidates 11 > gpurun_out/r03ac/line$r.json 2>> gpurun_out/r03ac/err.log || exit 1
  python3 -c "
import json
r=json.loads(open('gpurun_out/r03ac/line$r.json').read().strip().splitlines()[-1])
print(json.dumps({'kernel_ms': r['roofline']['kernel_ms'], 'sets': r['placement']['candidates_ms'], 'serial': r['box']['identity'].get('serial_number')}))" | tee -a gpurun_out/r03ac/summary.jsonl
done
