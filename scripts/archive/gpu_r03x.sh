#!/bin/bash
# Headline-only bench lines (default flags otherwise) in two fresh processes: is the tuned
# headline stable across processes on a box?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03x
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline > gpurun_out/r03x/line$r.json 2>> gpurun_out/r03x/err.log || exit 1
  python3 -c "
import json
r=json.loads(open('gpurun_out/r03x/line$r.json').read().strip().splitlines()[-1])
print(json.dumps({'kernel_ms': r['roofline']['kernel_ms'], 'frac': r['roofline']['frac'], 'ms_per_step': r['ms_per_step'], 'sets': r['placement']['candidates_ms'], 'pci': r['box']['identity']['pci'], 'serial': r['box']['identity'].get('serial_number')}))" | tee -a gpurun_out/r03x/summary.jsonl
done
