#!/bin/bash
# round 3: host call cost on the current libraries, and the per-rank exchange cost (the rank as its
# own periodic RCCL neighbour, J strips and 2-D tiles) with the self-explaining halo_ab block
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 -u scripts/call_overhead.py > gpurun_out/call_overhead_r03.log 2>&1 || exit 1
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm > gpurun_out/halo_self_j.json 2> gpurun_out/halo_self_j.err || exit 1
timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm --decomp 2d > gpurun_out/halo_self_2d.json 2> gpurun_out/halo_self_2d.err || exit 1
cat gpurun_out/call_overhead_r03.log
python3 -c "
import json
for f in ('gpurun_out/halo_self_j.json', 'gpurun_out/halo_self_2d.json'):
    r = json.load(open(f)); print(f, r['ms_per_step'], r.get('halo_ab'))
"
