#!/bin/bash
# Per-rank exchange overhead A/B on one GPU (rank = own periodic neighbour through RCCL):
# alternating processes per variant, one JSON summary line each -> gpurun_out/halo_ab.log
#   VARIANTS="1d:GTMI_HALO_BANDS=halo 1d:GTMI_HALO_BANDS=unpack_main 2d:GTMI_HALO_STREAM=main" ROUNDS=2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
for r in $(seq "${ROUNDS:-2}"); do
  for v in $VARIANTS; do
    dec=${v%%:*}; envs=${v#*:}
    extra=""; [ "$dec" = 2d ] && extra="--decomp 2d"
    line=$(env ${envs//,/ } timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm $extra 2>>gpurun_out/halo_ab.err) || exit 1
    echo "$v $(echo "$line" | python3 -c 'import json,sys; d=json.loads(sys.stdin.readlines()[-1]); a=d["halo_ab"]; print(a["plain_ms_per_step"], a["halo_ms_per_step"], a["overhead"])')" | tee -a gpurun_out/halo_ab.log
  done
done
