#!/bin/bash
# Round 6 (h): the driver's N>1 command shape end to end with this round's code, ranks sharing
# the one GPU of this box (gloo moves the halos through host memory; RCCL refuses two ranks on one
# device): 8 ranks in J strips (headline + the C5 leg) and 4 ranks as a 2x2 grid. Times are not
# scaling figures; the point is the flow and the line (dist, link probe, halo schedule, C5 leg).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06h}
mkdir -p $O
export GTMI_DIST_BACKEND=gloo GTMI_NO_COMPILE=1
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29527 \
  bench.py --gpus 8 --steps 5 --warmup 2 --placement-candidates 0 > $O/n8_jstrips.log 2>&1 || { tail -30 $O/n8_jstrips.log; exit 1; }
grep '^{"metric"' $O/n8_jstrips.log | cut -c1-300
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29528 \
  bench.py --gpus 4 --steps 5 --warmup 2 --placement-candidates 0 --decomp 2d > $O/n4_2d.log 2>&1 || { tail -30 $O/n4_2d.log; exit 1; }
grep '^{"metric"' $O/n4_2d.log | cut -c1-300
