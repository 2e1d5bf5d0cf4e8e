#!/bin/bash
# Round 5: the N>1 bench path end to end on real hardware, with ranks sharing the one GPU of this
# box (gloo moves the halos through host memory; RCCL refuses two ranks on one device). Launched
# exactly as the driver launches N>1 (torch.distributed.run, one process per rank); times are not
# meaningful (the ranks share one GPU), the point is the flow: rendezvous, link probe, halo
# exchange with overlap, barrier-bracketed timing, max over ranks, one JSON line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05zb}
mkdir -p $O
export GTMI_DIST_BACKEND=gloo
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 5 --warmup 2 --placement-candidates 0 > $O/n2_jstrips.log 2>&1 || { tail -30 $O/n2_jstrips.log; exit 1; }
grep '^{"metric"' $O/n2_jstrips.log | cut -c1-400
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 4 --steps 5 --warmup 2 --placement-candidates 0 --decomp 2d > $O/n4_2d.log 2>&1 || { tail -30 $O/n4_2d.log; exit 1; }
grep '^{"metric"' $O/n4_2d.log | cut -c1-400
