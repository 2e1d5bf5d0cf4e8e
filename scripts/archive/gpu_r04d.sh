#!/bin/bash
# Round 4 measurements: the default bench line (headline + extras + CPU baseline), the same
# command's hdiff kernel-trace stats, and the per-rank halo-exchange cost of both decompositions
# (rank as its own periodic neighbour through RCCL; in-process A/B against a plain launch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_hdiff -o kt -- python3 bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline > $O/kt_hdiff.log 2>&1 || { tail -30 $O/kt_hdiff.log; exit 1; }
grep '^{"metric"' $O/kt_hdiff.log
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
for d in jstrips 2d jstrips 2d; do
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm --decomp $d --placement-candidates 0 2>> $O/halo.err | tee -a $O/halo.log || exit 1
done
unset RANK LOCAL_RANK WORLD_SIZE MASTER_ADDR MASTER_PORT
# the N>1 path with in-place placement tuning in every rank (2 ranks on one GPU over gloo)
bash scripts/dist_rehearsal.sh > $O/dist_rehearsal.log 2>&1 || { tail -30 $O/dist_rehearsal.log; exit 1; }
cp gpurun_out/dist_*.json $O/ && cat $O/dist_rehearsal.log | tail -4
