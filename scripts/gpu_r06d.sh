#!/bin/bash
# Round 6 (d): C5 (BASELINE configs[4]) at its exact global size through the sharded path on one
# box: 8 ranks of 8192 x 1024 x 160 f32 sharing the GPU (gloo host-staged halos), every cell
# checked against the C oracle (tests/c5_sharded_check.py); the small version as the GPU test;
# then the hdiff_f32 traffic record on the library the exact-product fma re-keyed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06d}
mkdir -p $O
GTMI_NO_COMPILE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_c5_sharded.py -x -q -m gpu --timeout 280 \
  --timeout-method thread -p no:cacheprovider > $O/pytest_c5_sharded.log 2>&1 || { tail -30 $O/pytest_c5_sharded.log; exit 1; }
tail -1 $O/pytest_c5_sharded.log
GTMI_NO_COMPILE=1 GTMI_DIST_BACKEND=gloo OMP_NUM_THREADS=16 timeout -k 10 900 python -m torch.distributed.run --nnodes 1 \
  --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29571 tests/c5_sharded_check.py --ni 8192 --nj 1024 --nk 160 \
  > $O/c5_sharded_check.json 2> $O/c5_sharded_check.err || { tail -30 $O/c5_sharded_check.err; exit 1; }
cat $O/c5_sharded_check.json
[ -n "$SKIP_PMC" ] || { GTMI_NO_COMPILE=1 TAG=r06d CONFIGS="hdiff_f32" bash scripts/profile.sh > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }; }
echo done
