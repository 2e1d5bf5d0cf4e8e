#!/bin/bash
# Round 5: K-streaming buffer loads in the column kernels (kbuf): column goldens under kbuf on the
# GPU, interleaved A/B of vadv / tridiag / staged, and the wave-cycle split of vadv and tridiag
# with kbuf=1 next to r05a's kbuf=0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "column_options" --timeout 120 \
  --timeout-method thread -p no:cacheprovider > $O/pytest_kbuf.log 2>&1 || { tail -40 $O/pytest_kbuf.log; exit 1; }
tail -1 $O/pytest_kbuf.log
for cfg in vadv tridiag; do
  timeout -k 10 200 python3 scripts/sweep.py --config $cfg --variants "kbuf=0;kbuf=1" --rounds 9 > $O/sweep_$cfg.log 2>&1 \
    || { tail -20 $O/sweep_$cfg.log; exit 1; }
  echo "== $cfg"; cat $O/sweep_$cfg.log | grep -v Warn
done
CONFIGS="vadv tridiag" TAG=${TAG:-r05b} BENCH_OPTS="--opt kbuf=1" timeout -k 10 600 bash scripts/pmc_waits.sh > $O/waits.log 2>&1 \
  || { tail -30 $O/waits.log; exit 1; }
cp gpurun_out/waits_${TAG:-r05b}/summary.json $O/waits_summary.json
python3 -c "import json; d=json.load(open('$O/waits_summary.json')); [print(k, {x: d[k].get(x) for x in ('parked','stalled','active','L2_hit','issue_share_SCA','issue_share_VALU')}) for k in d]"
# staged tile geometry and lap5 work order (launch-size probe follow-up)
timeout -k 10 200 python3 scripts/sweep.py --config staged --variants "tile=1;tile_by=16;tile_bx=128;tile_bx=128,tile_by=4" --rounds 9 > $O/sweep_staged.log 2>&1 || { tail -20 $O/sweep_staged.log; exit 1; }
echo "== staged"; grep -v Warn $O/sweep_staged.log
for cfg in lap5 lap5_k160; do
  timeout -k 10 200 python3 scripts/sweep.py --config $cfg --variants "order=6;order=5;order=0" --rounds 9 > $O/sweep_$cfg.log 2>&1 || { tail -20 $O/sweep_$cfg.log; exit 1; }
  echo "== $cfg"; grep -v Warn $O/sweep_$cfg.log
done
