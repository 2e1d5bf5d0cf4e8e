#!/bin/bash
# parity tests + interleaved variant sweeps (one process per config)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
while read -r cfg variants; do
  [ -z "$cfg" ] && continue
  echo "== sweep $cfg"
  timeout -k 10 300 python scripts/sweep.py --config $cfg --variants "$variants" > gpurun_out/sweep_$cfg.log 2>&1
  rc=$?; grep -v Warning gpurun_out/sweep_$cfg.log | grep -v "cls = be" | tail -12
  [ $rc -eq 0 ] || exit $rc
done < scripts/sweep_list.txt
