#!/bin/bash
# interleaved variant sweeps only (scripts/sweep_list.txt: "<config> <variants>" per line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
while read -r cfg variants; do
  [ -z "$cfg" ] && continue
  echo "== sweep $cfg"
  timeout -k 10 400 python scripts/sweep.py --config $cfg --variants "$variants" > gpurun_out/sweep_$cfg.log 2>&1
  rc=$?; grep -v Warning gpurun_out/sweep_$cfg.log | grep -v "cls = be" | tail -14
  [ $rc -eq 0 ] || exit $rc
done < scripts/sweep_list.txt
