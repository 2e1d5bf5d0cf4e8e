#!/bin/bash
# Round 5: column-kernel block shape and block order re-swept on today's kernels (register band,
# LDS tail, head placement); last swept in round 1 before any of them existed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05s}
mkdir -p $O
for cfg in tridiag vadv; do
  timeout -k 10 400 python3 scripts/sweep.py --config $cfg --rounds 7 --variants "col_bx=64;col_bx=128;col_bx=256;col_order=0" \
    > $O/sweep_$cfg.log 2>&1 || { tail -20 $O/sweep_$cfg.log; exit 1; }
  grep -v Warn $O/sweep_$cfg.log
done
