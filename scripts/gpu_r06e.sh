#!/bin/bash
# Round 6 (e): the C5 tile's lane width. 4 f32 cells per 16-B lane (default) holds 129 VGPRs,
# 3 waves per SIMD; 2 cells per 8-B lane holds 70 (7 waves). Interleaved on shared buffers,
# every variant bit-checked against the first (scripts/sweep.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06e}
mkdir -p $O
GTMI_NO_COMPILE=1 timeout -k 10 400 python scripts/sweep.py --config hdiff_f32 --rounds 5 \
  --variants "vector=4;vector=2;vector=2,strip_align=16;vector=2,bufld=1;vector=2,strip_align=16,bufld=1" \
  > $O/sweep_f32_vector.log 2>&1 || { tail -20 $O/sweep_f32_vector.log; exit 1; }
grep -v "^built" $O/sweep_f32_vector.log
