#!/bin/bash
# Round 5: is hdiff's slow placement mode (first allocation 2.81 ms) also a latency effect that
# deeper row prefetch would hide? Prefetch variants x all-field placement sets in one process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05zl}
mkdir -p $O
GTMI_NO_COMPILE=1 timeout -k 10 500 python3 scripts/column_placement_probe.py --config hdiff --sets 5 --reps 5 --rounds 3 \
  --variants "jchunk=0;prefetch=3;prefetch=6;prefetch=8" > $O/matrix_hdiff.jsonl 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
cut -c1-200 $O/matrix_hdiff.jsonl
