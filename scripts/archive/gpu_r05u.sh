#!/bin/bash
# Round 5: the column kernels run ~12 % slower on a fresh process's first allocations (r05t) than
# in the bench line, where they follow the hdiff/lap5 configs. Allocation history, one process per
# history: fresh; 24 GB held before the fields; 24 GB allocated and freed before the fields (the
# fields carved out of that cached segment by torch's caching allocator).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05u}
mkdir -p $O
: > $O/alloc.jsonl
for cfg in tridiag vadv; do
  for h in "" "--pre-gb 24" "--pre-gb 24 --carve" "" "--pre-gb 24 --carve"; do
    timeout -k 10 120 python3 scripts/alloc_probe.py --config $cfg $h --tag "$cfg $h" 2>>$O/alloc.err | grep '^{' >> $O/alloc.jsonl || { tail -20 $O/alloc.err; exit 1; }
    tail -1 $O/alloc.jsonl | cut -c1-160
  done
done
