#!/bin/bash
# Round 5 (follow-up of r05v: 8 s of the hdiff workload first makes tridiag 1.80 -> 1.56 ms, a
# copy loop does not): which part of it? A few hdiff steps only; other configs; hdiff with its
# cached blocks released before the tridiag fields are allocated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05w}
mkdir -p $O
: > $O/alloc.jsonl
for h in "--warm-s 0.001 --warm-with hdiff" "--warm-s 8 --warm-with hdiff --empty-cache" "--warm-s 8 --warm-with lap5" \
         "--warm-s 8 --warm-with copy" "--warm-s 8 --warm-with staged" "--warm-s 0.001 --warm-with copy" ""; do
  timeout -k 10 120 python3 scripts/alloc_probe.py --config tridiag $h --tag "tridiag $h" 2>>$O/alloc.err | grep '^{' >> $O/alloc.jsonl || { tail -20 $O/alloc.err; exit 1; }
  tail -1 $O/alloc.jsonl | cut -c1-230
done
