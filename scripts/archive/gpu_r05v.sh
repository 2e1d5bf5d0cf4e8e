#!/bin/bash
# Round 5 (follow-up of r05u): is the bench line's faster tridiag/vadv the GPU's state after the
# earlier configs ran? 8 s of a torch copy loop, or of the hdiff workload, before the fields.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05v}
mkdir -p $O
: > $O/alloc.jsonl
for h in "" "--warm-s 8 --warm-with copy" "--warm-s 8 --warm-with hdiff" "" "--warm-s 8 --warm-with hdiff"; do
  timeout -k 10 120 python3 scripts/alloc_probe.py --config tridiag $h --tag "tridiag $h" 2>>$O/alloc.err | grep '^{' >> $O/alloc.jsonl || { tail -20 $O/alloc.err; exit 1; }
  tail -1 $O/alloc.jsonl | cut -c1-200
done
