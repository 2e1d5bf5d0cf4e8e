#!/bin/bash
# Round 5: the first allocations of a fresh process land in the slow placement mode on every box
# (tridiag 1.80 ms, hdiff 2.81 ms). One 24 GB block held first did not change that (r05u); do
# several medium blocks held first (the size of the fields themselves) move the fields to the
# fast mode?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05zd}
mkdir -p $O
: > $O/alloc.jsonl
for c in tridiag hdiff; do
  for h in "" "--pre-chunks 8 --pre-chunk-gb 1.5" "--pre-chunks 16 --pre-chunk-gb 1.5" "--pre-chunks 4 --pre-chunk-gb 5.4" ""; do
    timeout -k 10 150 python3 scripts/alloc_probe.py --config $c $h --tag "$c $h" 2>>$O/alloc.err | grep '^{' >> $O/alloc.jsonl || { tail -20 $O/alloc.err; exit 1; }
    python3 -c "import json; d=[json.loads(l) for l in open('$O/alloc.jsonl')][-1]; print(d['tag'], d['kernel_ms'])"
  done
done
