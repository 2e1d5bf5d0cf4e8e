#!/bin/bash
# Round 5: price the column kernels' memory streams with zero-record descriptors (kbuf_null:
# same instruction stream, chosen fields without memory traffic), and list the gfx950 counters.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05d}
mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters_list.txt 2>&1 || echo "rocprofv3 -L rc=$?"
timeout -k 10 300 python3 scripts/sweep.py --config vadv --rounds 7 --variants \
  "kbuf=1;kbuf=1,kbuf_null=*;kbuf=1,kbuf_null=ccol:dcol;kbuf=1,kbuf_null=u_pos;kbuf=1,kbuf_null=wcon;kbuf=1,kbuf_null=utens_stage" \
  > $O/sweep_vadv_null.log 2>&1 || { tail -20 $O/sweep_vadv_null.log; exit 1; }
grep -v Warn $O/sweep_vadv_null.log
timeout -k 10 300 python3 scripts/sweep.py --config tridiag --rounds 7 --variants \
  "kbuf=1;kbuf=1,kbuf_null=*;kbuf=1,kbuf_null=sup:rhs;kbuf=1,kbuf_null=inf:diag" \
  > $O/sweep_tridiag_null.log 2>&1 || { tail -20 $O/sweep_tridiag_null.log; exit 1; }
grep -v Warn $O/sweep_tridiag_null.log
