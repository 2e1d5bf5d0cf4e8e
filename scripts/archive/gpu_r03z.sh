#!/bin/bash
# Column kernels: register band (kreg) interleaved in one process on shared buffers, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03z
for c in tridiag vadv tridiag vadv; do
  echo "== $c" | tee -a gpurun_out/r03z/kreg.log
  timeout -k 10 300 python3 scripts/sweep.py --config $c --variants "kreg=0;kreg=16;kreg=32;kreg=48" --rounds 5 2>> gpurun_out/r03z/err.log | tee -a gpurun_out/r03z/kreg.log || exit 1
done
