#!/bin/bash
# Round 5: is the column kernels' issue stall an instruction-fetch stall? (vadv's kernel is 103 KB
# of code, tridiag's 46 KB, hdiff's 7 KB.) Instruction-cache and fetch counters per config, and
# for tridiag/vadv with a different register band (code size follows the band).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r05r}
CONFIGS="vadv tridiag hdiff" PASSES="E F" TAG=$T bash scripts/pmc_waits.sh || exit 1
CONFIGS="tridiag" PASSES="E F" TAG=$T VARIANT=kreg64 BENCH_OPTS="--opt kreg=64" bash scripts/pmc_waits.sh || exit 1
CONFIGS="vadv" PASSES="E F" TAG=$T VARIANT=kreg48 BENCH_OPTS="--opt kreg=48" bash scripts/pmc_waits.sh || exit 1
