#!/bin/bash
# Round 6 (o): the default bench command under rocprofv3 kernel-trace stats on the libraries
# rebuilt with DPP combining off (the GPU suite and smoke ran in the call before, same tree;
# the traffic records came from scripts/gpu_r06b.sh with TAG=r06o).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06o}
mkdir -p $O
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys_bench.log timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
  -d $O/kt_bench -o kt -- python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
grep '^{"metric"' $O/bench.json | cut -c1-300
