#!/bin/bash
# Round 6 (j): differential fuzz with every program built under the two-row tile geometry
# (tile_rows=2, 128x8 threads; the tile programs take it, the others ignore it), at the default
# level counts and at 120 levels (blocked tile levels).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export FUZZ_OPTS='{"tile_rows": 2, "tile_bx": 128, "tile_by": 8}'
TAG=r06j FUZZ_NK=0 bash scripts/gpu_r06g.sh && TAG=r06j FUZZ_NK=120 bash scripts/gpu_r06g.sh
