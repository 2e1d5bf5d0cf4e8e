#!/bin/bash
# Round 6 (b): PMC traffic records for every bench config on the round-6 libraries (the public
# header's corrected signature doc re-keyed every library, so the round-5 records no longer match
# the build keys the line reports): per config the bench line under kernel-trace stats, then
# FETCH_SIZE and WRITE_SIZE in separate passes (scripts/profile.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
GTMI_NO_COMPILE=1 TAG=${TAG:-r06b} CONFIGS="${CONFIGS:-hdiff lap5 tridiag hdiff_f32 copy vadv hdiff_blocks staged}" \
  bash scripts/profile.sh > gpurun_out/profile_${TAG:-r06b}.log 2>&1 || { tail -30 gpurun_out/profile_${TAG:-r06b}.log; exit 1; }
grep -E '^\{"metric"' gpurun_out/profile_${TAG:-r06b}.log | cut -c1-200
