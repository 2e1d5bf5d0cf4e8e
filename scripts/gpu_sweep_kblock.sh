#!/bin/bash
# column kernels: blocked K loads (kblock) vs one level at a time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
CONFIGS=copy VH="pointwise_plane=0;pointwise_plane=0,kblock=4;pointwise_plane=0,kblock=8;jmirror=1" bash scripts/gpu_sweep_plane.sh &&
CONFIGS="tridiag vadv" VH="kblock=0;kblock=2;kblock=4;kblock=8" bash scripts/gpu_sweep_plane.sh
