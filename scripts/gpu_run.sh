#!/bin/bash
# One GPU call: parity tests + smoke, rocprof profile of every bench config (TAG), then the
# column-sweep lab (LAB=1). Every GPU step has its own time limit; the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  bash scripts/gpu_tests.sh || exit $?
fi
if [ -n "${PYTEST_ONLY:-}" ]; then
  timeout -k 10 600 python -u -m pytest $PYTEST_ONLY -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_only.log 2>&1 || { tail -40 gpurun_out/pytest_only.log; exit 1; }
  tail -3 gpurun_out/pytest_only.log
fi
if [ -n "${CONFIGS:-}" ]; then
  CONFIGS="$CONFIGS" TAG=${TAG:-r02a} timeout -k 10 900 bash scripts/profile.sh > gpurun_out/profile.log 2>&1 \
    || { tail -30 gpurun_out/profile.log; exit 1; }
  echo "profile done"
  tail -3 gpurun_out/profile.log
fi
if [ "${LAB:-0}" = 1 ]; then
  timeout -k 10 300 ./scripts/lab/tridiag_lab ${LAB_REPS:-20} > gpurun_out/lab.log 2>&1 || { cat gpurun_out/lab.log; exit 1; }
  cat gpurun_out/lab.log
fi
if [ "${HALO:-0}" = 1 ]; then
  # per-rank cost of the J-strip exchange machinery: the rank is its own periodic neighbour
  # through RCCL; bench lines with and without the halo path, then a kernel trace of the halo run
  export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
  for m in halo unpack_main halo unpack_main; do
    GTMI_HALO_BANDS=$m timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm 2>> gpurun_out/halo.err | tee -a gpurun_out/halo.log || exit 1
  done
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm --no-overlap 2>> gpurun_out/halo.err | tee -a gpurun_out/halo.log || exit 1
  timeout -k 10 300 python3 bench.py --no-extra --no-cpu-baseline --steps 50 --halo-selfcomm --decomp 2d 2>> gpurun_out/halo.err | tee -a gpurun_out/halo.log || exit 1
  for m in halo unpack_main; do
    GTMI_HALO_BANDS=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/halo_kt_$m -o kt -- python3 bench.py --no-extra --no-cpu-baseline --steps 20 --halo-selfcomm > gpurun_out/halo_kt_$m.log 2>&1 || exit 1
  done
  unset RANK LOCAL_RANK WORLD_SIZE MASTER_ADDR MASTER_PORT
fi
if [ "${ROCTX:-0}" = 1 ]; then
  # ROCTX ranges of the stencil libraries (gtmi:<stencil>) and the halo copies, next to the kernels
  timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/roctx -o rt -- python3 bench.py --steps 3 --warmup 1 --no-extra --no-cpu-baseline > gpurun_out/roctx.log 2>&1 || { tail -20 gpurun_out/roctx.log; exit 1; }
  find gpurun_out/roctx -name "*marker*"
fi
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  cat gpurun_out/bench.json
fi
