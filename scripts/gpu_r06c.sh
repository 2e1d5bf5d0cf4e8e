#!/bin/bash
# Round 6 (c): the GPU suite, the C5 tile's fma rendering A/B, and: does
# gating the interior on the pack let RCCL's kernel run beside it? The J-strip halo path on one GPU, the rank its own periodic neighbour through RCCL:
#   1. the GPU suite incl. the gated halo variants (bit-exact vs the C oracle),
#   2. alternating-process A/B of the per-step exchange overhead (scripts/halo_ab.sh),
#   3. a kernel trace of one gated run (where RCCL's kernel lands relative to the interior).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06c}
mkdir -p $O
# the whole GPU suite on prebuilt libraries (the gated halo variants and the exact-product fma
# rendering, which re-keyed the f32 cast-tree libraries, among them), then smoke
GTMI_NO_COMPILE=1 GTMI_CACHE_LOG=$PWD/$O/build_keys.log bash scripts/gpu_tests.sh || exit $?
cp gpurun_out/pytest_gpu.log gpurun_out/smoke.log $O/
# C5 tile: the fma rendering against the separate multiply, interleaved on shared buffers
GTMI_NO_COMPILE=1 timeout -k 10 300 python scripts/sweep.py --config hdiff_f32 --variants "exact_fma=1;exact_fma=0" \
  --rounds 4 > $O/sweep_f32_fma.log 2>&1 || { tail -20 $O/sweep_f32_fma.log; exit 1; }
grep '^{' $O/sweep_f32_fma.log
rm -f gpurun_out/halo_ab.log
GTMI_NO_COMPILE=1 ROUNDS=${ROUNDS:-3} VARIANTS="1d:GTMI_HALO_GATE=0 1d:GTMI_HALO_GATE=1 1d:GTMI_HALO_GATE=1,GTMI_HALO_BANDS=halo" \
  bash scripts/halo_ab.sh || { tail -20 gpurun_out/halo_ab.err; exit 1; }
cp gpurun_out/halo_ab.log $O/halo_ab.log
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541
for v in 0 1; do
  GTMI_NO_COMPILE=1 GTMI_HALO_GATE=$v GTMI_HALO_BANDS=$([ $v = 1 ] && echo halo || echo unpack_main) timeout -k 10 300 \
    rocprofv3 --kernel-trace --output-format csv -d $O/kt_gate$v -o kt -- python3 bench.py --no-extra --no-cpu-baseline \
    --steps 10 --warmup 2 --sustain 0 --placement-candidates 0 --halo-selfcomm > $O/kt_gate$v.log 2>&1 || { tail -20 $O/kt_gate$v.log; exit 1; }
done
echo done
