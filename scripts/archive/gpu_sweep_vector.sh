set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --config hdiff_f32 --rounds 7 --variants "jchunk=0;vector=8;vector=8,prefetch=1;vector=2;vector=8,jchunk=16" > gpurun_out/sweep_f32.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_f32.log
timeout -k 10 300 python scripts/sweep.py --config hdiff --rounds 7 --variants "jchunk=0;vector=4;vector=4,prefetch=2" > gpurun_out/sweep_hdiff.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_hdiff.log
timeout -k 10 300 python scripts/sweep.py --config lap5 --rounds 7 --variants "jchunk=0;order=5;vector=4;vector=4,order=5" > gpurun_out/sweep_lap5.log 2>&1 || exit $?
grep '^{' gpurun_out/sweep_lap5.log
