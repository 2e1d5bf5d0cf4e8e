V="jmirror=0;jmirror=1;jmirror=1,jchunk=8;jmirror=1,jchunk=32;jmirror=0,jchunk=32;jmirror=1,jchunk=32,prefetch=6"
mkdir -p gpurun_out
timeout -k 10 300 python scripts/sweep.py --config hdiff --rounds 7 --variants "$V" > gpurun_out/sweep_hdiff.log 2>&1 &&
timeout -k 10 300 python scripts/sweep.py --config hdiff_f32 --rounds 7 --variants "$V" > gpurun_out/sweep_hdiff_f32.log 2>&1 &&
timeout -k 10 300 python scripts/sweep.py --config lap5 --rounds 7 --variants "$V" > gpurun_out/sweep_lap5.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
echo "rc=$?"; tail -3 gpurun_out/pytest_gpu.log
