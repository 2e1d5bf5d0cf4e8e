set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_tile.py tests/test_gpu_parity.py -k "tile or staged" -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_tile.log 2>&1 || { tail -30 gpurun_out/pt_tile.log; exit 1; }
tail -2 gpurun_out/pt_tile.log
timeout -k 10 200 python3 bench.py --config staged --no-cpu-baseline --no-extra --sustain 0 --placement-candidates 0 > gpurun_out/bench_staged.json 2> gpurun_out/bench_staged.err || exit 1
head -c 900 gpurun_out/bench_staged.json; echo
rm -f gpurun_out/alloc_probe.jsonl
for a in "--tag d1" "--pre-gb 16 --tag p16" "--pre-gb 48 --tag p48" "--tag d2" "--pre-gb 16 --post-free --tag p16f" "--pre-gb 100 --tag p100" "--tag d3"; do timeout -k 10 120 python3 -u scripts/alloc_probe.py $a >> gpurun_out/alloc_probe.jsonl 2>> gpurun_out/alloc_probe.err || exit 1; done
cat gpurun_out/alloc_probe.jsonl
timeout -k 10 300 ./scripts/lab/tridiag_lab 10 2 > gpurun_out/lab_live.log 2>&1 || { cat gpurun_out/lab_live.log; exit 1; }
cat gpurun_out/lab_live.log
