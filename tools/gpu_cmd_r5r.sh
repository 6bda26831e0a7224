set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_r5r.log 2>&1 || { tail -60 gpurun_out/tests_r5r.log; exit 1; }
tail -3 gpurun_out/tests_r5r.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r5r.json 2> gpurun_out/bench_r5r.err || { tail -30 gpurun_out/bench_r5r.err; exit 1; }
tail -c 1800 gpurun_out/bench_r5r.json
