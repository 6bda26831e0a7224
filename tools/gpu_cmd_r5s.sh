set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_r5s.log 2>&1 || { tail -60 gpurun_out/tests_r5s.log; exit 1; }
tail -3 gpurun_out/tests_r5s.log
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r5s.json 2> gpurun_out/bench_r5s.err || { tail -30 gpurun_out/bench_r5s.err; exit 1; }
tail -c 1500 gpurun_out/bench_r5s.json
bash tools/prof.sh kernel > gpurun_out/prof_kernel.log 2>&1 || { tail -20 gpurun_out/prof_kernel.log; exit 1; }
echo PROF_OK
timeout -k 10 400 python tools/host_latency.py --chunks 1,4 > gpurun_out/host_latency_final.txt 2>&1 || { tail -20 gpurun_out/host_latency_final.txt; exit 1; }
grep chunks gpurun_out/host_latency_final.txt
