set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_r5q_host.log 2>&1 || { tail -60 gpurun_out/tests_r5q_host.log; exit 1; }
tail -3 gpurun_out/tests_r5q_host.log
timeout -k 10 400 python tools/host_latency.py --chunks 1,2,3,4,6,8 > gpurun_out/host_latency.txt 2>&1 || { tail -20 gpurun_out/host_latency.txt; exit 1; }
grep chunks gpurun_out/host_latency.txt
