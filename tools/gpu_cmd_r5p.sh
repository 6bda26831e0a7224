set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python tools/host_latency.py > gpurun_out/host_latency.txt 2>&1 || { tail -20 gpurun_out/host_latency.txt; exit 1; }
cat gpurun_out/host_latency.txt
