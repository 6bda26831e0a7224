set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_r5y.json 2> gpurun_out/bench_r5y.err || { tail -30 gpurun_out/bench_r5y.err; exit 1; }
tail -c 2500 gpurun_out/bench_r5y.json
