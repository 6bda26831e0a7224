set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python bench.py --curve bn254 --n 4194304 --steps 40 --warmup 5 --no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/bench_bn254.json 2> gpurun_out/bench_bn254.err || { tail -30 gpurun_out/bench_bn254.err; exit 1; }
cat gpurun_out/bench_bn254.json
