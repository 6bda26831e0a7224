set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k boundaries > gpurun_out/tests_r5aq.log 2>&1 || { tail -40 gpurun_out/tests_r5aq.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/tests_r5aq.log | tail -12
