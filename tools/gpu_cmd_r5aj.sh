set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_r5aj.log 2>&1 || { tail -60 gpurun_out/tests_r5aj.log; exit 1; }
tail -2 gpurun_out/tests_r5aj.log
grep -n "accumulation_order" gpurun_out/tests_r5aj.log || true
