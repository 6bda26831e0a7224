set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > gpurun_out/gpu1.log 2>&1
rc=$?
tail -30 gpurun_out/gpu1.log
exit $rc
