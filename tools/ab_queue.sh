#!/bin/bash
# Accumulation work queue A/B (KZGMI_ACC_QUEUE = chunks per capped accumulation thread; 0 = the
# static one-round grid; base = the library before the queue): GPU tests on the new default, then
# the pipelined rate at 200 steps and at the driver's 20-step form (median of repeats), the
# single-batch latency, and BN254 2^22, alternating arms A/B/A.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=$PWD/kzg-batch-verification-scheme_amd/kzgmi
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
MIN="--no-cpu --msm-steps 0 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 --cfg4-msms 0"
arm() {  # label
  case "$1" in
    base) export KZGMI_LIB=$P/libkzgmi_base.so; unset KZGMI_ACC_QUEUE ;;
    q*) unset KZGMI_LIB; export KZGMI_ACC_QUEUE=${1#q} ;;
  esac
}
for a in base q0 q2 q4 q4 q2 q0 base; do
  arm $a
  for form in "200 24 4" "20 5 9"; do
    set -- $form
    timeout -k 10 300 python bench.py $MIN --steps $1 --warmup $2 --repeats $3 > gpurun_out/abq.json 2> gpurun_out/abq.err || { tail -5 gpurun_out/abq.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abq.json').read().strip().splitlines()[-1]);s=d['secondary'];print('$a', 'steps=$1', 'value %.1f' % d['value'], 'median %.1f' % s['repeats_median_batch_verifies_per_s'], 'single %.2f ms' % s['single_batch_latency_ms'], 'acc %.3f ms' % s['phase_ms_single_batch']['accumulate'])" || exit 1
  done
done
for a in base q2 q4 q2 base; do
  arm $a
  timeout -k 10 300 python bench.py $MIN --curve bn254 --n 4194304 --steps 40 --warmup 8 --repeats 3 > gpurun_out/abq.json 2> gpurun_out/abq.err || { tail -5 gpurun_out/abq.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abq.json').read().strip().splitlines()[-1]);s=d['secondary'];print('$a', 'bn254 2^22', 'value %.1f' % d['value'], 'median %.1f' % s['repeats_median_batch_verifies_per_s'], 'single %.2f ms' % s['single_batch_latency_ms'])" || exit 1
done
