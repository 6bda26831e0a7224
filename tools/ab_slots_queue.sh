#!/bin/bash
# Pipeline depth with the work-queue accumulation: --slots x KZGMI_HW_QUEUES arms alternated,
# pipelined 2^20 batch rate over 200 steps (median of repeats) and the driver's 20-step form.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
MIN="--no-cpu --msm-steps 0 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 --cfg4-msms 0"
for a in "16 24" "12 24" "20 24" "24 32" "16 32" "16 32" "24 32" "20 24" "12 24" "16 24"; do
  set -- $a
  for form in "200 24 4" "20 5 7"; do
    set -- $a $form
    KZGMI_HW_QUEUES=$2 timeout -k 10 300 python bench.py $MIN --slots $1 --steps $3 --warmup $4 --repeats $5 > gpurun_out/abs.json 2> gpurun_out/abs.err || { tail -5 gpurun_out/abs.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abs.json').read().strip().splitlines()[-1]);s=d['secondary'];print('slots=$1 queues=$2 steps=$3', 'value %.1f' % d['value'], 'median %.1f' % s['repeats_median_batch_verifies_per_s'])" || exit 1
  done
done
