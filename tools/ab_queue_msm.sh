#!/bin/bash
# Work-queue A/B for MSMs (KZGMI_ACC_QUEUE / KZGMI_ACC_QUEUE_MIN): 2^20 MSMs (64-entry chunks at the
# cap: the queue makes them 32) and configs[3]'s 2^24 MSM, plus the 2^20 batch rate, arms alternated.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ARGS="--no-cpu --steps 100 --warmup 16 --repeats 2 --msm-steps 96 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 --cfg4-msms 4"
for a in "0 32" "2 32" "2 64" "2 64" "2 32" "0 32"; do
  set -- $a
  KZGMI_ACC_QUEUE=$1 KZGMI_ACC_QUEUE_MIN=$2 timeout -k 10 300 python bench.py $ARGS > gpurun_out/abm.json 2> gpurun_out/abm.err || { tail -5 gpurun_out/abm.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abm.json').read().strip().splitlines()[-1]);s=d['secondary'];print('q=$1 min=$2', 'batch %.1f' % s['repeats_median_batch_verifies_per_s'], 'msm %.1f M' % (s['msm_pts_per_s']/1e6), 'msm1 %.2f ms' % s['msm_single_latency_ms'], 'cfg4 %.1f ms' % s['cfg4_msm_2e24']['ms_per_msm'])" || exit 1
done
