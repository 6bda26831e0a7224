#!/bin/bash
# Single-GPU pipeline depth beyond 14 slots: slots x HW queues (KZGMI_HW_QUEUES), 200 timed steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "14 16" "16 16" "16 24" "20 24" "24 32" "16 32"; do
  set -- $cfg
  KZGMI_HW_QUEUES=$2 timeout -k 10 200 python bench.py --no-cpu --steps 200 --warmup 24 --slots $1 --msm-steps 0 --compressed-steps 0 \
    --fs-steps 0 --trusted-steps 0 --commit-steps 0 > gpurun_out/sq.json 2> gpurun_out/sq.err || { tail -5 gpurun_out/sq.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sq.json').read().strip().splitlines()[-1]);print('slots $1 queues $2', round(d['value'],2))"
done
