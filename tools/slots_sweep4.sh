#!/bin/bash
# Single-GPU pipeline depth with the radix-29 accumulation: slots x HW queues, 200 timed steps, two passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for pass in 1 2; do
  for cfg in "12 24" "16 24" "20 24" "20 32"; do
    set -- $cfg
    KZGMI_HW_QUEUES=$2 timeout -k 10 200 python bench.py --no-cpu --steps 200 --warmup 24 --slots $1 --msm-steps 0 --compressed-steps 0 \
      --fs-steps 0 --trusted-steps 0 --commit-steps 0 > gpurun_out/s4.json 2> gpurun_out/s4.err || { tail -5 gpurun_out/s4.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/s4.json').read().strip().splitlines()[-1]);print('pass $pass slots $1 queues $2', round(d['value'],2))"
  done
done
