#!/bin/bash
# Single-GPU pipeline depth after the latency-tail work: batch-verifies/s vs slots (16 HW queues),
# two passes each, 200 timed steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for pass in 1 2; do
  for s in ${SLOTS:-6 8 10 12 14}; do
    timeout -k 10 200 python bench.py --no-cpu --steps 200 --warmup 24 --slots $s --msm-steps 0 --compressed-steps 0 \
      --fs-steps 0 --trusted-steps 0 --commit-steps 0 > gpurun_out/ss_$s.json 2> gpurun_out/ss_$s.err || { tail -5 gpurun_out/ss_$s.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ss_$s.json').read().strip().splitlines()[-1]);print('pass $pass slots $s', round(d['value'],2))"
  done
done
