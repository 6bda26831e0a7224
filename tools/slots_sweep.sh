#!/bin/bash
# Pipeline-depth sweep: batch-verifies/s for each "slots hw_queues" pair in $CFGS (default:
# the shipped 16 x 24 and its neighbours), $PASSES passes, $STEPS timed steps, headline leg
# only.  SHARDED=1 runs the multi-GPU pipeline at world 1 instead (8 slots + 2 combine lanes).
# (Replaces the round-1/2 variants slots_sweep2-4.sh: same runs, parameterised.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for pass in $(seq 1 ${PASSES:-2}); do
  for cfg in ${CFGS:-"12:24 16:24 20:24 16:16"}; do
    s=${cfg%%:*}; q=${cfg##*:}
    KZGMI_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu --steps ${STEPS:-200} --warmup 24 --slots $s \
      ${SHARDED:+--sharded} --msm-steps 0 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 \
      --cfg4-msms 0 > gpurun_out/sw.json 2> gpurun_out/sw.err || { tail -5 gpurun_out/sw.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/sw.json').read().strip().splitlines()[-1]);print('pass $pass slots $s queues $q', round(d['value'],2))"
  done
done
