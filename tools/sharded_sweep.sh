#!/bin/bash
# Sharded (world-1 RCCL) pipeline: batch and MSM rates vs slots in flight (+ 2 combine lanes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for s in ${SLOTS:-6 8 10}; do
  timeout -k 10 240 python bench.py --sharded --no-cpu --steps 120 --warmup 12 --msm-steps 48 --slots $s --cfg4-msms 0 --repeats 1 \
    --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 \
    > gpurun_out/sw_$s.json 2> gpurun_out/sw_$s.err || { tail -20 gpurun_out/sw_$s.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sw_$s.json').read().strip().splitlines()[-1]);print('slots $s', round(d['value'],2), 'msm', round(d['secondary']['msm_pts_per_s']/1e6,1), 'glv', round(d['secondary']['msm_trusted_g1_glv']['pts_per_s']/1e6,1))"
done
