#!/bin/bash
# configs[1] MSM rate vs the number of timed pipelined MSMs (the drain of the in-flight MSMs is
# inside the timed region): bash tools/msm_steps_check.sh 24 96 24 96
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in "$@"; do
  timeout -k 10 200 python bench.py --no-cpu --steps 40 --warmup 8 --repeats 1 --msm-steps $m --trusted-steps 0 \
    --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/m.json 2> gpurun_out/m.err || { tail -5 gpurun_out/m.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/m.json').read().strip().splitlines()[-1]);print(sys.argv[1], 'msm M pts/s', round(d['secondary']['msm_pts_per_s']/1e6,1))" $m
done
