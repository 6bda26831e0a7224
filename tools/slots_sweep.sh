#!/bin/bash
# Pipeline-depth sweep: batch-verifies/s vs slots and HW queues (single GPU and sharded).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {  # name, env, args
  env $2 timeout -k 10 200 python bench.py --no-cpu --steps 24 --warmup 8 --msm-steps 0 $3 > gpurun_out/sw_$1.json 2>gpurun_out/sw_$1.err || { tail -5 gpurun_out/sw_$1.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sw_$1.json').read().strip().splitlines()[-1]);print('$1', round(d['value'],2), {k:round(v,1) for k,v in d['secondary']['phase_ms_avg_in_timed_region'].items()})"
}
run default "X=1" ""
run sh_default "X=1" "--sharded"
run sh_s12 "X=1" "--sharded --slots 12"
run sh_s6 "X=1" "--sharded --slots 6"
