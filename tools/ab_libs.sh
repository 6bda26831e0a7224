#!/bin/bash
# A/B: single-batch phases and pipelined throughput for alternative library builds.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  timeout -k 10 200 python tools/phase_timing.py --lib "$lib" | cut -c1-400 || exit 1
  KZGMI_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu --steps 200 --warmup 24 --msm-steps 0 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 --cfg4-msms 0 > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail -5 gpurun_out/ab.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print('$lib', 'pipelined', round(d['value'],2))"
done
