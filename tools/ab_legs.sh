#!/bin/bash
# A/B of the secondary bench legs (configs[3] 2^24 MSM, compressed + subgroup batches) across
# library builds: bench.py with the main pipelined leg cut to a few steps.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  KZGMI_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu --steps 8 --warmup 4 --msm-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 ${LEG_ARGS:-} > gpurun_out/legs.json 2> gpurun_out/legs.err || { tail -5 gpurun_out/legs.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/legs.json').read().strip().splitlines()[-1]); s=d['secondary']
c=s.get('cfg4_msm_2e24') or {}; z=s.get('compressed_subgroup') or {}
print('$lib', 'cfg4_ms', c.get('ms_per_msm'), 'compressed/s', z.get('batch_verifies_per_s'), 'conv', (z.get('phase_ms_single_batch') or {}).get('convert'))"
done
