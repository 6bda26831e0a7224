#!/bin/bash
# A/B of library builds on configs[4] (BN254, n = 2^22 on one GPU): pipelined batch-verifies/s.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  KZGMI_LIB="$lib" timeout -k 10 300 python bench.py --curve bn254 --n 4194304 --no-cpu --steps 40 --warmup 8 --msm-steps 0 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 --cfg4-msms 0 > gpurun_out/abbn.json 2> gpurun_out/abbn.err || { tail -5 gpurun_out/abbn.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abbn.json').read().strip().splitlines()[-1]);print('$lib', 'bn254 pipelined', round(d['value'],2), 'reduce', round(d['secondary']['phase_ms_single_batch']['reduce'],3))"
done
