#!/bin/bash
# A/B of library builds on the scalar-prep / transcript-heavy legs: BN254 2^22 (scalar prep of
# 4 M tuples per batch) and the Fiat-Shamir batch leg.  bash tools/ab_fs.sh libA libB ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  KZGMI_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu --steps 40 --warmup 8 --repeats 1 --msm-steps 0 --trusted-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 --fs-steps 96 > gpurun_out/af.json 2> gpurun_out/af.err || { tail -5 gpurun_out/af.err; exit 1; }
  KZGMI_LIB="$lib" timeout -k 10 300 python bench.py --curve bn254 --n 4194304 --no-cpu --steps 40 --warmup 8 --repeats 1 --msm-steps 0 --trusted-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 --fs-steps 0 > gpurun_out/afb.json 2> gpurun_out/afb.err || { tail -5 gpurun_out/afb.err; exit 1; }
  python -c "import json,sys;d=json.loads(open('gpurun_out/af.json').read().strip().splitlines()[-1]);b=json.loads(open('gpurun_out/afb.json').read().strip().splitlines()[-1]);print(sys.argv[1], 'batch', round(d['value'],1), 'fs', round(d['secondary']['fiat_shamir']['batch_verifies_per_s'],1), 'bn254', round(b['value'],2), 'scalars ms', round(b['secondary']['phase_ms_single_batch']['scalars'],3))" $lib
done
