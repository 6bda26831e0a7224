#!/bin/bash
# A/B of library builds on the sort-heavy legs: configs[3] (2^24-point MSM), the prover commit
# (n = 2^20, one bucket set), the 2^20 MSM and configs[4] (BN254 n = 2^22).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  KZGMI_LIB="$lib" timeout -k 10 400 python bench.py --no-cpu --steps 40 --warmup 8 --repeats 1 --msm-steps 16 --cfg4-msms 6 --commit-steps 24 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 > gpurun_out/abs.json 2> gpurun_out/abs.err || { tail -5 gpurun_out/abs.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abs.json').read().strip().splitlines()[-1]);s=d['secondary'];c=s['cfg4_msm_2e24'];print('$lib', 'batch', round(d['value'],1), 'msm', round(s['msm_pts_per_s']/1e6,1), 'cfg4 ms', round(c['ms_per_msm'],2), 'cfg4 sort', round(c['phase_ms_single_msm']['sort'],2), 'commit/s', round(s['prover_commit']['commits_per_s'],1))"
  KZGMI_LIB="$lib" timeout -k 10 300 python bench.py --curve bn254 --n 4194304 --no-cpu --steps 40 --warmup 8 --repeats 1 --msm-steps 0 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 --cfg4-msms 0 > gpurun_out/absb.json 2> gpurun_out/absb.err || { tail -5 gpurun_out/absb.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/absb.json').read().strip().splitlines()[-1]);s=d['secondary'];print('$lib', 'bn254', round(d['value'],2), 'sort', round(s['phase_ms_single_batch']['sort'],2))"
done
