#!/bin/bash
# A/B of library builds on small and mid batch sizes: single-batch phases at n = 256 and 2^17,
# pipelined rates at 2^17 and 2^20.  bash tools/ab_chunk.sh libA libB ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  for n in 256 131072; do
    timeout -k 10 200 python tools/phase_timing.py --lib "$lib" --n $n --reps 6 | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);p=d['phases'];print('$lib', 'n=$n', 'sum %.3f' % sum(p.values()), {k: round(v,3) for k,v in p.items()})" || exit 1
  done
  KZGMI_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu --n 131072 --steps 400 --warmup 40 --repeats 1 --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/ac.json 2> gpurun_out/ac.err || { tail -5 gpurun_out/ac.err; exit 1; }
  KZGMI_LIB="$lib" timeout -k 10 300 python bench.py --no-cpu --steps 100 --warmup 16 --repeats 1 --msm-steps 48 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/ad.json 2> gpurun_out/ad.err || { tail -5 gpurun_out/ad.err; exit 1; }
  python -c "import json;a=json.loads(open('gpurun_out/ac.json').read().strip().splitlines()[-1]);b=json.loads(open('gpurun_out/ad.json').read().strip().splitlines()[-1]);print('$lib', '2^17', round(a['value'],1), '2^20', round(b['value'],1), 'msm', round(b['secondary']['msm_pts_per_s']/1e6,1))"
done
