#!/bin/bash
# Window width A/B (KZGMI_WBITS=16 forces c = 16; unset = the library's choice): single-batch
# phases at n = 256 / 2^17 / 2^18, pipelined rates at 2^17 / 2^18, MSM 2^18.  bash tools/ab_wbits.sh 16 auto 16 auto
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for w in "$@"; do
  if [ "$w" = auto ]; then unset KZGMI_WBITS; else export KZGMI_WBITS=$w; fi
  for n in 256 65536 131072; do
    timeout -k 10 200 python tools/phase_timing.py --n $n --reps 6 | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);p=d['phases'];print('w=$w', 'n=$n', 'ok', d['ok'], 'sum %.3f' % sum(p.values()), {k: round(v,3) for k,v in p.items()})" || exit 1
  done
  for n in 65536 131072 262144; do
    timeout -k 10 300 python bench.py --no-cpu --n $n --steps 300 --warmup 30 --repeats 1 --msm-steps 96 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/aw.json 2> gpurun_out/aw.err || { tail -5 gpurun_out/aw.err; exit 1; }
    python -c "import json;a=json.loads(open('gpurun_out/aw.json').read().strip().splitlines()[-1]);print('w=$w', 'n=$n', 'batch/s', round(a['value'],1), 'msm M pts/s', round(a['secondary']['msm_pts_per_s']/1e6,1))"
  done
done
