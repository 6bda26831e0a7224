#!/bin/bash
# Two-level bucket-piece join + balanced accumulation grid A/B (libkzgmi_base = neither,
# libkzgmi_fg = two-level join only, libkzgmi = both): single-batch phases at 2^16 / 2^17,
# pipelined rates at 2^16 / 2^17 / 2^20.  bash tools/ab_fix.sh base fg new base new
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = new ]; then unset KZGMI_LIB; else export KZGMI_LIB=$PWD/kzg-batch-verification-scheme_amd/kzgmi/libkzgmi_$v.so; fi
  for n in 65536 131072; do
    timeout -k 10 200 python tools/phase_timing.py --n $n --reps 6 | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);p=d['phases'];print('v=$v', 'n=$n', 'ok', d['ok'], 'sum %.3f' % sum(p.values()), {k: round(v,3) for k,v in p.items()})" || exit 1
  done
  for n in 65536 131072 1048576; do
    st=300; [ $n = 1048576 ] && st=120
    timeout -k 10 300 python bench.py --no-cpu --n $n --steps $st --warmup 20 --repeats 1 --msm-steps 48 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/af.json 2> gpurun_out/af.err || { tail -5 gpurun_out/af.err; exit 1; }
    python -c "import json;a=json.loads(open('gpurun_out/af.json').read().strip().splitlines()[-1]);print('v=$v', 'n=$n', 'batch/s', round(a['value'],1), 'msm M pts/s', round(a['secondary']['msm_pts_per_s']/1e6,1))"
  done
done
