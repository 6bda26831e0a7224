#!/bin/bash
# Inversion A/B (libkzgmi_base = bit-serial EEA for MSM results + x^(p-2) in the pairing;
# libkzgmi = word-level binary GCD for both): batch phases at n = 256 / 2^20, MSM latency.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = new ]; then unset KZGMI_LIB; else export KZGMI_LIB=$PWD/kzg-batch-verification-scheme_amd/kzgmi/libkzgmi_$v.so; fi
  for n in 256 1048576; do
    timeout -k 10 200 python tools/phase_timing.py --n $n --reps 6 | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);p=d['phases'];print('v=$v', 'n=$n', 'ok', d['ok'], 'sum %.3f' % sum(p.values()), {k: round(v,3) for k,v in p.items()})" || exit 1
  done
  for n in 256 131072 1048576; do
    timeout -k 10 200 python tools/msm_latency.py --n $n | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print('v=$v', 'msm n=$n', 'median_ms %.3f' % d['median_ms'])" || exit 1
  done
done
