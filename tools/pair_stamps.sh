#!/bin/bash
# Pairing interpreter phase stamps (KZ_PROBE_STAMPS builds given as arguments), one single batch each.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in "$@"; do
  echo "== $lib"
  timeout -k 10 200 python tools/phase_timing.py --lib kzg-batch-verification-scheme_amd/kzgmi/$lib --reps 1 > gpurun_out/stamps.log 2>&1 || { tail -5 gpurun_out/stamps.log; exit 1; }
  grep -a "PAIRSTAMP" gpurun_out/stamps.log | tail -8
done
