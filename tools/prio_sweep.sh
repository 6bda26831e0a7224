#!/bin/bash
# Tail-kernel wave priority (s_setprio) x pipeline depth: batch-verifies/s, 200 timed steps.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
L=kzg-batch-verification-scheme_amd/kzgmi
for cfg in "libkzgmi_noprio 12 16" "libkzgmi 12 16" "libkzgmi_noprio 16 24" "libkzgmi 16 24" "libkzgmi_noprio 24 32" "libkzgmi 24 32" "libkzgmi 8 16"; do
  set -- $cfg
  KZGMI_LIB=$L/$1.so KZGMI_HW_QUEUES=$3 timeout -k 10 200 python bench.py --no-cpu --steps 200 --warmup 24 --slots $2 --msm-steps 0 \
    --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 > gpurun_out/pq.json 2> gpurun_out/pq.err || { tail -5 gpurun_out/pq.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/pq.json').read().strip().splitlines()[-1]);print('$1 slots $2 queues $3', round(d['value'],2), {k: round(v,1) for k,v in d['secondary']['phase_ms_avg_in_timed_region'].items()})"
done
