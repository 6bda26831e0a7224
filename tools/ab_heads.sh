#!/bin/bash
# Regression A/B of library builds of earlier heads against the in-tree one (arms alternated):
# pipelined 2^20 batch rate over 200 steps (median of repeats) and the single-batch phases.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=$PWD/kzg-batch-verification-scheme_amd/kzgmi
MIN="--no-cpu --msm-steps 0 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 --cfg4-msms 0"
for a in "$@"; do
  if [ "$a" = head ]; then unset KZGMI_LIB; else export KZGMI_LIB=$P/libkzgmi_$a.so; fi
  timeout -k 10 300 python bench.py $MIN --steps 200 --warmup 24 --repeats 4 > gpurun_out/abh.json 2> gpurun_out/abh.err || { tail -5 gpurun_out/abh.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abh.json').read().strip().splitlines()[-1]);s=d['secondary'];print('$a', 'value %.1f' % d['value'], 'median %.1f' % s['repeats_median_batch_verifies_per_s'], 'single %.2f ms' % s['single_batch_latency_ms'], {k: round(v, 3) for k, v in s['phase_ms_single_batch'].items()})" || exit 1
done
