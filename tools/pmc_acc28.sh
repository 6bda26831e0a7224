#!/bin/bash
# SQ counters: radix-2^28 vs 32-bit accumulation kernel (BLS12-381, one n = 2^20 batch).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc28"
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex 'k_accumulate' --output-format csv -d "$OUT/a$i" -o run -- python3 "$R/tools/phase_timing.py" --reps 1 > "$OUT/a$i.log" 2>&1 || { tail -20 "$OUT/a$i.log"; exit 1; }
done
