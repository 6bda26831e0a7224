#!/bin/bash
# SQ counters for the accumulation kernel (one single batch via tools/phase_timing.py) and
# the Fp-multiply probe: instruction mix and where wave cycles go.  One --pmc pass per
# counter group (no trace domains combined with --pmc).
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/pmc_acc"
mkdir -p "$OUT"
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex 'k_accumulate|k_chain' --output-format csv -d "$OUT/p$i" -o run -- python3 "$R/tools/phase_timing.py" --reps 1 > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex 'k_chain' --output-format csv -d "$OUT/q$i" -o run -- "$R/tools/probes/fpmul_chain" > "$OUT/q$i.log" 2>&1 || { tail -20 "$OUT/q$i.log"; exit 1; }
done
find "$OUT" -name '*counter_collection*'
