#!/bin/bash
# Instruction-cache pressure of k_accumulate (single batches, tools/phase_timing.py): one pass,
# SQ/SQC counters only.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_icache
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
LIB=${1:-}; [ -n "$LIB" ] && [ "${LIB#/}" = "$LIB" ] && LIB=$R/$LIB
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU --kernel-include-regex 'k_accumulate' --output-format csv -d $OUT/ic -o ic -- python3 $R/tools/phase_timing.py --reps 2 ${LIB:+--lib $LIB} > $OUT/ic.log 2>&1 || { tail -20 $OUT/ic.log; exit 1; }
find $OUT -name '*counter_collection*'
