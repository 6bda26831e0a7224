#!/bin/bash
# SQ_INSTS_VALU / SQ_INSTS_SALU / SQ_WAVES of every kernel of single, non-pipelined batches
# (tools/phase_timing.py): each kernel's share of the chip's VALU issue per batch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_valu_all
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d $OUT/v -o v -- python3 $R/tools/phase_timing.py --reps 2 "$@" > $OUT/v.log 2>&1 || { tail -20 $OUT/v.log; exit 1; }
find $OUT -name '*counter_collection*' | head
