#!/bin/bash
# SQ counters of the shipped k_accumulate (single, non-pipelined batches; tools/phase_timing.py)
# in one pass (8 SQ slots), plus a FETCH_SIZE/WRITE_SIZE calibration pass that also counts
# k_pts_to29 (known bytes per launch: reads and rewrites every point once).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_sq
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex 'k_accumulate' --output-format csv -d $OUT/sq -o sq -- python3 $R/tools/phase_timing.py --reps 2 > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_accumulate|k_fixup' --output-format csv -d $OUT/fetch -o fetch -- python3 $R/tools/phase_timing.py --reps 2 > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_accumulate|k_fixup' --output-format csv -d $OUT/write -o write -- python3 $R/tools/phase_timing.py --reps 2 > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
find $OUT -name '*counter_collection*' | head
