#!/bin/bash
# SQ counters of k_accumulate<Bn254> on single configs[4]-size batches (n = 2^22, GLV):
# VALU instructions per addition and the wave-cycle split, for the VALU-floor estimate.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_sq_bn
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --kernel-include-regex 'k_accumulate' --output-format csv -d $OUT/sq -o sq -- python3 $R/tools/phase_timing.py --reps 2 --curve bn254 --n 4194304 > $OUT/sq.log 2>&1 || { tail -20 $OUT/sq.log; exit 1; }
find $OUT -name '*counter_collection*' | head
