#!/bin/bash
# rocprofv3 kernel trace of non-pipelined single batches (tools/phase_timing.py): per-kernel
# durations without the 12-slot pipeline's stretching.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/kt_single
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o kt -- python3 $R/tools/phase_timing.py --reps 4 "$@" > $OUT/run.log 2>&1 || { tail -20 $OUT/run.log; exit 1; }
