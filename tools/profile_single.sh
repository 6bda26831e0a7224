#!/bin/bash
# Judged profile of the dominant kernel on non-pipelined single batches (tools/phase_timing.py):
#   1) kernel trace + stats;  2) FETCH_SIZE  3) WRITE_SIZE  4) TCC_HIT/TCC_MISS -- counter
#   passes of their own, no trace domains, restricted to k_accumulate.
# Summarise locally: python3 tools/summarize_single.py gpurun_out/prof_single profiles/r01/rocprof_single
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_single
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/tools/phase_timing.py --reps 4 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  d=$(echo $c | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-include-regex 'k_accumulate' --output-format csv -d $OUT/$d -o $d -- python3 $R/tools/phase_timing.py --reps 2 > $OUT/$d.log 2>&1 || { tail -20 $OUT/$d.log; exit 1; }
done
find $OUT -name '*.csv' | head -20
