#!/bin/bash
# rocprofv3 passes for the judged profile (run on the GPU box), same bench command each time:
#   1) kernel trace + stats (CSV); 2) FETCH_SIZE and 3) WRITE_SIZE passes (separate, counters
#   only, no trace domains), restricted to the bucket-accumulation kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 24 --warmup 8 --no-cpu --msm-steps 0 --fs-steps 0 --compressed-steps 0 --trusted-steps 0 --commit-steps 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py $ARGS > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_accumulate<' --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py $ARGS > $OUT/fetch.log 2>&1 || { tail -20 $OUT/fetch.log; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_accumulate<' --output-format csv -d $OUT/write -o write -- python3 $R/bench.py $ARGS > $OUT/write.log 2>&1 || { tail -20 $OUT/write.log; exit 1; }
# summarise locally after the merge: python3 tools/summarize_profile.py gpurun_out/prof profiles/r01/rocprof
