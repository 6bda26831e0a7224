#!/bin/bash
# rocprofv3 passes on the GPU box (replaces round 1-3's profile*.sh / kt_*.sh / pmc_*.sh):
#   tools/prof.sh MODE [phase_timing.py args, e.g. --curve bn254 --n 4194304]
# MODE
#   kernel    kernel trace + stats of single, non-pipelined batches (tools/phase_timing.py): the
#             per-kernel durations the bench line's roofline.rocprof_kernel_avg_ms is checked against
#   traffic   FETCH_SIZE, WRITE_SIZE, TCC_HIT/TCC_MISS of k_accumulate: one counter pass each
#   sq        8 SQ counters of k_accumulate (VALU instructions per addition, wave-cycle split)
#   valu      SQ_INSTS_VALU / SALU / WAVES of every kernel of a batch
#   icache    instruction-cache counters of k_accumulate
#   pipelined kernel + memory-copy trace of a short pipelined bench (args: bench.py arguments)
# Counter passes never combine --pmc with trace domains, stay within the per-block counter
# limits, and run under their own `timeout -s KILL`.  Output: gpurun_out/prof_MODE/ (kernel and
# traffic share gpurun_out/prof_single/).  Summaries: python3 tools/summarize_single.py
# gpurun_out/prof_single profiles/<round>/rocprof_single; tools/summarize_sq.py gpurun_out/prof_sq ...
set -o pipefail
MODE=${1:?mode}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
# PROF_TAG: suffix of the output directory (e.g. _bn254 for a second curve's passes)
case $MODE in kernel|traffic) OUT=$R/gpurun_out/prof_single${PROF_TAG:-} ;; *) OUT=$R/gpurun_out/prof_$MODE${PROF_TAG:-} ;; esac
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PT="python3 $R/tools/phase_timing.py"
pmc() {  # pmc NAME REGEX COUNTERS...
  local name=$1 regex=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "$regex" --output-format csv -d "$OUT/$name" -o "$name" \
    -- $PT --reps 2 $ARGS > "$OUT/$name.log" 2>&1 || { tail -20 "$OUT/$name.log"; exit 1; }
}
ARGS="$*"
case $MODE in
  kernel)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/kt" -o kt -- $PT --reps 4 $ARGS \
      > "$OUT/kt.log" 2>&1 || { tail -20 "$OUT/kt.log"; exit 1; } ;;
  traffic)
    pmc fetch_size 'k_accumulate|k_fixup' FETCH_SIZE
    pmc write_size 'k_accumulate|k_fixup' WRITE_SIZE
    pmc tcc_hit_sum 'k_accumulate' TCC_HIT_sum TCC_MISS_sum ;;
  sq)
    pmc sq 'k_accumulate' SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU \
      SQ_WAIT_INST_ANY SQ_WAIT_ANY ;;
  valu)
    timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES --output-format csv -d "$OUT/v" -o v \
      -- $PT --reps 2 $ARGS > "$OUT/v.log" 2>&1 || { tail -20 "$OUT/v.log"; exit 1; } ;;
  icache)
    pmc ic 'k_accumulate' SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAVE_CYCLES \
      SQ_WAIT_INST_ANY SQ_INSTS_VALU ;;
  pipelined)
    timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/run" -o run \
      -- python3 "$R/bench.py" --no-cpu --repeats 1 $ARGS > "$OUT/run.log" 2>&1 || { tail -20 "$OUT/run.log"; exit 1; } ;;
  *) echo "unknown mode $MODE"; exit 2 ;;
esac
find "$OUT" -name '*stats*' -o -name '*counter_collection*' | head -20
