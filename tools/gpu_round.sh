#!/bin/bash
# One GPU-box session: parity tests, smoke, bench (+ optional sharded-pipeline bench and the
# rocprof passes of tools/prof.sh).  Every GPU step has its own time limit; steps chain with ||exit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -3 gpurun_out/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "${SHARDED:-}" ]; then
  timeout -k 10 600 python bench.py --sharded --no-cpu --msm-steps 0 > gpurun_out/bench_sharded.json 2> gpurun_out/bench_sharded.err || { tail -30 gpurun_out/bench_sharded.err; exit 1; }
  cat gpurun_out/bench_sharded.json
fi
if [ -n "${PROFILE:-}" ]; then  # the judged rocprof summaries: single-batch kernel trace + counter passes
  for m in kernel traffic sq; do bash tools/prof.sh $m > gpurun_out/prof_$m.log 2>&1 || { tail -20 gpurun_out/prof_$m.log; exit 1; }; done
fi
