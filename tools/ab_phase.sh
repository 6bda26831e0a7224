#!/bin/bash
# A/B of library builds on single-batch phase times (tools/phase_timing.py), each lib twice in
# A/B/A order: bash tools/ab_phase.sh libA libB ...
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for pass in 1 2; do
  for lib in "$@"; do
    timeout -k 10 200 python tools/phase_timing.py --lib "$lib" --reps 6 | cut -c1-600 || exit 1
  done
done
