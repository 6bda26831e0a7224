#!/bin/bash
# Round profile session: single-batch kernel trace + counter passes of the dominant kernel
# (tools/profile_single.sh, tools/pmc_sq_accumulate.sh), the full default bench, configs[4]
# (BN254 2^22, and its 2^19 per-GPU shard) and the 2^17-tuple batch (per-rank share of an 8-way strong split of 2^20).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
bash tools/profile_single.sh > gpurun_out/profile_single.log 2>&1 || { tail -20 gpurun_out/profile_single.log; exit 1; }
bash tools/pmc_sq_accumulate.sh > gpurun_out/pmc_sq.log 2>&1 || { tail -20 gpurun_out/pmc_sq.log; exit 1; }
cd "$R"
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
echo full; cut -c1-300 gpurun_out/bench_full.json
timeout -k 10 300 python bench.py --curve bn254 --n 4194304 --steps 40 --warmup 8 --no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/bench_bn254.json 2> gpurun_out/bench_bn254.err || { tail -30 gpurun_out/bench_bn254.err; exit 1; }
echo bn254; cut -c1-300 gpurun_out/bench_bn254.json
timeout -k 10 300 python bench.py --curve bn254 --n 524288 --steps 200 --warmup 20 --no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/bench_bn254_2e19.json 2> gpurun_out/bench_bn254_2e19.err || { tail -30 gpurun_out/bench_bn254_2e19.err; exit 1; }
echo bn254 2e19; cut -c1-300 gpurun_out/bench_bn254_2e19.json
timeout -k 10 300 python bench.py --n 131072 --steps 400 --warmup 40 --no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/bench_2e17.json 2> gpurun_out/bench_2e17.err || { tail -30 gpurun_out/bench_2e17.err; exit 1; }
echo 2e17; cut -c1-300 gpurun_out/bench_2e17.json
