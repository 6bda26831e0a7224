#!/bin/bash
# configs[4] (BN254, n = 2^22, one GPU) diagnosis: A/B of library builds (pipelined rate), then a
# kernel-trace summary of a short pipelined run and the accumulation's L2-miss traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; P=kzg-batch-verification-scheme_amd/kzgmi
bash tools/ab_bn254.sh $P/libkzgmi.so $P/libkzgmi_bn32.so $P/libkzgmi.so || exit 1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bn" -o run --output-format csv -- python3 "$R/bench.py" --curve bn254 --n 4194304 --steps 12 --warmup 4 --no-cpu --msm-steps 0 --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 --cfg4-msms 0 > "$R/gpurun_out/prof_bn.log" 2>&1 || { tail -20 "$R/gpurun_out/prof_bn.log"; exit 1; }
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex 'k_accumulate|k_fine_sort|k_bin_scatter' --output-format csv -d "$R/gpurun_out/pmc_bn_$tag" -o run -- python3 "$R/tools/phase_timing.py" --curve bn254 --n 4194304 --reps 1 > "$R/gpurun_out/pmc_bn_$tag.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc_bn_$tag.log"; exit 1; }
done
find "$R/gpurun_out" -name '*stats*' -path '*prof_bn*'
