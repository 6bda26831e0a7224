set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 10 --warmup 5 --no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 --h2d-steps 48 --bn254-steps 0 --shard17-steps 0 --repeats 1 --default-queues-steps 0 --detail-file ''"
timeout -k 10 1000 python tools/ab.py --rounds 3 --no-quiet --key h2d_pageable_per_s --key h2d_pinned_per_s --bench "$B" c8 c4:KZGMI_COPY_THREADS=4 c12:KZGMI_COPY_THREADS=12 c15:KZGMI_COPY_THREADS=15 > gpurun_out/ab_copy_threads.txt 2>&1 || { tail -30 gpurun_out/ab_copy_threads.txt; exit 1; }
tail -1 gpurun_out/ab_copy_threads.txt
