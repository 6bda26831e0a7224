set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python tools/ab.py --rounds 3 --no-quiet --key shard_2e17_rccl_world1_per_s --bench "--steps 10 --warmup 5 --no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 --h2d-steps 0 --bn254-steps 0 --shard17-steps 240 --repeats 1 --default-queues-steps 0 --detail-file ''" d4 d3:KZGMI_ACC_ORDER_SMALL=3 d5:KZGMI_ACC_ORDER_SMALL=5 > gpurun_out/ab_acc_order_shard17.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order_shard17.txt; exit 1; }
tail -1 gpurun_out/ab_acc_order_shard17.txt
