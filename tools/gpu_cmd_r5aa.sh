set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python tools/ab.py --rounds 5 --bench "--steps 20 --warmup 5" on off:KZGMI_ACC_ORDER=0,KZGMI_ACC_ORDER_SMALL=0 q4:KZGMI_HW_QUEUES=4 q4o:KZGMI_HW_QUEUES=4,KZGMI_ACC_ORDER=2 > gpurun_out/ab_acc_order_steps20.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order_steps20.txt; exit 1; }
tail -1 gpurun_out/ab_acc_order_steps20.txt
