set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab.py --rounds 3 q4:KZGMI_HW_QUEUES=4 q4o:KZGMI_HW_QUEUES=4,KZGMI_ACC_ORDER=2 q24:KZGMI_HW_QUEUES=24 > gpurun_out/ab_acc_order_q4.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order_q4.txt; exit 1; }
tail -1 gpurun_out/ab_acc_order_q4.txt
