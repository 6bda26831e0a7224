set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python tools/ab.py --rounds 3 o2 o0:KZGMI_ACC_ORDER=0 o3:KZGMI_ACC_ORDER=3 o4:KZGMI_ACC_ORDER=4 > gpurun_out/ab_acc_order.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order.txt; exit 1; }
tail -12 gpurun_out/ab_acc_order.txt
