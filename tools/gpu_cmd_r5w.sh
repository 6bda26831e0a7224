set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python tools/ab.py --rounds 3 --bench "--n 131072 --steps 600 --warmup 48" o4:KZGMI_ACC_ORDER=4 o0:KZGMI_ACC_ORDER=0 o6:KZGMI_ACC_ORDER=6 o8:KZGMI_ACC_ORDER=8 > gpurun_out/ab_acc_order_2e17b.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order_2e17b.txt; exit 1; }
tail -1 gpurun_out/ab_acc_order_2e17b.txt
timeout -k 10 600 python tools/ab.py --rounds 2 --bench "--curve bn254 --steps 200" o2 o3:KZGMI_ACC_ORDER=3 o4:KZGMI_ACC_ORDER=4 > gpurun_out/ab_acc_order_bn254b.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order_bn254b.txt; exit 1; }
tail -1 gpurun_out/ab_acc_order_bn254b.txt
