set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_r5x.log 2>&1 || { tail -60 gpurun_out/tests_r5x.log; exit 1; }
tail -2 gpurun_out/tests_r5x.log
timeout -k 10 500 python tools/ab.py --rounds 3 new off:KZGMI_ACC_ORDER=0,KZGMI_ACC_ORDER_SMALL=0 > gpurun_out/ab_acc_order_final.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order_final.txt; exit 1; }
tail -1 gpurun_out/ab_acc_order_final.txt
timeout -k 10 500 python tools/ab.py --rounds 3 --bench "--n 131072 --steps 600 --warmup 48" new off:KZGMI_ACC_ORDER=0,KZGMI_ACC_ORDER_SMALL=0 > gpurun_out/ab_acc_order_final_2e17.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order_final_2e17.txt; exit 1; }
tail -1 gpurun_out/ab_acc_order_final_2e17.txt
timeout -k 10 500 python tools/ab.py --rounds 3 --bench "--n 262144 --steps 400 --warmup 48" new off:KZGMI_ACC_ORDER=0,KZGMI_ACC_ORDER_SMALL=0 o2:KZGMI_ACC_ORDER_SMALL=2 > gpurun_out/ab_acc_order_final_2e18.txt 2>&1 || { tail -30 gpurun_out/ab_acc_order_final_2e18.txt; exit 1; }
tail -1 gpurun_out/ab_acc_order_final_2e18.txt
