set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python tools/ab.py --rounds 4 --bench "--steps 20 --warmup 5" f2 f0:KZGMI_FRONT_ORDER=0 f1:KZGMI_FRONT_ORDER=1 f4:KZGMI_FRONT_ORDER=4 > gpurun_out/ab_front_order_steps20.txt 2>&1 || { tail -30 gpurun_out/ab_front_order_steps20.txt; exit 1; }
tail -1 gpurun_out/ab_front_order_steps20.txt
timeout -k 10 600 python tools/ab.py --rounds 2 f2 f0:KZGMI_FRONT_ORDER=0 > gpurun_out/ab_front_order_steps200.txt 2>&1 || { tail -30 gpurun_out/ab_front_order_steps200.txt; exit 1; }
tail -1 gpurun_out/ab_front_order_steps200.txt
