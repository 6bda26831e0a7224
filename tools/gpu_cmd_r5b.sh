set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python tools/ab.py --rounds 2 --bench "--steps 100 --warmup 16" s24 s4:KZGMI_HW_QUEUES=4 s4p:KZGMI_HW_QUEUES=4,KZGMI_STREAM_PRIO=1 s24p:KZGMI_STREAM_PRIO=1 l4a2:KZGMI_HW_QUEUES=4,KZGMI_LANES=2,KZGMI_ACC_LANES=2 s4x8:KZGMI_HW_QUEUES=4,KZGMI_BENCH_SLOTS=8,KZGMI_STREAM_PRIO=1 > gpurun_out/ab_prio.txt 2>&1 || { tail -30 gpurun_out/ab_prio.txt; exit 1; }
tail -1 gpurun_out/ab_prio.txt
timeout -k 10 400 python tools/ab.py --rounds 2 --bench "--steps 240 --warmup 16 --n 131072" s24 s4:KZGMI_HW_QUEUES=4 s4p:KZGMI_HW_QUEUES=4,KZGMI_STREAM_PRIO=1 l4a2:KZGMI_HW_QUEUES=4,KZGMI_LANES=2,KZGMI_ACC_LANES=2 > gpurun_out/ab_prio_2e17.txt 2>&1 || { tail -30 gpurun_out/ab_prio_2e17.txt; exit 1; }
tail -1 gpurun_out/ab_prio_2e17.txt
