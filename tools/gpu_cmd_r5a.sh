set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_r5a.log 2>&1 || { tail -60 gpurun_out/tests_r5a.log; exit 1; }
tail -3 gpurun_out/tests_r5a.log
timeout -k 10 500 python tools/ab.py --rounds 2 --bench "--steps 100 --warmup 16" lanes24 lanes4:KZGMI_HW_QUEUES=4 slots24:KZGMI_LANES=0 slots4:KZGMI_LANES=0,KZGMI_HW_QUEUES=4 > gpurun_out/ab_lanes.txt 2>&1 || { tail -30 gpurun_out/ab_lanes.txt; exit 1; }
tail -1 gpurun_out/ab_lanes.txt
timeout -k 10 400 python tools/ab.py --rounds 2 --bench "--steps 240 --warmup 16 --n 131072" lanes24 lanes4:KZGMI_HW_QUEUES=4 slots24:KZGMI_LANES=0 > gpurun_out/ab_lanes_2e17.txt 2>&1 || { tail -30 gpurun_out/ab_lanes_2e17.txt; exit 1; }
tail -1 gpurun_out/ab_lanes_2e17.txt
