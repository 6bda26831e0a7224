set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python tools/ab.py --rounds 4 --bench "--steps 20 --warmup 5" s16 s8:KZGMI_BENCH_SLOTS=8 s6:KZGMI_BENCH_SLOTS=6 s12:KZGMI_BENCH_SLOTS=12 > gpurun_out/ab_slots_steps20.txt 2>&1 || { tail -30 gpurun_out/ab_slots_steps20.txt; exit 1; }
tail -1 gpurun_out/ab_slots_steps20.txt
timeout -k 10 700 python tools/ab.py --rounds 2 s16 s8:KZGMI_BENCH_SLOTS=8 s12:KZGMI_BENCH_SLOTS=12 > gpurun_out/ab_slots_steps200.txt 2>&1 || { tail -30 gpurun_out/ab_slots_steps200.txt; exit 1; }
tail -1 gpurun_out/ab_slots_steps200.txt
