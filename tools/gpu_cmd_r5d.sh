set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/probes/batch_affine/ba_wave > gpurun_out/ba_wave.txt 2>&1 || { cat gpurun_out/ba_wave.txt; exit 1; }
cat gpurun_out/ba_wave.txt
bash tools/prof.sh kernel > gpurun_out/prof_kernel.log 2>&1 || { tail -20 gpurun_out/prof_kernel.log; exit 1; }
bash tools/prof.sh traffic > gpurun_out/prof_traffic.log 2>&1 || { tail -20 gpurun_out/prof_traffic.log; exit 1; }
bash tools/prof.sh sq > gpurun_out/prof_sq.log 2>&1 || { tail -20 gpurun_out/prof_sq.log; exit 1; }
echo PROF_OK
