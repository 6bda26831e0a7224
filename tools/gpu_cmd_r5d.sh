set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/probes/batch_affine/ba_wave > gpurun_out/ba_wave.txt 2>&1 || { cat gpurun_out/ba_wave.txt; exit 1; }
cat gpurun_out/ba_wave.txt
bash tools/prof.sh kernel > gpurun_out/prof_kernel.log 2>&1 || { tail -20 gpurun_out/prof_kernel.log; exit 1; }
bash tools/prof.sh traffic > gpurun_out/prof_traffic.log 2>&1 || { tail -20 gpurun_out/prof_traffic.log; exit 1; }
bash tools/prof.sh sq > gpurun_out/prof_sq.log 2>&1 || { tail -20 gpurun_out/prof_sq.log; exit 1; }
echo PROF_OK
for cv in bls12_381 bn254; do
  timeout -k 10 200 python tools/phase_timing.py --reps 1 --curve $cv --n 65536 --lib kzg-batch-verification-scheme_amd/build_stamps/libkzgmi.so > gpurun_out/stamps_$cv.txt 2>&1 || { tail -20 gpurun_out/stamps_$cv.txt; exit 1; }
done
grep -h "PAIRSTAMP" gpurun_out/stamps_bls12_381.txt | tail -10
