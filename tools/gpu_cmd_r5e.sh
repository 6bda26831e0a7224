set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/probes/batch_affine/ba_wave > gpurun_out/ba_wave.txt 2>&1 || { cat gpurun_out/ba_wave.txt; exit 1; }
cat gpurun_out/ba_wave.txt
for b in build_stamps build_stamps2; do
  timeout -k 10 200 python tools/phase_timing.py --reps 1 --curve bls12_381 --n 65536 --lib kzg-batch-verification-scheme_amd/$b/libkzgmi.so > gpurun_out/${b}_bls.txt 2>&1 || { tail -20 gpurun_out/${b}_bls.txt; exit 1; }
  grep -h "PAIRSTAMP" gpurun_out/${b}_bls.txt | tail -10
done
