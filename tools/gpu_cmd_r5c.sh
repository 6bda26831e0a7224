set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_r5c.log 2>&1 || { tail -60 gpurun_out/tests_r5c.log; exit 1; }
tail -3 gpurun_out/tests_r5c.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r5c.json 2> gpurun_out/bench_r5c.err || { tail -30 gpurun_out/bench_r5c.err; exit 1; }
tail -c 3000 gpurun_out/bench_r5c.json
for cv in bls12_381 bn254; do
  timeout -k 10 200 python tools/phase_timing.py --reps 1 --curve $cv --n 65536 --lib kzg-batch-verification-scheme_amd/build_stamps/libkzgmi.so > gpurun_out/stamps_$cv.txt 2>&1 || { tail -20 gpurun_out/stamps_$cv.txt; exit 1; }
done
grep -h "PAIRSTAMP" gpurun_out/stamps_bls12_381.txt | tail -12
bash tools/prof.sh kernel > gpurun_out/prof_kernel.log 2>&1 || { tail -20 gpurun_out/prof_kernel.log; exit 1; }
echo PROF_OK
