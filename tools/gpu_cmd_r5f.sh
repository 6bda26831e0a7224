set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 tools/probes/batch_affine/ba_wave > gpurun_out/ba_wave.txt 2>&1 || { cat gpurun_out/ba_wave.txt; exit 1; }
grep -v "^  mismatch" gpurun_out/ba_wave.txt
: > gpurun_out/ab_combine.txt
for r in 1 2 3; do
  for v in build_ref kzgmi; do
    for n in 1048576 256; do
      echo "round $r lib $v n $n" >> gpurun_out/ab_combine.txt
      timeout -k 10 120 python tools/phase_timing.py --reps 10 --n $n --lib kzg-batch-verification-scheme_amd/$v/libkzgmi.so >> gpurun_out/ab_combine.txt 2>&1 || { tail -20 gpurun_out/ab_combine.txt; exit 1; }
    done
  done
done
grep -A1 "^round" gpurun_out/ab_combine.txt | grep -o '"combine": [0-9.]*\|"reduce": [0-9.]*\|^round.*' | paste - - - 
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_r5f.log 2>&1 || { tail -60 gpurun_out/tests_r5f.log; exit 1; }
tail -3 gpurun_out/tests_r5f.log
