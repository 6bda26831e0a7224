set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/ab_mulsplit.txt
for r in 1 2 3; do
  for v in build_ref kzgmi; do
    for n in 1048576 256; do
      echo "round $r lib $v n $n" >> gpurun_out/ab_mulsplit.txt
      timeout -k 10 120 python tools/phase_timing.py --reps 10 --n $n --lib kzg-batch-verification-scheme_amd/$v/libkzgmi.so >> gpurun_out/ab_mulsplit.txt 2>&1 || { tail -20 gpurun_out/ab_mulsplit.txt; exit 1; }
    done
  done
done
python tools/ab_phases.py gpurun_out/ab_mulsplit.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_r5j.log 2>&1 || { tail -60 gpurun_out/tests_r5j.log; exit 1; }
tail -3 gpurun_out/tests_r5j.log
