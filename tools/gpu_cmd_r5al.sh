set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_r5al.log 2>&1 || { tail -60 gpurun_out/tests_r5al.log; exit 1; }
tail -2 gpurun_out/tests_r5al.log
: > gpurun_out/ab_bn254_naf.txt
for r in 1 2 3; do
  for v in build_ref kzgmi; do
    for n in 65536 256; do
      echo "round $r lib $v n $n" >> gpurun_out/ab_bn254_naf.txt
      timeout -k 10 120 python tools/phase_timing.py --curve bn254 --reps 10 --n $n --lib kzg-batch-verification-scheme_amd/$v/libkzgmi.so >> gpurun_out/ab_bn254_naf.txt 2>&1 || { tail -20 gpurun_out/ab_bn254_naf.txt; exit 1; }
    done
  done
done
python tools/ab_phases.py gpurun_out/ab_bn254_naf.txt pairing,combine,reduce
