set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tests_r5n.log 2>&1 || { tail -60 gpurun_out/tests_r5n.log; exit 1; }
tail -3 gpurun_out/tests_r5n.log
: > gpurun_out/ab_small_bn.txt
for r in 1 2; do
  for st in 0 4096; do
    for n in 64 256 1024; do
      echo "round $r lib small$st n $n" >> gpurun_out/ab_small_bn.txt
      KZGMI_SMALL_TERMS=$st timeout -k 10 120 python tools/phase_timing.py --curve bn254 --reps 10 --n $n >> gpurun_out/ab_small_bn.txt 2>&1 || { tail -20 gpurun_out/ab_small_bn.txt; exit 1; }
    done
  done
done
python tools/ab_phases.py gpurun_out/ab_small_bn.txt accumulate,reduce,combine,pairing
