set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_r5aw.log 2>&1 || { tail -60 gpurun_out/tests_r5aw.log; exit 1; }
tail -2 gpurun_out/tests_r5aw.log
KZGMI_SORT_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread -k "boundaries or ragged or golden" > gpurun_out/tests_r5aw_split.log 2>&1 || { tail -60 gpurun_out/tests_r5aw_split.log; exit 1; }
tail -2 gpurun_out/tests_r5aw_split.log
: > gpurun_out/ab_fixup_crowded.txt
for r in 1 2 3; do
  for v in build_ref kzgmi; do
    for n in 1048576 131072; do
      echo "round $r lib $v n $n" >> gpurun_out/ab_fixup_crowded.txt
      timeout -k 10 120 python tools/phase_timing.py --reps 10 --n $n --lib kzg-batch-verification-scheme_amd/$v/libkzgmi.so >> gpurun_out/ab_fixup_crowded.txt 2>&1 || { tail -20 gpurun_out/ab_fixup_crowded.txt; exit 1; }
    done
  done
done
python tools/ab_phases.py gpurun_out/ab_fixup_crowded.txt sort,accumulate,reduce
timeout -k 10 700 python tools/ab.py --rounds 3 --bench "--n 131072 --steps 600 --warmup 48" new ref:lib=kzg-batch-verification-scheme_amd/build_ref/libkzgmi.so > gpurun_out/ab_fixup_crowded_2e17.txt 2>&1 || { tail -30 gpurun_out/ab_fixup_crowded_2e17.txt; exit 1; }
tail -1 gpurun_out/ab_fixup_crowded_2e17.txt
