set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_cmd_r5ah.sh || exit 1
: > gpurun_out/ab_tile8192.txt
for r in 1 2 3; do
  for v in kzgmi build_t8; do
    for n in 1048576 131072; do
      echo "round $r lib $v n $n" >> gpurun_out/ab_tile8192.txt
      timeout -k 10 120 python tools/phase_timing.py --reps 10 --n $n --lib kzg-batch-verification-scheme_amd/$v/libkzgmi.so >> gpurun_out/ab_tile8192.txt 2>&1 || { tail -20 gpurun_out/ab_tile8192.txt; exit 1; }
    done
  done
done
python tools/ab_phases.py gpurun_out/ab_tile8192.txt sort,accumulate,reduce
