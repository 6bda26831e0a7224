set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_single gpurun_out/prof_single_ref
bash tools/prof.sh kernel --lib $GRAFT_REPO_ROOT/kzg-batch-verification-scheme_amd/build_ref/libkzgmi.so > gpurun_out/prof_kref.log 2>&1 || { tail -20 gpurun_out/prof_kref.log; exit 1; }
mv gpurun_out/prof_single gpurun_out/prof_single_ref
bash tools/prof.sh kernel > gpurun_out/prof_knew.log 2>&1 || { tail -20 gpurun_out/prof_knew.log; exit 1; }
: > gpurun_out/ab_set_shift2.txt
for r in 1 2 3; do
  for v in build_ref kzgmi; do
    for n in 1048576 131072; do
      echo "round $r lib $v n $n" >> gpurun_out/ab_set_shift2.txt
      timeout -k 10 120 python tools/phase_timing.py --reps 10 --n $n --lib kzg-batch-verification-scheme_amd/$v/libkzgmi.so >> gpurun_out/ab_set_shift2.txt 2>&1 || { tail -20 gpurun_out/ab_set_shift2.txt; exit 1; }
    done
  done
done
python tools/ab_phases.py gpurun_out/ab_set_shift2.txt sort,accumulate,reduce
