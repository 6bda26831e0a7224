set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/prof.sh kernel --n 131072 > gpurun_out/prof_k17.log 2>&1 || { tail -20 gpurun_out/prof_k17.log; exit 1; }
mv gpurun_out/prof_single gpurun_out/prof_single17
bash tools/prof.sh kernel > gpurun_out/prof_k20.log 2>&1 || { tail -20 gpurun_out/prof_k20.log; exit 1; }
ls gpurun_out/prof_single/kt
