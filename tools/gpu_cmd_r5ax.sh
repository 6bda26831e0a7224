set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_single
bash tools/prof.sh kernel --n 131072 > gpurun_out/prof_k17b.log 2>&1 || { tail -20 gpurun_out/prof_k17b.log; exit 1; }
