set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W2=1 TORCHRUN=1 STEPS=60 bash tools/scale_rehearsal.sh > gpurun_out/scale_r5an.log 2>&1 || { tail -30 gpurun_out/scale_r5an.log; exit 1; }
cat gpurun_out/scale_r5an.log | tail -5
