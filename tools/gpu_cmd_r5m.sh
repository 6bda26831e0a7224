set -o pipefail
mkdir -p gpurun_out/prof17
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof17/kt -o kt -- python3 $GRAFT_REPO_ROOT/tools/phase_timing.py --reps 8 --n 131072 > $GRAFT_REPO_ROOT/gpurun_out/prof17/kt.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof17/kt.log; exit 1; }
cd $GRAFT_REPO_ROOT
ls gpurun_out/prof17/kt
