set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/prof.sh pipelined --n 131072 --steps 200 --warmup 48 --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 --h2d-steps 0 --bn254-steps 0 --shard17-steps 0 --default-queues-steps 0 > gpurun_out/prof_pipe17.log 2>&1 || { tail -20 gpurun_out/prof_pipe17.log; exit 1; }
mv gpurun_out/prof_pipelined gpurun_out/prof_pipelined17
bash tools/prof.sh pipelined --steps 60 --warmup 16 --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 --h2d-steps 0 --bn254-steps 0 --shard17-steps 0 --default-queues-steps 0 > gpurun_out/prof_pipe.log 2>&1 || { tail -20 gpurun_out/prof_pipe.log; exit 1; }
ls gpurun_out/prof_pipelined/run
