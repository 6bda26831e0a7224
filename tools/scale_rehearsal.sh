#!/bin/bash
# Multi-GPU bench path on the 1-GPU box: (1) the sharded pipeline at world 1 over RCCL (the
# per-rank rate the N-GPU runs are built from), (2) with W2=1: `bench.py --gpus 2` started
# directly (no torchrun: bench.py's own launcher, kzgmi/launch.py, starts the 2 ranks), both
# ranks on the one GPU over gloo (KZGMI_DIST_BACKEND=gloo; RCCL refuses two ranks per device) --
# exercises the launcher, every collective, the strong-scaled leg and rank 0's report.  With
# TORCHRUN=1 the 2 ranks start the driver's way instead (python -m torch.distributed.run ...
# bench.py --gpus 2, default legs), still over gloo on the one GPU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --sharded --no-cpu --steps ${STEPS:-120} --warmup 12 --msm-steps 12 \
  --compressed-steps 0 --fs-steps 0 --trusted-steps 0 --commit-steps 0 \
  > gpurun_out/sharded_w1.json 2> gpurun_out/sharded_w1.err || { tail -20 gpurun_out/sharded_w1.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/sharded_w1.json').read().strip().splitlines()[-1]);print('sharded w1', round(d['value'],2), 'strong', d['secondary'].get('strong_scaling_batch_per_s'), 'msm', d['headline']['msm_pts_per_s_2e20'])"
if [ -n "${W2:-}" ]; then
  if [ -n "${TORCHRUN:-}" ]; then  # exactly the driver's N = 2 command line, default legs
    L="python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611"
    A="--gpus 2 --steps 20 --warmup 5"
  else
    L="python"; A="--gpus 2 --no-cpu --steps 24 --warmup 6 --msm-steps 6 --slots 3 --cfg4-msms 2"
  fi
  KZGMI_DIST_BACKEND=gloo timeout -k 10 500 $L bench.py $A > gpurun_out/gloo_w2.json 2> gpurun_out/gloo_w2.err || { tail -30 gpurun_out/gloo_w2.err; exit 1; }
  python -c "import json;d=[json.loads(l) for l in open('gpurun_out/gloo_w2.json') if l.startswith('{')][-1];print('gloo w2', d['n_gpus'], round(d['value'],2), 'strong', d['secondary'].get('strong_scaling_batch_per_s'), 'msm', d['headline']['msm_pts_per_s_2e20'])"
fi
