set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
Q="--no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 --h2d-steps 0 --bn254-steps 0 --shard17-steps 0 --repeats 5 --default-queues-steps 0 --detail-file ''"
: > gpurun_out/warmup_sweep.txt
for r in 1 2; do
for w in 5 16 32; do
  echo "round $r warmup $w" >> gpurun_out/warmup_sweep.txt
  eval timeout -k 10 200 python bench.py --steps 20 --warmup $w $Q > gpurun_out/ws.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ws.json').read().strip().splitlines()[-1]);print(d['value'], d['secondary'].get('repeats_median_batch_verifies_per_s'))" >> gpurun_out/warmup_sweep.txt
done
done
cat gpurun_out/warmup_sweep.txt
