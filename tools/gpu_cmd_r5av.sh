set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof_single
bash tools/prof.sh kernel > gpurun_out/prof_k20.log 2>&1 || { tail -20 gpurun_out/prof_k20.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/bench_r5av.json 2> gpurun_out/bench_r5av.err || { tail -30 gpurun_out/bench_r5av.err; exit 1; }
tail -c 1500 gpurun_out/bench_r5av.json
cp gpurun_out/bench_detail.json gpurun_out/bench_r5av_detail.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r5av_driver.json 2> gpurun_out/bench_r5av_driver.err || { tail -30 gpurun_out/bench_r5av_driver.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_r5av_driver.json').read().strip().splitlines()[-1]);print('driver form', d['value'], d['headline'])"
