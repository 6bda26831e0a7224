set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_r5ay.log 2>&1 || { tail -60 gpurun_out/tests_r5ay.log; exit 1; }
tail -2 gpurun_out/tests_r5ay.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r5ay.json 2> gpurun_out/bench_r5ay.err || { tail -30 gpurun_out/bench_r5ay.err; exit 1; }
cp gpurun_out/bench_detail.json gpurun_out/bench_r5ay_detail.json
python -c "import json;d=json.loads(open('gpurun_out/bench_r5ay.json').read().strip().splitlines()[-1]);print('full', d['value'], d['headline'], d['secondary']['shard_2e17_rccl_world1_per_s'], d['secondary']['default_hw_queues_frac'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r5ay_driver.json 2> gpurun_out/bench_r5ay_driver.err || { tail -30 gpurun_out/bench_r5ay_driver.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_r5ay_driver.json').read().strip().splitlines()[-1]);print('driver form', d['value'], d['headline'])"
