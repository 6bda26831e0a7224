set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_r5ad.json 2> gpurun_out/bench_r5ad.err || { tail -30 gpurun_out/bench_r5ad.err; exit 1; }
tail -c 1800 gpurun_out/bench_r5ad.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r5ad_driver.json 2> gpurun_out/bench_r5ad_driver.err || { tail -30 gpurun_out/bench_r5ad_driver.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_r5ad_driver.json').read().strip().splitlines()[-1]);print('driver form', d['value'], d['headline'])"
