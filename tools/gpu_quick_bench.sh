set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 60 --warmup 8 --no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/bq.json 2> gpurun_out/bq.err || { tail -30 gpurun_out/bq.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bq.json'));s=d['secondary'];print(d['value'], s['repeats_median_batch_verifies_per_s'], [round(x,1) for x in s['repeats_batch_verifies_per_s']])"
timeout -k 10 300 python bench.py --curve bn254 --n 524288 --steps 200 --warmup 20 --no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 --cfg4-msms 0 > gpurun_out/bq_bn.json 2> gpurun_out/bq_bn.err || { tail -30 gpurun_out/bq_bn.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bq_bn.json'));s=d['secondary'];print('bn254 2^19', d['value'], s['repeats_median_batch_verifies_per_s'], s['phase_ms_single_batch'])"
