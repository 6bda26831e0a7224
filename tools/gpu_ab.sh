#!/bin/bash
# GPU tests, then A/B of the default library against the given variants: BLS12-381 pipelined
# rate (tools/ab_libs.sh) and configs[4] BN254 (tools/ab_bn254.sh), alternating builds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
P=kzg-batch-verification-scheme_amd/kzgmi
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/tests.log 2>&1 || { tail -40 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
libs="$P/libkzgmi.so"
for v in "$@"; do libs="$libs $P/$v $P/libkzgmi.so"; done
bash tools/ab_libs.sh $libs || exit 1
bash tools/ab_bn254.sh $libs || exit 1
