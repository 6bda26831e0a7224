"""Synchronous single-MSM latency (kzgmi_msm_g1 on HBM-resident points and scalars), median of
--reps calls after one warm call; --lib times another build (A/B).

python tools/msm_latency.py [--n N] [--reps R] [--curve C] [--lib path/to/libkzgmi.so]
"""
import argparse
import hashlib
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-batch-verification-scheme_amd"))
ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1 << 20)
ap.add_argument("--reps", type=int, default=15)
ap.add_argument("--lib", default=None)
ap.add_argument("--curve", default="bls12_381")
args = ap.parse_args()
if args.lib:
    os.environ["KZGMI_LIB"] = args.lib

import torch  # noqa: E402
import kzgmi  # noqa: E402

ctx = kzgmi.Context(0, 1)
curve, n = args.curve, args.n
g1b = 2 * kzgmi.FP_BYTES[curve]
C = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
P = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
z = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
y = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
ctx.gen_tuples(curve, 0x1234567, hashlib.sha256(b"m").digest(), n, C, z, y, P)
ref = ctx.msm_g1(curve, C, z, n=n)
runs = []
for _ in range(args.reps):
    torch.cuda.synchronize()
    a = time.perf_counter()
    r = ctx.msm_g1(curve, C, z, n=n)
    runs.append((time.perf_counter() - a) * 1e3)
    assert r == ref
print(json.dumps({"lib": kzgmi.LIB_PATH, "n": n, "msm_latency_ms_median": statistics.median(runs),
                  "runs": [round(x, 3) for x in runs]}))
