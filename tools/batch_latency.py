#!/usr/bin/env python3
"""Single-batch latency A/B: synchronous kzgmi_batch_verify_device on HBM-resident inputs, the
median of --reps calls after two warm calls, plus one profiled pass of phase times (the phases
are the slot stream's marks: with the split accumulation they are the critical path).

    python tools/batch_latency.py [--rounds R] [--n N] [--curve C] [--reps K] VARIANT [VARIANT ...]

VARIANT is `label[:KEY=VAL[,KEY=VAL...]]` as in tools/ab.py (KEY an environment variable, or
`lib` = another libkzgmi.so).  Variants alternate within each round (boxes drift).
"""
import argparse
import hashlib
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(args):
    sys.path.insert(0, os.path.join(ROOT, "kzg-batch-verification-scheme_amd"))
    import torch
    import kzgmi
    ctx = kzgmi.Context(0, 1)
    curve, n = args.curve, args.n
    g2 = kzgmi.G2_GENERATOR[curve]
    tau = 0x1234567
    srs = ctx.load_srs(curve, g2, ctx.g2_mul(curve, g2, tau))
    g1b = 2 * kzgmi.FP_BYTES[curve]
    C = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    P = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    z = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    y = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.gen_tuples(curve, tau, hashlib.sha256(b"t").digest(), n, C, z, y, P)
    seed = hashlib.sha256(b"v").digest()
    for _ in range(2):
        assert ctx.batch_verify(srs, C, z, y, P, seed=seed, n=n) is True
    torch.cuda.synchronize()
    runs = []
    for _ in range(args.reps):
        a = time.perf_counter()
        ok = ctx.batch_verify(srs, C, z, y, P, seed=seed, n=n)
        runs.append((time.perf_counter() - a) * 1e3)
        assert ok is True
    ctx.set_profiling(True)
    for _ in range(4):
        assert ctx.batch_verify(srs, C, z, y, P, seed=seed, n=n) is True
    ph = ctx.phase_ms()
    print(json.dumps({"latency_ms": statistics.median(runs), "min_ms": min(runs), "phases": ph}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="*")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=1 << 20)
    ap.add_argument("--curve", default="bls12_381")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--child", action="store_true")
    args = ap.parse_args()
    if args.child:
        return child(args)
    variants = []
    for spec in args.variants:
        label, _, kvs = spec.partition(":")
        env = {}
        for kv in filter(None, kvs.split(",")):
            k, _, v = kv.partition("=")
            env["KZGMI_LIB" if k == "lib" else k] = (os.path.join(ROOT, v) if k == "lib" and not os.path.isabs(v) else v)
        variants.append((label, env))
    res = {label: [] for label, _ in variants}
    for r in range(args.rounds):
        for label, env in variants:
            p = subprocess.run(["timeout", "-k", "10", "240", sys.executable, os.path.abspath(__file__), "--child",
                                "--n", str(args.n), "--curve", args.curve, "--reps", str(args.reps)],
                               env=dict(os.environ, **env), capture_output=True, text=True)
            if p.returncode:
                print(p.stderr[-3000:], file=sys.stderr)
                return p.returncode
            d = json.loads(p.stdout.strip().splitlines()[-1])
            res[label].append(d["latency_ms"])
            print(json.dumps({"round": r, "variant": label, "env": env, **d}), flush=True)
    print(json.dumps({"summary": {k: {"median_ms": statistics.median(v), "runs": v} for k, v in res.items()},
                      "n": args.n, "curve": args.curve}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
