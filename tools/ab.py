#!/usr/bin/env python3
"""A/B runner for timing experiments on the GPU box (replaces round 1-3's per-experiment
tools/ab_*.sh scripts).

    python tools/ab.py [--rounds R] [--bench "ARGS"] [--phases] VARIANT [VARIANT ...]

VARIANT is `label[:KEY=VAL[,KEY=VAL...]]`; KEY is an environment variable (KZGMI_ACC_QUEUE,
KZGMI_WBITS, KZGMI_HW_QUEUES, KZGMI_COPY_THREADS, ...) or `lib`, a path to another build of
libkzgmi.so (sets KZGMI_LIB).  Every round runs every variant once, in order (A B C A B C ...),
because boxes differ by several percent in the same build and drift during a session: only
alternated runs in one call compare.  Each run is `bench.py ARGS` (default: the pipelined
configs[2] rate alone) under its own time limit; with --phases also tools/phase_timing.py
(single-batch phase times).  Prints one JSON line per run and a summary (median `value` per
variant, and any --key fields from the bench line's `secondary`).

Examples:
  python tools/ab.py base q4:KZGMI_ACC_QUEUE=4
  python tools/ab.py --rounds 3 new base:lib=kzg-batch-verification-scheme_amd/build_ref/libkzgmi.so
  python tools/ab.py --bench "--curve bn254 --n 4194304 --steps 40" base w13:KZGMI_WBITS=13
"""
import argparse
import json
import os
import shlex
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUIET = ("--no-cpu --msm-steps 0 --trusted-steps 0 --fs-steps 0 --commit-steps 0 --compressed-steps 0 "
         "--cfg4-msms 0 --h2d-steps 0 --bn254-steps 0 --shard17-steps 0 --repeats 1 --default-queues-steps 0 --detail-file ''")


def parse_variant(spec):
    label, _, kvs = spec.partition(":")
    env = {}
    for kv in filter(None, kvs.split(",")):
        k, _, v = kv.partition("=")
        if k == "lib":
            env["KZGMI_LIB"] = v if os.path.isabs(v) else os.path.join(ROOT, v)
        else:
            env[k] = v
    return label, env


def get(d, dotted):
    for part in dotted.split("."):
        if not isinstance(d, dict):
            return None
        d = d.get(part)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--bench", default="--steps 200 --warmup 24", help="bench.py arguments (plus the quiet set)")
    ap.add_argument("--no-quiet", action="store_true", help="do not add the flags that skip the secondary legs")
    ap.add_argument("--phases", action="store_true", help="also time single-batch phases (tools/phase_timing.py)")
    ap.add_argument("--key", action="append", default=[], help="secondary.* field to summarise too")
    ap.add_argument("--timeout", type=int, default=300)
    args = ap.parse_args()
    variants = [parse_variant(v) for v in args.variants]
    out_dir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out_dir, exist_ok=True)
    results = {label: [] for label, _ in variants}
    extra = {label: {k: [] for k in args.key} for label, _ in variants}
    bench_args = shlex.split(args.bench) + ([] if args.no_quiet else shlex.split(QUIET))
    for r in range(args.rounds):
        for label, env in variants:
            e = dict(os.environ, **env)
            if args.phases:
                p = subprocess.run(["timeout", "-k", "10", "200", sys.executable, os.path.join(ROOT, "tools", "phase_timing.py")],
                                   env=e, capture_output=True, text=True)
                if p.returncode:
                    print(p.stderr[-2000:], file=sys.stderr)
                    return p.returncode
                print(json.dumps({"round": r, "variant": label, "phases": json.loads(p.stdout.strip().splitlines()[-1])}),
                      flush=True)
            p = subprocess.run(["timeout", "-k", "10", str(args.timeout), sys.executable, os.path.join(ROOT, "bench.py")]
                               + bench_args, env=e, capture_output=True, text=True)
            if p.returncode:
                print(p.stderr[-3000:], file=sys.stderr)
                return p.returncode
            d = json.loads(p.stdout.strip().splitlines()[-1])
            results[label].append(d["value"])
            row = {"round": r, "variant": label, "env": env, "value": d["value"], "ms_per_step": d["ms_per_step"]}
            for k in args.key:
                v = get(d.get("secondary", {}), k)
                extra[label][k].append(v)
                row[k] = v
            print(json.dumps(row), flush=True)
    summary = {label: {"median": statistics.median(v), "runs": v} for label, v in results.items()}
    for label in summary:
        for k, vs in extra[label].items():
            nums = [x for x in vs if isinstance(x, (int, float))]
            summary[label][k] = statistics.median(nums) if nums else None
    print(json.dumps({"summary": summary, "bench_args": bench_args}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
