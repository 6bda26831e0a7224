#!/usr/bin/env python3
"""Pipelined G1 MSM rate at one size through the three paths bench.py uses (GPU box):
ctx.msm_g1_async over `--slots` slots, and kzgmi.distributed.ShardedMsmPipeline at world 1 over
RCCL in the eager and the deferred schedule.  Prints ms per MSM of each.

python tools/msm_pipe_check.py [--log-n 21] [--slots 4] [--msms 24]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-batch-verification-scheme_amd"))
# as bench.py: the box exports GPU_MAX_HW_QUEUES=4 (HIP's default); force the pipeline's 24 --
# with 4, streams share hardware queues and a stream's GPU-side wait blocks the others behind it
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("KZGMI_HW_QUEUES", "24")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import kzgmi  # noqa: E402
from kzgmi.distributed import ShardedMsmPipeline  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--log-n", type=int, default=21)
ap.add_argument("--slots", type=int, default=4)
ap.add_argument("--msms", type=int, default=24)
ap.add_argument("--eager-slots", type=int, default=0, help="slots of the eager schedule (default --slots)")
ap.add_argument("--only", default="", help="run only this schedule (direct / eager / deferred)")
args = ap.parse_args()
curve, n = "bls12_381", 1 << args.log_n
ctx = kzgmi.Context(0, 16)
gen = torch.Generator(device="cuda").manual_seed(5)
k = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=gen)
k[:, 0] &= 0x3F
s = torch.randint(0, 256, (n, 32), dtype=torch.uint8, device="cuda", generator=gen)
s[:, 0] &= 0x3F
p = torch.empty(n * 96, dtype=torch.uint8, device="cuda")
ctx.gen_g1(curve, k.reshape(-1), n, p)
s = s.reshape(-1)
torch.cuda.synchronize()


def direct(slots):
    res, q = [], [0]

    def sub():
        sl = q[0] % slots
        if q[0] >= slots:
            res.append(ctx.msm_wait(sl))
        ctx.msm_g1_async(curve, sl, p, s, n)
        q[0] += 1

    def drain():
        first = q[0] % slots if q[0] >= slots else 0
        for i in range(min(q[0], slots)):
            res.append(ctx.msm_wait((first + i) % slots))
        q[0] = 0
    return sub, drain, res


def sharded(eager, slots, lanes):
    pipe = ShardedMsmPipeline(ctx, curve, slots=slots, lanes=lanes, eager=eager)
    res = []
    return (lambda: res.extend(pipe.submit(p, s, n))), (lambda: res.extend(pipe.drain())), res


os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29551")
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
es = args.eager_slots or args.slots
for name, mk in (("direct", lambda: direct(args.slots)), ("eager%d" % es, lambda: sharded(True, es, 0)),
                 ("deferred", lambda: sharded(False, args.slots, 2)), ("direct", lambda: direct(args.slots))):
    if args.only and not name.startswith(args.only):
        continue
    sub, drain, res = mk()
    for _ in range(args.slots):
        sub()
    drain()
    torch.cuda.synchronize()
    a = time.perf_counter()
    calls = []
    for _ in range(args.msms):
        c0 = time.perf_counter()
        sub()
        calls.append(1e3 * (time.perf_counter() - c0))
    drain()
    torch.cuda.synchronize()
    dt = time.perf_counter() - a
    assert len(set(res)) == 1
    print("%-9s n=2^%d slots=%d: %.2f ms per MSM, %.1f M pts/s; host ms per submit: first %s, median %.2f"
          % (name, args.log_n, args.slots, 1e3 * dt / args.msms, n * args.msms / dt / 1e6,
             " ".join("%.2f" % x for x in calls[:6]), sorted(calls)[len(calls) // 2]), flush=True)
dist.destroy_process_group()
