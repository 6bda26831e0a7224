#!/usr/bin/env python3
"""Host time of one pipelined enqueue (kzgmi_batch_verify_device_async through the Python binding)
against the GPU time it starts: times K back-to-back async submissions on K idle slots, with and
without phase profiling, at n = 2^20 and 2^17.

    python tools/enqueue_time.py
"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kzg-batch-verification-scheme_amd"))


def main():
    import torch
    import kzgmi
    slots = 16
    ctx = kzgmi.Context(0, slots)
    curve = "bls12_381"
    g2 = kzgmi.G2_GENERATOR[curve]
    tau = 0x1234567
    srs = ctx.load_srs(curve, g2, ctx.g2_mul(curve, g2, tau))
    for n in (1 << 20, 1 << 17):
        ctx.reserve(curve, n)
        g1b = 2 * kzgmi.FP_BYTES[curve]
        C = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
        P = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
        z = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        y = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
        ctx.gen_tuples(curve, tau, hashlib.sha256(b"t").digest(), n, C, z, y, P)
        seed = hashlib.sha256(b"v").digest()
        for prof in (False, True, False):
            ctx.set_profiling(prof)
            for rep in range(3):
                torch.cuda.synchronize()
                ts = []
                for s in range(slots):
                    a = time.perf_counter()
                    ctx.batch_verify_async(srs, s, C, z, y, P, n, seed=seed)
                    ts.append(time.perf_counter() - a)
                for s in range(slots):
                    assert ctx.wait(s)
                ts.sort()
                print("n=2^%d profiling=%d rep %d: enqueue ms min %.3f median %.3f max %.3f first %.3f" % (
                    n.bit_length() - 1, prof, rep, 1e3 * ts[0], 1e3 * ts[len(ts) // 2], 1e3 * ts[-1], 1e3 * ts[0]),
                    flush=True)
        ctx.set_profiling(False)


if __name__ == "__main__":
    main()
