"""Parity at BASELINE.json's full sizes, HIP path vs the C oracle.

The oracle (OpenMP, the GPU box's host cores) finishes these in seconds, so the check is the
strongest one available: bit-exact combined points A and B (or the MSM result) plus the
verdict, and the size-independent property that one corrupted evaluation flips the verdict.
Inputs are generated on the device (kzgmi_gen_tuples / kzgmi_gen_g1; their host restatement
is checked in test_gpu_parity.py) and copied to the host for the oracle.
"""
import hashlib

import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

from oracle import oracle as O  # noqa: E402  (checker only)
from oracle.pyspec import curves as pc  # noqa: E402
from oracle.pyspec import kzg as pk  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    import kzgmi
    c = kzgmi.Context(0, 1)
    yield c
    c.close()


def _host(t):
    return t.cpu().numpy().tobytes()


def _gen_batch(ctx, curve, n, tau, seed):
    import torch
    g1b = 2 * pc.CURVES[curve].fp_bytes
    Cm = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    P = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    z = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    y = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.gen_tuples(curve, tau, seed, n, Cm, z, y, P)
    return Cm, z, y, P


@pytest.mark.parametrize("curve,log_n,seed_no", [("bls12_381", 20, 4), ("bn254", 22, 5)])
def test_full_batch_vs_oracle(ctx, curve, log_n, seed_no):
    """cfg 3 (BLS12-381, n = 2^20) and cfg 5 (BN254, n = 2^22): A, B, verdict bit-exact."""
    C = pc.CURVES[curve]
    n, tau = 1 << log_n, 0xC0FFEE + seed_no
    Cm, z, y, P = _gen_batch(ctx, curve, n, tau, hashlib.sha256(b"cfg%d" % seed_no).digest())
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    vseed = hashlib.sha256(b"cfg%d-verify" % seed_no).digest()
    assert ctx.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n) is True
    A, B = ctx.last_combination(curve)
    hb = [_host(t) for t in (Cm, z, y, P)]
    ok, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, vseed, want_ab=True)
    assert ok is True and A == Ao and B == Bo
    # negative run (cfg 3 "plus one negative run with a corrupted y"): last tuple's y
    y[32 * (n - 1) + 31] ^= 1
    assert ctx.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n) is False


def test_full_msm_vs_oracle(ctx):
    """cfg 2: BLS12-381 MSM, n = 2^20, points k_i G1 with k_i uniform in Fr, uniform scalars."""
    import random
    import torch
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n = 1 << 20
    rng = random.Random(2)
    ks = b"".join(pk.fr_to_bytes(rng.randrange(C.r)) for _ in range(n))
    rng = random.Random(3)
    sc = b"".join(pk.fr_to_bytes(rng.randrange(C.r)) for _ in range(n))
    d_k = torch.frombuffer(bytearray(ks), dtype=torch.uint8).cuda()
    pts = torch.empty(n * 2 * C.fp_bytes, dtype=torch.uint8, device="cuda")
    ctx.gen_g1(curve, d_k, n, pts)
    d_sc = torch.frombuffer(bytearray(sc), dtype=torch.uint8).cuda()
    got = ctx.msm_g1(curve, pts, d_sc, n=n)
    assert got == O.msm_g1(curve, _host(pts), sc, n)


def test_sharded_msm_cfg4(ctx):
    """cfg 4 at its real size on one device: G1 MSM n = 2^24 as 8 shards of 2^21 points
    (msm_partial, one per would-be GPU) + msm_combine, checked through the discrete-log
    identity sum_i s_i [k_i] G1 = [sum_i k_i s_i mod r] G1: points k_i G1 from
    the GPU generator (its restatement is checked in test_gpu_parity.py), the dot product
    and the final scalar multiple on the oracle.  Every shard's partial is checked the same
    way."""
    import numpy as np
    import torch
    curve = "bls12_381"
    C = pc.CURVES[curve]
    shards, m = 8, 1 << 21
    n = shards * m
    rs = np.random.default_rng(4)
    ks = rs.integers(0, 256, size=(n, 32), dtype=np.uint8)
    ks[:, 0] &= 0x3F                      # < 2^254: canonical Fr (r > 2^254)
    sc = rs.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sc[:, 0] &= 0x3F
    g1b = 2 * C.fp_bytes
    pb = ctx.partial_bytes(curve)
    pts = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    d_k = torch.from_numpy(ks.reshape(-1)).cuda()
    ctx.gen_g1(curve, d_k, n, pts)
    del d_k
    d_sc = torch.from_numpy(sc.reshape(-1)).cuda()
    parts = torch.empty(shards * pb, dtype=torch.uint8, device="cuda")
    for k in range(shards):
        ctx.msm_partial(curve, pts[k * m * g1b:(k + 1) * m * g1b], d_sc[k * m * 32:(k + 1) * m * 32], m,
                        parts[k * pb:(k + 1) * pb])
    got = ctx.msm_combine(curve, parts, shards)
    kb, sb = ks.tobytes(), sc.tobytes()
    want = O.g1_mul_gen(curve, pk.fr_to_bytes(O.fr_dot(curve, kb, sb, n)), 1)
    assert got == want
    enc = ctx.partial_encode(curve, parts, shards)
    for k in (0, shards - 1):
        lo, hi = k * m * 32, (k + 1) * m * 32
        assert enc[k] == O.g1_mul_gen(curve, pk.fr_to_bytes(O.fr_dot(curve, kb[lo:hi], sb[lo:hi], m)), 1), k


def test_sharded_batch_cfg5_bn254(ctx):
    """cfg 5 shape on one device: BN254 batch of 2^22 tuples as 8 shards of 2^19 (global index
    offsets, one per would-be GPU): every shard's A_k, B_k equals the oracle's combination of
    the same range, the combined A, B equal the oracle's unsharded batch, the verdict is True,
    and a corrupted y in shard 5 flips it."""
    import torch
    curve = "bn254"
    C = pc.CURVES[curve]
    shards, m = 8, 1 << 19
    n, tau = shards * m, 0xC0FFEE + 55
    Cm, z, y, P = _gen_batch(ctx, curve, n, tau, hashlib.sha256(b"cfg5-sharded").digest())
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    seed = hashlib.sha256(b"cfg5-sharded-verify").digest()
    g1b = 2 * C.fp_bytes
    pb = ctx.partial_bytes(curve)
    hb = [_host(t) for t in (Cm, z, y, P)]
    parts = torch.empty(shards * 2 * pb, dtype=torch.uint8, device="cuda")

    def run(yt):
        for k in range(shards):
            lo, hi = k * m, (k + 1) * m
            ctx.batch_partial(srs, Cm[lo * g1b:hi * g1b], z[lo * 32:hi * 32], yt[lo * 32:hi * 32],
                              P[lo * g1b:hi * g1b], m, lo, seed, parts[k * 2 * pb:(k + 1) * 2 * pb])
        return ctx.batch_combine(srs, parts, shards)

    assert run(y) is True
    AB = ctx.last_combination(curve)
    enc = ctx.partial_encode(curve, parts, 2 * shards)
    for k in range(shards):
        lo, hi = k * m, (k + 1) * m
        want = O.batch_combination(curve, hb[0][lo * g1b:hi * g1b], hb[1][lo * 32:hi * 32], hb[2][lo * 32:hi * 32],
                                   hb[3][lo * g1b:hi * g1b], m, lo, g2, tg2, seed)
        assert (enc[2 * k], enc[2 * k + 1]) == want, k
    ok, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, seed, want_ab=True)
    assert ok is True and AB == (Ao, Bo)
    y2 = y.clone()
    y2[32 * (5 * m + 123) + 31] ^= 1
    assert run(y2) is False


@pytest.mark.parametrize("curve,n,trusted", [("bls12_381", 300007, False), ("bls12_381", 262143, True),
                                             ("bn254", 524289, False),
                                             # 2^15 < n <= 2^17: 13-bit windows (api.hip call_wbits)
                                             ("bls12_381", 100003, False), ("bls12_381", 70001, True),
                                             ("bn254", 90001, False)])
def test_ragged_batch_vs_oracle(ctx, curve, n, trusted):
    """Non-power-of-two batches: the accumulation's per-thread runs, the last partial round and
    the bucket pieces joined by k_fixup do not divide evenly.  A, B and the verdict bit-exact vs
    the oracle (with and without the GLV split that trusted_g1 enables), then one corrupted
    proof flips the verdict.  The mid sizes run the 13-bit window width."""
    C = pc.CURVES[curve]
    tau = 0xBADC0DE + n
    Cm, z, y, P = _gen_batch(ctx, curve, n, tau, hashlib.sha256(b"ragged%d" % n).digest())
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    vseed = hashlib.sha256(b"ragged-verify%d" % n).digest()
    assert ctx.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n, trusted_g1=trusted) is True
    A, B = ctx.last_combination(curve)
    hb = [_host(t) for t in (Cm, z, y, P)]
    ok, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, vseed, want_ab=True)
    assert ok is True and A == Ao and B == Bo
    # swap two proofs (both stay valid curve points): the check must fail
    g1b = 2 * C.fp_bytes
    P2 = P.clone()
    P2[:g1b] = P[(n - 1) * g1b:]
    P2[(n - 1) * g1b:] = P[:g1b]
    assert ctx.batch_verify(srs, Cm, z, y, P2, seed=vseed, n=n, trusted_g1=trusted) is False


@pytest.mark.parametrize("curve,n,trusted", [("bls12_381", 393213, False), ("bls12_381", 393213, True),
                                             ("bn254", 655361, False),
                                             # 2^16 < n <= 2^17: 13-bit windows (20; 10 with GLV)
                                             ("bls12_381", 100003, False), ("bls12_381", 120001, True),
                                             ("bn254", 131071, False)])
def test_ragged_msm_vs_oracle(ctx, curve, n, trusted):
    """Mid-size, non-power-of-two MSMs with uniform 255-bit scalars (16 windows; 8 with GLV on
    trusted BLS12-381 points; 20 and 10 for the 13-bit width of the smaller sizes): bit-exact vs
    the oracle."""
    import numpy as np
    import torch
    C = pc.CURVES[curve]
    rs = np.random.default_rng(n + trusted)
    # scalars < 2^253 < r, big-endian, uniform in their range
    ks = rs.integers(0, 256, size=(n, 32), dtype=np.uint8)
    ks[:, 0] &= 0x1F
    sc = rs.integers(0, 256, size=(n, 32), dtype=np.uint8)
    sc[:, 0] &= 0x1F
    d_k = torch.from_numpy(ks.reshape(-1).copy()).cuda()
    pts = torch.empty(n * 2 * C.fp_bytes, dtype=torch.uint8, device="cuda")
    ctx.gen_g1(curve, d_k, n, pts)
    d_sc = torch.from_numpy(sc.reshape(-1).copy()).cuda()
    ctx.set_trusted_g1(trusted)
    try:
        got = ctx.msm_g1(curve, pts, d_sc, n=n)
    finally:
        ctx.set_trusted_g1(False)
    assert got == O.msm_g1(curve, _host(pts), sc.tobytes(), n)


# the path switches of a batch call: the one-wave-per-term small path up to 4096 MSM terms (3n + 1
# for BLS12-381, 4n + 2 for BN254's GLV halves), 13-bit windows from 2^15 + 1 tuples, 16-bit
# windows and the 2^23-entry accumulation order depth above 2^17 (api.hip run_msm_core, call_wbits)
@pytest.mark.parametrize("curve,n", [("bls12_381", 1365), ("bls12_381", 1366), ("bls12_381", 32768),
                                     ("bls12_381", 32769), ("bls12_381", 131072), ("bls12_381", 131073),
                                     ("bn254", 1023), ("bn254", 1024), ("bn254", 32769)])
def test_batch_path_boundaries_vs_oracle(ctx, curve, n):
    """A, B and the verdict bit-exact vs the oracle on both sides of every size switch, then a
    corrupted y in the middle tuple flips the verdict."""
    C = pc.CURVES[curve]
    tau = 0xB0DA + n
    Cm, z, y, P = _gen_batch(ctx, curve, n, tau, hashlib.sha256(b"boundary%d" % n).digest())
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    vseed = hashlib.sha256(b"boundary-verify%d" % n).digest()
    assert ctx.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n) is True
    A, B = ctx.last_combination(curve)
    hb = [_host(t) for t in (Cm, z, y, P)]
    ok, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, vseed, want_ab=True)
    assert ok is True and A == Ao and B == Bo
    y[32 * (n // 2) + 31] ^= 1
    assert ctx.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n) is False


def _context_env(slots, **env):
    import os
    import kzgmi
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return kzgmi.Context(0, slots)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.mark.parametrize("curve,log_n", [("bls12_381", 17), ("bls12_381", 20), ("bn254", 17), ("bn254", 20)])
def test_split_accumulation_vs_oracle(curve, log_n):
    """The split accumulation (api.hip run_msm_core): MSM#0's bucket sets accumulate in one
    launch, then MSM#1's in a second one over the sorted range after them, while MSM#0's
    reduction and window combination run on the slot's side stream.  Forced on
    (KZGMI_SPLIT_ACC=1) and off (=0): A, B and the verdict bit-exact vs the oracle, a corrupted
    y flips the verdict; the split with the first launch's piece joins on the slot stream and the
    side stream at the slot's priority (KZGMI_SPLIT_SIDEFIX=0, KZGMI_SPLIT_SIDEPRIO=0); the
    other order (MSM#1's sets first, its tail on the side stream: KZGMI_SPLIT_REV=0); then the
    forced split pipelined on 4 slots with corrupted batches in flight between valid ones (each
    verdict checked)."""
    import torch
    C = pc.CURVES[curve]
    n, tau = 1 << log_n, 0x5B117 + log_n
    gen = _context_env(1)
    try:
        Cm, z, y, P = _gen_batch(gen, curve, n, tau, hashlib.sha256(b"split%d" % log_n).digest())
    finally:
        gen.close()
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    vseed = hashlib.sha256(b"split-verify%d" % log_n).digest()
    hb = [_host(t) for t in (Cm, z, y, P)]
    ok, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, vseed, want_ab=True)
    assert ok is True
    ybad = y.clone()
    ybad[32 * (n // 3) + 31] ^= 1
    for env in ({"KZGMI_SPLIT_ACC": "1"}, {"KZGMI_SPLIT_ACC": "0"}, {"KZGMI_SPLIT_ACC": "1", "KZGMI_SPLIT_SIDEFIX": "0", "KZGMI_SPLIT_SIDEPRIO": "0"},
                {"KZGMI_SPLIT_ACC": "1", "KZGMI_SPLIT_REV": "0"}, {"KZGMI_SPLIT_ACC": "1", "KZGMI_SPLIT_REV": "0", "KZGMI_SPLIT_SIDEFIX": "0"}):
        c = _context_env(1, **env)
        try:
            srs = c.load_srs(curve, g2, tg2)
            assert c.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n) is True, env
            assert c.last_combination(curve) == (Ao, Bo), env
            assert c.batch_verify(srs, Cm, z, ybad, P, seed=vseed, n=n) is False, env
            del srs
        finally:
            c.close()
    c = _context_env(4, KZGMI_SPLIT_ACC="1")
    try:
        srs = c.load_srs(curve, g2, tg2)
        want = [True, False, True, True, False, True]
        for i, w in enumerate(want):
            if i >= 4:
                assert c.wait(i % 4) is want[i - 4], i - 4
            c.batch_verify_async(srs, i % 4, Cm, z, y if w else ybad, P, n, seed=vseed)
        for i in range(len(want) - 4, len(want)):
            assert c.wait(i % 4) is want[i], i
        torch.cuda.synchronize()
        del srs
    finally:
        c.close()


@pytest.mark.parametrize("curve,n", [("bls12_381", 1 << 17), ("bn254", 100003), ("bls12_381", 300007)])
def test_sort_full_bins_fallback_vs_oracle(curve, n):
    """The sort launcher's set-table fallback (launch_msm.hip: a call with more bucket sets than
    the SetShift table holds sorts every set in full-width coarse bins instead of aborting),
    forced at every size with KZGMI_SORT_FULL_BINS=1: at 13-bit windows (2^17 tuples, where the
    top windows' per-set bin widths differ) and 16-bit ones, A, B and the verdict bit-exact vs
    the oracle, a corrupted y flips it."""
    C = pc.CURVES[curve]
    tau = 0xF0B1 + n
    c = _context_env(1, KZGMI_SORT_FULL_BINS="1")
    try:
        Cm, z, y, P = _gen_batch(c, curve, n, tau, hashlib.sha256(b"fullbins%d" % n).digest())
        g2 = pk.g2_to_bytes(C.g2, C)
        tg2 = O.g2_mul(curve, g2, tau)
        srs = c.load_srs(curve, g2, tg2)
        vseed = hashlib.sha256(b"fullbins-verify%d" % n).digest()
        assert c.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n) is True
        A, B = c.last_combination(curve)
        hb = [_host(t) for t in (Cm, z, y, P)]
        ok, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, vseed, want_ab=True)
        assert ok is True and A == Ao and B == Bo
        y[32 * (n // 2) + 31] ^= 1
        assert c.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n) is False
        del srs
    finally:
        c.close()
