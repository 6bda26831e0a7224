"""Fiat-Shamir / powers-of-r randomisers on the GPU vs the oracle.

The GPU derives r from a parallel Merkle transcript (csrc/fs.hpp); the spec restates it in
oracle/pyspec/kzg.py (fs_challenge) and tests/fsref.py (byte level, hashlib).  The combined
points A, B of r_i = r^i batches are checked bit-exactly against the C oracle's powers mode.
"""
import hashlib

import pytest

pytestmark = pytest.mark.gpu

from fsref import fs_challenge_bytes  # noqa: E402
from oracle import oracle as O  # noqa: E402  (checker only)
from oracle.pyspec import curves as pc  # noqa: E402
from oracle.pyspec import kzg as pk  # noqa: E402

CURVES = ["bls12_381", "bn254"]


def h(x):
    return bytes.fromhex(x)


@pytest.fixture(scope="module")
def ctx():
    import kzgmi
    c = kzgmi.Context(0, 2)
    yield c
    c.close()


def _dev(b):
    import torch
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()


def _host(t):
    return t.cpu().numpy().tobytes()


def _gen(ctx, curve, n, tau, tag):
    import torch
    g1b = 2 * pc.CURVES[curve].fp_bytes
    Cm = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    P = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    z = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    y = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.gen_tuples(curve, tau, hashlib.sha256(tag).digest(), n, Cm, z, y, P)
    return Cm, z, y, P


@pytest.mark.parametrize("curve", CURVES)
def test_fs_golden(ctx, curve, golden):
    C = pc.CURVES[curve]
    for n in ([4, 16, 256] if curve == "bls12_381" else [4, 16, 64]):
        g = golden("%s_batch_n%d.json" % (curve, n))
        cm, pf, zb, yb = h(g["commitments"]), h(g["proofs"]), h(g["zs"]), h(g["ys"])
        r = fs_challenge_bytes(curve, cm, zb, yb, pf, n)
        assert ctx.fs_challenge(curve, _dev(cm), _dev(zb), _dev(yb), _dev(pf), n) == r
        cc, pc_ = O.g1_compress(curve, cm, n), O.g1_compress(curve, pf, n)
        assert ctx.fs_challenge(curve, _dev(cc), _dev(zb), _dev(yb), _dev(pc_), n, compressed=True) == r
        srs = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]))
        # Fiat-Shamir mode = the seeded 127-bit randomisers with seed = be32(r)
        ok, A, B = O.batch_verify(curve, cm, zb, yb, pf, n, h(g["g2"]), h(g["tau_g2"]), r.to_bytes(32, "big"),
                                  want_ab=True)
        assert ok is True
        assert ctx.batch_verify(srs, cm, zb, yb, pf, fiat_shamir=True) is True
        assert ctx.last_combination(curve) == (A, B)
        assert ctx.batch_verify(srs, cc, zb, yb, pc_, fiat_shamir=True, compressed=True, subgroup_check=True) is True
        assert ctx.last_combination(curve) == (A, B)
        # powers mode with the same r: r_i = r^i
        okp, Ap, Bp = O.batch_verify_powers(curve, cm, zb, yb, pf, n, h(g["g2"]), h(g["tau_g2"]), r)
        assert okp is True
        assert ctx.batch_verify(srs, cm, zb, yb, pf, challenge=r) is True
        assert ctx.last_combination(curve) == (Ap, Bp)
        yb2 = bytearray(yb)
        yb2[32 * (n - 1) + 31] ^= 1
        assert ctx.batch_verify(srs, cm, zb, bytes(yb2), pf, fiat_shamir=True) is False


@pytest.mark.parametrize("curve", CURVES)
def test_powers_arbitrary_r(ctx, curve, golden):
    import kzgmi
    C = pc.CURVES[curve]
    g = golden("%s_batch_n16.json" % curve)
    cm, pf, zb, yb = h(g["commitments"]), h(g["proofs"]), h(g["zs"]), h(g["ys"])
    srs = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]))
    for r in [1, 2, C.r - 1, 0x1234567890ABCDEF << 100]:
        ok, A, B = O.batch_verify_powers(curve, cm, zb, yb, pf, 16, h(g["g2"]), h(g["tau_g2"]), r)
        assert ctx.batch_verify(srs, cm, zb, yb, pf, challenge=r) is ok
        assert ctx.last_combination(curve) == (A, B)
    with pytest.raises(kzgmi.KzgmiError) as e:  # r >= modulus is non-canonical
        ctx.batch_verify(srs, cm, zb, yb, pf, challenge=C.r)
    assert e.value.code == -4


@pytest.mark.parametrize("curve,n", [("bls12_381", 3 * 4096 + 100), ("bn254", 9000)])
def test_fs_multichunk_and_shards(ctx, curve, n):
    """Several 4096-leaf subtrees (non-power-of-two n); 4096-aligned shards: gathered subtree
    roots give the same r; shard partials seeded with be32(r) (the Fiat-Shamir randomisers) and
    with r^(offset + i) (powers mode) each combine to the whole."""
    import torch
    C = pc.CURVES[curve]
    tau = 31337
    Cm, z, y, P = _gen(ctx, curve, n, tau, b"fs-" + curve.encode())
    hb = [_host(t) for t in (Cm, z, y, P)]
    r = fs_challenge_bytes(curve, hb[0], hb[1], hb[2], hb[3], n)
    assert ctx.fs_challenge(curve, Cm, z, y, P, n) == r
    g1b = 2 * C.fp_bytes
    cut = 2 * 4096
    nch = (n + 4095) // 4096
    dg = torch.empty(nch * 32, dtype=torch.uint8, device="cuda")
    ctx.fs_chunk_digests(curve, Cm[:cut * g1b], z[:cut * 32], y[:cut * 32], P[:cut * g1b], cut, 0, dg[:64])
    ctx.fs_chunk_digests(curve, Cm[cut * g1b:], z[cut * 32:], y[cut * 32:], P[cut * g1b:], n - cut, cut, dg[64:])
    assert ctx.fs_challenge_from_digests(curve, dg, nch, n) == r
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    pb = ctx.partial_bytes(curve)
    parts = torch.empty(2 * 2 * pb, dtype=torch.uint8, device="cuda")
    for kw in ({"seed": r.to_bytes(32, "big")}, {"seed": None, "challenge": r}):
        for k, (lo, hi) in enumerate([(0, cut), (cut, n)]):
            ctx.batch_partial_async(srs, 0, Cm[lo * g1b:hi * g1b], z[lo * 32:hi * 32], y[lo * 32:hi * 32],
                                    P[lo * g1b:hi * g1b], hi - lo, lo, out=parts[2 * k * pb:2 * (k + 1) * pb], **kw)
            assert ctx.wait(0) is True
        assert ctx.batch_combine(srs, parts, 2) is True
    assert ctx.batch_verify(srs, Cm, z, y, P, n=n, fiat_shamir=True) is True
    ok, A, B = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, r.to_bytes(32, "big"), want_ab=True)
    assert ok is True and ctx.last_combination(curve) == (A, B)


@pytest.mark.slow
def test_fs_full_size(ctx):
    """cfg 3 size with Fiat-Shamir randomisers: r, A, B bit-exact; negative run rejected."""
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n, tau = 1 << 20, 0x5EED
    Cm, z, y, P = _gen(ctx, curve, n, tau, b"fs-full")
    hb = [_host(t) for t in (Cm, z, y, P)]
    r = fs_challenge_bytes(curve, hb[0], hb[1], hb[2], hb[3], n)
    assert ctx.fs_challenge(curve, Cm, z, y, P, n) == r
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    assert ctx.batch_verify(srs, Cm, z, y, P, n=n, fiat_shamir=True) is True
    ok, A, B = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, r.to_bytes(32, "big"), want_ab=True)
    assert ok is True and ctx.last_combination(curve) == (A, B)
    y[5] ^= 1
    assert ctx.batch_verify(srs, Cm, z, y, P, n=n, fiat_shamir=True) is False


def test_sharded_fs_rccl_world1(ctx):
    """kzgmi.distributed Fiat-Shamir flow on the device over a world-1 RCCL group."""
    import os
    import socket
    import torch
    import torch.distributed as dist
    from kzgmi.distributed import fs_challenge_sharded, sharded_batch_verify
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n, tau = 5000, 4711
    Cm, z, y, P = _gen(ctx, curve, n, tau, b"fs-rccl")
    g2 = pk.g2_to_bytes(C.g2, C)
    srs = ctx.load_srs(curve, g2, O.g2_mul(curve, g2, tau))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    created = not dist.is_initialized()
    if created:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        r = fs_challenge_sharded(ctx, curve, Cm, z, y, P, n, 0, n)
        assert r == ctx.fs_challenge(curve, Cm, z, y, P, n)
        assert sharded_batch_verify(ctx, srs, Cm, z, y, P, n, 0, None, fiat_shamir=True, n_total=n) is True
        y[7] ^= 1
        assert sharded_batch_verify(ctx, srs, Cm, z, y, P, n, 0, None, fiat_shamir=True, n_total=n) is False
    finally:
        if created:
            dist.destroy_process_group()
