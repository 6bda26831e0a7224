"""Prover-side commitments with a fixed SRS base vs the oracle.

commit(coeffs) must equal the plain MSM over [tau^i]_1 (C oracle) and [p(tau)]_1; an end-to-end
KZG round trip (commit p, commit the quotient (p - y) / (X - z) as the proof, batch-verify on
the GPU) closes the loop with the verifier.
"""
import random

import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)
from oracle.pyspec import curves as pc  # noqa: E402
from oracle.pyspec import kzg as pk  # noqa: E402

CURVES = ["bls12_381", "bn254"]
TAU = 0x1F2E3D4C5B6A7988


@pytest.fixture(scope="module")
def ctx():
    import kzgmi
    c = kzgmi.Context(0, 2)
    yield c
    c.close()


def _powers(curve, n, tau=TAU):
    C = pc.CURVES[curve]
    sc, x = [], 1
    for _ in range(n):
        sc.append(pk.fr_to_bytes(x))
        x = x * tau % C.r
    return O.g1_mul_gen(curve, b"".join(sc), n)


def _fr(vals):
    return b"".join(pk.fr_to_bytes(v) for v in vals)


def _quotient(coeffs, z, r):
    """(p(X) - p(z)) / (X - z) by synthetic division (coefficients low to high)."""
    n = len(coeffs)
    q = [0] * (n - 1)
    acc = 0
    for i in range(n - 1, 0, -1):
        acc = (acc * z + coeffs[i]) % r
        q[i - 1] = acc
    return q


@pytest.mark.parametrize("curve", CURVES)
def test_commit_matches_msm(ctx, curve):
    C = pc.CURVES[curve]
    n = 300
    powers = _powers(curve, n)
    ck = ctx.load_commit_key(curve, powers)
    rng = random.Random(5)
    g1b = 2 * C.fp_bytes
    for m in [1, 2, 17, 64, 299, 300]:
        cs = [rng.randrange(C.r) for _ in range(m)]
        got = ctx.commit(ck, _fr(cs))
        assert got == O.msm_g1(curve, powers[:m * g1b], _fr(cs), m), m
        p_tau = sum(c * pow(TAU, i, C.r) for i, c in enumerate(cs)) % C.r
        assert got == O.g1_mul_gen(curve, pk.fr_to_bytes(p_tau), 1), m
    # edge scalars: zeros, r - 1, a single nonzero high coefficient
    for cs in [[0] * 50, [C.r - 1] * 50, [0] * 49 + [7]]:
        assert ctx.commit(ck, _fr(cs)) == O.msm_g1(curve, powers[:50 * g1b], _fr(cs), 50)
    assert ctx.commit(ck, b"") == pk.g1_to_bytes(None, C)


@pytest.mark.parametrize("curve", CURVES)
def test_commit_async_slots(ctx, curve):
    """Pipelined commits: two in flight on slots 0/1, results in order, bit-exact."""
    import torch
    C = pc.CURVES[curve]
    n = 200
    powers = _powers(curve, n)
    ck = ctx.load_commit_key(curve, powers)
    rng = random.Random(8)
    g1b = 2 * C.fp_bytes
    css = [[rng.randrange(C.r) for _ in range(m)] for m in (200, 37, 0)]
    dev = [torch.frombuffer(bytearray(_fr(cs) or bytes(32)), dtype=torch.uint8).cuda() for cs in css]
    want = [O.msm_g1(curve, powers[:len(cs) * g1b], _fr(cs), len(cs)) for cs in css]
    ctx.commit_async(ck, 0, dev[0], len(css[0]))
    ctx.commit_async(ck, 1, dev[1], len(css[1]))
    assert ctx.msm_wait(1) == want[1]
    ctx.commit_async(ck, 1, dev[2], 0)
    assert ctx.msm_wait(0) == want[0]
    assert ctx.msm_wait(1) == want[2] == pk.g1_to_bytes(None, C)


@pytest.mark.parametrize("curve", CURVES)
def test_commit_errors(ctx, curve):
    import kzgmi
    C = pc.CURVES[curve]
    ck = ctx.load_commit_key(curve, _powers(curve, 8))
    with pytest.raises(kzgmi.KzgmiError) as e:
        ctx.commit(ck, _fr([1] * 9))  # more coefficients than powers
    assert e.value.code == -1
    with pytest.raises(kzgmi.KzgmiError) as e:
        ctx.commit(ck, pk.fr_to_bytes(1) + C.r.to_bytes(32, "big"))
    assert e.value.code == -4
    bad = bytearray(_powers(curve, 2))
    bad[2 * C.fp_bytes - 1] ^= 1
    with pytest.raises(kzgmi.KzgmiError) as e:
        ctx.load_commit_key(curve, bytes(bad))
    assert e.value.code == -3


@pytest.mark.parametrize("curve", CURVES)
def test_prover_verifier_round_trip(ctx, curve):
    """Commitments and opening proofs from the commit key, checked by the GPU batch verifier."""
    C = pc.CURVES[curve]
    deg = 128
    ck = ctx.load_commit_key(curve, _powers(curve, deg))
    g2 = pk.g2_to_bytes(C.g2, C)
    srs = ctx.load_srs(curve, g2, O.g2_mul(curve, g2, TAU))
    rng = random.Random(9)
    cm, zs, ys, pf = [], [], [], []
    for _ in range(8):
        coeffs = [rng.randrange(C.r) for _ in range(deg)]
        z = rng.randrange(C.r)
        y = sum(c * pow(z, i, C.r) for i, c in enumerate(coeffs)) % C.r
        cm.append(ctx.commit(ck, _fr(coeffs)))
        pf.append(ctx.commit(ck, _fr(_quotient(coeffs, z, C.r))))
        zs.append(pk.fr_to_bytes(z))
        ys.append(pk.fr_to_bytes(y))
    args = [b"".join(v) for v in (cm, zs, ys, pf)]
    assert ctx.batch_verify(srs, *args, seed=bytes(32)) is True
    ys[3] = pk.fr_to_bytes((int.from_bytes(ys[3], "big") + 1) % C.r)
    assert ctx.batch_verify(srs, args[0], args[1], b"".join(ys), args[3], seed=bytes(32)) is False


def test_commit_key_outliving_context(golden):
    import gc
    import kzgmi
    c = kzgmi.Context(0, 1)
    ck = c.load_commit_key("bn254", _powers("bn254", 4))
    c.close()
    del ck
    gc.collect()
    c2 = kzgmi.Context(0, 1)
    ck2 = c2.load_commit_key("bn254", _powers("bn254", 4))
    assert c2.commit(ck2, _fr([1, 0, 0, 0])) == O.g1_mul_gen("bn254", pk.fr_to_bytes(1), 1)
    c2.close()


@pytest.mark.slow
def test_commit_full_size(ctx):
    """n = 2^20 powers (cfg 2 size), random coefficients: bit-exact vs the oracle MSM."""
    import torch
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n = 1 << 20
    rng = random.Random(12)
    ks = _fr([rng.randrange(C.r) for _ in range(n)])
    d_k = torch.frombuffer(bytearray(ks), dtype=torch.uint8).cuda()
    pts = torch.empty(n * 2 * C.fp_bytes, dtype=torch.uint8, device="cuda")
    ctx.gen_g1(curve, d_k, n, pts)   # stand-in SRS: n independent random G1 points
    hp = pts.cpu().numpy().tobytes()
    ck = ctx.load_commit_key(curve, hp)
    cs = _fr([rng.randrange(C.r) for _ in range(n)])
    assert ctx.commit(ck, cs) == O.msm_g1(curve, hp, cs, n)
    d_cs = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    assert ctx.commit(ck, d_cs) == O.msm_g1(curve, hp, cs, n)
