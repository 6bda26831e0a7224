"""GLV endomorphism on the GPU: bit-exact vs the C oracle.

GLV regroups the same sum (k P = k0 P + k1 phi(P)) for P in G1, so every result must equal
the oracle's plain double-and-add MSM / batch combination exactly, with GLV on or off.  On
BLS12-381 (cofactor > 1) the split is used only for points declared or checked to be in G1
(kzgmi_set_trusted_g1, KZGMI_FLAG_TRUSTED_G1 / KZGMI_FLAG_SUBGROUP_CHECK); a non-member point
in an undeclared MSM must still give the plain result.  Scalars come from
oracle/pyspec/glv.edge_scalars (0, 1, r - 1, +-lambda, Babai rounding boundaries, the
largest halves of a random search); the decomposition itself is pinned on the CPU in
tests/test_glv.py.
"""
import hashlib
import random

import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)
from oracle.pyspec import curves as pc  # noqa: E402
from oracle.pyspec import glv  # noqa: E402
from oracle.pyspec import kzg as pk  # noqa: E402

CURVES = ["bls12_381", "bn254"]


@pytest.fixture(scope="module")
def ctx():
    import kzgmi
    c = kzgmi.Context(0, 2)
    c.set_trusted_g1(True)
    yield c
    c.set_glv(msm=True, batch=True)
    c.close()


def _points(curve, n, seed):
    C = pc.CURVES[curve]
    rng = random.Random(seed)
    return O.g1_mul_gen(curve, b"".join(pk.fr_to_bytes(rng.randrange(C.r)) for _ in range(n)), n)


@pytest.mark.parametrize("curve", CURVES)
def test_msm_edge_scalars_glv_on_off(ctx, curve):
    C = pc.CURVES[curve]
    ks = glv.edge_scalars(curve, 96)
    n = len(ks)
    pts = bytearray(_points(curve, n, 5))
    g1b = 2 * C.fp_bytes
    pts[3 * g1b:4 * g1b] = pts[7 * g1b:8 * g1b]          # a duplicated point
    inf = bytearray(g1b)
    if curve == "bls12_381":
        inf[0] = 0x40
    pts[11 * g1b:12 * g1b] = inf                           # the point at infinity
    pts = bytes(pts)
    sc = b"".join(pk.fr_to_bytes(k) for k in ks)
    want = O.msm_g1(curve, pts, sc, n)
    for on in (True, False):
        ctx.set_glv(msm=on)
        assert ctx.msm_g1(curve, pts, sc) == want, on
        for m in (1, 2, 13):                               # prefixes: tiny MSMs
            assert ctx.msm_g1(curve, pts[:m * g1b], sc[:m * 32]) == O.msm_g1(curve, pts[:m * g1b], sc[:m * 32], m)
    ctx.set_glv(msm=True)


@pytest.mark.parametrize("curve", CURVES)
def test_msm_random_glv(ctx, curve):
    C = pc.CURVES[curve]
    rng = random.Random(19)
    for n in [1, 3, 4097, 20000]:
        pts = _points(curve, n, n)
        sc = b"".join(pk.fr_to_bytes(rng.randrange(C.r)) for _ in range(n))
        assert ctx.msm_g1(curve, pts, sc) == O.msm_g1(curve, pts, sc, n), n


def test_msm_non_subgroup_point_untrusted(ctx):
    """BLS12-381 MSM over a point outside G1: without the trusted-G1 declaration the plain
    (non-GLV) result, bit-exact vs the oracle; the declaration is per context."""
    from pointcases import non_subgroup_points
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n = 40
    pts = bytearray(_points(curve, n, 8))
    pts[96 * 3:96 * 4] = pk.g1_to_bytes(non_subgroup_points(1, seed=4)[0], C)
    pts = bytes(pts)
    sc = b"".join(pk.fr_to_bytes(k) for k in glv.edge_scalars(curve, n)[:n])
    try:
        ctx.set_trusted_g1(False)
        assert ctx.msm_g1(curve, pts, sc) == O.msm_g1(curve, pts, sc, n)
    finally:
        ctx.set_trusted_g1(True)


def _batch(ctx, torch, curve, n, tau, seed):
    C = pc.CURVES[curve]
    g1b = 2 * C.fp_bytes
    Cm = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    P = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    z = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    y = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.gen_tuples(curve, tau, seed, n, Cm, z, y, P)
    return Cm, z, y, P


@pytest.mark.parametrize("curve", CURVES)
def test_batch_verify_glv_modes(ctx, curve):
    """Batch verification with the GLV split of s_i, t (and r^i): A, B bit-exact vs the oracle
    in the random-randomiser and powers-of-r modes; corrupted batches rejected."""
    import torch
    C = pc.CURVES[curve]
    n, tau = 3001, 0xABCDEF123
    seed = hashlib.sha256(b"glv-batch").digest()
    Cm, z, y, P = _batch(ctx, torch, curve, n, tau, seed)
    g2 = pk.g2_to_bytes(C.g2, C)
    tg2 = O.g2_mul(curve, g2, tau)
    srs = ctx.load_srs(curve, g2, tg2)
    hb = [t.cpu().numpy().tobytes() for t in (Cm, z, y, P)]
    vseed = hashlib.sha256(b"glv-verify").digest()
    ok_o, Ao, Bo = O.batch_verify(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, vseed, want_ab=True)
    r = random.Random(4).randrange(C.r)
    okp, Ap, Bp = O.batch_verify_powers(curve, hb[0], hb[1], hb[2], hb[3], n, g2, tg2, r)
    ybad = y.clone()
    ybad[32 * 2000 + 31] ^= 1
    try:
        for on in (True, False):
            ctx.set_glv(msm=True, batch=on)
            for tr in (True, False):
                assert ctx.batch_verify(srs, Cm, z, y, P, seed=vseed, n=n, trusted_g1=tr) is True
                assert ctx.last_combination(curve) == (Ao, Bo), (on, tr)
                assert ctx.batch_verify(srs, Cm, z, y, P, n=n, challenge=r, trusted_g1=tr) is True
                assert ctx.last_combination(curve) == (Ap, Bp), (on, tr)
                assert ctx.batch_verify(srs, Cm, z, y, P, n=n, fiat_shamir=True, trusted_g1=tr) is True
                assert ctx.batch_verify(srs, Cm, z, ybad, P, seed=vseed, n=n, trusted_g1=tr) is False
                assert ctx.batch_verify(srs, Cm, z, ybad, P, n=n, fiat_shamir=True, trusted_g1=tr) is False
    finally:
        ctx.set_glv(msm=True, batch=True)
    assert ok_o and okp


def test_set_glv_rejects_in_flight(ctx):
    import kzgmi
    import torch
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n = 300
    pts = torch.frombuffer(bytearray(_points(curve, n, 1)), dtype=torch.uint8).cuda()
    sc = torch.frombuffer(bytearray(b"".join(pk.fr_to_bytes(i * 977 + 5) for i in range(n))), dtype=torch.uint8).cuda()
    ctx.msm_g1_async(curve, 1, pts, sc, n)
    with pytest.raises(kzgmi.KzgmiError):
        ctx.set_glv(msm=False)
    got = ctx.msm_wait(1)
    assert got == O.msm_g1(curve, pts.cpu().numpy().tobytes(), sc.cpu().numpy().tobytes(), n)
    del C
