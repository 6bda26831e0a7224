"""Compressed G1 inputs + subgroup checks on the GPU vs the oracle.

Bar: bit-exact.  The GPU decompresses with a (p+1)/4 square root and tests subgroup
membership with the endomorphism identity phi(P) = [-x^2]P; the oracle decompresses
independently and checks membership by definition ([r]P == O), so agreement pins both.
"""
import hashlib

import pytest

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)
from oracle.pyspec import curves as pc  # noqa: E402
from oracle.pyspec import kzg as pk  # noqa: E402
from pointcases import invalid_compressed, subgroup_cases  # noqa: E402

CURVES = ["bls12_381", "bn254"]


def h(x):
    return bytes.fromhex(x)


@pytest.fixture(scope="module")
def ctx():
    import kzgmi
    c = kzgmi.Context(0, 1)
    yield c
    c.close()


def _dev(b):
    import torch
    return torch.frombuffer(bytearray(b), dtype=torch.uint8).cuda()


@pytest.mark.parametrize("curve", CURVES)
@pytest.mark.parametrize("n", [4, 16, 256])
def test_compressed_golden_batch(ctx, curve, n, golden):
    """Golden batches in compressed form: same verdict and same A, B as the uncompressed run."""
    if curve == "bn254" and n == 256:
        n = 64
    C = pc.CURVES[curve]
    g = golden("%s_batch_n%d.json" % (curve, n))
    srs = ctx.load_srs(curve, h(g["g2"]), h(g["tau_g2"]))
    Cm, P = h(g["commitments"]), h(g["proofs"])
    cc, pc_ = O.g1_compress(curve, Cm, n), O.g1_compress(curve, P, n)
    for flags in [dict(compressed=True), dict(compressed=True, subgroup_check=True)]:
        assert ctx.batch_verify(srs, cc, h(g["zs"]), h(g["ys"]), pc_, seed=h(g["seed"]), **flags) is True
        A, B = ctx.last_combination(curve)
        assert A == h(g["valid"]["A"]) and B == h(g["valid"]["B"])
        # device-resident form
        assert ctx.batch_verify(srs, _dev(cc), _dev(h(g["zs"])), _dev(h(g["ys"])), _dev(pc_), seed=h(g["seed"]),
                                n=n, **flags) is True
    # uncompressed + subgroup check
    assert ctx.batch_verify(srs, Cm, h(g["zs"]), h(g["ys"]), P, seed=h(g["seed"]), subgroup_check=True) is True
    ys = bytearray(h(g["ys"]))
    ys[31] ^= 1
    assert ctx.batch_verify(srs, cc, h(g["zs"]), bytes(ys), pc_, seed=h(g["seed"]), compressed=True) is False


@pytest.mark.parametrize("curve", CURVES)
def test_gpu_compress_matches_oracle(ctx, curve):
    import random
    import torch
    C = pc.CURVES[curve]
    n = 3000
    rng = random.Random(8)
    pts = O.g1_mul_gen(curve, b"".join(pk.fr_to_bytes(rng.randrange(C.r)) for _ in range(n)), n)
    pts += pk.g1_to_bytes(None, C)  # infinity
    n += 1
    out = torch.empty(n * C.fp_bytes, dtype=torch.uint8, device="cuda")
    ctx.g1_compress(curve, _dev(pts), n, out)
    comp = out.cpu().numpy().tobytes()
    assert comp == O.g1_compress(curve, pts, n)
    ctx.g1_validate(curve, out, n, compressed=True)
    ctx.g1_validate(curve, out, n, compressed=True, subgroup_check=True)


@pytest.mark.parametrize("curve", CURVES)
def test_invalid_compressed_errors(ctx, curve):
    import kzgmi
    C = pc.CURVES[curve]
    good = pk.g1_to_bytes_compressed(C.g1, C)
    for enc, want in invalid_compressed(C):
        with pytest.raises(kzgmi.KzgmiError) as e:
            ctx.g1_validate(curve, _dev(good + enc + good), 3, compressed=True)
        assert e.value.code == want, enc.hex()
        assert O.g1_decompress(curve, enc, 1)[0] == want


def test_subgroup_check_cases(ctx):
    """Per point: GPU endomorphism test == oracle definition, incl. small-order components."""
    import kzgmi
    C = pc.BLS12_381
    for P, member in subgroup_cases():
        enc = pk.g1_to_bytes(P, C)
        assert O.g1_subgroup_check("bls12_381", enc, 1) is member
        ctx.g1_validate("bls12_381", _dev(enc), 1)  # on the curve either way
        if member:
            ctx.g1_validate("bls12_381", _dev(enc), 1, subgroup_check=True)
            ctx.g1_validate("bls12_381", _dev(pk.g1_to_bytes_compressed(P, C)), 1, compressed=True,
                            subgroup_check=True)
        else:
            for b, comp in [(enc, False), (pk.g1_to_bytes_compressed(P, C), True)]:
                with pytest.raises(kzgmi.KzgmiError) as e:
                    ctx.g1_validate("bls12_381", _dev(b), 1, compressed=comp, subgroup_check=True)
                assert e.value.code == kzgmi.ERR_NOT_IN_SUBGROUP


def test_batch_with_non_subgroup_point(ctx, golden):
    """A proof outside G1: rejected with KZGMI_ERR_NOT_IN_SUBGROUP under the flag; without it
    the batch is merely checked (the verdict is False since the tuple is not an opening)."""
    import kzgmi
    from pointcases import non_subgroup_points
    C = pc.BLS12_381
    g = golden("bls12_381_batch_n16.json")
    srs = ctx.load_srs("bls12_381", h(g["g2"]), h(g["tau_g2"]))
    P = bytearray(h(g["proofs"]))
    P[96 * 5:96 * 6] = pk.g1_to_bytes(non_subgroup_points(1, seed=9)[0], C)
    args = (srs, h(g["commitments"]), h(g["zs"]), h(g["ys"]), bytes(P))
    with pytest.raises(kzgmi.KzgmiError) as e:
        ctx.batch_verify(*args, seed=h(g["seed"]), subgroup_check=True)
    assert e.value.code == kzgmi.ERR_NOT_IN_SUBGROUP
    assert ctx.batch_verify(*args, seed=h(g["seed"])) is False
    ok, A, B = O.batch_verify("bls12_381", h(g["commitments"]), h(g["zs"]), h(g["ys"]), bytes(P), 16, h(g["g2"]),
                              h(g["tau_g2"]), h(g["seed"]), want_ab=True)
    assert ok is False and ctx.last_combination("bls12_381") == (A, B)


@pytest.mark.slow
def test_full_size_compressed_subgroup(ctx):
    """cfg 3 size (n = 2^20) with compressed inputs + subgroup checks: same A, B as uncompressed."""
    import torch
    curve = "bls12_381"
    C = pc.CURVES[curve]
    n, tau = 1 << 20, 0xABCDEF
    g1b = 2 * C.fp_bytes
    Cm = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    P = torch.empty(n * g1b, dtype=torch.uint8, device="cuda")
    z = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    y = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    ctx.gen_tuples(curve, tau, hashlib.sha256(b"cmp").digest(), n, Cm, z, y, P)
    g2 = pk.g2_to_bytes(C.g2, C)
    srs = ctx.load_srs(curve, g2, O.g2_mul(curve, g2, tau))
    seed = hashlib.sha256(b"cmp-verify").digest()
    assert ctx.batch_verify(srs, Cm, z, y, P, seed=seed, n=n) is True
    ab = ctx.last_combination(curve)
    cc = torch.empty(n * C.fp_bytes, dtype=torch.uint8, device="cuda")
    pp = torch.empty(n * C.fp_bytes, dtype=torch.uint8, device="cuda")
    ctx.g1_compress(curve, Cm, n, cc)
    ctx.g1_compress(curve, P, n, pp)
    assert ctx.batch_verify(srs, cc, z, y, pp, seed=seed, n=n, compressed=True, subgroup_check=True) is True
    assert ctx.last_combination(curve) == ab
