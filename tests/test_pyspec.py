"""Known-answer checks pinning the Python spec (SURVEY.md Appendix A constants and identities).

The reference has no vectors (LICENSE only), so the spec is pinned by public curve facts:
primality of p and r, curve/twist membership and order of the generators, the polynomial
parametrisations, and the final-exponentiation decompositions the fast paths rely on.
"""
import pytest
import sympy

from oracle.pyspec import curves as pc
from oracle.pyspec import kzg as pk

X_BLS = -0xD201000000010000


def test_bls_constants():
    C = pc.BLS12_381
    assert sympy.isprime(C.p) and sympy.isprime(C.r)
    x = X_BLS
    assert C.r == x ** 4 - x ** 2 + 1
    assert C.p == (x - 1) ** 2 * (x ** 4 - x ** 2 + 1) // 3 + x
    assert C.p.bit_length() == 381 and C.r.bit_length() == 255


def test_bn_constants():
    C = pc.BN254
    u = pc.BN254_U
    assert sympy.isprime(C.p) and sympy.isprime(C.r)
    assert C.p == 36 * u ** 4 + 36 * u ** 3 + 24 * u ** 2 + 6 * u + 1
    assert C.r == 36 * u ** 4 + 36 * u ** 3 + 18 * u ** 2 + 6 * u + 1


@pytest.mark.parametrize("C", [pc.BLS12_381, pc.BN254])
def test_generators(C):
    assert pc.g1_on_curve(C.g1, C)
    assert pc.g2_on_curve(C.g2, C)
    assert pc.g1_mul(C.g1, C.r, C) is None
    assert pc.g2_mul(C.g2, C.r, C) is None
    # encodings round-trip
    assert pk.g1_from_bytes(pk.g1_to_bytes(C.g1, C), C) == C.g1
    assert pk.g2_from_bytes(pk.g2_to_bytes(C.g2, C), C) == C.g2
    assert pk.g1_from_bytes(pk.g1_to_bytes(None, C), C) is None


def test_bls_g1_generator_small_y():
    C = pc.BLS12_381
    assert C.g1[1] <= (C.p - 1) // 2


def test_final_exponent_decompositions():
    C = pc.BLS12_381
    p, r, x = C.p, C.r, X_BLS
    lam = (p ** 4 - p ** 2 + 1) // r
    assert (p ** 4 - p ** 2 + 1) % r == 0
    assert 3 * lam == (x - 1) ** 2 * (x + p) * (x ** 2 + p ** 2 - 1) + 3
    C = pc.BN254
    p, r, u = C.p, C.r, pc.BN254_U
    lam = (p ** 4 - p ** 2 + 1) // r
    l3, l2 = 1, 6 * u * u + 1
    l1 = -36 * u ** 3 - 18 * u ** 2 - 12 * u + 1
    l0 = -36 * u ** 3 - 30 * u ** 2 - 18 * u - 2
    assert lam == l0 + l1 * p + l2 * p ** 2 + l3 * p ** 3


def test_randomizer_rule():
    seed = bytes(range(32))
    r = [pk.randomizer(seed, i) for i in range(64)]
    assert all(0 < v < 2 ** 127 for v in r)
    assert len(set(r)) == 64


def test_encoding_rejections():
    C = pc.BLS12_381
    b = bytearray(pk.g1_to_bytes(C.g1, C))
    b[0] |= 0x80
    with pytest.raises(ValueError):
        pk.g1_from_bytes(bytes(b), C)
    with pytest.raises(ValueError):
        pk.fr_from_bytes(C.r.to_bytes(32, "big"), C)
