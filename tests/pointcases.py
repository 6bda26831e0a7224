"""Deterministic G1 test cases for compressed inputs and subgroup checks.

Built from the Python spec (test infrastructure): on-curve BLS12-381 points outside the
order-r subgroup (random ones and ones of small order 3 and 11 -- the cofactor is
3 * 11^2 * 10177^2 * 859267^2 * 52437899^2), and invalid compressed encodings labelled with
the error class the boundary must return.
"""
import random

from oracle.pyspec import curves as pc
from oracle.pyspec import kzg as pk

BLS = pc.BLS12_381
X_ABS = 0xD201000000010000
COFACTOR = (X_ABS + 1) ** 2 // 3
ERR_ENCODING, ERR_NOT_ON_CURVE, ERR_NOT_IN_SUBGROUP = -2, -3, -7


def _random_curve_point(C, rng):
    while True:
        x = rng.randrange(C.p)
        rhs = (x * x * x + C.b) % C.p
        y = pow(rhs, (C.p + 1) // 4, C.p)
        if y * y % C.p == rhs:
            return (x, y if rng.random() < 0.5 else C.p - y)


def non_subgroup_points(count, seed=1):
    """Random on-curve BLS12-381 points outside G1 (checked by definition)."""
    rng = random.Random(seed)
    out = []
    while len(out) < count:
        P = _random_curve_point(BLS, rng)
        if not pc.g1_in_subgroup(P, BLS):
            out.append(P)
    return out


def small_order_point(ell, seed=2):
    """A point of prime order ell | cofactor: the ell-Sylow component of a random curve point
    ([#E / ell^v] R), multiplied by ell until the next multiple would vanish."""
    assert COFACTOR % ell == 0
    v, h = 0, COFACTOR
    while h % ell == 0:
        h //= ell
        v += 1
    rng = random.Random(seed)
    while True:
        T = pc.g1_mul_unreduced(_random_curve_point(BLS, rng), h * BLS.r, BLS)
        if T is None:
            continue
        while pc.g1_mul_unreduced(T, ell, BLS) is not None:
            T = pc.g1_mul_unreduced(T, ell, BLS)
        return T


def subgroup_cases():
    """[(point, in_subgroup)]: G1 points, random non-members, small-order points and
    G1 points shifted by small-order points."""
    rng = random.Random(7)
    g1 = [pc.g1_mul(BLS.g1, rng.randrange(1, BLS.r), BLS) for _ in range(4)]
    bad = non_subgroup_points(4)
    t3, t11 = small_order_point(3), small_order_point(11)
    shifted = [pc.g1_add(g1[0], t3, BLS), pc.g1_add(g1[1], t11, BLS)]
    return [(P, True) for P in g1] + [(P, False) for P in bad + [t3, t11] + shifted]


def invalid_compressed(C, seed=3):
    """[(encoding, expected error)] for curve C's compressed format."""
    rng = random.Random(seed)
    n = C.fp_bytes
    good = pk.g1_to_bytes_compressed(pc.g1_mul(C.g1, rng.randrange(1, C.r), C), C)
    cases = []
    # x = p (non-canonical) with valid flag bits
    xb = bytearray(C.p.to_bytes(n, "big"))
    xb[0] |= 0x80
    cases.append((bytes(xb), ERR_ENCODING))
    # x with no square root of x^3 + b
    while True:
        x = rng.randrange(C.p)
        rhs = (x * x * x + C.b) % C.p
        if pow(rhs, (C.p - 1) // 2, C.p) == C.p - 1:
            break
    xb = bytearray(x.to_bytes(n, "big"))
    xb[0] |= 0x80
    cases.append((bytes(xb), ERR_NOT_ON_CURVE))
    # flag errors
    if C.name == "bls12_381":
        b = bytearray(good)
        b[0] &= 0x7F                      # compression bit missing
        cases.append((bytes(b), ERR_ENCODING))
        cases.append((bytes([0xC0]) + bytes(n - 2) + b"\x01", ERR_ENCODING))  # infinity + junk
        cases.append((bytes([0xE0]) + bytes(n - 1), ERR_ENCODING))            # infinity + sign
    else:
        b = bytearray(good)
        b[0] &= 0x3F                      # 0b00 marker
        cases.append((bytes(b), ERR_ENCODING))
        cases.append((bytes([0x40]) + bytes(n - 2) + b"\x01", ERR_ENCODING))  # infinity + junk
    return cases


def invalid_uncompressed(C, rng):
    """[(encoding, expected error or None = valid identity)] for curve C's uncompressed format
    (rules of oracle/pyspec/kzg.py g1_from_bytes)."""
    n = C.fp_bytes
    P = pc.g1_mul(C.g1, rng.randrange(1, C.r), C)
    cases = [(C.p.to_bytes(n, "big") + P[1].to_bytes(n, "big"), -2),            # x = p
             (P[0].to_bytes(n, "big") + (C.p + 1).to_bytes(n, "big"), -2),      # y = p + 1
             (P[0].to_bytes(n, "big") + ((P[1] + 1) % C.p).to_bytes(n, "big"), -3),
             ((P[0] + 1).to_bytes(n, "big") + P[1].to_bytes(n, "big"), -3),
             (bytes(2 * n), -3 if C.name == "bls12_381" else None),            # (0, 0)
             (pk.g1_to_bytes(None, C), None)]
    if C.name == "bls12_381":
        cases += [(bytes([0x80]) + bytes(2 * n - 1), -2),                        # compression bit
                  (bytes([0x40]) + bytes(2 * n - 2) + b"\x01", -2),              # infinity + junk
                  (bytes([0x20 | P[0] >> (8 * n - 8)]) + P[0].to_bytes(n, "big")[1:] + P[1].to_bytes(n, "big"), -2)]
    return cases
