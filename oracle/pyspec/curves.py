"""Pure-Python big-int specification of BLS12-381 and BN254 (TEST INFRASTRUCTURE ONLY).

This module is part of the oracle (see oracle/README.md).  It is never imported by the
product path (`kzg-batch-verification-scheme_amd/`).  It exists to pin the C oracle and the
HIP kernels with an implementation that shares no code and no representation with them:
plain Python ints, affine/Jacobian formulas written from the textbook definitions.

Parity status: **parity unpinned by the reference** -- the reference snapshot holds only
`/root/reference/LICENSE:1-201`.  The spec follows BASELINE.json:5
(north_star) and SURVEY.md Appendix A (curve constants, checked in tests/test_pyspec.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

# ----------------------------------------------------------------------------- Fp2
# Fp2 = Fp[u]/(u^2 + 1) for both curves; elements are (c0, c1) meaning c0 + c1*u.


def fp2_add(a, b, p):
    return ((a[0] + b[0]) % p, (a[1] + b[1]) % p)


def fp2_sub(a, b, p):
    return ((a[0] - b[0]) % p, (a[1] - b[1]) % p)


def fp2_neg(a, p):
    return ((-a[0]) % p, (-a[1]) % p)


def fp2_mul(a, b, p):
    return ((a[0] * b[0] - a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)


def fp2_inv(a, p):
    n = (a[0] * a[0] + a[1] * a[1]) % p
    ni = pow(n, -1, p)
    return (a[0] * ni % p, (-a[1]) * ni % p)


def fp2_is_zero(a):
    return a[0] == 0 and a[1] == 0


# ----------------------------------------------------------------------------- params


@dataclass(frozen=True)
class CurveParams:
    name: str
    p: int
    r: int
    b: int                      # E: y^2 = x^3 + b
    xi: Tuple[int, int]         # Fp6 non-residue, xi = w^6
    beta: int                   # u = w^6 - beta in the flat Fp12 (xi = beta + u)
    twist: str                  # 'M' (b' = b*xi) or 'D' (b' = b/xi)
    g1: Tuple[int, int]
    g2: Tuple[Tuple[int, int], Tuple[int, int]]
    loop: int                   # |ate loop parameter|
    loop_negative: bool         # BLS12-381: x < 0 -> conjugate the Miller value
    bn_frobenius_lines: bool    # BN: two extra lines with pi(Q), -pi^2(Q)
    fp_bytes: int

    @property
    def b2(self):
        """Twist coefficient b' in Fp2."""
        if self.twist == "M":
            return fp2_mul((self.b, 0), self.xi, self.p)
        return fp2_mul((self.b, 0), fp2_inv(self.xi, self.p), self.p)


BLS12_381 = CurveParams(
    name="bls12_381",
    p=0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB,
    r=0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
    b=4,
    xi=(1, 1),
    beta=1,
    twist="M",
    g1=(
        0x17F1D3A73197D7942695638C4FA9AC0FC3688C4F9774B905A14E3A3F171BAC586C55E83FF97A1AEFFB3AF00ADB22C6BB,
        0x08B3F481E3AAA0F1A09E30ED741D8AE4FCF5E095D5D00AF600DB18CB2C04B3EDD03CC744A2888AE40CAA232946C5E7E1,
    ),
    g2=(
        (
            0x024AA2B2F08F0A91260805272DC51051C6E47AD4FA403B02B4510B647AE3D1770BAC0326A805BBEFD48056C8C121BDB8,
            0x13E02B6052719F607DACD3A088274F65596BD0D09920B61AB5DA61BBDC7F5049334CF11213945D57E5AC7D055D042B7E,
        ),
        (
            0x0CE5D527727D6E118CC9CDC6DA2E351AADFD9BAA8CBDD3A76D429A695160D12C923AC9CC3BACA289E193548608B82801,
            0x0606C4A02EA734CC32ACD2B02BC28B99CB3E287E85A763AF267492AB572E99AB3F370D275CEC1DA1AAA9075FF05F79BE,
        ),
    ),
    loop=0xD201000000010000,
    loop_negative=True,
    bn_frobenius_lines=False,
    fp_bytes=48,
)

BN254_U = 4965661367192848881

BN254 = CurveParams(
    name="bn254",
    p=21888242871839275222246405745257275088696311157297823662689037894645226208583,
    r=21888242871839275222246405745257275088548364400416034343698204186575808495617,
    b=3,
    xi=(9, 1),
    beta=9,
    twist="D",
    g1=(1, 2),
    g2=(
        (
            10857046999023057135944570762232829481370756359578518086990519993285655852781,
            11559732032986387107991004021392285783925812861821192530917403151452391805634,
        ),
        (
            8495653923123431417604973247489272438418190587263600148770280649306958101930,
            4082367875863433681332203403145435568316851327593401208105741076214120093531,
        ),
    ),
    loop=6 * BN254_U + 2,
    loop_negative=False,
    bn_frobenius_lines=True,
    fp_bytes=32,
)

CURVES = {"bls12_381": BLS12_381, "bn254": BN254}

# ----------------------------------------------------------------------------- G1 (Fp)
# Affine points are (x, y) tuples; the point at infinity is None.

G1Point = Optional[Tuple[int, int]]


def g1_on_curve(P: G1Point, C: CurveParams) -> bool:
    if P is None:
        return True
    x, y = P
    return (y * y - x * x * x - C.b) % C.p == 0


def g1_neg(P: G1Point, C: CurveParams) -> G1Point:
    if P is None:
        return None
    return (P[0], (-P[1]) % C.p)


def g1_add(P: G1Point, Q: G1Point, C: CurveParams) -> G1Point:
    p = C.p
    if P is None:
        return Q
    if Q is None:
        return P
    x1, y1 = P
    x2, y2 = Q
    if x1 == x2:
        if (y1 + y2) % p == 0:
            return None
        lam = 3 * x1 * x1 * pow(2 * y1, -1, p) % p
    else:
        lam = (y2 - y1) * pow(x2 - x1, -1, p) % p
    x3 = (lam * lam - x1 - x2) % p
    y3 = (lam * (x1 - x3) - y1) % p
    return (x3, y3)


# Jacobian (X, Y, Z) with x = X/Z^2, y = Y/Z^3 -- used only to make scalar
# multiplication fast enough for fixture generation.
def _jac_dbl(P, p):
    X, Y, Z = P
    if Z == 0 or Y == 0:
        return (1, 1, 0)
    A = X * X % p
    B = Y * Y % p
    Cc = B * B % p
    D = 2 * ((X + B) * (X + B) - A - Cc) % p
    E = 3 * A % p
    F = E * E % p
    X3 = (F - 2 * D) % p
    Y3 = (E * (D - X3) - 8 * Cc) % p
    Z3 = 2 * Y * Z % p
    return (X3, Y3, Z3)


def _jac_add_affine(P, q, p):
    X1, Y1, Z1 = P
    if Z1 == 0:
        return (q[0], q[1], 1)
    x2, y2 = q
    Z1Z1 = Z1 * Z1 % p
    U2 = x2 * Z1Z1 % p
    S2 = y2 * Z1 * Z1Z1 % p
    H = (U2 - X1) % p
    Rr = (S2 - Y1) % p
    if H == 0:
        if Rr == 0:
            return _jac_dbl(P, p)
        return (1, 1, 0)
    HH = H * H % p
    HHH = H * HH % p
    V = X1 * HH % p
    X3 = (Rr * Rr - HHH - 2 * V) % p
    Y3 = (Rr * (V - X3) - Y1 * HHH) % p
    Z3 = Z1 * H % p
    return (X3, Y3, Z3)


def _jac_to_affine(P, p):
    X, Y, Z = P
    if Z == 0:
        return None
    zi = pow(Z, -1, p)
    zi2 = zi * zi % p
    return (X * zi2 % p, Y * zi2 * zi % p)


def g1_mul(P: G1Point, k: int, C: CurveParams) -> G1Point:
    """Left-to-right double-and-add; k is reduced mod r (the group order)."""
    if P is None:
        return None
    k %= C.r
    if k == 0:
        return None
    p = C.p
    R = (1, 1, 0)
    for bit in bin(k)[2:]:
        R = _jac_dbl(R, p)
        if bit == "1":
            R = _jac_add_affine(R, P, p)
    return _jac_to_affine(R, p)


def g1_mul_unreduced(P: G1Point, k: int, C: CurveParams) -> G1Point:
    """[k]P without reducing k mod r (for points that may lie outside the order-r subgroup)."""
    if P is None or k == 0:
        return None
    p = C.p
    R = (1, 1, 0)
    for bit in bin(k)[2:]:
        R = _jac_dbl(R, p)
        if bit == "1":
            R = _jac_add_affine(R, P, p)
    return _jac_to_affine(R, p)


def g1_in_subgroup(P: G1Point, C: CurveParams) -> bool:
    """Definition: [r]P == O (the fast endomorphism test on the GPU is checked against this)."""
    return g1_mul_unreduced(P, C.r, C) is None


def g1_msm(points, scalars, C: CurveParams) -> G1Point:
    """Naive sum of k_i * P_i (definition of the MSM)."""
    acc = None
    for P, k in zip(points, scalars):
        acc = g1_add(acc, g1_mul(P, k, C), C)
    return acc


# ----------------------------------------------------------------------------- G2 (Fp2, twist)

G2Point = Optional[Tuple[Tuple[int, int], Tuple[int, int]]]


def g2_on_curve(Q: G2Point, C: CurveParams) -> bool:
    if Q is None:
        return True
    p = C.p
    x, y = Q
    lhs = fp2_mul(y, y, p)
    rhs = fp2_add(fp2_mul(fp2_mul(x, x, p), x, p), C.b2, p)
    return lhs == rhs


def g2_neg(Q: G2Point, C: CurveParams) -> G2Point:
    if Q is None:
        return None
    return (Q[0], fp2_neg(Q[1], C.p))


def g2_add(P: G2Point, Q: G2Point, C: CurveParams) -> G2Point:
    p = C.p
    if P is None:
        return Q
    if Q is None:
        return P
    x1, y1 = P
    x2, y2 = Q
    if x1 == x2:
        if fp2_is_zero(fp2_add(y1, y2, p)):
            return None
        lam = fp2_mul(fp2_mul((3, 0), fp2_mul(x1, x1, p), p), fp2_inv(fp2_add(y1, y1, p), p), p)
    else:
        lam = fp2_mul(fp2_sub(y2, y1, p), fp2_inv(fp2_sub(x2, x1, p), p), p)
    x3 = fp2_sub(fp2_sub(fp2_mul(lam, lam, p), x1, p), x2, p)
    y3 = fp2_sub(fp2_mul(lam, fp2_sub(x1, x3, p), p), y1, p)
    return (x3, y3)


def g2_mul(Q: G2Point, k: int, C: CurveParams) -> G2Point:
    """Double-and-add over the raw integer k (not reduced: used for r*Q == O checks)."""
    R = None
    for bit in bin(k)[2:] if k > 0 else "":
        R = g2_add(R, R, C)
        if bit == "1":
            R = g2_add(R, Q, C)
    return R
