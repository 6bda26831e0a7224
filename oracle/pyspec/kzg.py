"""KZG batch-verification specification (TESTS ONLY; golden-fixture generator).

Defines, for the whole repo, the exact semantics the C oracle and the HIP product must
reproduce bit for bit (spec source: BASELINE.json:5; reference: none, LICENSE only):

Encodings (big-endian, canonical):
  * Fr scalar: 32 bytes, value < r.
  * G1 BLS12-381: 96 bytes x||y; infinity = 0x40 followed by 95 zero bytes (ZCash flags,
    uncompressed).  G1 BN254: 64 bytes x||y; infinity = 64 zero bytes (EIP-196).
  * G2: x.c1||x.c0||y.c1||y.c0 (imaginary part first); BLS infinity = 0x40 || zeros,
    BN254 infinity = zeros.

Randomisers (counter mode, shard-local): r_i = (int_be(SHA256(seed || le64(i))[0:16]) >> 1),
replaced by 1 if zero.  127-bit randomisers => soundness error <= 2^-127 per batch; the
127-bit bound keeps the top signed window of a 16-bit Pippenger digit split carry-free.

Batch check (n tuples (C_i, z_i, y_i, pi_i), SRS {G1, [1]_2, [tau]_2}):
  A = sum r_i pi_i
  B = sum r_i C_i + sum (r_i z_i mod r) pi_i + ((-sum r_i y_i) mod r) G1
  accept  <=>  e(A, [tau]_2) * e(-B, [1]_2) == 1      (n == 0 accepts)
"""
from __future__ import annotations

import hashlib
import random
from typing import List, Optional, Sequence

from .curves import (CurveParams, G1Point, G2Point, g1_add, g1_mul, g1_neg, g1_on_curve,
                     g2_mul, g2_on_curve)
from .pairing import multi_pairing_is_one

INF_FLAG = 0x40


# ----------------------------------------------------------------------------- encodings


def fr_to_bytes(k: int) -> bytes:
    return int(k).to_bytes(32, "big")


def fr_from_bytes(b: bytes, C: CurveParams) -> int:
    k = int.from_bytes(b, "big")
    if k >= C.r:
        raise ValueError("non-canonical scalar")
    return k


def g1_size(C: CurveParams) -> int:
    return 2 * C.fp_bytes


def g2_size(C: CurveParams) -> int:
    return 4 * C.fp_bytes


def g1_to_bytes(P: G1Point, C: CurveParams) -> bytes:
    n = C.fp_bytes
    if P is None:
        if C.name == "bls12_381":
            return bytes([INF_FLAG]) + bytes(2 * n - 1)
        return bytes(2 * n)
    return P[0].to_bytes(n, "big") + P[1].to_bytes(n, "big")


def g1_from_bytes(b: bytes, C: CurveParams) -> G1Point:
    n = C.fp_bytes
    if len(b) != 2 * n:
        raise ValueError("bad length")
    if C.name == "bls12_381":
        flags = b[0] & 0xE0
        if flags & 0x80:
            raise ValueError("compressed encoding not accepted")
        if flags & INF_FLAG:
            if (b[0] & 0x3F) or any(b[1:]):
                raise ValueError("bad infinity encoding")
            return None
        if flags & 0x20:
            raise ValueError("sort flag set on uncompressed point")
    elif not any(b):
        return None
    x = int.from_bytes(b[:n], "big")
    y = int.from_bytes(b[n:], "big")
    if x >= C.p or y >= C.p:
        raise ValueError("non-canonical coordinate")
    P = (x, y)
    if not g1_on_curve(P, C):
        raise ValueError("point not on curve")
    return P


def g1_to_bytes_compressed(P: G1Point, C: CurveParams) -> bytes:
    """BLS12-381: 48 B ZCash (0x80 compressed | 0x40 infinity | 0x20 larger y).
    BN254: 32 B gnark-crypto (top bits 0b10 smaller y, 0b11 larger y, 0b01 infinity)."""
    n = C.fp_bytes
    if C.name == "bls12_381":
        if P is None:
            return bytes([0xC0]) + bytes(n - 1)
        b = bytearray(P[0].to_bytes(n, "big"))
        b[0] |= 0x80 | (0x20 if P[1] > (C.p - 1) // 2 else 0)
        return bytes(b)
    if P is None:
        return bytes([0x40]) + bytes(n - 1)
    b = bytearray(P[0].to_bytes(n, "big"))
    b[0] |= 0xC0 if P[1] > (C.p - 1) // 2 else 0x80
    return bytes(b)


def g1_from_bytes_compressed(b: bytes, C: CurveParams) -> G1Point:
    """Inverse of g1_to_bytes_compressed; ValueError on any invalid encoding, 'not on curve'
    when x^3 + b has no square root."""
    n = C.fp_bytes
    if len(b) != n:
        raise ValueError("bad length")
    b0 = b[0]
    if C.name == "bls12_381":
        if not b0 & 0x80:
            raise ValueError("compression flag missing")
        if b0 & 0x40:
            if b0 != 0xC0 or any(b[1:]):
                raise ValueError("bad infinity encoding")
            return None
        larger = bool(b0 & 0x20)
        x = int.from_bytes(bytes([b0 & 0x1F]) + b[1:], "big")
    else:
        m = b0 & 0xC0
        if m == 0x40:
            if b0 != 0x40 or any(b[1:]):
                raise ValueError("bad infinity encoding")
            return None
        if m == 0x00:
            raise ValueError("not a compressed encoding")
        larger = m == 0xC0
        x = int.from_bytes(bytes([b0 & 0x3F]) + b[1:], "big")
    if x >= C.p:
        raise ValueError("non-canonical coordinate")
    rhs = (x * x * x + C.b) % C.p
    y = pow(rhs, (C.p + 1) // 4, C.p)
    if y * y % C.p != rhs:
        raise ValueError("point not on curve")
    if y == 0 and larger:
        raise ValueError("bad sign flag")
    if (y > (C.p - 1) // 2) != larger:
        y = C.p - y
    return (x, y)


def g2_to_bytes(Q: G2Point, C: CurveParams) -> bytes:
    n = C.fp_bytes
    if Q is None:
        if C.name == "bls12_381":
            return bytes([INF_FLAG]) + bytes(4 * n - 1)
        return bytes(4 * n)
    (x0, x1), (y0, y1) = Q
    return b"".join(v.to_bytes(n, "big") for v in (x1, x0, y1, y0))


def g2_from_bytes(b: bytes, C: CurveParams) -> G2Point:
    n = C.fp_bytes
    if len(b) != 4 * n:
        raise ValueError("bad length")
    if C.name == "bls12_381":
        if b[0] & 0x80:
            raise ValueError("compressed encoding not accepted")
        if b[0] & INF_FLAG:
            return None
    elif not any(b):
        return None
    v = [int.from_bytes(b[i * n:(i + 1) * n], "big") for i in range(4)]
    if any(x >= C.p for x in v):
        raise ValueError("non-canonical coordinate")
    Q = ((v[1], v[0]), (v[3], v[2]))
    if not g2_on_curve(Q, C):
        raise ValueError("point not on twist")
    return Q


# ----------------------------------------------------------------------------- randomisers


def randomizer(seed: bytes, i: int) -> int:
    assert len(seed) == 32
    h = hashlib.sha256(seed + int(i).to_bytes(8, "little")).digest()
    r = int.from_bytes(h[:16], "big") >> 1
    return r if r else 1


# ----------------------------------------------------------------------------- verify


def batch_combination(commitments: Sequence[G1Point], zs, ys, proofs: Sequence[G1Point],
                      seed: bytes, C: CurveParams, offset: int = 0, powers_of=None):
    """Return (A, B) as affine points.  `offset` = global index of tuple 0 (sharding).
    powers_of = r: Fiat-Shamir / powers mode, r_i = r^(offset + i) instead of the seed rule."""
    A = None
    B = None
    t = 0
    for i, (Ci, z, y, Pi) in enumerate(zip(commitments, zs, ys, proofs)):
        ri = pow(powers_of, offset + i, C.r) if powers_of is not None else randomizer(seed, offset + i)
        A = g1_add(A, g1_mul(Pi, ri, C), C)
        B = g1_add(B, g1_mul(Ci, ri, C), C)
        B = g1_add(B, g1_mul(Pi, ri * z % C.r, C), C)
        t = (t + ri * y) % C.r
    B = g1_add(B, g1_mul(C.g1, (-t) % C.r, C), C)
    return A, B


def batch_verify_points(commitments, zs, ys, proofs, srs_g2, srs_tau_g2, seed, C) -> bool:
    if len(commitments) == 0:
        return True
    A, B = batch_combination(commitments, zs, ys, proofs, seed, C)
    return multi_pairing_is_one([(A, srs_tau_g2), (g1_neg(B, C), srs_g2)], C)


def verify_single(Cm, z, y, Pi, srs_g2, srs_tau_g2, C) -> bool:
    """e(pi, [tau]_2 - [z]_2) == e(C - [y]_1, [1]_2)  (textbook KZG check)."""
    from .curves import g2_add, g2_neg
    tz = g2_add(srs_tau_g2, g2_neg(g2_mul(srs_g2, z % C.r, C), C), C)
    lhs = g1_add(Cm, g1_neg(g1_mul(C.g1, y, C), C), C)
    return multi_pairing_is_one([(Pi, tz), (g1_neg(lhs, C), srs_g2)], C)


# ----------------------------------------------------------------------------- generators


def toy_srs(tau: int, C: CurveParams):
    return C.g1, C.g2, g2_mul(C.g2, tau % C.r, C)


def valid_tuples(n: int, tau: int, rng: random.Random, C: CurveParams):
    """n valid openings of degree-1 polynomials under a known toy tau (test only).

    c_i, z_i, y_i uniform in Fr; q_i = (c_i - y_i) / (tau - z_i); C_i = c_i G1, pi_i = q_i G1.
    """
    out = []
    for _ in range(n):
        c = rng.randrange(C.r)
        z = rng.randrange(C.r)
        while z == tau % C.r:
            z = rng.randrange(C.r)
        y = rng.randrange(C.r)
        q = (c - y) * pow(tau - z, -1, C.r) % C.r
        out.append((g1_mul(C.g1, c, C), z, y, g1_mul(C.g1, q, C), c, q))
    return out


def poly_eval(coeffs: List[int], x: int, r: int) -> int:
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % r
    return acc


def poly_commit_and_open(coeffs: List[int], z: int, tau: int, C: CurveParams):
    """Genuine KZG: commit with powers of tau, open at z via synthetic division."""
    r = C.r
    powers = [pow(tau, i, r) for i in range(len(coeffs))]
    srs = [g1_mul(C.g1, s, C) for s in powers]

    def commit(cs):
        acc = None
        for c, Pw in zip(cs, srs):
            acc = g1_add(acc, g1_mul(Pw, c, C), C)
        return acc

    y = poly_eval(coeffs, z, r)
    # q(X) = (f(X) - y) / (X - z) by synthetic division
    d = len(coeffs) - 1
    q = [0] * d
    if d:
        q[d - 1] = coeffs[d] % r
        for k in range(d - 1, 0, -1):
            q[k - 1] = (coeffs[k] + z * q[k]) % r
    return commit(coeffs), y, commit(q)


# ------------------------------------------------------------------ Fiat-Shamir transcript
# (device implementation csrc/fs.hpp, C-ABI KZGMI_FLAG_FIAT_SHAMIR)
FS_LEAF_TAG = b"KZGMI_FS_LEAF_V1"
FS_ROOT_TAG = b"KZGMI_FS_ROOT_V1"
FS_CHUNK = 4096


def fs_leaf(i: int, c_comp: bytes, p_comp: bytes, z: int, y: int) -> bytes:
    return hashlib.sha256(FS_LEAF_TAG + i.to_bytes(8, "big") + c_comp + p_comp + z.to_bytes(32, "big")
                          + y.to_bytes(32, "big")).digest()


def merkle_root(nodes: List[bytes]) -> bytes:
    """Binary Merkle root of a power-of-two list; node = SHA256(left || right)."""
    assert nodes and len(nodes) & (len(nodes) - 1) == 0
    while len(nodes) > 1:
        nodes = [hashlib.sha256(nodes[k] + nodes[k + 1]).digest() for k in range(0, len(nodes), 2)]
    return nodes[0]


def fs_slots(n: int) -> int:
    slots = FS_CHUNK
    while slots < n:
        slots *= 2
    return slots


def fs_challenge(commitments: Sequence[G1Point], zs, ys, proofs: Sequence[G1Point], C: CurveParams) -> int:
    """r = int_be(SHA256(ROOT_TAG || be64(n) || merkle_root(leaves, zero-padded to
    max(4096, next_pow2(n)) slots))) mod r, 1 if 0; leaves over compressed encodings."""
    n = len(commitments)
    leaves = [fs_leaf(i, g1_to_bytes_compressed(commitments[i], C), g1_to_bytes_compressed(proofs[i], C), zs[i], ys[i])
              for i in range(n)]
    leaves += [bytes(32)] * (fs_slots(n) - n)
    h = hashlib.sha256(FS_ROOT_TAG + n.to_bytes(8, "big") + merkle_root(leaves)).digest()
    r = int.from_bytes(h, "big") % C.r
    return r if r else 1


def fs_seed(commitments, zs, ys, proofs, C: CurveParams) -> bytes:
    """KZGMI_FLAG_FIAT_SHAMIR randomisers: the counter-mode r_i of `randomizer` seeded with
    be32(fs_challenge(...)), i.e. batch_combination(..., seed=fs_seed(...))."""
    return fs_challenge(commitments, zs, ys, proofs, C).to_bytes(32, "big")
