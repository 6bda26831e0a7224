"""GLV scalar decomposition spec (TEST INFRASTRUCTURE ONLY).

Independent restatement (plain Python ints, derived from the curve parameters in
curves.py, sharing nothing with tools/gen_params.py) of what csrc/glv.hpp computes:

    phi(x, y) = (beta x, y) = [lam] P on G1,  lam^2 + lam + 1 = 0 (mod r)
    k = k0 + k1 lam (mod r) with (k0, k1) = (k, 0) - round(b1) v1 - round(b2) v2 (Babai)

where v1, v2 is the reduced basis of {(a, b) : a + b lam = 0 mod r} from the extended
Euclidean algorithm on (r, lam) (Gallant-Lambert-Vanstone 2001; Guide to ECC Alg. 3.74),
and BLS12-381 pins lam = -x^2 (the eigenvalue of the subgroup-test phi).  The GPU result of
an MSM does not depend on the decomposition (GLV only regroups the same sum), so parity is
pinned by the C oracle's plain MSM; this module pins the decomposition itself.

Parity status: unpinned by the reference (which holds no code).
"""
from __future__ import annotations

import random
from functools import lru_cache
from typing import List, Tuple

from . import curves as pc


@lru_cache(maxsize=None)
def params(curve: str):
    """(beta, lam, v1, v2) for `curve` (det(v1, v2) = +r, v2.b > 0, v1.b < 0)."""
    C = pc.CURVES[curve]
    p, r = C.p, C.r

    def cube_roots(m):
        g = 2
        while pow(g, (m - 1) // 3, m) == 1:
            g += 1
        w = pow(g, (m - 1) // 3, m)
        return [w, w * w % m]

    lams = cube_roots(r)
    if curve == "bls12_381":
        x = 0xD201000000010000
        lams = [(-x * x) % r]
    G = C.g1
    for beta in cube_roots(p):
        for lam in lams:
            if (beta * G[0] % p, G[1]) == pc.g1_mul(G, lam, C):
                break
        else:
            continue
        break
    else:
        raise AssertionError("no matching (beta, lambda)")
    # extended Euclid on (r, lam): s_i r + t_i lam = r_i; stop at the first r_i < sqrt(r)
    rs, ts = [r, lam], [0, 1]
    while rs[-1] * rs[-1] >= r:
        q = rs[-2] // rs[-1]
        rs.append(rs[-2] - q * rs[-1])
        ts.append(ts[-2] - q * ts[-1])
    m = len(rs) - 1
    v1 = (rs[m], -ts[m])
    q = rs[m - 1] // rs[m]
    c1 = (rs[m - 1], -ts[m - 1])
    c2 = (rs[m - 1] - q * rs[m], -(ts[m - 1] - q * ts[m]))
    v2 = c1 if c1[0] ** 2 + c1[1] ** 2 <= c2[0] ** 2 + c2[1] ** 2 else c2
    if v1[0] * v2[1] - v1[1] * v2[0] < 0:
        v2 = (-v2[0], -v2[1])
    return beta, lam, v1, v2


def _round_div(a: int, b: int) -> int:
    """round(a / b) for a >= 0, b > 0 (b odd: no ties)."""
    return (2 * a + b) // (2 * b)


def decompose(curve: str, k: int) -> Tuple[int, int]:
    """(k0, k1) with k = k0 + k1 lam (mod r), |k0|, |k1| < 2^127 (signed)."""
    C = pc.CURVES[curve]
    _, _, v1, v2 = params(curve)
    det = v1[0] * v2[1] - v1[1] * v2[0]
    assert det == C.r
    c1 = _round_div(k * v2[1], det)
    c2 = _round_div(-k * v1[1], det)
    return k - c1 * v1[0] - c2 * v2[0], -c1 * v1[1] - c2 * v2[1]


def phi(curve: str, P):
    if P is None:
        return None
    C = pc.CURVES[curve]
    beta = params(curve)[0]
    return (beta * P[0] % C.p, P[1])


def edge_scalars(curve: str, count: int = 64, seed: int = 1) -> List[int]:
    """Scalars at the edges of the decomposition: 0, 1, r - 1, lam, -lam, Babai rounding
    boundaries (k g / r within one unit of m + 1/2 for both multipliers g) and the scalars with
    the largest |k0|, |k1| among a random search."""
    C = pc.CURVES[curve]
    r = C.r
    _, lam, v1, v2 = params(curve)
    rng = random.Random(seed)
    out = [0, 1, 2, r - 1, r - 2, lam, r - lam, (r - 1) // 2, (r + 1) // 2, (1 << 127) - 1, 1 << 127,
           (1 << 128) - 1, 1 << 128]
    for g in (v2[1], -v1[1]):
        for _ in range(count // 4):
            mq = rng.randrange(max(1, g))
            k = ((2 * mq + 1) * r) // (2 * g)  # k g / r just below mq + 1/2
            out += [k % r, (k + 1) % r]
    best = []
    for _ in range(20000):
        k = rng.randrange(r)
        k0, k1 = decompose(curve, k)
        best.append((max(abs(k0), abs(k1)), k))
    best.sort(reverse=True)
    out += [k for _, k in best[:count // 4]]
    return [k % r for k in out][:max(count, 13)]
