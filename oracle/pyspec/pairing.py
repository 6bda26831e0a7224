"""Optimal-ate pairing in a FLAT Fp12 = Fp[w]/(w^12 - 2*beta*w^6 + beta^2 + 1) (TESTS ONLY).

Deliberately structured differently from the C oracle and the HIP kernels (which use the
Fp2 -> Fp6 -> Fp12 tower, projective line coefficients and an x-chain final exponentiation):

* Fp12 elements are length-12 coefficient lists over Fp in the basis 1, w, ..., w^11.
* Q in E'(Fp2) is walked with AFFINE twist arithmetic; every line is evaluated at P by
  untwisting into E(Fp12) with plain Fp12 multiplications.
* The final exponentiation is a naive square-and-multiply by 3*(p^12 - 1)/r.

The cube is part of the definition used across the repo: the fast hard part (HIP kernels
and the C oracle) computes f^(3*(p^4-p^2+1)/r) for BLS12-381 (Hayashida-Hayasaka-Teruya),
so every implementation here returns e(P, Q)^3 for BLS12-381.  For BN254 the exponent is
exactly (p^12 - 1)/r.  Both are non-degenerate bilinear maps (gcd(3, r) = 1).

Spec source: BASELINE.json:5 ("multi-Miller-loop + final exponentiation"), SURVEY.md 3.1.
Reference: none (/root/reference/LICENSE:1-201 only) -- parity unpinned by the reference.
"""
from __future__ import annotations

from .curves import CurveParams, fp2_inv, fp2_mul, fp2_sub, fp2_add, fp2_is_zero, fp2_neg

# ----------------------------------------------------------------------------- flat Fp12


def _modpoly(C: CurveParams):
    # w^12 = 2*beta*w^6 - (beta^2 + 1)   because u = w^6 - beta and u^2 = -1
    return (2 * C.beta) % C.p, (-(C.beta * C.beta + 1)) % C.p


def f12_one():
    return [1] + [0] * 11


def f12_mul(a, b, C: CurveParams):
    p = C.p
    t = [0] * 23
    for i, ai in enumerate(a):
        if ai:
            for j, bj in enumerate(b):
                t[i + j] += ai * bj
    c6, c0 = _modpoly(C)
    for k in range(22, 11, -1):
        v = t[k] % p
        if v:
            t[k - 6] += v * c6
            t[k - 12] += v * c0
    return [x % p for x in t[:12]]


def f12_pow(a, e: int, C: CurveParams):
    r = f12_one()
    for bit in bin(e)[2:]:
        r = f12_mul(r, r, C)
        if bit == "1":
            r = f12_mul(r, a, C)
    return r


def f12_from_fp2(c, C: CurveParams):
    """c0 + c1*u with u = w^6 - beta."""
    out = [0] * 12
    out[0] = (c[0] - C.beta * c[1]) % C.p
    out[6] = c[1] % C.p
    return out


def f12_from_fp(x, C: CurveParams):
    return [x % C.p] + [0] * 11


def f12_w_power(k: int, C: CurveParams):
    """w^k for 0 <= k < 12."""
    out = [0] * 12
    out[k] = 1
    return out


def f12_inv_w_power(k: int, C: CurveParams):
    """w^-k = w^(6-k) / xi  (since w^6 = xi), for 1 <= k <= 6."""
    xi_inv = fp2_inv(C.xi, C.p)
    return f12_mul(f12_w_power(6 - k, C), f12_from_fp2(xi_inv, C), C)


def flat_to_tower(f, C: CurveParams):
    """Convert a flat Fp12 into the tower coefficient order used by the C/HIP code.

    Tower: Fp12 = Fp6[w]/(w^2 - v), Fp6 = Fp2[v]/(v^3 - xi).  An element
    (a0 + a1 v + a2 v^2) + (b0 + b1 v + b2 v^2) w equals
    a0 + b0 w + a1 w^2 + b1 w^3 + a2 w^4 + b2 w^5.  Returned as the 12 Fp values
    [a0.c0, a0.c1, a1.c0, a1.c1, a2.c0, a2.c1, b0.c0, b0.c1, b1.c0, b1.c1, b2.c0, b2.c1].
    """
    p = C.p
    coeff = []  # Fp2 coefficient of w^k, k = 0..5
    for k in range(6):
        y = f[k + 6] % p
        x = (f[k] + C.beta * f[k + 6]) % p
        coeff.append((x, y))
    order = [0, 2, 4, 1, 3, 5]
    out = []
    for k in order:
        out.extend(coeff[k])
    return out


# ----------------------------------------------------------------------------- lines


def _untwist_factors(C: CurveParams):
    """Fp12 constants (cx, cy) with x = x' * cx, y = y' * cy mapping E'(Fp2) -> E(Fp12)."""
    if C.twist == "M":  # x = x'/w^2, y = y'/w^3
        return f12_inv_w_power(2, C), f12_inv_w_power(3, C)
    return f12_w_power(2, C), f12_w_power(3, C)  # D-type: x = x' w^2, y = y' w^3


def _line(T, lam, P, C: CurveParams, consts):
    """Line through the twist point T with twist slope lam, evaluated at P (affine in Fp).

    Untwisted: slope m = lam * cy/cx; line(P) = m*(xP - xT) - (yP - yT).
    """
    cx, cy, cy_over_cx = consts
    xT = f12_mul(f12_from_fp2(T[0], C), cx, C)
    yT = f12_mul(f12_from_fp2(T[1], C), cy, C)
    m = f12_mul(f12_from_fp2(lam, C), cy_over_cx, C)
    dx = [(a - b) % C.p for a, b in zip(f12_from_fp(P[0], C), xT)]
    dy = [(a - b) % C.p for a, b in zip(f12_from_fp(P[1], C), yT)]
    t = f12_mul(m, dx, C)
    return [(a - b) % C.p for a, b in zip(t, dy)]


def _vertical(T, P, C: CurveParams, consts):
    cx = consts[0]
    xT = f12_mul(f12_from_fp2(T[0], C), cx, C)
    return [(a - b) % C.p for a, b in zip(f12_from_fp(P[0], C), xT)]


def _step(T, Q, P, C, consts):
    """Return (line value at P, T + Q) for T, Q on the twist (affine)."""
    p = C.p
    if T is None or Q is None:
        return f12_one(), (Q if T is None else T)
    if T[0] == Q[0]:
        if fp2_is_zero(fp2_add(T[1], Q[1], p)):
            return _vertical(T, P, C, consts), None
        lam = fp2_mul(fp2_mul((3, 0), fp2_mul(T[0], T[0], p), p),
                      fp2_inv(fp2_add(T[1], T[1], p), p), p)
    else:
        lam = fp2_mul(fp2_sub(Q[1], T[1], p), fp2_inv(fp2_sub(Q[0], T[0], p), p), p)
    l = _line(T, lam, P, C, consts)
    x3 = fp2_sub(fp2_sub(fp2_mul(lam, lam, p), T[0], p), Q[0], p)
    y3 = fp2_sub(fp2_mul(lam, fp2_sub(T[0], x3, p), p), T[1], p)
    return l, (x3, y3)


def _frobenius_twist(Q, C: CurveParams):
    """pi_p on E'(Fp2) via untwist-frobenius-twist: (conj(x) * gx, conj(y) * gy)."""
    p = C.p
    # psi(x', y') = (x'^p * xi^((p-1)/3), y'^p * xi^((p-1)/2)) for the D-type BN twist
    def fp2_pow(a, e):
        r = (1, 0)
        for bit in bin(e)[2:]:
            r = fp2_mul(r, r, p)
            if bit == "1":
                r = fp2_mul(r, a, p)
        return r
    gx = fp2_pow(C.xi, (p - 1) // 3)
    gy = fp2_pow(C.xi, (p - 1) // 2)
    x, y = Q
    xc = (x[0], (-x[1]) % p)
    yc = (y[0], (-y[1]) % p)
    return (fp2_mul(xc, gx, p), fp2_mul(yc, gy, p))


def miller_loop(P, Q, C: CurveParams):
    """f_{loop,Q}(P) in the flat Fp12 (plus BN Frobenius lines / BLS conjugation)."""
    if P is None or Q is None:
        return f12_one()
    cx, cy = _untwist_factors(C)
    # cy/cx: M-type w^-3/w^-2 = w^-1 ; D-type w^3/w^2 = w
    cy_over_cx = f12_inv_w_power(1, C) if C.twist == "M" else f12_w_power(1, C)
    consts = (cx, cy, cy_over_cx)
    f = f12_one()
    T = Q
    bits = bin(C.loop)[3:]
    for bit in bits:
        l, T = _step(T, T, P, C, consts)
        f = f12_mul(f12_mul(f, f, C), l, C)
        if bit == "1":
            l, T = _step(T, Q, P, C, consts)
            f = f12_mul(f, l, C)
    if C.bn_frobenius_lines:
        Q1 = _frobenius_twist(Q, C)
        Q2 = _frobenius_twist(Q1, C)
        Q2 = (Q2[0], fp2_neg(Q2[1], C.p))
        l, T = _step(T, Q1, P, C, consts)
        f = f12_mul(f, l, C)
        l, T = _step(T, Q2, P, C, consts)
        f = f12_mul(f, l, C)
    if C.loop_negative:
        # f_{-|x|} = 1/f_{|x|} up to factors killed by the final exponentiation;
        # 1/f == f^(p^6) after the easy part, so use the p^6 power (conjugation).
        f = f12_pow(f, C.p ** 6, C)
    return f


def final_exponent(C: CurveParams) -> int:
    e = (C.p ** 12 - 1) // C.r
    return 3 * e if C.name == "bls12_381" else e


def final_exp(f, C: CurveParams):
    return f12_pow(f, final_exponent(C), C)


def pairing(P, Q, C: CurveParams):
    """e(P, Q) (cubed for BLS12-381, see module docstring) as a flat Fp12."""
    return final_exp(miller_loop(P, Q, C), C)


def multi_pairing_is_one(pairs, C: CurveParams) -> bool:
    f = f12_one()
    for P, Q in pairs:
        f = f12_mul(f, miller_loop(P, Q, C), C)
    return final_exp(f, C) == f12_one()
