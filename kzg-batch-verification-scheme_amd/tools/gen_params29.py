"""Generates csrc/params29_gen.hpp: the Fp constants of the radix-2^29 accumulation arithmetic
(csrc/field29.hpp) for both curves -- BLS12-381 in 14 x 29-bit limbs (R29 = 2^406) and BN254 in
9 x 29-bit limbs (R29 = 2^261): p, -p^-1 mod 2^32, the Montgomery conversions to/from the
32-bit-limb domain (R = 2^384 / 2^256), biased multiples of p for carry-free subtraction, the
small multiples of p for the exact zero test, and the ROLE constants -- which biased multiple
each subtraction of the accumulation loop and its doubling uses.

The roles differ per curve because the headroom differs: R29 / p is 2^25 for BLS12-381 but only
~169 for BN254, so a Montgomery product of inputs below a p and b p returns below
(a b p / R29 + 1) p, and on BN254 that is only < 2p while a b < 169.  check_bounds() below runs
the value bounds of every step (in units of p) through the loop until they are stable and
asserts each precondition: a bias k p is at least the subtrahend's bound, the zero-tested values
stay below NKP p, and every product's output stays within the bounds its consumers assume.

python3 kzg-batch-verification-scheme_amd/tools/gen_params29.py > kzg-batch-verification-scheme_amd/csrc/params29_gen.hpp
"""
from fractions import Fraction

W = 29
MASK = (1 << W) - 1

CURVES = [
    # name, p, limbs, 32-bit-limb Montgomery exponent, curve b, NKP, roles (multiples of p)
    ("Bls12_381Fp29",
     0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab,
     14, 384, 4, 20,
     dict(ACC_NEG=8, ACC_P=16, ACC_R=16, ACC_X3=8, ACC_QX=16, ACC_PPP=8, DBL_X=8, DBL_QX=16, DBL_Y=8)),
    ("Bn254Fp29",
     0x30644e72e131a029b85045b68181585d97816a916871ca8d3c208c16d87cfd47,
     9, 256, 3, 12,
     dict(ACC_NEG=2, ACC_P=8, ACC_R=4, ACC_X3=4, ACC_QX=8, ACC_PPP=2, DBL_X=4, DBL_QX=8, DBL_Y=2)),
]
# bucket records (x29_add / x29_dbl inputs and outputs, both curves): x < 10p, y < 16p, zz, zzz < 2p
REC = dict(x=10, y=16, z=2)


def limbs(x, n):
    out = []
    for _ in range(n - 1):
        out.append(x & MASK)
        x >>= W
    out.append(x)
    return out


def biased(k, p, n):
    """k p with limbs 0..n-2 moved into [2^29, 2^30) (borrowing from the next limb)."""
    b = limbs(k * p, n)
    b[0] += 1 << W
    for i in range(1, n - 1):
        b[i] += (1 << W) - 1
    b[n - 1] -= 1
    assert sum(v << (W * i) for i, v in enumerate(b)) == k * p
    assert all((1 << W) <= v < (1 << (W + 1)) for v in b[:n - 1]) and b[n - 1] >= 0
    return b


def biased3(k, p, n):
    """k p with limbs 0..n-2 in [3 (2^29 - 1), 2^31): the bias of sub3_29 (a + B - s - 2t in one
    carry pass, s and t normalised, so every limb's s + 2t <= 3 (2^29 - 1) <= B_i)."""
    b = limbs(k * p, n)
    b[0] += 3 << W
    for i in range(1, n - 1):
        b[i] += (3 << W) - 3
    b[n - 1] -= 3
    assert sum(v << (W * i) for i, v in enumerate(b)) == k * p
    assert all(3 * ((1 << W) - 1) <= v < (1 << 31) for v in b[:n - 1]) and b[n - 1] >= 0
    return b


def check_bounds(p, n, nkp, roles):
    """Value bounds (units of p) of the accumulation loop (msm.hpp acc_loop29), its doubling
    (dbl_affine29), the record addition/doubling (x29_add, x29_dbl) and the on-curve test."""
    R = 1 << (W * n)
    lim = Fraction(R, p)  # values must stay representable: < 2^(29 n)
    def mont(a, b):       # (a p)(b p)/R + p, in units of p
        assert a < lim and b < lim
        return Fraction(a) * b * p / R + 1
    def mont2(a, b, c, d):
        assert max(a, b, c, d) < lim
        return (Fraction(a) * b + Fraction(c) * d) * p / R + 1
    ro = {k: Fraction(v) for k, v in roles.items()}
    # points come out of a Montgomery product with canonical inputs (fp_to29, k_convert_points
    # <To29>): below (p / R29 + 1) p, NOT below p -- on BN254 that is 1.006 p, so negating q.y
    # needs a bias of 2p (a bias of 1p goes negative for ~0.3 % of the points)
    qin = mont(1, 1)
    assert ro["ACC_NEG"] >= qin
    # dbl_affine29: the running sum := 2q (q.x < qin p, q.y < ACC_NEG p)
    qx, qy = qin, ro["ACC_NEG"]
    U = 2 * qy
    V = mont(U, U); Wd = mont(U, V); S = mont(qx, V); M = 3 * mont(qx, qx)
    assert ro["DBL_X"] >= 2 * S
    dx = mont(M, M) + ro["DBL_X"]
    assert ro["DBL_QX"] >= dx
    t = mont(M, S + ro["DBL_QX"]); w = mont(Wd, qy)
    assert ro["DBL_Y"] >= w
    dy = t + ro["DBL_Y"]
    # the loop from a bucket start (x = q.x, y = q.y, zz = zzz = ONE < p) to a fixed point
    X, Y, Z = max(qx, dx), max(qy, dy), max(Fraction(1), V, Wd)
    for _ in range(50):
        U2, S2 = mont(qx, Z), mont(qy, Z)
        assert ro["ACC_P"] >= X and ro["ACC_R"] >= Y
        P, Rr = U2 + ro["ACC_P"], S2 + ro["ACC_R"]
        assert P < nkp and Rr < nkp, "zero test range"
        PP = mont(P, P); PPP = mont(P, PP); Q2 = mont(X, PP)
        assert ro["ACC_X3"] >= PPP + 2 * Q2
        X3 = mont(Rr, Rr) + ro["ACC_X3"]
        assert ro["ACC_QX"] >= X3 and ro["ACC_PPP"] >= PPP
        # neg_lazy29 (ACC_PPP - PPP limb by limb, no carries): the top limb must not go negative
        assert limbs(roles["ACC_PPP"] * p, n)[n - 1] - 1 >= (int(PPP * p) >> (W * (n - 1))) + 1
        Y3 = mont2(Rr, Q2 + ro["ACC_QX"], Y, ro["ACC_PPP"])
        Zn = max(Z, mont(Z, PP), mont(Z, PPP))
        Xn, Yn = max(X, X3), max(Y, Y3)
        if (Xn, Yn, Zn) == (X, Y, Z):
            break
        X, Y, Z = Xn, Yn, Zn
    else:
        raise AssertionError("loop bounds do not settle")
    assert X < REC["x"] and Y < REC["y"] and Z < REC["z"], "flushed records within the record bounds"
    # x29_add on records (B2, B8, B16) and x29_dbl (B4, B8, B16)
    x, y, z = (Fraction(REC[k]) for k in "xyz")
    U1, S1 = mont(x, z), mont(y, z)
    P, Rr = U1 + 2, S1 + 2
    assert 2 >= U1 and 2 >= S1 and P < nkp and Rr < nkp
    PP = mont(P, P); PPP = mont(P, PP); Q2 = mont(U1, PP)
    assert 8 >= PPP + 2 * Q2
    X3 = mont(Rr, Rr) + 8
    assert 16 >= X3 and 8 >= PPP
    Y3 = mont2(Rr, Q2 + 16, S1, 8)
    ZZ = mont(mont(z, z), PP); ZZZ = mont(mont(z, z), PPP)
    assert X3 < REC["x"] and Y3 < REC["y"] and ZZ < REC["z"] and ZZZ < REC["z"]
    U = 2 * y
    V = mont(U, U); Wd = mont(U, V); S = mont(x, V); M = 3 * mont(x, x)
    assert 4 >= 2 * S
    X3 = mont(M, M) + 4
    assert 8 >= X3 and 16 >= y
    Y3 = mont2(M, S + 8, Wd, 16)
    assert X3 < REC["x"] and Y3 < REC["y"] and mont(V, z) < REC["z"] and mont(Wd, z) < REC["z"]
    # to32: canon29 needs mont(record, TO32 < p) < 2p
    assert mont(max(REC.values()), 1) < 2
    # k_convert_points<To29>: y^2 - (x^3 + b) with B4, zero-tested
    rhs = mont(mont(1, 1), 1) + 1
    assert 4 >= rhs and mont(1, 1) + 4 < nkp
    return dict(X=float(X), Y=float(Y), Z=float(Z))


def arr(v):
    return "{" + ", ".join("0x%xu" % x for x in v) + "}"


def emit(name, p, n, r32, b, nkp, roles):
    R29 = 1 << (W * n)
    assert p < R29 and (n - 1) * W < p.bit_length()
    bounds = check_bounds(p, n, nkp, roles)
    inv = (-pow(p, -1, 1 << 32)) % (1 << 32)
    print("struct %s {  // R29 = 2^%d; loop bounds x < %.2fp, y < %.2fp, zz, zzz < %.2fp"
          % (name, W * n, bounds["X"], bounds["Y"], bounds["Z"]))
    print("  static constexpr int N = %d;" % n)
    print("  static constexpr uint32_t MOD[N] = %s;" % arr(limbs(p, n)))
    print("  static constexpr uint32_t INV = 0x%xu;  // -p^-1 mod 2^32 (used mod 2^29)" % inv)
    print("  static constexpr uint32_t ONE[N] = %s;  // R29 mod p" % arr(limbs(R29 % p, n)))
    e29 = 2 * W * n - r32
    print("  static constexpr uint32_t TO29[N] = %s;  // 2^%d mod p: mont29(x 2^%d, TO29) = x R29"
          % (arr(limbs((1 << e29) % p, n)), e29, r32))
    print("  static constexpr uint32_t TO32[N] = %s;  // 2^%d mod p: mont29(x R29, TO32) = x 2^%d"
          % (arr(limbs((1 << r32) % p, n)), r32, r32))
    print("  static constexpr uint32_t R2[N] = %s;  // R29^2 mod p: mont29(x, R2) = x R29" % arr(limbs(R29 * R29 % p, n)))
    print("  static constexpr uint32_t BCURVE[N] = %s;  // %d R29 mod p (y^2 = x^3 + %d)" % (arr(limbs(b * R29 % p, n)), b, b))
    for k in (1, 2, 4, 8, 16, 32, 64):
        print("  static constexpr uint32_t B%d[N] = %s;  // %d p, biased limbs" % (k, arr(biased(k, p, n)), k))
    for k in (4, 8):
        print("  static constexpr uint32_t C%d[N] = %s;  // %d p, limbs in [3 (2^29 - 1), 2^31) (sub3_29)"
              % (k, arr(biased3(k, p, n)), k))
    print("  // roles (tools/gen_params29.py check_bounds): the bias of each subtraction in acc_loop29 / dbl_affine29")
    for role, k in roles.items():
        kind = "C" if role == "ACC_X3" else "B"
        print("  static constexpr const uint32_t (&%s)[N] = %s%d;" % (role, kind, k))
    print("  static constexpr const uint32_t (&ACC_X3_B)[N] = B%d;  // ACC_X3 for two carry passes (A/B build)"
          % roles["ACC_X3"])
    print("  static constexpr int NKP = %d;" % nkp)
    print("  static constexpr uint32_t KP_LO[NKP] = %s;  // low limb of k p" % arr([(k * p) & MASK for k in range(nkp)]))
    print("  static constexpr uint32_t KP[NKP][N] = {%s};  // k p" % ", ".join(arr(limbs(k * p, n)) for k in range(nkp)))
    print("};\n")


def main():
    print("// GENERATED by tools/gen_params29.py -- do not edit.  Fp in radix 2^29: BLS12-381 (14 limbs,")
    print("// R29 = 2^406) and BN254 (9 limbs, R29 = 2^261).")
    print("#pragma once")
    print("#include <cstdint>\n")
    print("namespace kzgmi {\n")
    for c in CURVES:
        emit(*c)
    print("}  // namespace kzgmi")


if __name__ == "__main__":
    main()
