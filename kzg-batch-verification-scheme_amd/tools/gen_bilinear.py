"""Generate csrc/bilinear_gen.hpp: one-round bilinear programs for the wavefront-parallel pairing.

Every Fp12 operation of the pairing (Karatsuba multiplication, complex squaring,
Granger-Scott cyclotomic squaring, sparse line products, Frobenius, the steps of the Fp12
inversion, line evaluation) has the shape

    out_k = sum_t c_kt * X_t  +  sum_j d_kj * (L_j . R_j)

where X_t are input Fp coefficients, L_j / R_j are linear forms (small integer coefficients)
over the inputs (or constants), and c, d are small integers.  Symbolically executing the
tower formulas with "linear-form" field elements yields those tables.  On the GPU one
workgroup evaluates a table in one round: lane j computes L_j, R_j and one Montgomery
product, then lane k sums its output -- the latency of ONE Fp product instead of ~54 in a row.

Sources: 0 = operand A, 1 = operand B, 2 = constant table (Frobenius gammas, per curve).
Reference: none (LICENSE only); formulas as in csrc/tower.hpp; tables are self-checked here
numerically against direct tower arithmetic on random inputs, and on the GPU against the oracle.

    python kzg-batch-verification-scheme_amd/tools/gen_bilinear.py
"""
import os
import random

# ----------------------------------------------------------------------------- symbolic Fp


class Ctx:
    def __init__(self):
        self.prods = []   # list of (left dict, right dict)
        self.cache = {}

    def product(self, L, R):
        # canonical, deduplicate identical products
        key = (tuple(sorted(L.items())), tuple(sorted(R.items())))
        key2 = (key[1], key[0])
        if key in self.cache:
            return self.cache[key]
        if key2 in self.cache:
            return self.cache[key2]
        j = len(self.prods)
        self.prods.append((dict(L), dict(R)))
        self.cache[key] = j
        return j


class S:
    """Symbolic Fp element: linear form {atom: coeff}; atom = ('A'|'B'|'K', i) or ('P', j)."""
    ctx = None

    def __init__(self, d=None):
        self.d = {k: v for k, v in (d or {}).items() if v != 0}

    @staticmethod
    def atom(src, i):
        return S({(src, i): 1})

    @staticmethod
    def zero():
        return S()

    def __add__(self, o):
        d = dict(self.d)
        for k, v in o.d.items():
            d[k] = d.get(k, 0) + v
        return S(d)

    def __sub__(self, o):
        d = dict(self.d)
        for k, v in o.d.items():
            d[k] = d.get(k, 0) - v
        return S(d)

    def __neg__(self):
        return S({k: -v for k, v in self.d.items()})

    def smul(self, c):
        return S({k: v * c for k, v in self.d.items()})

    def is_zero(self):
        return not self.d

    def __mul__(self, o):
        if self.is_zero() or o.is_zero():
            return S()
        for k in list(self.d) + list(o.d):
            assert k[0] != "P", "operand depends on a product: not a one-round map"
        # pure constant x constant never happens here
        j = S.ctx.product(self.d, o.d)
        return S({("P", j): 1})


# ----------------------------------------------------------------------------- tower (symbolic)
class F2:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    @staticmethod
    def zero():
        return F2(S.zero(), S.zero())

    def __add__(self, o): return F2(self.c0 + o.c0, self.c1 + o.c1)
    def __sub__(self, o): return F2(self.c0 - o.c0, self.c1 - o.c1)
    def __neg__(self): return F2(-self.c0, -self.c1)
    def dbl(self): return self + self
    def conj(self): return F2(self.c0, -self.c1)
    def is_zero(self): return self.c0.is_zero() and self.c1.is_zero()

    def __mul__(self, o):
        if self.is_zero() or o.is_zero():
            return F2.zero()
        if self.c1.is_zero() and o.c1.is_zero():
            return F2(self.c0 * o.c0, S.zero())
        if self.c1.is_zero():
            return F2(self.c0 * o.c0, self.c0 * o.c1)
        if o.c1.is_zero():
            return F2(self.c0 * o.c0, self.c1 * o.c0)
        t0 = self.c0 * o.c0
        t1 = self.c1 * o.c1
        t2 = (self.c0 + self.c1) * (o.c0 + o.c1)
        return F2(t0 - t1, t2 - t0 - t1)

    def sqr(self):
        if self.c1.is_zero():
            return F2(self.c0 * self.c0, S.zero())
        t = self.c0 * self.c1
        return F2((self.c0 + self.c1) * (self.c0 - self.c1), t + t)

    def mul_fp(self, s):
        return F2(self.c0 * s, self.c1 * s)

    def mul_xi(self, curve):
        if curve == "bls12_381":
            return F2(self.c0 - self.c1, self.c0 + self.c1)
        return F2(self.c0.smul(9) - self.c1, self.c0 + self.c1.smul(9))


class F6:
    def __init__(self, c0, c1, c2, curve):
        self.c0, self.c1, self.c2, self.cv = c0, c1, c2, curve

    def __add__(self, o): return F6(self.c0 + o.c0, self.c1 + o.c1, self.c2 + o.c2, self.cv)
    def __sub__(self, o): return F6(self.c0 - o.c0, self.c1 - o.c1, self.c2 - o.c2, self.cv)
    def __neg__(self): return F6(-self.c0, -self.c1, -self.c2, self.cv)
    def mul_v(self): return F6(self.c2.mul_xi(self.cv), self.c0, self.c1, self.cv)

    def __mul__(self, b):
        a = self
        t0, t1, t2 = a.c0 * b.c0, a.c1 * b.c1, a.c2 * b.c2
        c0 = t0 + ((a.c1 + a.c2) * (b.c1 + b.c2) - t1 - t2).mul_xi(self.cv)
        c1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1 + t2.mul_xi(self.cv)
        c2 = (a.c0 + a.c2) * (b.c0 + b.c2) - t0 - t2 + t1
        return F6(c0, c1, c2, self.cv)

    def mul_f2(self, s): return F6(self.c0 * s, self.c1 * s, self.c2 * s, self.cv)


class F12:
    def __init__(self, c0, c1):
        self.c0, self.c1 = c0, c1

    def __mul__(self, b):
        a = self
        t0 = a.c0 * b.c0
        t1 = a.c1 * b.c1
        c1 = (a.c0 + a.c1) * (b.c0 + b.c1) - t0 - t1
        return F12(t0 + t1.mul_v(), c1)

    def sqr(self):
        ab = self.c0 * self.c1
        t = (self.c0 + self.c1) * (self.c0 + self.c1.mul_v())
        return F12(t - ab - ab.mul_v(), ab + ab)

    def conj(self): return F12(self.c0, -self.c1)

    def coeffs(self):  # tower order: c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2 (each c0, c1)
        out = []
        for f6 in (self.c0, self.c1):
            for f2 in (f6.c0, f6.c1, f6.c2):
                out += [f2.c0, f2.c1]
        return out


def f12_from(src, cv):
    a = [S.atom(src, i) for i in range(12)]
    f2 = [F2(a[2 * k], a[2 * k + 1]) for k in range(6)]
    return F12(F6(f2[0], f2[1], f2[2], cv), F6(f2[3], f2[4], f2[5], cv))


def fp4_sqr(a, b, cv):
    t0 = a.sqr()
    t1 = b.sqr()
    return t1.mul_xi(cv) + t0, (a + b).sqr() - t0 - t1


def cyclo_sqr(f, cv):
    z0, z1 = f.c0.c0, f.c1.c1
    z2, z3 = f.c1.c0, f.c0.c2
    z4, z5 = f.c0.c1, f.c1.c2
    t0, t1 = fp4_sqr(z0, z1, cv)
    t2, t3 = fp4_sqr(z2, z3, cv)
    t4, t5 = fp4_sqr(z4, z5, cv)
    r00 = (t0 - z0).dbl() + t0
    r11 = (t1 + z1).dbl() + t1
    xt5 = t5.mul_xi(cv)
    r10 = (xt5 + z2).dbl() + xt5
    r02 = (t4 - z3).dbl() + t4
    r01 = (t2 - z4).dbl() + t2
    r12 = (t3 + z5).dbl() + t3
    return F12(F6(r00, r01, r02, cv), F6(r10, r11, r12, cv))


def line_f12(a, b, c, cv):
    """Sparse line as an Fp12: M-type a + b w^2 + c w^3; D-type a + b w + c w^3."""
    z = F2.zero()
    if cv == "bls12_381":
        return F12(F6(a, b, z, cv), F6(z, c, z, cv))
    return F12(F6(a, z, z, cv), F6(b, c, z, cv))


def line_from(src, cv):
    x = [S.atom(src, i) for i in range(6)]
    return line_f12(F2(x[0], x[1]), F2(x[2], x[3]), F2(x[4], x[5]), cv)


# ----------------------------------------------------------------------------- programs
def build_op(fn, cv):
    S.ctx = Ctx()
    outs = fn(cv)
    prods = S.ctx.prods
    return prods, outs


def op_mul(cv):
    return (f12_from("A", cv) * f12_from("B", cv)).coeffs()


def op_sqr(cv):
    return f12_from("A", cv).sqr().coeffs()


def op_cyc(cv):
    return cyclo_sqr(f12_from("A", cv), cv).coeffs()


def op_conj(cv):
    return f12_from("A", cv).conj().coeffs()


def op_line(cv):  # f * line(B)
    return (f12_from("A", cv) * line_from("B", cv)).coeffs()


def op_ll(cv):  # line(A) * line(B)
    return (line_from("A", cv) * line_from("B", cv)).coeffs()


def op_frob(k):
    def fn(cv):
        f = f12_from("A", cv)
        out = []
        # w^i order: c0.c0 w0, c1.c0 w1, c0.c1 w2, c1.c1 w3, c0.c2 w4, c1.c2 w5
        pos = {("c0", 0): 0, ("c1", 0): 1, ("c0", 1): 2, ("c1", 1): 3, ("c0", 2): 4, ("c1", 2): 5}
        res = {}
        for half in ("c0", "c1"):
            f6 = getattr(f, half)
            for j, f2 in enumerate((f6.c0, f6.c1, f6.c2)):
                i = pos[(half, j)]
                y = f2.conj() if k & 1 else f2
                if i > 0:
                    g = F2(S.atom("K", 12 * (k - 1) + 2 * i), S.atom("K", 12 * (k - 1) + 2 * i + 1))
                    y = y * g
                res[(half, j)] = y
        for half in ("c0", "c1"):
            for j in range(3):
                out += [res[(half, j)].c0, res[(half, j)].c1]
        return out
    return fn


# Fp12 inverse, split in one-round stages (A/B = stage inputs)
def op_inv_norm(cv):  # A = f (12) -> t = c0^2 - v c1^2 (Fp6, 6)
    f = f12_from("A", cv)
    t = f.c0 * f.c0 - (f.c1 * f.c1).mul_v()
    return [t.c0.c0, t.c0.c1, t.c1.c0, t.c1.c1, t.c2.c0, t.c2.c1]


def f6_from(src, cv):
    a = [S.atom(src, i) for i in range(6)]
    return F6(F2(a[0], a[1]), F2(a[2], a[3]), F2(a[4], a[5]), cv)


def op_inv6_t(cv):  # A = a (Fp6) -> (t0, t1, t2)
    a = f6_from("A", cv)
    t0 = a.c0.sqr() - (a.c1 * a.c2).mul_xi(cv)
    t1 = a.c2.sqr().mul_xi(cv) - a.c0 * a.c1
    t2 = a.c1.sqr() - a.c0 * a.c2
    return [t0.c0, t0.c1, t1.c0, t1.c1, t2.c0, t2.c1]


def op_inv6_d(cv):  # A = a (Fp6), B = t (Fp6) -> d = a0 t0 + xi (a2 t1 + a1 t2) (Fp2)
    a = f6_from("A", cv)
    t = f6_from("B", cv)
    d = a.c0 * t.c0 + (a.c2 * t.c1 + a.c1 * t.c2).mul_xi(cv)
    return [d.c0, d.c1]


def op_inv2_n(cv):  # A = d (Fp2) -> d0^2 + d1^2
    d0, d1 = S.atom("A", 0), S.atom("A", 1)
    return [d0 * d0 + d1 * d1]


def op_inv2_fin(cv):  # A = d (2), B = ninv (1) -> (d0 ninv, -d1 ninv)
    d0, d1, ni = S.atom("A", 0), S.atom("A", 1), S.atom("B", 0)
    return [d0 * ni, -(d1 * ni)]


def op_inv6_fin(cv):  # A = t (6), B = dinv (2) -> t * dinv (Fp6)
    t = f6_from("A", cv)
    di = F2(S.atom("B", 0), S.atom("B", 1))
    r = t.mul_f2(di)
    return [r.c0.c0, r.c0.c1, r.c1.c0, r.c1.c1, r.c2.c0, r.c2.c1]


def op_inv12_fin(cv):  # A = f (12), B = tinv (Fp6) -> (c0 tinv, -c1 tinv)
    f = f12_from("A", cv)
    ti = f6_from("B", cv)
    r = F12(f.c0 * ti, -(f.c1 * ti))
    return r.coeffs()


def op_leval(cv):
    """Line value at a homogeneous G1 point.  A = (c.c0, c.c1, lam.c0, lam.c1), B = (X, Y, Z).
    M-type: (c Z, lam X, -Y);  D-type: (-Y, lam X, c Z)  as 3 Fp2 = 6 Fp."""
    c = F2(S.atom("A", 0), S.atom("A", 1))
    lam = F2(S.atom("A", 2), S.atom("A", 3))
    X, Y, Z = S.atom("B", 0), S.atom("B", 1), S.atom("B", 2)
    cz = c.mul_fp(Z)
    lx = lam.mul_fp(X)
    ny = F2(-Y, S.zero())
    if cv == "bls12_381":
        parts = (cz, lx, ny)
    else:
        parts = (ny, lx, cz)
    out = []
    for p in parts:
        out += [p.c0, p.c1]
    return out


OPS = [
    ("MUL", op_mul), ("SQR", op_sqr), ("CYC", op_cyc), ("CONJ", op_conj), ("LINE", op_line), ("LL", op_ll),
    ("FROB1", op_frob(1)), ("FROB2", op_frob(2)), ("FROB3", op_frob(3)),
    ("INV_NORM", op_inv_norm), ("INV6_T", op_inv6_t), ("INV6_D", op_inv6_d), ("INV2_N", op_inv2_n),
    ("INV2_FIN", op_inv2_fin), ("INV6_FIN", op_inv6_fin), ("INV12_FIN", op_inv12_fin), ("LEVAL", op_leval),
]

SRC = {"A": 0, "B": 1, "K": 2}

# ----------------------------------------------------------------------------- numeric self-check
P = {"bls12_381": 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB,
     "bn254": 21888242871839275222246405745257275088696311157297823662689037894645226208583}
XI = {"bls12_381": (1, 1), "bn254": (9, 1)}


def f2m(a, b, p):
    return ((a[0] * b[0] - a[1] * b[1]) % p, (a[0] * b[1] + a[1] * b[0]) % p)


def f2pow(a, e, p):
    r = (1, 0)
    for bit in bin(e)[2:]:
        r = f2m(r, r, p)
        if bit == "1":
            r = f2m(r, a, p)
    return r


def consts(cv):
    p = P[cv]
    out = []
    for k in (1, 2, 3):
        for i in range(6):
            g = f2pow(XI[cv], i * (p ** k - 1) // 6, p)
            out += [g[0], g[1]]
    return out


def evaluate(prods, outs, A, B, K, p):
    def ev(d, pv):
        s = 0
        for (src, i), c in d.items():
            if src == "A":
                s += c * A[i]
            elif src == "B":
                s += c * B[i]
            elif src == "K":
                s += c * K[i]
            else:
                s += c * pv[i]
        return s % p
    pv = [ev(L, None) * ev(R, None) % p for L, R in prods]
    return [ev(o.d, pv) for o in outs]


# direct numeric tower for the check (schoolbook over w: Fp12 = Fp2[w]/(w^6 - xi))
def to_w(c12):
    # tower coeff order -> w-power order list of Fp2
    f2 = [(c12[2 * k], c12[2 * k + 1]) for k in range(6)]  # c0.c0,c0.c1,c0.c2,c1.c0,c1.c1,c1.c2
    return [f2[0], f2[3], f2[1], f2[4], f2[2], f2[5]]


def from_w(w):
    order = [w[0], w[2], w[4], w[1], w[3], w[5]]
    out = []
    for x in order:
        out += [x[0], x[1]]
    return out


def wmul(a, b, cv):
    p = P[cv]
    r = [(0, 0)] * 12
    for i in range(6):
        for j in range(6):
            t = f2m(a[i], b[j], p)
            r[i + j] = ((r[i + j][0] + t[0]) % p, (r[i + j][1] + t[1]) % p)
    out = []
    for k in range(6):
        hi = f2m(r[k + 6], XI[cv], p)
        out.append(((r[k][0] + hi[0]) % p, (r[k][1] + hi[1]) % p))
    return out


def selfcheck(cv, tables):
    p = P[cv]
    rnd = random.Random(1)
    K = consts(cv)
    A = [rnd.randrange(p) for _ in range(12)]
    B = [rnd.randrange(p) for _ in range(12)]
    prods, outs = tables["MUL"]
    assert evaluate(prods, outs, A, B, K, p) == from_w(wmul(to_w(A), to_w(B), cv)), "MUL"
    prods, outs = tables["SQR"]
    assert evaluate(prods, outs, A, B, K, p) == from_w(wmul(to_w(A), to_w(A), cv)), "SQR"
    # frobenius = A^(p^k)
    for k in (1, 2, 3):
        prods, outs = tables["FROB%d" % k]
        got = evaluate(prods, outs, A, B, K, p)
        w = to_w(A)
        r = [(1, 0)] + [(0, 0)] * 5
        # naive power would be too slow; check frob1 via frob1(a*b) == frob1(a)*frob1(b)
        got_b = evaluate(prods, outs, B, A, K, p)
        ab = from_w(wmul(to_w(A), to_w(B), cv))
        got_ab = evaluate(prods, outs, ab, A, K, p)
        assert got_ab == from_w(wmul(to_w(got), to_w(got_b), cv)), "FROB%d multiplicative" % k
        del r, w
    # inverse pipeline
    f = A

    def run(name, X, Y=None):
        pr, ou = tables[name]
        return evaluate(pr, ou, X, Y or [0] * 12, K, p)
    t = run("INV_NORM", f)
    t6 = run("INV6_T", t)
    d = run("INV6_D", t, t6)
    nrm = run("INV2_N", d)
    ni = [pow(nrm[0], -1, p)]
    di = run("INV2_FIN", d, ni)
    ti = run("INV6_FIN", t6, di)
    finv = run("INV12_FIN", f, ti)
    one = from_w(wmul(to_w(f), to_w(finv), cv))
    assert one == [1] + [0] * 11, "INV"
    # sparse line products
    L = [rnd.randrange(p) for _ in range(6)]
    L2 = [rnd.randrange(p) for _ in range(6)]

    def line_full(x):
        z = (0, 0)
        a, b, c = (x[0], x[1]), (x[2], x[3]), (x[4], x[5])
        if cv == "bls12_381":
            w = [a, z, b, c, z, z]
        else:
            w = [a, b, z, c, z, z]
        return from_w(w)
    assert run("LINE", A, L) == from_w(wmul(to_w(A), to_w(line_full(L)), cv)), "LINE"
    assert run("LL", L, L2) == from_w(wmul(to_w(line_full(L)), to_w(line_full(L2)), cv)), "LL"
    assert run("CONJ", A) == A[:6] + [(-x) % p for x in A[6:]], "CONJ"



# ----------------------------------------------------------------------------- pairing bytecode
# Register file (in Fp units, LDS): [K consts 36][E lines NL*12][P 6][SCAL 4][G0..G15 x 12]
K_ROUND, K_ROUND2, K_COPY, K_INV, K_CYCRUN = 0, 1, 2, 3, 4
OPNUM = {name: i for i, (name, _) in enumerate(OPS)}
NONE = 0xFFFF
LOOP = {"bls12_381": 0xD201000000010000, "bn254": 6 * 4965661367192848881 + 2}
XABS = 0xD201000000010000
BN_U = 4965661367192848881


def naf(k):
    """Non-adjacent form of k > 0, least significant digit first."""
    d = []
    while k:
        z = 2 - (k & 3) if k & 1 else 0
        d.append(z)
        k = (k - z) >> 1
    return d


def loop_digits(cv):
    """The Miller loop's digits below the top one, most significant first (csrc/params_gen.hpp
    LOOP / LOOP_NEG): |x| in binary for BLS12-381, the NAF of 6u + 2 for BN254."""
    lp = LOOP[cv]
    d = naf(lp) if cv == "bn254" else [(lp >> i) & 1 for i in range(lp.bit_length())]
    assert d[-1] == 1 and sum(v << i if v >= 0 else -(1 << i) for i, v in enumerate(d)) == lp
    return d[-2::-1]


def num_lines(cv):
    n = sum(1 + (dg != 0) for dg in loop_digits(cv))
    return n if cv == "bls12_381" else n + 2


class Prog:
    def __init__(self, cv):
        self.cv = cv
        self.nl = num_lines(cv)
        self.R_K = 0
        self.R_E = 36
        self.R_P = self.R_E + 12 * self.nl
        self.R_SCAL = self.R_P + 6
        self.R_G = self.R_SCAL + 4
        self.NG = 16
        self.NR = self.R_G + 12 * self.NG
        self.code = []

    def g(self, i):
        assert 0 <= i < self.NG
        return self.R_G + 12 * i

    def e(self, idx):  # E[idx][0] (12 contiguous: pair 0 then pair 1)
        return self.R_E + 12 * idx

    def op(self, name, a, b, out):
        self._check_alias(name, a, b, out)
        self.code.append([K_ROUND, OPNUM[name], a, NONE if b is None else b, out, 0, 0, 0, 0, 0])

    def op2(self, n1, a1, b1, o1, n2, a2, b2, o2):
        # the two ops of a round run concurrently and write their outputs straight into the register
        # file (pairing_par.hpp): neither output block may overlap any input block of the round or
        # the other output block
        self._check_alias(n1, a1, b1, o1)
        self._check_alias(n2, a2, b2, o2)
        wa1, wb1, no1 = op_shape(n1, self.cv)
        wa2, wb2, no2 = op_shape(n2, self.cv)
        for o, no, name in ((o1, no1, n1), (o2, no2, n2)):
            for x, w in ((a1, wa1), (b1, wb1), (a2, wa2), (b2, wb2)):
                assert not _overlap(o, no, x, w), "%s: output block overlaps an input block of the round" % name
        assert not _overlap(o1, no1, o2, no2), "%s/%s: output blocks overlap" % (n1, n2)
        self.code.append([K_ROUND2, OPNUM[n1], a1, NONE if b1 is None else b1, o1,
                          OPNUM[n2], a2, NONE if b2 is None else b2, o2, 0])

    def copy(self, dst, src):
        self.code.append([K_COPY, 0, src, NONE, dst, 0, 0, 0, 0, 0])

    def inv(self, dst, src):
        self.code.append([K_INV, 0, src, NONE, dst, 0, 0, 0, 0, 0])

    def _check_alias(self, name, a, b, out):
        # outputs are written straight into the register file with no barrier after the round's
        # reads (pairing_par.hpp): the output block [out, out + no) must be disjoint from every
        # input block [a, a + wa), [b, b + wb) -- as ranges, not just distinct starts (an operand may
        # address into the middle of a block, like LL's e(idx) + 6)
        wa, wb, no = op_shape(name, self.cv)
        assert not _overlap(out, no, a, wa), "%s: output block overlaps input A" % name
        assert not _overlap(out, no, b, wb), "%s: output block overlaps input B" % name


def _overlap(x, nx, y, ny):
    """[x, x + nx) and [y, y + ny) intersect (y None or ny 0: no operand)."""
    if y is None or nx == 0 or ny == 0:
        return False
    return x < y + ny and y < x + nx


_SHAPES = {}


def op_shape(name, cv):
    """(words read from A, words read from B, words written) of an op, from its symbolic form."""
    key = (name, cv)
    if key not in _SHAPES:
        saved = S.ctx
        prods, outs = build_op(dict(OPS)[name], cv)
        S.ctx = saved
        w = {"A": 0, "B": 0}
        forms = [f for L, R in prods for f in (L, R)] + [getattr(o, "d", {}) for o in outs]
        for f in forms:
            for k in f:
                if isinstance(k, tuple) and k[0] in w:
                    w[k[0]] = max(w[k[0]], k[1] + 1)
        _SHAPES[key] = (w["A"], w["B"], len(outs))
    return _SHAPES[key]


def build_program(cv):
    P = Prog(cv)
    f, t, g = P.g(0), P.g(1), P.g(2)
    idx = 0
    first = True
    for dg in loop_digits(cv):
        if first:
            P.op("LL", P.e(idx), P.e(idx) + 6, f)
            first = False
        else:
            P.op2("SQR", f, None, t, "LL", P.e(idx), P.e(idx) + 6, g)
            P.op("MUL", t, g, f)
        idx += 1
        if dg:  # the precomputed lines through T and +-Q
            P.op("LL", P.e(idx), P.e(idx) + 6, g)
            P.op("MUL", f, g, t)
            P.copy(f, t)
            idx += 1
    if cv == "bls12_381":
        P.op("CONJ", f, None, t)
        P.copy(f, t)
    else:
        for _ in range(2):
            P.op("LL", P.e(idx), P.e(idx) + 6, g)
            P.op("MUL", f, g, t)
            P.copy(f, t)
            idx += 1
    assert idx == P.nl
    # ---- easy part
    r3, r4, r5, r6, r7 = P.g(3), P.g(4), P.g(5), P.g(6), P.g(7)
    sc = P.R_SCAL
    P.op("INV_NORM", f, None, r3)
    P.op("INV6_T", r3, None, r4)
    P.op("INV6_D", r3, r4, r5)
    P.op("INV2_N", r5, None, sc)
    P.inv(sc + 1, sc)
    P.op("INV2_FIN", r5, sc + 1, r6)
    P.op("INV6_FIN", r4, r6, r3)
    P.op("INV12_FIN", f, r3, r4)
    P.op("CONJ", f, None, r5)
    P.op("MUL", r5, r4, g)
    P.op("FROB2", g, None, r5)
    P.op("MUL", r5, g, r6)           # r6 = gg (cyclotomic)
    gg = r6

    def cyclo_pow(dst, a, tmp, e, conj_reg=None):
        # ping-pong between dst and tmp; a copy only if the result ends in tmp.  conj_reg: signed
        # digits (NAF) -- a^-1 = conj(a) in the cyclotomic subgroup, one CONJ round into conj_reg
        digits = naf(e)[-2::-1] if conj_reg is not None else [(e >> i) & 1 for i in range(e.bit_length() - 2, -1, -1)]
        if conj_reg is not None and -1 in digits:
            P.op("CONJ", a, None, conj_reg)
        cur, oth = None, None
        for dg in digits:
            src = a if cur is None else cur
            nxt = tmp if cur != tmp else dst
            P.op("CYC", src, None, nxt)
            cur = nxt
            if dg:
                nxt = dst if cur == tmp else tmp
                P.op("MUL", cur, a if dg > 0 else conj_reg, nxt)
                cur = nxt
        if cur != dst:
            P.copy(dst, cur)

    def conj(dst, src):
        P.op("CONJ", src, None, dst)

    res = P.g(15)
    if cv == "bls12_381":
        X = XABS
        cyclo_pow(r3, gg, t, X); conj(r4, r3); conj(r5, gg); P.op("MUL", r4, r5, r3)      # a = g^(x-1)
        cyclo_pow(r4, r3, t, X); conj(r5, r4); conj(r4, r3); P.op("MUL", r5, r4, r3)      # a = a^(x-1)
        cyclo_pow(r4, r3, t, X); conj(r5, r4); P.op("FROB1", r3, None, r4); P.op("MUL", r5, r4, f)  # b
        cyclo_pow(r3, f, t, X); conj(r4, r3); cyclo_pow(r3, r4, t, X); conj(r5, r3)       # b^(x^2)
        P.op("FROB2", f, None, r3); P.op("MUL", r5, r3, r4); conj(r3, f); P.op("MUL", r4, r3, r5)  # c
        P.op("CYC", gg, None, r3); P.op("MUL", r3, gg, r4)                                  # g^3
        P.op("MUL", r5, r4, res)
    else:
        U = BN_U
        fu, fu2, fu3 = P.g(8), P.g(9), P.g(10)
        ca = P.g(12)  # conj of the base: free until k_a below
        cyclo_pow(fu, gg, t, U, ca)   # u in NAF: 24 nonzero digits instead of 28 set bits
        cyclo_pow(fu2, fu, t, U, ca)
        cyclo_pow(fu3, fu2, t, U, ca)
        sq = lambda d, a: P.op("CYC", a, None, d)  # noqa: E731
        mul = lambda d, a, b: P.op("MUL", a, b, d)  # noqa: E731
        x1, x2, x3 = r4, r5, r7
        k_t2, k_a, k_b, k_c, k_d, k_e = P.g(11), P.g(12), P.g(13), P.g(14), P.g(3), P.g(0)
        sq(x1, fu2); sq(x2, x1); mul(t, x2, x1); mul(k_t2, t, gg)             # t2 = fu2^6 g
        sq(x3, x2); sq(g, x3); mul(x2, g, x3); mul(k_a, x2, t)                # fu2^30
        mul(k_b, g, x1)                                                       # fu2^18
        sq(x1, fu3); sq(x2, x1); sq(x3, x2); sq(x1, x3); sq(g, x1)             # g = fu3^32, x2 = fu3^4
        mul(k_c, g, x2)                                                       # fu3^36
        sq(x1, fu); sq(x2, x1); sq(x3, x2); mul(k_d, x3, x2)                  # fu^12
        sq(g, x3); mul(k_e, g, x1)                                            # fu^18
        mul(x1, k_c, k_b); mul(x2, x1, k_d); conj(x1, x2); mul(x3, x1, gg)     # t1
        mul(x1, k_c, k_a); mul(x2, x1, k_e); sq(g, gg); mul(t, x2, g); conj(x1, t)  # t0
        P.op("FROB1", x3, None, x2); mul(t, x1, x2)
        P.op("FROB2", k_t2, None, x2); mul(x1, t, x2)
        P.op("FROB3", gg, None, x2); mul(res, x1, x2)
    return P, res


def compress_cyc_runs(P):
    """Runs of >= 2 chained cyclotomic squarings (cyclo_pow's zero digits: s0 -> u, u -> v, v -> u,
    ...) become one K_CYCRUN [4, n, s0, u, v]: the interpreter runs the n rounds back to back
    without decoding each (pairing_par.hpp)."""
    cyc = OPNUM["CYC"]
    out, i = [], 0
    code = P.code
    while i < len(code):
        ins = code[i]
        if ins[0] == K_ROUND and ins[1] == cyc:
            s0, u = ins[2], ins[4]
            j, cur, other = i + 1, u, None
            while j < len(code) and code[j][0] == K_ROUND and code[j][1] == cyc and code[j][2] == cur:
                o = code[j][4]
                if other is None:
                    if o in (cur, s0) and o != s0:
                        break
                    if o == cur:
                        break
                    other = o
                elif o != (other if cur == u else u):
                    break
                cur = o
                j += 1
            n = j - i
            if n >= 2 and other is not None:
                out.append([K_CYCRUN, n, s0, u, other, 0, 0, 0, 0, 0])
                i = j
                continue
        out.append(ins)
        i += 1
    P.code = out


def check_program(cv, tables, P, res):
    """Run the bytecode numerically on random line values and compare with a direct
    evaluation (Miller product over the same lines, naive final exponentiation)."""
    p = globals()["P"][cv]
    rnd = random.Random(7)
    K = consts(cv)
    R = [0] * P.NR
    R[P.R_K:P.R_K + 36] = K
    nl = P.nl
    for i in range(nl * 12):
        R[P.R_E + i] = rnd.randrange(p)
    names = [n for n, _ in OPS]
    for ins in P.code:
        kind = ins[0]
        if kind in (K_ROUND, K_ROUND2):
            insts = [ins[1:5]] + ([ins[5:9]] if kind == K_ROUND2 else [])
            outs = []
            for opn, a, b, o in insts:
                pr, ou = tables[names[opn]]
                A = R[a:a + 12]
                B = R[b:b + 12] if b != NONE else [0] * 12
                outs.append((o, evaluate(pr, ou, A, B, K, p)))
            for o, vals in outs:
                R[o:o + len(vals)] = vals
        elif kind == K_CYCRUN:
            pr, ou = tables["CYC"]
            src, dst = ins[2], ins[3]
            for _ in range(ins[1]):
                R[dst:dst + 12] = evaluate(pr, ou, R[src:src + 12], [0] * 12, K, p)
                src, dst = dst, (ins[4] if dst == ins[3] else ins[3])
        elif kind == K_COPY:
            R[ins[4]:ins[4] + 12] = R[ins[2]:ins[2] + 12]
        elif kind == K_INV:
            R[ins[4]] = pow(R[ins[2]], -1, p)
    got = R[res:res + 12]

    def line_full(x):
        z = (0, 0)
        a, b, c = (x[0], x[1]), (x[2], x[3]), (x[4], x[5])
        return from_w([a, z, b, c, z, z] if cv == "bls12_381" else [a, b, z, c, z, z])
    one = [1] + [0] * 11
    f = one
    idx = 0
    first = True
    for dg in loop_digits(cv):
        l = from_w(wmul(to_w(line_full(R[P.R_E + 12 * idx:P.R_E + 12 * idx + 6])),
                        to_w(line_full(R[P.R_E + 12 * idx + 6:P.R_E + 12 * idx + 12])), cv))
        f = l if first else from_w(wmul(to_w(from_w(wmul(to_w(f), to_w(f), cv))), to_w(l), cv))
        first = False
        idx += 1
        if dg:
            l = from_w(wmul(to_w(line_full(R[P.R_E + 12 * idx:P.R_E + 12 * idx + 6])),
                            to_w(line_full(R[P.R_E + 12 * idx + 6:P.R_E + 12 * idx + 12])), cv))
            f = from_w(wmul(to_w(f), to_w(l), cv))
            idx += 1
    if cv == "bls12_381":
        f = f[:6] + [(-x) % p for x in f[6:]]
    else:
        for _ in range(2):
            l = from_w(wmul(to_w(line_full(R[P.R_E + 12 * idx:P.R_E + 12 * idx + 6])),
                            to_w(line_full(R[P.R_E + 12 * idx + 6:P.R_E + 12 * idx + 12])), cv))
            f = from_w(wmul(to_w(f), to_w(l), cv))
            idx += 1
    r_ord = {"bls12_381": 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001,
             "bn254": 21888242871839275222246405745257275088548364400416034343698204186575808495617}[cv]
    e = (p ** 12 - 1) // r_ord * (3 if cv == "bls12_381" else 1)
    acc = one
    w = to_w(f)
    a = to_w(acc)
    for bit in bin(e)[2:]:
        a = wmul(a, a, cv)
        if bit == "1":
            a = wmul(a, w, cv)
    want = from_w(a)
    assert got == want, "bytecode program mismatch for %s" % cv

# ----------------------------------------------------------------------------- emit
def emit():
    lines = ["// GENERATED by tools/gen_bilinear.py -- do not edit.",
             "// One-round bilinear programs for the wavefront-parallel pairing (pairing_par.hpp).",
             "#pragma once", "#include <hip/hip_runtime.h>", "#include <cstdint>", "namespace kzgmi {", ""]
    stats = {}
    for cv, tag in (("bls12_381", "Bls"), ("bn254", "Bn")):
        tables = {name: build_op(fn, cv) for name, fn in OPS}
        selfcheck(cv, tables)
        # flatten: terms are (src<<5 | idx, coeff)
        terms = []
        desc = []
        for name, _ in OPS:
            prods, outs = tables[name]
            base_prod = len(terms)
            prod_idx = []
            for L, R in prods:
                for side in (L, R):
                    prod_idx.append(len(terms))
                    for (src, i), c in sorted(side.items()):
                        terms.append((SRC[src] << 6 | i, c))
                    terms.append((255, 0))  # end marker
            out_idx = []
            for o in outs:
                out_idx.append(len(terms))
                for (src, i), c in sorted(o.d.items(), key=lambda kv: (kv[0][0] != "P", kv[0])):
                    code = (3 << 6 | i) if src == "P" else (SRC[src] << 6 | i)
                    terms.append((code, c))
                terms.append((255, 0))
            desc.append((name, len(prods), len(outs), prod_idx, out_idx))
            stats[(cv, name)] = (len(prods), len(outs), max([len(o.d) for o in outs] or [0]))
        assert len(terms) < 65536
        pfx = "k%s_" % tag
        nl = 12 if cv == "bls12_381" else 8
        R = 1 << (32 * nl)
        Kv = [k * R % p_mod for k in consts(cv)] if (p_mod := P[cv]) else []
        lines.append("static __constant__ uint8_t %sTERM_CODE[%d] = {%s};" % (pfx, len(terms), ", ".join(str(t[0]) for t in terms)))
        lines.append("static __constant__ int8_t %sTERM_COEF[%d] = {%s};" % (pfx, len(terms), ", ".join(str(t[1]) for t in terms)))
        lines.append("static __constant__ uint32_t %sK[36][%d] = {%s};" % (pfx, nl, ", ".join(
            "{" + ", ".join("0x%08xu" % ((v >> (32 * i)) & 0xffffffff) for i in range(nl)) + "}" for v in Kv)))
        for name, np_, no, pidx, oidx in desc:
            lines.append("// %s: %d products, %d outputs" % (name, np_, no))
            lines.append("static __constant__ uint16_t %s%s_P[%d] = {%s};" % (pfx, name, max(1, len(pidx)), ", ".join(map(str, pidx or [0]))))
            lines.append("static __constant__ uint16_t %s%s_O[%d] = {%s};" % (pfx, name, len(oidx), ", ".join(map(str, oidx))))
        prog, res = build_program(cv)
        n_before = len(prog.code)
        compress_cyc_runs(prog)
        print("%s: %d instructions, %d after CYC runs" % (cv, n_before, len(prog.code)))
        check_program(cv, tables, prog, res)
        flat = [v for ins in prog.code for v in ins]
        lines.append("static __constant__ uint16_t %sPROG[%d] = {%s};" % (pfx, len(flat), ", ".join(map(str, flat))))
        lines.append("struct %sOpsInfo {" % tag)
        lines.append("  static constexpr int NTERMS = %d;" % len(terms))
        lines.append("  static constexpr int NPROG = %d, R_K = %d, R_E = %d, R_P = %d, R_SCAL = %d, R_G = %d, NR = %d, R_RES = %d;" % (
            len(prog.code), prog.R_K, prog.R_E, prog.R_P, prog.R_SCAL, prog.R_G, prog.NR, res))
        stats[(cv, "PROGRAM")] = (len(prog.code), sum(1 for i in prog.code if i[0] in (0, 1)), 0)
        for name, np_, no, pidx, oidx in desc:
            lines.append("  static constexpr int %s_NP = %d, %s_NO = %d;" % (name, np_, name, no))
        lines.append("};")
        lines.append("")
    lines.append("}  // namespace kzgmi")
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc", "bilinear_gen.hpp")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    for k, v in sorted(stats.items()):
        print("%-10s %-10s products=%3d outputs=%2d max_out_terms=%d" % (k[0], k[1], v[0], v[1], v[2]))
    print("wrote", path)


if __name__ == "__main__":
    emit()
