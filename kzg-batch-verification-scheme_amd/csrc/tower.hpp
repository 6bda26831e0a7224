// Extension-field tower for the pairing (hot-path row a7 of SURVEY.md 8a).
//
//   Fp2 = Fp[u]/(u^2+1),  Fp6 = Fp2[v]/(v^3 - xi),  Fp12 = Fp6[w]/(w^2 - v)
//   BLS12-381: xi = 1+u (M-type twist);  BN254: xi = 9+u (D-type twist).
//
// Algorithms: Karatsuba Fp2/Fp6 products, complex squaring, Granger-Scott cyclotomic
// squaring, sparse products with the line shapes of each twist, Frobenius via precomputed
// gamma_{k,i} = xi^(i(p^k-1)/6) (tools/gen_params.py).  Reference: none (LICENSE only);
// checked against the C oracle / Python spec (tests/test_gpu_parity.py).
#pragma once
#include "field.hpp"
#include "params_gen.hpp"

#define KZ_CALL __device__ __noinline__

namespace kzgmi {

// Field multiplication as a real call: the tower/pairing path is latency-bound and a fully
// inlined Fp12 product (54 Fp products) costs minutes of compile time per instance.
template <class P>
KZ_CALL Fp<P> fp_mul_c(const Fp<P>& a, const Fp<P>& b) { return fp_mul(a, b); }

// ============================================================================ curve traits
struct Bls12_381 {
  using FpP = Bls12_381FpParams;
  using FrP = Bls12_381FrParams;
  using K = Bls12_381Consts;
  static constexpr bool M_TWIST = true;
  static constexpr int FP_BYTES = 48;
  static constexpr int ID = 0;
};
struct Bn254 {
  using FpP = Bn254FpParams;
  using FrP = Bn254FrParams;
  using K = Bn254Consts;
  static constexpr bool M_TWIST = false;
  static constexpr int FP_BYTES = 32;
  static constexpr int ID = 1;
};

// ============================================================================ Fp2
template <class Cv>
struct Fp2 {
  using F = Fp<typename Cv::FpP>;
  F c0, c1;
  KZ_DEV static Fp2 zero() { return {F::zero(), F::zero()}; }
  KZ_DEV static Fp2 one() { return {F::one(), F::zero()}; }
  KZ_DEV bool is_zero() const { return c0.is_zero() && c1.is_zero(); }
  KZ_DEV bool operator==(const Fp2& o) const { return c0 == o.c0 && c1 == o.c1; }
};

template <class Cv> KZ_DEV Fp2<Cv> f2_add(const Fp2<Cv>& a, const Fp2<Cv>& b) { return {fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)}; }
template <class Cv> KZ_DEV Fp2<Cv> f2_sub(const Fp2<Cv>& a, const Fp2<Cv>& b) { return {fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)}; }
template <class Cv> KZ_DEV Fp2<Cv> f2_neg(const Fp2<Cv>& a) { return {fp_neg(a.c0), fp_neg(a.c1)}; }
template <class Cv> KZ_DEV Fp2<Cv> f2_dbl(const Fp2<Cv>& a) { return {fp_dbl(a.c0), fp_dbl(a.c1)}; }
template <class Cv> KZ_DEV Fp2<Cv> f2_conj(const Fp2<Cv>& a) { return {a.c0, fp_neg(a.c1)}; }

template <class Cv>
KZ_CALL Fp2<Cv> f2_mul(const Fp2<Cv>& a, const Fp2<Cv>& b) {
  auto t0 = fp_mul_c(a.c0, b.c0);
  auto t1 = fp_mul_c(a.c1, b.c1);
  auto t2 = fp_mul_c(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return {fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1)};
}
template <class Cv>
KZ_CALL Fp2<Cv> f2_sqr(const Fp2<Cv>& a) {
  auto t = fp_mul_c(a.c0, a.c1);
  return {fp_mul_c(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1)), fp_dbl(t)};
}
template <class Cv>
KZ_DEV Fp2<Cv> f2_mul_fp(const Fp2<Cv>& a, const typename Fp2<Cv>::F& s) { return {fp_mul_c(a.c0, s), fp_mul_c(a.c1, s)}; }

// multiply by xi
template <class Cv>
KZ_DEV Fp2<Cv> f2_mul_xi(const Fp2<Cv>& a) {
  if constexpr (Cv::ID == 0) {  // (a0 + a1 u)(1 + u) = (a0 - a1) + (a0 + a1) u
    return {fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)};
  } else {  // (a0 + a1 u)(9 + u) = (9a0 - a1) + (a0 + 9a1) u
    auto n0 = fp_add(fp_mul8(a.c0), a.c0);
    auto n1 = fp_add(fp_mul8(a.c1), a.c1);
    return {fp_sub(n0, a.c1), fp_add(a.c0, n1)};
  }
}
template <class Cv>
KZ_CALL Fp2<Cv> f2_inv(const Fp2<Cv>& a) {
  auto n = fp_add(fp_mul_c(a.c0, a.c0), fp_mul_c(a.c1, a.c1));
  auto ni = fp_inv(n);
  return {fp_mul_c(a.c0, ni), fp_neg(fp_mul_c(a.c1, ni))};
}
template <class Cv>
KZ_DEV Fp2<Cv> f2_const(const uint32_t (&c)[2][Cv::FpP::N]) {
  return {Fp2<Cv>::F::from_const(c[0]), Fp2<Cv>::F::from_const(c[1])};
}

// ============================================================================ Fp6
template <class Cv>
struct Fp6 {
  Fp2<Cv> c0, c1, c2;
  KZ_DEV static Fp6 zero() { return {Fp2<Cv>::zero(), Fp2<Cv>::zero(), Fp2<Cv>::zero()}; }
  KZ_DEV static Fp6 one() { return {Fp2<Cv>::one(), Fp2<Cv>::zero(), Fp2<Cv>::zero()}; }
};
template <class Cv> KZ_DEV Fp6<Cv> f6_add(const Fp6<Cv>& a, const Fp6<Cv>& b) { return {f2_add(a.c0, b.c0), f2_add(a.c1, b.c1), f2_add(a.c2, b.c2)}; }
template <class Cv> KZ_DEV Fp6<Cv> f6_sub(const Fp6<Cv>& a, const Fp6<Cv>& b) { return {f2_sub(a.c0, b.c0), f2_sub(a.c1, b.c1), f2_sub(a.c2, b.c2)}; }
template <class Cv> KZ_DEV Fp6<Cv> f6_neg(const Fp6<Cv>& a) { return {f2_neg(a.c0), f2_neg(a.c1), f2_neg(a.c2)}; }
// v * (a0 + a1 v + a2 v^2) = xi a2 + a0 v + a1 v^2
template <class Cv> KZ_DEV Fp6<Cv> f6_mul_v(const Fp6<Cv>& a) { return {f2_mul_xi(a.c2), a.c0, a.c1}; }

template <class Cv>
KZ_CALL Fp6<Cv> f6_mul(const Fp6<Cv>& a, const Fp6<Cv>& b) {
  auto t0 = f2_mul(a.c0, b.c0);
  auto t1 = f2_mul(a.c1, b.c1);
  auto t2 = f2_mul(a.c2, b.c2);
  // c0 = t0 + xi((a1+a2)(b1+b2) - t1 - t2)
  auto c0 = f2_add(t0, f2_mul_xi(f2_sub(f2_sub(f2_mul(f2_add(a.c1, a.c2), f2_add(b.c1, b.c2)), t1), t2)));
  // c1 = (a0+a1)(b0+b1) - t0 - t1 + xi t2
  auto c1 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c1), f2_add(b.c0, b.c1)), t0), t1), f2_mul_xi(t2));
  // c2 = (a0+a2)(b0+b2) - t0 - t2 + t1
  auto c2 = f2_add(f2_sub(f2_sub(f2_mul(f2_add(a.c0, a.c2), f2_add(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
}
template <class Cv>
KZ_CALL Fp6<Cv> f6_sqr(const Fp6<Cv>& a) {  // CH-SQR2
  auto s0 = f2_sqr(a.c0);
  auto ab = f2_mul(a.c0, a.c1);
  auto s1 = f2_dbl(ab);
  auto s2 = f2_sqr(f2_add(f2_sub(a.c0, a.c1), a.c2));
  auto bc = f2_mul(a.c1, a.c2);
  auto s3 = f2_dbl(bc);
  auto s4 = f2_sqr(a.c2);
  auto c0 = f2_add(f2_mul_xi(s3), s0);
  auto c1 = f2_add(f2_mul_xi(s4), s1);
  auto c2 = f2_sub(f2_sub(f2_add(f2_add(s1, s2), s3), s0), s4);
  return {c0, c1, c2};
}
template <class Cv>
KZ_DEV Fp6<Cv> f6_mul_fp2(const Fp6<Cv>& a, const Fp2<Cv>& s) { return {f2_mul(a.c0, s), f2_mul(a.c1, s), f2_mul(a.c2, s)}; }

template <class Cv>
KZ_CALL Fp6<Cv> f6_inv(const Fp6<Cv>& a) {
  auto t0 = f2_sub(f2_sqr(a.c0), f2_mul_xi(f2_mul(a.c1, a.c2)));
  auto t1 = f2_sub(f2_mul_xi(f2_sqr(a.c2)), f2_mul(a.c0, a.c1));
  auto t2 = f2_sub(f2_sqr(a.c1), f2_mul(a.c0, a.c2));
  auto d = f2_add(f2_mul(a.c0, t0), f2_mul_xi(f2_add(f2_mul(a.c2, t1), f2_mul(a.c1, t2))));
  auto di = f2_inv(d);
  return {f2_mul(t0, di), f2_mul(t1, di), f2_mul(t2, di)};
}

// ============================================================================ Fp12
template <class Cv>
struct Fp12 {
  Fp6<Cv> c0, c1;
  KZ_DEV static Fp12 one() { return {Fp6<Cv>::one(), Fp6<Cv>::zero()}; }
};

template <class Cv>
KZ_CALL Fp12<Cv> f12_mul(const Fp12<Cv>& a, const Fp12<Cv>& b) {
  auto t0 = f6_mul(a.c0, b.c0);
  auto t1 = f6_mul(a.c1, b.c1);
  auto c1 = f6_sub(f6_sub(f6_mul(f6_add(a.c0, a.c1), f6_add(b.c0, b.c1)), t0), t1);
  auto c0 = f6_add(t0, f6_mul_v(t1));
  return {c0, c1};
}
template <class Cv>
KZ_CALL Fp12<Cv> f12_sqr(const Fp12<Cv>& a) {  // complex squaring
  auto ab = f6_mul(a.c0, a.c1);
  auto t = f6_mul(f6_add(a.c0, a.c1), f6_add(a.c0, f6_mul_v(a.c1)));
  auto c0 = f6_sub(f6_sub(t, ab), f6_mul_v(ab));
  auto c1 = f6_add(ab, ab);
  return {c0, c1};
}
template <class Cv>
KZ_DEV Fp12<Cv> f12_conj(const Fp12<Cv>& a) { return {a.c0, f6_neg(a.c1)}; }

template <class Cv>
KZ_CALL Fp12<Cv> f12_inv(const Fp12<Cv>& a) {
  // (c0 + c1 w)^-1 = (c0 - c1 w) / (c0^2 - v c1^2)
  auto t = f6_sub(f6_mul(a.c0, a.c0), f6_mul_v(f6_mul(a.c1, a.c1)));
  auto ti = f6_inv(t);
  return {f6_mul(a.c0, ti), f6_neg(f6_mul(a.c1, ti))};
}

template <class Cv>
KZ_DEV bool f12_is_one(const Fp12<Cv>& a) {
  auto one = Fp2<Cv>::one();
  return a.c0.c0 == one && a.c0.c1.is_zero() && a.c0.c2.is_zero() && a.c1.c0.is_zero() &&
         a.c1.c1.is_zero() && a.c1.c2.is_zero();
}

// Frobenius f -> f^(p^k), k = 1..3.  Coefficient of w^i (i = 0..5) is multiplied by
// gamma_{k,i} after conjugation (odd k).  w^i order: c0.c0=w^0, c1.c0=w^1, c0.c1=w^2,
// c1.c1=w^3, c0.c2=w^4, c1.c2=w^5.
template <class Cv, int k>
KZ_CALL Fp12<Cv> f12_frob(const Fp12<Cv>& a) {
  using K = typename Cv::K;
  auto fr = [&](const Fp2<Cv>& x, int i) {
    Fp2<Cv> y = (k & 1) ? f2_conj(x) : x;
    if (i == 0) return y;
    return f2_mul(y, f2_const<Cv>(K::FROB[k - 1][i]));
  };
  Fp12<Cv> r;
  r.c0.c0 = fr(a.c0.c0, 0);
  r.c1.c0 = fr(a.c1.c0, 1);
  r.c0.c1 = fr(a.c0.c1, 2);
  r.c1.c1 = fr(a.c1.c1, 3);
  r.c0.c2 = fr(a.c0.c2, 4);
  r.c1.c2 = fr(a.c1.c2, 5);
  return r;
}

// Granger-Scott cyclotomic squaring (valid after the easy part of the final exponentiation).
// View f as Fp4^3: pairs (g0,g1) = (c0.c0, c1.c1), (g2,g3) = (c1.c0, c0.c2), (g4,g5) = (c0.c1, c1.c2).
template <class Cv>
KZ_DEV void fp4_sqr(Fp2<Cv>& r0, Fp2<Cv>& r1, const Fp2<Cv>& a, const Fp2<Cv>& b) {
  auto t0 = f2_sqr(a);
  auto t1 = f2_sqr(b);
  r0 = f2_add(f2_mul_xi(t1), t0);
  r1 = f2_sub(f2_sub(f2_sqr(f2_add(a, b)), t0), t1);
}
template <class Cv>
KZ_CALL Fp12<Cv> f12_cyclo_sqr(const Fp12<Cv>& f) {
  Fp2<Cv> t0, t1, t2, t3, t4, t5;
  fp4_sqr(t0, t1, f.c0.c0, f.c1.c1);
  fp4_sqr(t2, t3, f.c1.c0, f.c0.c2);
  fp4_sqr(t4, t5, f.c0.c1, f.c1.c2);
  Fp12<Cv> r;
  // z0 = 3 t0 - 2 z0 ; z1 = 3 t1 + 2 z1   (z0 = c0.c0, z1 = c1.c1)
  r.c0.c0 = f2_add(f2_dbl(f2_sub(t0, f.c0.c0)), t0);
  r.c1.c1 = f2_add(f2_dbl(f2_add(t1, f.c1.c1)), t1);
  // z2 (c1.c0) = 3 xi t5 + 2 z2 ; z3 (c0.c2) = 3 t4 - 2 z3
  auto xt5 = f2_mul_xi(t5);
  r.c1.c0 = f2_add(f2_dbl(f2_add(xt5, f.c1.c0)), xt5);
  r.c0.c2 = f2_add(f2_dbl(f2_sub(t4, f.c0.c2)), t4);
  // z4 (c0.c1) = 3 t2 - 2 z4 ; z5 (c1.c2) = 3 t3 + 2 z5
  r.c0.c1 = f2_add(f2_dbl(f2_sub(t2, f.c0.c1)), t2);
  r.c1.c2 = f2_add(f2_dbl(f2_add(t3, f.c1.c2)), t3);
  return r;
}

// ---------------------------------------------------------------------------- sparse lines
// M-type (BLS12-381) line, scaled by w^3:  l = a + b w^2 + c w^3  -> (c0.c0, c0.c1, c1.c1)
// D-type (BN254)   line:                  l = a + b w   + c w^3  -> (c0.c0, c1.c0, c1.c1)
template <class Cv>
KZ_CALL Fp12<Cv> f12_mul_line(const Fp12<Cv>& f, const Fp2<Cv>& a, const Fp2<Cv>& b, const Fp2<Cv>& c) {
  Fp12<Cv> l;
  l.c0 = Fp6<Cv>::zero();
  l.c1 = Fp6<Cv>::zero();
  if constexpr (Cv::M_TWIST) {
    // l.c0 = (a, b, 0), l.c1 = (0, c, 0)
    // f*l = (f0 + f1 w)(L0 + L1 w) with L0 = a + b v, L1 = c v
    auto t0 = [&]() {  // f0 * (a + b v)
      auto x0 = f2_mul(f.c0.c0, a);
      auto x1 = f2_mul(f.c0.c1, b);
      // (f00 + f01 v + f02 v^2)(a + b v) = f00 a + (f00 b + f01 a) v + (f01 b + f02 a) v^2 + f02 b v^3
      Fp6<Cv> r;
      r.c0 = f2_add(x0, f2_mul_xi(f2_mul(f.c0.c2, b)));
      r.c1 = f2_sub(f2_sub(f2_mul(f2_add(f.c0.c0, f.c0.c1), f2_add(a, b)), x0), x1);
      r.c2 = f2_add(x1, f2_mul(f.c0.c2, a));
      return r;
    }();
    auto t1 = f6_mul_v(f6_mul_fp2(f.c1, c));  // f1 * (c v)
    // c0 = f0 L0 + v (f1 L1) ; c1 = f0 L1 + f1 L0 = (f0+f1)(L0+L1) - f0L0 - f1L1
    Fp6<Cv> L01;
    L01.c0 = a; L01.c1 = f2_add(b, c); L01.c2 = Fp2<Cv>::zero();
    auto s = f6_add(f.c0, f.c1);
    // s * (a + (b+c) v)
    auto y0 = f2_mul(s.c0, a);
    auto y1 = f2_mul(s.c1, L01.c1);
    Fp6<Cv> m;
    m.c0 = f2_add(y0, f2_mul_xi(f2_mul(s.c2, L01.c1)));
    m.c1 = f2_sub(f2_sub(f2_mul(f2_add(s.c0, s.c1), f2_add(a, L01.c1)), y0), y1);
    m.c2 = f2_add(y1, f2_mul(s.c2, a));
    Fp12<Cv> r;
    r.c0 = f6_add(t0, f6_mul_v(t1));
    r.c1 = f6_sub(f6_sub(m, t0), t1);
    return r;
  } else {
    // L0 = a (Fp2 scalar in Fp6), L1 = b + c v
    auto t0 = f6_mul_fp2(f.c0, a);
    auto t1 = [&]() {  // f1 * (b + c v)
      auto x0 = f2_mul(f.c1.c0, b);
      auto x1 = f2_mul(f.c1.c1, c);
      Fp6<Cv> r;
      r.c0 = f2_add(x0, f2_mul_xi(f2_mul(f.c1.c2, c)));
      r.c1 = f2_sub(f2_sub(f2_mul(f2_add(f.c1.c0, f.c1.c1), f2_add(b, c)), x0), x1);
      r.c2 = f2_add(x1, f2_mul(f.c1.c2, b));
      return r;
    }();
    auto s = f6_add(f.c0, f.c1);
    // s * (a + b + c v)
    auto ab = f2_add(a, b);
    auto y0 = f2_mul(s.c0, ab);
    auto y1 = f2_mul(s.c1, c);
    Fp6<Cv> m;
    m.c0 = f2_add(y0, f2_mul_xi(f2_mul(s.c2, c)));
    m.c1 = f2_sub(f2_sub(f2_mul(f2_add(s.c0, s.c1), f2_add(ab, c)), y0), y1);
    m.c2 = f2_add(y1, f2_mul(s.c2, ab));
    Fp12<Cv> r;
    r.c0 = f6_add(t0, f6_mul_v(t1));
    r.c1 = f6_sub(f6_sub(m, t0), t1);
    return r;
  }
}

}  // namespace kzgmi
