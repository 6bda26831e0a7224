// Two-pair multi-Miller loop + final exponentiation (hot-path row a7 of SURVEY.md 8a).
//
// The G2 side of the KZG check is fixed per SRS ({[1]_2, [tau]_2}), so every Miller-loop
// line is precomputed once by k_precompute_lines and stored as (c = yT - lam xT, lam).
// Evaluated at a homogeneous G1 point (X', Y', Z') = (X ZZZ, Y ZZ, ZZ ZZZ) built straight from
// the MSM's XYZZ output (no inversion):
//   M-type (BLS12-381, line scaled by w^3 Z'):  c Z' + (lam X') w^2 - Y' w^3
//   D-type (BN254, line scaled by Z'):          -Y' + (lam X') w + (c Z') w^3
// Final exponentiation: easy part f^((p^6-1)(p^2+1)), then
//   BLS12-381: 3(p^4-p^2+1)/r = (x-1)^2 (x+p)(x^2+p^2-1) + 3   (Hayashida-Hayasaka-Teruya)
//   BN254:     (p^4-p^2+1)/r  = l0 + l1 p + l2 p^2 + p^3 with l2 = 6u^2+1,
//              l1 = -36u^3-18u^2-12u+1, l0 = -36u^3-30u^2-18u-2
// (both identities are checked numerically in tests/test_pyspec.py).  The BLS12-381 result
// is therefore e^3, matching oracle/pyspec/pairing.py.  Reference: none (LICENSE only).
#pragma once
#include "common.hpp"

namespace kzgmi {

template <class Cv>
struct Line {
  Fp2<Cv> c, lam;
};

template <class Cv>
struct G2Aff {
  Fp2<Cv> x, y;
};

// digit i of the Miller loop scalar: +1 (LOOP), -1 (LOOP_NEG: BN254's 6u + 2 runs in NAF, 21
// additions of +-Q instead of 36 of Q), or 0
template <class Cv>
KZ_DEV int loop_digit(int i) {
  return (int)((Cv::K::LOOP[i >> 5] >> (i & 31)) & 1) - (int)((Cv::K::LOOP_NEG[i >> 5] >> (i & 31)) & 1);
}

template <class Cv>
constexpr int num_lines() {
  int n = 0;
  for (int i = Cv::K::LOOP_BITS - 2; i >= 0; --i) {
    n += 1;
    n += ((Cv::K::LOOP[i >> 5] | Cv::K::LOOP_NEG[i >> 5]) >> (i & 31)) & 1;
  }
  return Cv::M_TWIST ? n : n + 2;
}

template <class Cv>
KZ_DEV G2Aff<Cv> g2_frob(const G2Aff<Cv>& q) {
  using K = typename Cv::K;
  return {f2_mul(f2_conj(q.x), f2_const<Cv>(K::FROB[0][2])), f2_mul(f2_conj(q.y), f2_const<Cv>(K::FROB[0][3]))};
}

// T = T + Q (Q != +-T) and T = 2T, recording the line.
template <class Cv>
KZ_DEV void line_add(G2Aff<Cv>& T, const G2Aff<Cv>& Q, Line<Cv>& L) {
  auto lam = f2_mul(f2_sub(Q.y, T.y), f2_inv(f2_sub(Q.x, T.x)));
  L.lam = lam;
  L.c = f2_sub(T.y, f2_mul(lam, T.x));
  auto x3 = f2_sub(f2_sub(f2_sqr(lam), T.x), Q.x);
  auto y3 = f2_sub(f2_mul(lam, f2_sub(T.x, x3)), T.y);
  T.x = x3;
  T.y = y3;
}
template <class Cv>
KZ_DEV void line_dbl(G2Aff<Cv>& T, Line<Cv>& L) {
  auto x2 = f2_sqr(T.x);
  auto lam = f2_mul(f2_add(f2_dbl(x2), x2), f2_inv(f2_dbl(T.y)));
  L.lam = lam;
  L.c = f2_sub(T.y, f2_mul(lam, T.x));
  auto x3 = f2_sub(f2_sqr(lam), f2_dbl(T.x));
  auto y3 = f2_sub(f2_mul(lam, f2_sub(T.x, x3)), T.y);
  T.x = x3;
  T.y = y3;
}

// One thread per G2 point (2 threads).  Input: affine twist points in Montgomery form.
template <class Cv>
__global__ void k_precompute_lines(const G2Aff<Cv>* __restrict__ q_in, Line<Cv>* __restrict__ lines) {
  int k = threadIdx.x;
  if (k >= 2) return;
  constexpr int NL = num_lines<Cv>();
  Line<Cv>* out = lines + k * NL;
  G2Aff<Cv> Q = q_in[k];
  const G2Aff<Cv> negQ = {Q.x, f2_neg(Q.y)};
  G2Aff<Cv> T = Q;
  int idx = 0;
  for (int i = Cv::K::LOOP_BITS - 2; i >= 0; --i) {
    line_dbl(T, out[idx++]);
    const int d = loop_digit<Cv>(i);
    if (d) line_add(T, d > 0 ? Q : negQ, out[idx++]);  // the line through T and -Q for a -1 digit
  }
  if constexpr (!Cv::M_TWIST) {
    G2Aff<Cv> Q1 = g2_frob(Q);
    G2Aff<Cv> Q2 = g2_frob(Q1);
    Q2.y = f2_neg(Q2.y);
    line_add(T, Q1, out[idx++]);
    line_add(T, Q2, out[idx++]);
  }
}

template <class Cv>
struct Homog {
  Fp<typename Cv::FpP> X, Y, Z;
};

template <class Cv>
KZ_DEV Homog<Cv> homog_from_xyzz(const Xyzz<Cv>& p, bool negate) {
  Homog<Cv> h;
  h.X = fp_mul(p.x, p.zzz);
  h.Y = fp_mul(p.y, p.zz);
  if (negate) h.Y = fp_neg(h.Y);
  h.Z = fp_mul(p.zz, p.zzz);
  return h;
}

template <class Cv>
KZ_DEV Fp12<Cv> mul_line_at(const Fp12<Cv>& f, const Line<Cv>& L, const Homog<Cv>& P) {
  using F = Fp<typename Cv::FpP>;
  Fp2<Cv> ny = {fp_neg(P.Y), F::zero()};
  Fp2<Cv> b = f2_mul_fp(L.lam, P.X);
  Fp2<Cv> cz = f2_mul_fp(L.c, P.Z);
  if constexpr (Cv::M_TWIST) return f12_mul_line(f, cz, b, ny);
  else return f12_mul_line(f, ny, b, cz);
}

// f = prod_k f_{loop, Q_k}(P_k) with precomputed lines; P_k skipped if flagged infinity.
template <class Cv>
KZ_DEV Fp12<Cv> miller2(const Line<Cv>* lines, const Homog<Cv> (&P)[2], const bool (&skip)[2]) {
  constexpr int NL = num_lines<Cv>();
  Fp12<Cv> f = Fp12<Cv>::one();
  int idx = 0;
  for (int i = Cv::K::LOOP_BITS - 2; i >= 0; --i) {
    f = f12_sqr(f);
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if (!skip[k]) f = mul_line_at(f, lines[k * NL + idx], P[k]);
    ++idx;
    if (loop_digit<Cv>(i)) {  // the precomputed line through T and +-Q
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (!skip[k]) f = mul_line_at(f, lines[k * NL + idx], P[k]);
      ++idx;
    }
  }
  if constexpr (Cv::M_TWIST) {
    f = f12_conj(f);  // x < 0
  } else {
    for (int e = 0; e < 2; ++e) {
#pragma unroll
      for (int k = 0; k < 2; ++k)
        if (!skip[k]) f = mul_line_at(f, lines[k * NL + idx], P[k]);
      ++idx;
    }
  }
  return f;
}

// g^e for a 64-bit e by cyclotomic square-and-multiply (g in the cyclotomic subgroup)
template <class Cv>
KZ_DEV Fp12<Cv> cyclo_pow_u64(const Fp12<Cv>& g, uint64_t e) {
  Fp12<Cv> acc = g;
  int top = 63 - __builtin_clzll(e);
  for (int i = top - 1; i >= 0; --i) {
    acc = f12_cyclo_sqr(acc);
    if ((e >> i) & 1) acc = f12_mul(acc, g);
  }
  return acc;
}

template <class Cv>
KZ_DEV Fp12<Cv> final_exp(const Fp12<Cv>& f) {
  // easy part
  Fp12<Cv> g = f12_mul(f12_conj(f), f12_inv(f));
  g = f12_mul(f12_frob<Cv, 2>(g), g);
  if constexpr (Cv::ID == 0) {
    const uint64_t X = Cv::K::X_ABS;  // x = -X
    auto pow_x = [&](const Fp12<Cv>& a) { return f12_conj(cyclo_pow_u64(a, X)); };  // a^x
    Fp12<Cv> a = f12_mul(pow_x(g), f12_conj(g));            // g^(x-1)
    a = f12_mul(pow_x(a), f12_conj(a));                      // g^((x-1)^2)
    Fp12<Cv> b = f12_mul(pow_x(a), f12_frob<Cv, 1>(a));      // a^(x+p)
    Fp12<Cv> c = f12_mul(f12_mul(pow_x(pow_x(b)), f12_frob<Cv, 2>(b)), f12_conj(b));  // b^(x^2+p^2-1)
    Fp12<Cv> g3 = f12_mul(f12_cyclo_sqr(g), g);
    return f12_mul(c, g3);
  } else {
    const uint64_t U = Cv::K::U;
    Fp12<Cv> fu = cyclo_pow_u64(g, U);
    Fp12<Cv> fu2 = cyclo_pow_u64(fu, U);
    Fp12<Cv> fu3 = cyclo_pow_u64(fu2, U);
    auto sq = [&](const Fp12<Cv>& a) { return f12_cyclo_sqr(a); };
    // powers by small constants
    Fp12<Cv> fu2_2 = sq(fu2), fu2_4 = sq(fu2_2), fu2_6 = f12_mul(fu2_4, fu2_2);
    Fp12<Cv> fu2_16 = sq(sq(fu2_4)), fu2_18 = f12_mul(fu2_16, fu2_2);
    Fp12<Cv> fu2_30 = f12_mul(f12_mul(fu2_16, sq(fu2_4)), fu2_6);  // 16 + 8 + 6
    Fp12<Cv> fu3_4 = sq(sq(fu3)), fu3_32 = sq(sq(sq(fu3_4))), fu3_36 = f12_mul(fu3_32, fu3_4);
    Fp12<Cv> fu_2 = sq(fu), fu_4 = sq(fu_2), fu_8 = sq(fu_4), fu_12 = f12_mul(fu_8, fu_4);
    Fp12<Cv> fu_16 = sq(fu_8), fu_18 = f12_mul(fu_16, fu_2);
    // g^l2 = fu2^6 g ; g^l1 = conj(fu3^36 fu2^18 fu^12) g ; g^l0 = conj(fu3^36 fu2^30 fu^18 g^2)
    Fp12<Cv> t2 = f12_mul(fu2_6, g);
    Fp12<Cv> t1 = f12_mul(f12_conj(f12_mul(f12_mul(fu3_36, fu2_18), fu_12)), g);
    Fp12<Cv> t0 = f12_conj(f12_mul(f12_mul(f12_mul(fu3_36, fu2_30), fu_18), sq(g)));
    Fp12<Cv> r = f12_mul(t0, f12_frob<Cv, 1>(t1));
    r = f12_mul(r, f12_frob<Cv, 2>(t2));
    r = f12_mul(r, f12_frob<Cv, 3>(g));
    return r;
  }
}

}  // namespace kzgmi
