// G1 group arithmetic on gfx950 (hot-path row a4 of SURVEY.md 8a).
//
// Accumulators use XYZZ coordinates (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2), the cheapest
// inversion-free mixed addition for a = 0 curves: madd-2008-s = 8M + 2S, add-2008-s =
// 12M + 2S, dbl-2008-s-1 = 6M + 3S (Explicit-Formulas Database).  Infinity is ZZ = 0.
// Inputs are affine Montgomery points (96 B for BLS12-381) -- the layout the bucket
// accumulation gathers through (see msm.hip).  Reference: none (LICENSE only).
#pragma once
#include "tower.hpp"

namespace kzgmi {

// In HBM, affine points sit at a power-of-two stride (BLS12-381: 96 -> 128 B, BN254 64 B as
// is) so that each bucket-accumulation gather touches exactly one 128-B line (BLS12-381's 96 B
// at a 96-B stride touched 1.5 on average: L2-miss traffic of k_accumulate measured 211 B per
// window term, profiles/r01/rocprof_single/pmc_accumulate_single.json).  The slot also holds the
// point in the accumulation's radix-2^29 form in place (msm.hpp store_pt29: 112 B of limbs on
// BLS12-381, 64 B packed on BN254).
template <class Cv>
constexpr int kAffineAlign = 2 * Cv::FpP::N * 4 == 96 ? 128 : 2 * Cv::FpP::N * 4;

template <class Cv>
struct alignas(kAffineAlign<Cv>) Affine {
  using F = Fp<typename Cv::FpP>;
  F x, y;
};

template <class Cv>
struct Xyzz {
  using F = Fp<typename Cv::FpP>;
  F x, y, zz, zzz;
  KZ_DEV static Xyzz inf() { return {F::one(), F::one(), F::zero(), F::zero()}; }
  KZ_DEV bool is_inf() const { return zz.is_zero(); }
};

template <class Cv>
KZ_DEV Xyzz<Cv> xyzz_from_affine(const Affine<Cv>& a) {
  using F = typename Xyzz<Cv>::F;
  return {a.x, a.y, F::one(), F::one()};
}

// 2P, P in XYZZ
template <class Cv>
KZ_DEV Xyzz<Cv> xyzz_dbl(const Xyzz<Cv>& p) {
  auto U = fp_dbl(p.y);
  auto V = fp_sqr(U);
  auto W = fp_mul(U, V);
  auto S = fp_mul(p.x, V);
  auto M = fp_mul3(fp_sqr(p.x));
  Xyzz<Cv> r;
  r.x = fp_sub(fp_sqr(M), fp_dbl(S));
  r.y = fp_sub(fp_mul(M, fp_sub(S, r.x)), fp_mul(W, p.y));
  r.zz = fp_mul(V, p.zz);
  r.zzz = fp_mul(W, p.zzz);
  return r;  // p = inf (zz = 0) gives zz = zzz = 0 again
}

// 2Q, Q affine (mdbl-2008-s-1)
template <class Cv>
KZ_DEV Xyzz<Cv> xyzz_dbl_affine(const Affine<Cv>& q) {
  auto U = fp_dbl(q.y);
  auto V = fp_sqr(U);
  auto W = fp_mul(U, V);
  auto S = fp_mul(q.x, V);
  auto M = fp_mul3(fp_sqr(q.x));
  Xyzz<Cv> r;
  r.x = fp_sub(fp_sqr(M), fp_dbl(S));
  r.y = fp_sub(fp_mul(M, fp_sub(S, r.x)), fp_mul(W, q.y));
  r.zz = V;
  r.zzz = W;
  return r;
}

// P + Q, P in XYZZ, Q affine (not infinity).  madd-2008-s with the exceptional cases.
template <class Cv>
KZ_DEV Xyzz<Cv> xyzz_add_affine(const Xyzz<Cv>& p, const Affine<Cv>& q) {
  using F = typename Xyzz<Cv>::F;
  if (p.is_inf()) return xyzz_from_affine(q);
  auto U2 = fp_mul(q.x, p.zz);
  auto S2 = fp_mul(q.y, p.zzz);
  auto P = fp_sub(U2, p.x);
  auto R = fp_sub(S2, p.y);
  if (P.is_zero()) {
    if (R.is_zero()) return xyzz_dbl_affine(q);
    return Xyzz<Cv>::inf();
  }
  auto PP = fp_sqr(P);
  auto PPP = fp_mul(P, PP);
  auto Q = fp_mul(p.x, PP);
  Xyzz<Cv> r;
  r.x = fp_sub(fp_sub(fp_sqr(R), PPP), fp_dbl(Q));
  r.y = fp_sub(fp_mul(R, fp_sub(Q, r.x)), fp_mul(p.y, PPP));
  r.zz = fp_mul(p.zz, PP);
  r.zzz = fp_mul(p.zzz, PPP);
  (void)F::zero();
  return r;
}

// Canonical coordinates of a lazily reduced ([0, 2p), field.hpp "lazy reduction") point: the
// bucket-accumulation loop (msm.hpp k_accumulate) keeps its running sum that way.
template <class Cv>
KZ_DEV Xyzz<Cv> xyzz_canon(const Xyzz<Cv>& p) {
  return {fp_canon(p.x), fp_canon(p.y), fp_canon(p.zz), fp_canon(p.zzz)};
}

// P + Q, both XYZZ.  add-2008-s with the exceptional cases.
template <class Cv>
KZ_DEV Xyzz<Cv> xyzz_add(const Xyzz<Cv>& p, const Xyzz<Cv>& q) {
  if (p.is_inf()) return q;
  if (q.is_inf()) return p;
  auto U1 = fp_mul(p.x, q.zz);
  auto U2 = fp_mul(q.x, p.zz);
  auto S1 = fp_mul(p.y, q.zzz);
  auto S2 = fp_mul(q.y, p.zzz);
  auto P = fp_sub(U2, U1);
  auto R = fp_sub(S2, S1);
  if (P.is_zero()) {
    if (R.is_zero()) return xyzz_dbl(p);
    return Xyzz<Cv>::inf();
  }
  auto PP = fp_sqr(P);
  auto PPP = fp_mul(P, PP);
  auto Q = fp_mul(U1, PP);
  Xyzz<Cv> r;
  r.x = fp_sub(fp_sub(fp_sqr(R), PPP), fp_dbl(Q));
  r.y = fp_sub(fp_mul(R, fp_sub(Q, r.x)), fp_mul(S1, PPP));
  r.zz = fp_mul(fp_mul(p.zz, q.zz), PP);
  r.zzz = fp_mul(fp_mul(p.zzz, q.zzz), PPP);
  return r;
}

// Call (non-inlined) forms for everything outside the bucket-accumulation hot loop:
// reductions, window combination, generators, fix-ups.  Keeps code size and compile time
// bounded (a fully inlined point addition is ~12k instructions).
template <class Cv>
__device__ __noinline__ Xyzz<Cv> xyzz_add_c(const Xyzz<Cv>& p, const Xyzz<Cv>& q) { return xyzz_add(p, q); }
template <class Cv>
__device__ __noinline__ Xyzz<Cv> xyzz_dbl_c(const Xyzz<Cv>& p) { return xyzz_dbl(p); }
template <class Cv>
__device__ __noinline__ Xyzz<Cv> xyzz_add_affine_c(const Xyzz<Cv>& p, const Affine<Cv>& q) { return xyzz_add_affine(p, q); }
template <class P>
__device__ __noinline__ Fp<P> fp_inv_c(const Fp<P>& a) { return fp_inv(a); }

template <class Cv>
KZ_DEV Xyzz<Cv> xyzz_neg(const Xyzz<Cv>& p) { return {p.x, fp_neg(p.y), p.zz, p.zzz}; }

// XYZZ -> affine; returns false for infinity.  One inversion of ZZ*ZZZ.
template <class Cv>
KZ_DEV bool xyzz_to_affine(const Xyzz<Cv>& p, Affine<Cv>& out) {
  if (p.is_inf()) return false;
  auto I = fp_inv_c(fp_mul(p.zz, p.zzz));
  out.x = fp_mul(p.x, fp_mul(p.zzz, I));
  out.y = fp_mul(p.y, fp_mul(p.zz, I));
  return true;
}

template <class Cv>
KZ_DEV bool affine_on_curve(const Affine<Cv>& a) {
  using F = typename Affine<Cv>::F;
  auto l = fp_sqr(a.y);
  auto r = fp_add(fp_mul(fp_sqr(a.x), a.x), F::from_const(Cv::K::B_M));
  return l == r;
}

}  // namespace kzgmi
