// Compressed G1 inputs and the G1 subgroup check ("point decompression
// (48 B -> affine) + G1 subgroup check on the GPU", the step in front of batch_verify for
// Ethereum-format inputs).  Reference: none (LICENSE only); semantics fixed by
// oracle/pyspec/kzg.py (g1_from_bytes_compressed) and checked against the C oracle.
//
// Formats (big-endian x, flags in the top bits of byte 0):
//   BLS12-381, 48 B (ZCash):  0x80 compressed (required), 0x40 infinity (then byte 0 = 0xc0,
//                             rest zero), 0x20 y is the larger root (y > (p-1)/2)
//   BN254, 32 B (gnark-crypto): top two bits 0b10 smaller root, 0b11 larger root,
//                             0b01 infinity (rest zero); 0b00 is invalid here
// y = (x^3 + b)^((p+1)/4) (both p = 3 mod 4), rejected unless it squares back.
//
// Subgroup test (BLS12-381 only; BN254 G1 has cofactor 1): P in G1 <=> phi(P) = [-x^2] P with
// phi(x, y) = (beta x, y) (Scott, "A note on group membership tests for G1, G2 and GT on
// BLS pairing-friendly curves", 2021).  [x^2]P = [|x|]([|x|]P): 2 x 63 doublings + 2 x 5
// additions in Jacobian coordinates, one thread per point; beta is chosen in
// tools/gen_params.py by checking the identity on the generator.
#pragma once
#include <type_traits>

#include "field29.hpp"
#include "kernels.hpp"

namespace kzgmi {

// ---- BLS12-381 in radix 2^29 (field29.hpp): the square root's 375 squarings and the
// membership test's 126 doublings are throughput-bound chains of products, and a radix-29
// squaring is 301 mads instead of ~650 VALU instructions for a 32-bit-limb product (round 2:
// the convert phase of a compressed 2^20 batch 59 -> ~40 ms).  Value bounds per step below.
using Q29 = Bls12_381Fp29;
using G29 = F29<Q29>;

KZ_DEV G29 sel8_29(uint32_t k, const G29 (&t)[8]) {
  G29 r = t[0];
#pragma unroll
  for (int j = 1; j < 8; ++j)
    if (k == (uint32_t)j) r = t[j];
  return r;
}

// (x^3 + b)^((p+1)/4) for BLS12-381 in radix 2^29: the generated width-4 window of fp_pow_sqrt
template <class P>
KZ_DEV Fp<P> fp_pow_sqrt29(const Fp<P>& a) {
  const G29 x = fp_to29<Q29>(a);
  const G29 x2 = sqr29(x);
  G29 t[8];
  t[0] = x;
#pragma unroll
  for (int j = 1; j < 8; ++j) t[j] = mul29(t[j - 1], x2);
  G29 acc = sel8_29((uint32_t)P::SQRT_FIRST, t);
  for (int s = 0; s < P::SQRT_STEPS; ++s) {
    const int nsq = P::SQRT_SQR[s];
    for (int q = 0; q < nsq; ++q) acc = sqr29(acc);
    const uint32_t k = P::SQRT_IDX[s];
    if (k != 255u) acc = mul29(acc, sel8_29(k, t));
  }
  return fp_from29<Q29, P>(acc);
}

KZ_DEV G29 dbl29(const G29& a) { return add3_29(a, a, G29::zero()); }

// a = 0 Jacobian point in radix 2^29 with an explicit infinity flag (exact; no zero test of Z)
struct Jac29 {
  G29 x, y, z;
  bool inf;
};

// dbl-2009-l.  Inputs X < 34p, Y < 18p, Z < 8p  ->  X3 < 34p, Y3 < 18p, Z3 < 4p
KZ_DEV Jac29 jac29_dbl(const Jac29& p) {
  const G29 A = sqr29(p.x), B = sqr29(p.y), C = sqr29(B);                        // < 2p
  const G29 D0 = sqr29(add3_29(p.x, B, G29::zero()));                           // < 2p
  const G29 D = dbl29(sub29(sub29(D0, A, Q29::B2), C, Q29::B2));                // < 12p
  const G29 E = add3_29(A, A, A);                                              // < 6p
  Jac29 r;
  r.x = sub29(sqr29(E), dbl29(D), Q29::B32);                                    // < 34p
  r.y = sub29(mul29(E, sub29(D, r.x, Q29::B64)), dbl29(dbl29(dbl29(C))), Q29::B16);  // < 18p
  r.z = dbl29(mul29(p.y, p.z));                                                 // < 4p
  r.inf = p.inf;
  return r;
}

// v == 0 mod p for any v < 2^12 p (one product by the Montgomery one brings it below 2p)
KZ_DEV bool zero29(const G29& v) { return is_zero29(mul29(v, G29::from_const(Q29::ONE))); }

// p + q, q affine (< 2p; madd-2007-bl).  p: X < 34p, Y < 18p, Z < 8p -> X3, Y3, Z3 < 8p
__device__ __noinline__ Jac29 jac29_add_affine(const Jac29& p, const G29& qx, const G29& qy) {
  if (p.inf) return {qx, qy, G29::from_const(Q29::ONE), false};
  const G29 Z1Z1 = sqr29(p.z);
  const G29 U2 = mul29(qx, Z1Z1);
  const G29 S2 = mul29(qy, mul29(p.z, Z1Z1));
  const G29 H = sub29(U2, p.x, Q29::B64);                                       // < 66p
  const G29 rr = dbl29(sub29(S2, p.y, Q29::B32));                               // < 68p
  if (zero29(H)) {
    if (zero29(rr)) return jac29_dbl({qx, qy, G29::from_const(Q29::ONE), false});
    Jac29 o = p;
    o.inf = true;
    return o;
  }
  const G29 HH = sqr29(H);
  const G29 I = dbl29(dbl29(HH));                                               // < 8p
  const G29 J = mul29(H, I), V = mul29(p.x, I);
  Jac29 r;
  r.x = sub29(sub29(sqr29(rr), J, Q29::B2), dbl29(V), Q29::B4);                 // < 8p
  r.y = sub29(mul29(rr, sub29(V, r.x, Q29::B8)), dbl29(mul29(p.y, J)), Q29::B4);  // < 6p
  r.z = sub29(sub29(sqr29(add3_29(p.z, H, G29::zero())), Z1Z1, Q29::B2), HH, Q29::B2);  // < 6p
  r.inf = false;
  return r;
}

// p + q, both Jacobian (add-2007-bl); inputs as jac29_dbl's outputs -> X3 < 8p, Y3 < 6p, Z3 < 2p
__device__ __noinline__ Jac29 jac29_add(const Jac29& p, const Jac29& q) {
  if (p.inf) return q;
  if (q.inf) return p;
  const G29 Z1Z1 = sqr29(p.z), Z2Z2 = sqr29(q.z);
  const G29 U1 = mul29(p.x, Z2Z2), U2 = mul29(q.x, Z1Z1);
  const G29 S1 = mul29(p.y, mul29(q.z, Z2Z2)), S2 = mul29(q.y, mul29(p.z, Z1Z1));
  const G29 H = sub29(U2, U1, Q29::B2);                                         // < 4p
  const G29 rr = dbl29(sub29(S2, S1, Q29::B2));                                 // < 8p
  if (is_zero29(H)) {
    if (is_zero29(rr)) return jac29_dbl(p);
    Jac29 o = p;
    o.inf = true;
    return o;
  }
  const G29 I = sqr29(dbl29(H));
  const G29 J = mul29(H, I), V = mul29(U1, I);
  Jac29 r;
  r.x = sub29(sub29(sqr29(rr), J, Q29::B2), dbl29(V), Q29::B4);                 // < 8p
  r.y = sub29(mul29(rr, sub29(V, r.x, Q29::B8)), dbl29(mul29(S1, J)), Q29::B4);   // < 6p
  r.z = mul29(sub29(sub29(sqr29(add3_29(p.z, q.z, G29::zero())), Z1Z1, Q29::B2), Z2Z2, Q29::B2), H);  // < 2p
  r.inf = false;
  return r;
}

// dst = src through empty asm statements: a value the compiler cannot merge with src, so src
// keeps its registers and only dst lives in the call frame
KZ_DEV void g29_opaque_copy(G29& d, const G29& s) {
#pragma unroll
  for (int k = 0; k < Q29::N; ++k) asm volatile("" : "=v"(d.v[k]) : "0"(s.v[k]));
}
KZ_DEV void jac29_opaque_copy(Jac29& d, const Jac29& s) {
  g29_opaque_copy(d.x, s.x);
  g29_opaque_copy(d.y, s.y);
  g29_opaque_copy(d.z, s.z);
  d.inf = s.inf;
}

// [|x|] q (BLS parameter bit pattern), radix 2^29: the doublings run in call-free loops between
// the parameter's few set bits and the (out-of-line) additions sit between the loops.  One loop
// over all 63 bits with the conditional call inside kept the running point in the call frame:
// ~40 scratch dwordx4 stores + loads per doubling, 0.65 KB of scratch per lane.
template <class Cv, bool AFFINE>
KZ_DEV Jac29 mul_by_x_abs29(const Jac29& q, const G29& qx, const G29& qy) {
  constexpr uint64_t X = Cv::K::X_ABS;
  static_assert(X >> 63, "top bit set: the chain starts from q");
  Jac29 acc = q;  // top bit
  int b = 63;     // acc = [X >> b] q
  for (int k = 62; k >= 0; --k) {
    if (!((X >> k) & 1)) continue;  // uniform, compile-time pattern: the set bits below the top
#pragma unroll 1
    for (int i = 0; i < b - k; ++i) acc = jac29_dbl(acc);
    // the call's in-memory arguments are copies made here: acc (and q) stay register values in
    // the doubling loops instead of living in the call frame
    Jac29 arg;
    jac29_opaque_copy(arg, acc);
    if constexpr (AFFINE) {
      G29 ax, ay;
      g29_opaque_copy(ax, qx);
      g29_opaque_copy(ay, qy);
      acc = jac29_add_affine(arg, ax, ay);
    } else {
      Jac29 aq;
      jac29_opaque_copy(aq, q);
      acc = jac29_add(arg, aq);
    }
    b = k;
  }
#pragma unroll 1
  for (int i = 0; i < b; ++i) acc = jac29_dbl(acc);
  return acc;
}

// raw (standard-form) a > b
template <class P>
KZ_DEV bool fp_raw_gt(const Fp<P>& a, const uint32_t (&b)[P::N]) {
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < P::N; ++i) (void)__builtin_subc(b[i], a.v[i], bw, &bw);
  return bw != 0;
}

template <class Cv>
__global__ void __launch_bounds__(256) k_decompress_points(const uint8_t* __restrict__ bytes, uint32_t n,
                                                           Affine<Cv>* __restrict__ pts, uint8_t* __restrict__ inf,
                                                           uint32_t* __restrict__ err) {
  using P = typename Cv::FpP;
  using F = Fp<P>;
  constexpr int N = P::N;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[N];
  load_words(bytes + (size_t)i * 4 * N, w);
  const uint32_t b0 = w[0] & 0xffu;  // first byte = low byte of the little-endian word
  uint32_t rest = w[0] & ~0xffu;
#pragma unroll
  for (int k = 1; k < N; ++k) rest |= w[k];
  bool is_inf = false, larger = false, bad = false;
  if constexpr (Cv::ID == 0) {
    if (!(b0 & 0x80u)) bad = true;
    else if (b0 & 0x40u) { is_inf = true; bad = b0 != 0xc0u || rest != 0; }
    else larger = (b0 & 0x20u) != 0;
    w[0] &= ~0xe0u;
  } else {
    const uint32_t m = b0 & 0xc0u;
    if (m == 0x40u) { is_inf = true; bad = b0 != 0x40u || rest != 0; }
    else if (m == 0x80u) larger = false;
    else if (m == 0xc0u) larger = true;
    else bad = true;
    w[0] &= ~0xc0u;
  }
  if (bad) { raise_err(err, DERR_ENCODING); is_inf = true; }
  Affine<Cv> a;
  a.x = F::zero();
  a.y = F::zero();
  if (!is_inf) {
    F x = fp_from_be_words<P>(w, 0);
    if (!fp_raw_lt_mod(x)) {
      raise_err(err, DERR_ENCODING);
      is_inf = true;
    } else {
      a.x = fp_to_mont(x);
      const F rhs = fp_add(fp_mul(fp_sqr(a.x), a.x), F::from_const(Cv::K::B_M));
      F y;
      if constexpr (Cv::ID == 0) y = fp_pow_sqrt29(rhs);
      else y = fp_pow_sqrt(rhs);
      if (!(fp_sqr(y) == rhs)) {
        raise_err(err, DERR_NOT_ON_CURVE);
        is_inf = true;
      } else {
        const F yraw = fp_from_mont(y);
        if (yraw.is_zero() && larger) { raise_err(err, DERR_ENCODING); is_inf = true; }
        if (fp_raw_gt(yraw, P::HALF) != larger) y = fp_neg(y);
        a.y = y;
      }
    }
    if (is_inf) { a.x = F::zero(); a.y = F::zero(); }
  }
  uint32_t o[2 * N];
#pragma unroll
  for (int k = 0; k < N; ++k) { o[k] = a.x.v[k]; o[N + k] = a.y.v[k]; }
  store_words(reinterpret_cast<uint8_t*>(pts + i), o);
  inf[i] = is_inf ? 1 : 0;
}

// one uncompressed G1 encoding (as loaded little-endian words) -> its compressed encoding
// (same word layout; no validation)
template <class Cv>
KZ_DEV void compress_encoding(const uint32_t (&w)[2 * Cv::FpP::N], uint32_t (&o)[Cv::FpP::N]) {
  using P = typename Cv::FpP;
  constexpr int N = P::N;
  uint32_t any = 0;
#pragma unroll
  for (int k = 0; k < 2 * N; ++k) any |= w[k];
#pragma unroll
  for (int k = 0; k < N; ++k) o[k] = w[k];
  const bool is_inf = Cv::ID == 0 ? (w[0] & 0x40u) != 0 : any == 0;
  if (is_inf) {
#pragma unroll
    for (int k = 0; k < N; ++k) o[k] = 0;
    o[0] = Cv::ID == 0 ? 0xc0u : 0x40u;
  } else {
    const bool larger = fp_raw_gt(fp_from_be_words<P>(w, N), P::HALF);
    o[0] |= Cv::ID == 0 ? (0x80u | (larger ? 0x20u : 0u)) : (larger ? 0xc0u : 0x80u);
  }
}

// uncompressed G1 encodings -> compressed (no validation: a test/bench input utility)
template <class Cv>
__global__ void __launch_bounds__(256) k_compress_points(const uint8_t* __restrict__ in, uint32_t n,
                                                         uint8_t* __restrict__ out) {
  constexpr int N = Cv::FpP::N;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[2 * N], o[N];
  load_words(in + (size_t)i * 8 * N, w);
  compress_encoding<Cv>(w, o);
  store_words(out + (size_t)i * 4 * N, o);
}

// ---- Jacobian coordinates for the membership test (x = X/Z^2, y = Y/Z^3, infinity Z = 0):
// the test is ~126 doublings, and a = 0 Jacobian doubling (dbl-2009-l, 2M + 5S = 7 products)
// is cheaper than XYZZ doubling (6M + 3S = 9); the 10 additions cost a little more (madd
// 7M + 4S, add 11M + 5S vs 8M + 2S, 12M + 2S): ~1020 instead of ~1255 products per point.
template <class Cv>
struct Jac {
  using F = Fp<typename Cv::FpP>;
  F x, y, z;
  KZ_DEV bool is_inf() const { return z.is_zero(); }
};

template <class Cv>
KZ_DEV Jac<Cv> jac_dbl(const Jac<Cv>& p) {
  auto A = fp_sqr(p.x);
  auto B = fp_sqr(p.y);
  auto C = fp_sqr(B);
  auto D = fp_dbl(fp_sub(fp_sub(fp_sqr(fp_add(p.x, B)), A), C));
  auto E = fp_mul3(A);
  auto Fv = fp_sqr(E);
  Jac<Cv> r;
  r.x = fp_sub(Fv, fp_dbl(D));
  r.y = fp_sub(fp_mul(E, fp_sub(D, r.x)), fp_mul8(C));
  r.z = fp_dbl(fp_mul(p.y, p.z));
  return r;  // Z = 0 stays 0
}

// p + q, q affine (madd-2007-bl) with the exceptional cases
template <class Cv>
KZ_DEV Jac<Cv> jac_add_affine(const Jac<Cv>& p, const Affine<Cv>& q) {
  using F = typename Jac<Cv>::F;
  if (p.is_inf()) return {q.x, q.y, F::one()};
  auto Z1Z1 = fp_sqr(p.z);
  auto U2 = fp_mul(q.x, Z1Z1);
  auto S2 = fp_mul(q.y, fp_mul(p.z, Z1Z1));
  auto H = fp_sub(U2, p.x);
  auto rr = fp_dbl(fp_sub(S2, p.y));
  if (H.is_zero()) {
    if (rr.is_zero()) return jac_dbl(Jac<Cv>{q.x, q.y, F::one()});
    return {F::one(), F::one(), F::zero()};
  }
  auto HH = fp_sqr(H);
  auto I = fp_mul4(HH);
  auto J = fp_mul(H, I);
  auto V = fp_mul(p.x, I);
  Jac<Cv> r;
  r.x = fp_sub(fp_sub(fp_sqr(rr), J), fp_dbl(V));
  r.y = fp_sub(fp_mul(rr, fp_sub(V, r.x)), fp_dbl(fp_mul(p.y, J)));
  r.z = fp_sub(fp_sub(fp_sqr(fp_add(p.z, H)), Z1Z1), HH);
  return r;
}

// p + q, both Jacobian (add-2007-bl) with the exceptional cases
template <class Cv>
KZ_DEV Jac<Cv> jac_add(const Jac<Cv>& p, const Jac<Cv>& q) {
  using F = typename Jac<Cv>::F;
  if (p.is_inf()) return q;
  if (q.is_inf()) return p;
  auto Z1Z1 = fp_sqr(p.z);
  auto Z2Z2 = fp_sqr(q.z);
  auto U1 = fp_mul(p.x, Z2Z2);
  auto U2 = fp_mul(q.x, Z1Z1);
  auto S1 = fp_mul(p.y, fp_mul(q.z, Z2Z2));
  auto S2 = fp_mul(q.y, fp_mul(p.z, Z1Z1));
  auto H = fp_sub(U2, U1);
  auto rr = fp_dbl(fp_sub(S2, S1));
  if (H.is_zero()) {
    if (rr.is_zero()) return jac_dbl(p);
    return {F::one(), F::one(), F::zero()};
  }
  auto I = fp_sqr(fp_dbl(H));
  auto J = fp_mul(H, I);
  auto V = fp_mul(U1, I);
  Jac<Cv> r;
  r.x = fp_sub(fp_sub(fp_sqr(rr), J), fp_dbl(V));
  r.y = fp_sub(fp_mul(rr, fp_sub(V, r.x)), fp_dbl(fp_mul(S1, J)));
  r.z = fp_mul(fp_sub(fp_sub(fp_sqr(fp_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return r;
}

// [|x|] q by the fixed bit pattern of the BLS parameter (uniform control flow)
template <class Cv, class Base>
KZ_DEV Jac<Cv> mul_by_x_abs(const Base& q, const Jac<Cv>& q_jac) {
  constexpr uint64_t X = Cv::K::X_ABS;
  Jac<Cv> acc = q_jac;  // top bit
  for (int b = 62; b >= 0; --b) {
    acc = jac_dbl(acc);
    if ((X >> b) & 1) {
      if constexpr (std::is_same_v<Base, Affine<Cv>>) acc = jac_add_affine(acc, q);
      else acc = jac_add(acc, q);
    }
  }
  return acc;
}

// Waves per SIMD the membership test is compiled for: 2 (256 VGPRs, no scratch in the doubling
// loops) ran compressed batches at 22.5/s against 19.9 with the compiler's own choice (284
// registers, 1 wave), 22.2 at 3 waves and 21.9 at 4 (profiles/r04/ab_subgroup_check.txt).
#ifndef KZ_SGC_WAVES
#define KZ_SGC_WAVES 2
#endif
template <class Cv>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KZ_SGC_WAVES)))
k_subgroup_check(const Affine<Cv>* __restrict__ pts,
                                                        const uint8_t* __restrict__ inf, uint32_t n,
                                                        uint32_t* __restrict__ err) {
  static_assert(Cv::ID == 0, "BN254 G1 has cofactor 1: no subgroup check");
  using P = typename Cv::FpP;
  using F = Fp<P>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || inf[i]) return;
  const Affine<Cv> p = pts[i];
  // [x^2] p in radix 2^29 (the 126 doublings), then back to the 32-bit form for the comparison
  const G29 px = fp_to29<Q29>(p.x), py = fp_to29<Q29>(p.y);
  const Jac29 q1 = mul_by_x_abs29<Cv, true>({px, py, G29::from_const(Q29::ONE), false}, px, py);
  const Jac29 r2 = mul_by_x_abs29<Cv, false>(q1, px, py);
  const Jac<Cv> q2{fp_from29<Q29, P>(r2.x), fp_from29<Q29, P>(r2.y), r2.inf ? F::zero() : fp_from29<Q29, P>(r2.z)};
  // p in G1 <=> q2 == -phi(p) = (beta x, -y): X2 == beta x Z2^2 and Y2 == -y Z2^3, q2 finite
  const F bx = fp_mul(F::from_const(Cv::K::BETA_M), p.x);
  const F z2 = fp_sqr(q2.z);
  const bool ok = !r2.inf && !q2.is_inf() && q2.x == fp_mul(bx, z2) && q2.y == fp_mul(fp_neg(p.y), fp_mul(z2, q2.z));
  if (!ok) raise_err(err, DERR_NOT_IN_SUBGROUP);
}

}  // namespace kzgmi
