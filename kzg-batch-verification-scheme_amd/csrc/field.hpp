// Montgomery prime-field arithmetic for gfx950 (CDNA4), 32-bit limbs in VGPRs.
//
// Hot-path layer L1 of SURVEY.md section 1 ("Fp<Params> Montgomery mul/sqr/add ... in
// registers", BASELINE.json:5).  Reference: none -- /root/reference holds only LICENSE
// (LICENSE:1-201); the semantics are fixed by oracle/pyspec and checked against the C oracle.
//
// Design notes (MI355X):
//  * Limbs are 32-bit so every limb product is one v_mad_u64_u32 (32x32+64 -> 64); measured
//    ~27 T mad/s chip-wide on MI355X (scratch/ubench.hip), i.e. the multiply pipe, not HBM,
//    bounds every kernel built on this (SURVEY.md section 7 "the real roofline is not HBM").
//  * Multiplication is CIOS with the "no-carry" shortcut: every modulus used here has its
//    top limb < 0x7ffffffe (BLS12-381 p/r, BN254 p/r), so the t[N]/t[N+1] words of textbook
//    CIOS are never needed and the loop keeps N+0 words live.
//  * Carry chains use __builtin_addc/__builtin_subc -> v_add_co_u32 / v_addc_co_u32.
//  * Everything is fully unrolled with compile-time limb indices so the limbs stay in VGPRs
//    (runtime-indexed arrays would go to scratch: cdna_hip_programming.md 5.4 rule 20).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "bingcd.hpp"

#define KZ_DEV __device__ __forceinline__

namespace kzgmi {

template <class P>
struct Fp {
  static constexpr int N = P::N;
  uint32_t v[N];

  KZ_DEV static Fp zero() { Fp r; _Pragma("unroll") for (int i = 0; i < N; ++i) r.v[i] = 0; return r; }
  KZ_DEV static Fp one() { Fp r; _Pragma("unroll") for (int i = 0; i < N; ++i) r.v[i] = P::ONE[i]; return r; }
  KZ_DEV static Fp from_const(const uint32_t (&c)[N]) { Fp r; _Pragma("unroll") for (int i = 0; i < N; ++i) r.v[i] = c[i]; return r; }
  KZ_DEV bool is_zero() const {
    uint32_t x = 0;
    _Pragma("unroll") for (int i = 0; i < N; ++i) x |= v[i];
    return x == 0;
  }
  KZ_DEV bool operator==(const Fp& o) const {
    uint32_t x = 0;
    _Pragma("unroll") for (int i = 0; i < N; ++i) x |= v[i] ^ o.v[i];
    return x == 0;
  }
  KZ_DEV bool operator!=(const Fp& o) const { return !(*this == o); }
};

// ---------------------------------------------------------------------------- add/sub
template <class P>
KZ_DEV Fp<P> fp_add(const Fp<P>& a, const Fp<P>& b) {
  constexpr int N = P::N;
  Fp<P> s, d;
  uint32_t c = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) d.v[i] = __builtin_subc(s.v[i], P::MOD[i], bw, &bw);
  // a + b < 2p < 2^(32N): no carry out of s; s >= p iff no borrow
  _Pragma("unroll") for (int i = 0; i < N; ++i) s.v[i] = bw ? s.v[i] : d.v[i];
  return s;
}

template <class P>
KZ_DEV Fp<P> fp_sub(const Fp<P>& a, const Fp<P>& b) {
  constexpr int N = P::N;
  Fp<P> d, e;
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) d.v[i] = __builtin_subc(a.v[i], b.v[i], bw, &bw);
  uint32_t c = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) e.v[i] = __builtin_addc(d.v[i], P::MOD[i], c, &c);
  _Pragma("unroll") for (int i = 0; i < N; ++i) d.v[i] = bw ? e.v[i] : d.v[i];
  return d;
}

template <class P>
KZ_DEV Fp<P> fp_dbl(const Fp<P>& a) { return fp_add(a, a); }

template <class P>
KZ_DEV Fp<P> fp_neg(const Fp<P>& a) {
  constexpr int N = P::N;
  Fp<P> d;
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) d.v[i] = __builtin_subc(P::MOD[i], a.v[i], bw, &bw);
  bool z = a.is_zero();
  _Pragma("unroll") for (int i = 0; i < N; ++i) d.v[i] = z ? 0u : d.v[i];
  return d;
}

template <class P>
KZ_DEV Fp<P> fp_select(bool c, const Fp<P>& a, const Fp<P>& b) {
  Fp<P> r;
  _Pragma("unroll") for (int i = 0; i < P::N; ++i) r.v[i] = c ? a.v[i] : b.v[i];
  return r;
}


// ---------------------------------------------------------------------------- mul (product scanning)
// Same result as fp_mul (CIOS), different schedule: column-wise (FIPS) Montgomery with a
// 96-bit column accumulator {acc64, top}.  Each limb product is ONE v_mad_u64_u32 that
// accumulates into the 64-bit pair and writes its carry-out to an SGPR pair, plus ONE
// v_addc_co_u32 folding that carry into `top`.  hipcc's lowering of the CIOS form needs a
// zero-extended 64-bit addend per product (~3 extra v_mov/v_lshl_add per product: measured
// 803 v_mov_b32 per BLS12-381 product in the probe kernel's ISA); this form needs none.
// Each multiply-add is its own asm statement, so hipcc pads every boundary with `s_nop 0`
// (~1 nop per product).  Fusing 2-4 (a*b, m*p) pairs per statement removes them but measured
// no gain (tools/probes/macfuse.hip: 63.2 vs 64.1 G 12x12 products/s -- other waves fill the
// pad) and produced wrong products inside the library kernels (not in the isolated probe).
// Cause (tools/probes/asm_clobber.hip): the fused statements declared the accumulators "+v"
// without early clobber, so hipcc could give an accumulator the register of an input that a
// LATER instruction of the same statement still reads (register allocation decides, hence
// library-only); every output written before a later read needs "&".  The one-product-per-
// statement form below cannot alias and stays (the fusion gained nothing anyway).
KZ_DEV void mac32(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(top)
      : "v"(a), "v"(b));
}
KZ_DEV void mac32s(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b_uniform) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cc), "+v"(top)
      : "v"(a), "s"(b_uniform));
}

// First multiply-add of a column: the carry word starts from this product's carry-out
// (v_addc 0 + 0 + cc) instead of a zeroed register -- hipcc otherwise spends one v_mov per
// column materialising top = 0 (measured: 161 of the 351 v_mov_b32 in the accumulation's
// mixed addition were such zero moves).
KZ_DEV void mac32_first(uint64_t& acc, uint32_t& top, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32_e64 %2, %1, 0, 0, %1"
      : "+v"(acc), "=&s"(cc), "=v"(top)
      : "v"(a), "v"(b));
}

// One column scan for every product form.  TWO: (a b + c d) R^-1 with ONE reduction (the a b,
// c d and m p terms of a column go into the same 96-bit accumulator: <= 36 limb products per
// column).  Returns t = (a b [+ c d] + m p) / R before any final correction.
template <class P, bool TWO>
KZ_DEV Fp<P> mont_scan(const Fp<P>& a, const Fp<P>& b, const Fp<P>& c, const Fp<P>& d) {
  constexpr int N = P::N;
  uint32_t m[N];
  Fp<P> t;
  uint64_t acc = 0;
  uint32_t top;  // written by each column's first multiply-add (mac32_first)
  _Pragma("unroll") for (int k = 0; k < N; ++k) {
    _Pragma("unroll") for (int i = 0; i < k; ++i) {
      if (i == 0) mac32_first(acc, top, a.v[i], b.v[k - i]);
      else mac32(acc, top, a.v[i], b.v[k - i]);
      if constexpr (TWO) mac32(acc, top, c.v[i], d.v[k - i]);
      mac32s(acc, top, m[i], P::MOD[k - i]);
    }
    if (k == 0) mac32_first(acc, top, a.v[k], b.v[0]);
    else mac32(acc, top, a.v[k], b.v[0]);
    if constexpr (TWO) mac32(acc, top, c.v[k], d.v[0]);
    m[k] = (uint32_t)acc * P::INV;
    mac32s(acc, top, m[k], P::MOD[0]);  // low word becomes 0
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  _Pragma("unroll") for (int k = N; k < 2 * N - 1; ++k) {
    _Pragma("unroll") for (int i = k - N + 1; i < N; ++i) {
      if (i == k - N + 1) mac32_first(acc, top, a.v[i], b.v[k - i]);
      else mac32(acc, top, a.v[i], b.v[k - i]);
      if constexpr (TWO) mac32(acc, top, c.v[i], d.v[k - i]);
      mac32s(acc, top, m[i], P::MOD[k - i]);
    }
    t.v[k - N] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
  }
  t.v[N - 1] = (uint32_t)acc;  // < 2^(32N) for every caller's input bound: no further words
  return t;
}

// t >= M ? t - M : t  for a modulus-sized constant M (P::MOD or P::MOD2)
template <class P>
KZ_DEV Fp<P> fp_csub(const Fp<P>& t, const uint32_t (&M)[P::N]) {
  Fp<P> r, d;
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < P::N; ++i) d.v[i] = __builtin_subc(t.v[i], M[i], bw, &bw);
  _Pragma("unroll") for (int i = 0; i < P::N; ++i) r.v[i] = bw ? t.v[i] : d.v[i];
  return r;
}

// canonical inputs < p: (ab + mp)/R < 2p, one conditional subtraction
template <class P>
KZ_DEV Fp<P> fp_mul_ps(const Fp<P>& a, const Fp<P>& b) {
  return fp_csub<P>(mont_scan<P, false>(a, b, a, b), P::MOD);
}

// ---------------------------------------------------------------------------- lazy reduction
// For the bucket-accumulation loop only: values live in [0, 2p) ("lazy") instead of [0, p).
// With 4p < R (BLS12-381: 4p/R = 0.41, BN254: 0.76) the product-scanning Montgomery product
// of two lazy inputs is (ab + mp)/R < p (4p/R + 1) < 2p, so it can skip its final
// conditional subtraction (24 of its 661 VALU instructions); additions and subtractions keep
// the range with one conditional correction by 2p, and zero tests accept {0, p}.  Values are
// made canonical (fp_canon) before they leave the loop.
template <class P>
constexpr bool kFourPBelowR = P::MOD[P::N - 1] < (1u << 30);  // 4p < R = 2^(32N)
template <class P>
constexpr bool kEightPBelowR = P::MOD[P::N - 1] < (1u << 29);

template <class P>
KZ_DEV Fp<P> fp_mul_lazy(const Fp<P>& a, const Fp<P>& b) {
  static_assert(kFourPBelowR<P>, "lazy reduction needs 4p < R");
  return mont_scan<P, false>(a, b, a, b);  // < 2p
}

// (a b + c d) R^-1, lazy inputs <= 2p: < p (8p/R + 1), i.e. < 2p when 8p < R (BLS12-381:
// 8p/R = 0.82); BN254 (8p/R = 1.51, < 2.51p) folds 2p once more.  Replaces two products and an
// addition: 432 instead of 576 multiply-adds.
template <class P>
KZ_DEV Fp<P> fp_mul2_lazy(const Fp<P>& a, const Fp<P>& b, const Fp<P>& c, const Fp<P>& d) {
  static_assert(kFourPBelowR<P>, "lazy reduction needs 4p < R");
  const Fp<P> t = mont_scan<P, true>(a, b, c, d);
  if constexpr (kEightPBelowR<P>) return t;
  else return fp_csub<P>(t, P::MOD2);  // < 2p
}

template <class P>
KZ_DEV Fp<P> fp_neg_lazy(const Fp<P>& a) {  // a < 2p -> 2p - a in (0, 2p] (= -a mod p)
  Fp<P> d;
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < P::N; ++i) d.v[i] = __builtin_subc(P::MOD2[i], a.v[i], bw, &bw);
  return d;
}

template <class P>
KZ_DEV Fp<P> fp_rsub_mod(const Fp<P>& a) {  // a <= p -> p - a in [0, p] (lazy -a)
  Fp<P> d;
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < P::N; ++i) d.v[i] = __builtin_subc(P::MOD[i], a.v[i], bw, &bw);
  return d;
}

template <class P>
KZ_DEV Fp<P> fp_sub_lazy(const Fp<P>& a, const Fp<P>& b) {  // a, b < 2p -> a - b mod p, < 2p
  constexpr int N = P::N;
  Fp<P> d, e;
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) d.v[i] = __builtin_subc(a.v[i], b.v[i], bw, &bw);
  uint32_t c = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) e.v[i] = __builtin_addc(d.v[i], P::MOD2[i], c, &c);
  _Pragma("unroll") for (int i = 0; i < N; ++i) d.v[i] = bw ? e.v[i] : d.v[i];
  return d;
}

template <class P>
KZ_DEV Fp<P> fp_add_lazy(const Fp<P>& a, const Fp<P>& b) {  // a, b < 2p -> a + b mod p, < 2p
  constexpr int N = P::N;
  Fp<P> s, d;
  uint32_t c = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < N; ++i) d.v[i] = __builtin_subc(s.v[i], P::MOD2[i], bw, &bw);
  // a + b < 4p < 2^(32N): no carry out of s; s >= 2p iff no borrow
  _Pragma("unroll") for (int i = 0; i < N; ++i) s.v[i] = bw ? s.v[i] : d.v[i];
  return s;
}

template <class P>
KZ_DEV bool fp_is_zero_lazy(const Fp<P>& a) {  // a < 2p: a = 0 mod p <=> a in {0, p}
  uint32_t z = 0, q = 0;
  _Pragma("unroll") for (int i = 0; i < P::N; ++i) { z |= a.v[i]; q |= a.v[i] ^ P::MOD[i]; }
  return z == 0 || q == 0;
}

template <class P>
KZ_DEV Fp<P> fp_canon(const Fp<P>& a) {  // a < 2p -> a mod p
  return fp_csub<P>(a, P::MOD);
}

// Default multiplication used by every kernel.
template <class P>
KZ_DEV Fp<P> fp_mul(const Fp<P>& a, const Fp<P>& b) {
  return fp_mul_ps(a, b);
}

template <class P>
KZ_DEV Fp<P> fp_sqr(const Fp<P>& a) { return fp_mul(a, a); }

// small constant multiples by addition chains
template <class P>
KZ_DEV Fp<P> fp_mul3(const Fp<P>& a) { return fp_add(fp_add(a, a), a); }
template <class P>
KZ_DEV Fp<P> fp_mul4(const Fp<P>& a) { Fp<P> t = fp_add(a, a); return fp_add(t, t); }
template <class P>
KZ_DEV Fp<P> fp_mul8(const Fp<P>& a) { return fp_dbl(fp_mul4(a)); }

// ---------------------------------------------------------------------------- conversions
template <class P>
KZ_DEV Fp<P> fp_to_mont(const Fp<P>& raw) { return fp_mul(raw, Fp<P>::from_const(P::R2)); }

template <class P>
KZ_DEV Fp<P> fp_from_mont(const Fp<P>& a) {
  Fp<P> one = Fp<P>::zero();
  one.v[0] = 1;
  return fp_mul(a, one);
}

// raw (standard-form) value < modulus ?
template <class P>
KZ_DEV bool fp_raw_lt_mod(const Fp<P>& raw) {
  uint32_t bw = 0;
  _Pragma("unroll") for (int i = 0; i < P::N; ++i) (void)__builtin_subc(raw.v[i], P::MOD[i], bw, &bw);
  return bw != 0;
}

// ---------------------------------------------------------------------------- pow / inverse
// x^((p+1)/4) (square-root candidate, p = 3 mod 4) by the width-4 sliding-window schedule
// generated into P::SQRT_* (tools/gen_params.py window_steps): 375 squarings + 78
// multiplications + 8 for the odd-power table on BLS12-381, instead of 380 + 190 for plain
// square-and-multiply.  The schedule is the same for every lane (uniform loop bounds and
// table indices), the table lives in 8 named registers selected by v_cndmask.
template <class P>
KZ_DEV Fp<P> fp_sel8(uint32_t k, const Fp<P>& t0, const Fp<P>& t1, const Fp<P>& t2, const Fp<P>& t3,
                     const Fp<P>& t4, const Fp<P>& t5, const Fp<P>& t6, const Fp<P>& t7) {
  Fp<P> r = t0;
  r = fp_select(k == 1, t1, r);
  r = fp_select(k == 2, t2, r);
  r = fp_select(k == 3, t3, r);
  r = fp_select(k == 4, t4, r);
  r = fp_select(k == 5, t5, r);
  r = fp_select(k == 6, t6, r);
  r = fp_select(k == 7, t7, r);
  return r;
}

template <class P>
KZ_DEV Fp<P> fp_pow_sqrt(const Fp<P>& a) {
  const Fp<P> a2 = fp_sqr(a);
  const Fp<P> t0 = a, t1 = fp_mul(t0, a2), t2 = fp_mul(t1, a2), t3 = fp_mul(t2, a2);
  const Fp<P> t4 = fp_mul(t3, a2), t5 = fp_mul(t4, a2), t6 = fp_mul(t5, a2), t7 = fp_mul(t6, a2);
  Fp<P> acc = fp_sel8<P>(P::SQRT_FIRST, t0, t1, t2, t3, t4, t5, t6, t7);
  for (int s = 0; s < P::SQRT_STEPS; ++s) {
    const int nsq = P::SQRT_SQR[s];
    for (int q = 0; q < nsq; ++q) acc = fp_sqr(acc);
    const uint32_t k = P::SQRT_IDX[s];
    if (k != 255u) acc = fp_mul(acc, fp_sel8<P>(k, t0, t1, t2, t3, t4, t5, t6, t7));
  }
  return acc;
}

// a^-1 in Montgomery form (0 -> 0) for the single-lane tails (MSM result -> affine, the
// pairing's Fp inversion): the word-level binary GCD of bingcd.hpp on the raw Montgomery value
// aR, giving (aR)^-1, then two Montgomery products by R^2: (aR)^-1 R^2 = a^-1 R.
template <class P>
KZ_DEV Fp<P> fp_inv(const Fp<P>& a) {
  constexpr int N = P::N;
  uint32_t y[N], m[N], r[N];
  _Pragma("unroll") for (int i = 0; i < N; ++i) { y[i] = a.v[i]; m[i] = P::MOD[i]; }
  // canonical y < p (lazily reduced inputs stay below a few p)
  for (int k = 0; k < 4; ++k) {
    uint32_t d[N], bw = 0;
    _Pragma("unroll") for (int i = 0; i < N; ++i) d[i] = __builtin_subc(y[i], m[i], bw, &bw);
    if (bw) break;
    _Pragma("unroll") for (int i = 0; i < N; ++i) y[i] = d[i];
  }
  BinGcd<N>::inv(y, m, P::BITS, r);
  Fp<P> x;
  _Pragma("unroll") for (int i = 0; i < N; ++i) x.v[i] = r[i];
  const Fp<P> r2 = Fp<P>::from_const(P::R2);
  return fp_mul(fp_mul(x, r2), r2);
}

// ---------------------------------------------------------------------------- bytes
// 32-bit big-endian word -> host order
KZ_DEV uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

}  // namespace kzgmi
