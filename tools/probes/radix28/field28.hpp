// ARCHIVED EXPERIMENT (not built): radix-2^28 accumulation, measured slower in situ -- see
// profiles/r01/probes/radix28.txt.  Needed the Fp28 constants tools/gen_params.py emitted then.
// Carry-free radix-2^28 Montgomery arithmetic for the bucket-accumulation kernel.
//
// Why (measured, tools/probes/fp28.hip and the k_accumulate SQ counters in DESIGN.md): the
// accumulation is VALU-issue bound at ~6.8k instructions per mixed addition, and in the
// 32-bit-limb multiply half of the instructions are `v_addc` carry handling.  With 28-bit
// limbs in 32-bit words every column of product scanning fits a 64-bit accumulator
// (2N products < 2^56 each + carry < 2^63), so a limb product is ONE v_mad_u64_u32:
// 74-77 G products/s vs 58-61 G for the 32-bit form (BLS12-381, equal results).
//
// Representation: Q::N limbs (14 for BLS12-381, R = 2^392; 10 for BN254, R = 2^280),
// Montgomery form a*R28 mod p, LAZILY reduced: values are only known to lie below a stated
// multiple of p.  R28/p > 2047 (BLS) so mul28 returns < 2p for any inputs whose product is
// < 2047 p^2 (t = (ab + mp)/R < ab/R + p).  Limbs are kept normalised (< 2^28, top limb
// holding the rest) by one signed carry pass after every add/sub.  Callers track bounds;
// the accumulation kernel (msm28.hpp) documents them per step.
#pragma once
#include "field.hpp"
#include "params_gen.hpp"

namespace kzgmi {

constexpr uint32_t M28 = (1u << 28) - 1;

template <class Q>
struct F28 {
  static constexpr int N = Q::N;
  uint32_t v[N];
  KZ_DEV static F28 from_const(const uint32_t (&c)[N]) {
    F28 r;
    _Pragma("unroll") for (int i = 0; i < N; ++i) r.v[i] = c[i];
    return r;
  }
};

// a * b / R28 mod p (< 2p when a*b < 2047 p^2; inputs normalised)
template <class Q>
KZ_DEV F28<Q> mul28(const F28<Q>& a, const F28<Q>& b) {
  constexpr int N = Q::N;
  uint32_t m[N];
  F28<Q> t;
  uint64_t acc = 0;
  _Pragma("unroll") for (int k = 0; k < N; ++k) {
    _Pragma("unroll") for (int i = 0; i < k; ++i) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)m[i] * Q::MOD[k - i];
    }
    acc += (uint64_t)a.v[k] * b.v[0];
    m[k] = ((uint32_t)acc * Q::INV) & M28;
    acc += (uint64_t)m[k] * Q::MOD[0];  // low 28 bits become 0
    acc >>= 28;
  }
  _Pragma("unroll") for (int k = N; k < 2 * N - 1; ++k) {
    _Pragma("unroll") for (int i = k - N + 1; i < N; ++i) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)m[i] * Q::MOD[k - i];
    }
    t.v[k - N] = (uint32_t)acc & M28;
    acc >>= 28;
  }
  t.v[N - 1] = (uint32_t)acc;
  return t;
}

// signed carry pass over limb values x_i (each in (-2^30, 2^30)); result must be >= 0
template <int N>
KZ_DEV void norm28(int32_t (&x)[N], uint32_t (&out)[N]) {
  int32_t carry = 0;
  _Pragma("unroll") for (int i = 0; i < N - 1; ++i) {
    const int32_t t = x[i] + carry;
    out[i] = (uint32_t)t & M28;
    carry = t >> 28;  // arithmetic
  }
  out[N - 1] = (uint32_t)(x[N - 1] + carry);
}

// a + KP - b, normalised (KP a multiple of p at least b's bound)
template <class Q>
KZ_DEV F28<Q> sub28(const F28<Q>& a, const F28<Q>& b, const uint32_t (&kp)[Q::N]) {
  int32_t x[Q::N];
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) x[i] = (int32_t)(a.v[i] + kp[i]) - (int32_t)b.v[i];
  F28<Q> r;
  norm28<Q::N>(x, r.v);
  return r;
}
// a + KP - b - 2c, normalised
template <class Q>
KZ_DEV F28<Q> sub2_28(const F28<Q>& a, const F28<Q>& b, const F28<Q>& c, const uint32_t (&kp)[Q::N]) {
  int32_t x[Q::N];
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i)
    x[i] = (int32_t)(a.v[i] + kp[i]) - (int32_t)b.v[i] - 2 * (int32_t)c.v[i];
  F28<Q> r;
  norm28<Q::N>(x, r.v);
  return r;
}
// k * a, normalised (small k)
template <class Q, int K>
KZ_DEV F28<Q> smul28(const F28<Q>& a) {
  int32_t x[Q::N];
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) x[i] = K * (int32_t)a.v[i];
  F28<Q> r;
  norm28<Q::N>(x, r.v);
  return r;
}

template <class Q>
KZ_DEV bool all_zero28(const F28<Q>& a) {
  uint32_t x = 0;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) x |= a.v[i];
  return x == 0;
}
// a < 2p (normalised): a == 0 mod p
template <class Q>
KZ_DEV bool is_zero_lt2p(const F28<Q>& a) {
  uint32_t z = 0, e = 0;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) { z |= a.v[i]; e |= a.v[i] ^ Q::MOD[i]; }
  return z == 0 || e == 0;
}
// a < 2p (normalised) -> canonical a mod p
template <class Q>
KZ_DEV F28<Q> canon_lt2p(const F28<Q>& a) {
  int32_t x[Q::N];
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) x[i] = (int32_t)a.v[i] - (int32_t)Q::MOD[i];
  F28<Q> d;
  norm28<Q::N>(x, d.v);
  const bool neg = (int32_t)d.v[Q::N - 1] < 0;
  F28<Q> r;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) r.v[i] = neg ? a.v[i] : d.v[i];
  return r;
}

// 32-bit little-endian words <-> 28-bit limbs (same integer)
template <class Q, int NW>
KZ_DEV F28<Q> unpack28(const uint32_t (&w)[NW]) {
  F28<Q> r;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) {
    const int bit = 28 * i, wi = bit >> 5, sh = bit & 31;
    const uint64_t lo = (wi < NW ? (uint64_t)w[wi] : 0) | (wi + 1 < NW ? (uint64_t)w[wi + 1] << 32 : 0);
    r.v[i] = (uint32_t)(lo >> sh) & M28;
  }
  return r;
}
template <class Q, int NW>
KZ_DEV void pack32(const F28<Q>& a, uint32_t (&w)[NW]) {  // a canonical (< p < 2^(32 NW))
  _Pragma("unroll") for (int j = 0; j < NW; ++j) {
    const int bit = 32 * j, li = bit / 28, sh = bit % 28;
    uint64_t x = (uint64_t)a.v[li] >> sh;  // sh in {0, 4, ..., 24}: two limbs cover the word
    if (li + 1 < Q::N) x |= (uint64_t)a.v[li + 1] << (28 - sh);
    w[j] = (uint32_t)x;
  }
}

}  // namespace kzgmi
