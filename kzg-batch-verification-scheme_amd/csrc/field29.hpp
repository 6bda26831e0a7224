// Radix-2^29 Montgomery arithmetic: the bucket accumulation (msm.hpp k_accumulate) and
// everything around it that is full-chip or on the pipeline's critical path -- the point
// conversion and on-curve test (kernels.hpp), the piece join and both bucket-sum reductions
// (msm.hpp x29_add), and on BLS12-381 square roots and the subgroup check (points.hpp).
// BLS12-381: 14 limbs of 29 bits in 32-bit VGPRs, R29 = 2^406; BN254: 9 limbs, R29 = 2^261.
//
// Why: the accumulation is VALU-issue bound, and in the 32-bit-limb product (field.hpp) every
// limb product costs TWO issue slots, the v_mad_u64_u32 and the v_addc_co_u32 folding its
// carry-out (tools/probes/mad_rate.hip: both full rate).  With 29-bit limbs every column of
// the product -- at most 2N (a b) + N (m p) products < 2^58 plus the carry -- fits the 64-bit
// accumulator, so a limb product is ONE v_mad_u64_u32: 2N^2 mads + ~4 column ops x (2N - 1)
// (BLS12-381 392 mads instead of 288 x 2 + column moves; BN254 162 instead of 128 x 2).
// Additions and subtractions pay a carry pass instead (sub29: a + B - b with B a multiple of p
// whose limbs are biased into [2^29, 2^30), so no limb goes negative).  Measured in one harness
// (tools/probes/radix29/acc29.hip): the BLS12-381 mixed addition runs 1.17-1.22x faster than
// the 32-bit lazy form, and it fits 108 VGPRs without spills.
//
// Value bounds (all values are normalised: limbs 0..N-2 < 2^29): a product of inputs below
// a p and b p returns below (a b p / R29 + 1) p -- < 2p for a b < 2^24 on BLS12-381 but only
// for a b < ~169 on BN254 -- so callers track the bounds of sums and differences and pick the
// bias B_k with k p >= the subtrahend's bound.  The accumulation loop names its biases by role
// (Q::ACC_*, Q::DBL_*), chosen per curve and checked step by step by tools/gen_params29.py.
// Reference: none (LICENSE only); checked bit-exactly against the C oracle through the MSM and
// batch parity tests, which all run through this path.
#pragma once
#include "field.hpp"
#include <type_traits>
#include "params29_gen.hpp"

namespace kzgmi {

constexpr uint32_t M29 = (1u << 29) - 1;

// the radix-2^29 parameters of a curve's base field (Cv::ID 0: BLS12-381, 1: BN254)
template <class Cv>
using Fp29Of = std::conditional_t<Cv::ID == 0, Bls12_381Fp29, Bn254Fp29>;

template <class Q>
struct F29 {
  static constexpr int N = Q::N;
  uint32_t v[N];
  KZ_DEV static F29 zero() { F29 r; _Pragma("unroll") for (int i = 0; i < N; ++i) r.v[i] = 0; return r; }
  KZ_DEV static F29 from_const(const uint32_t (&c)[N]) {
    F29 r;
    _Pragma("unroll") for (int i = 0; i < N; ++i) r.v[i] = c[i];
    return r;
  }
};

KZ_DEV void mad29(uint64_t& acc, uint32_t a, uint32_t b) {
  uint64_t cc;  // carry-out unused: column sums stay below 2^64
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
}
KZ_DEV void mad29s(uint64_t& acc, uint32_t a, uint32_t b_uniform) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "s"(b_uniform));
}

// Column terms issued up to 4 per asm statement: hipcc pads every inline-asm statement that
// writes a VGPR with an s_nop before the next VALU reads it (it cannot see that the statement
// has no dst-sel forwarding hazard), so one mad per statement costs one s_nop per mad; the
// hardware interlocks a plain dependent v_mad_u64_u32 chain by itself.  The carry-out SGPR is
// early-clobber ("=&s": an "s" input read by a later instruction must not share it); the
// accumulator is "+v" -- its register holds its own (64-bit, runtime) value on entry, so no
// 32-bit input can share it (field.hpp mac32 note: the aliasing case is an accumulator whose
// value equals an input).  (One mad per statement measured 1 % slower, profiles/HISTORY.md.)
template <int K, int I, int CNT, int NX, int NY>
KZ_DEV void vv_run(uint64_t& acc, const uint32_t (&x)[NX], const uint32_t (&y)[NY]) {
  uint64_t cc;
  if constexpr (CNT >= 4) {
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %4, %5, %0\n\t"
        "v_mad_u64_u32 %0, %1, %6, %7, %0\n\tv_mad_u64_u32 %0, %1, %8, %9, %0"
        : "+v"(acc), "=&s"(cc)
        : "v"(x[I]), "v"(y[K - I]), "v"(x[I + 1]), "v"(y[K - I - 1]), "v"(x[I + 2]), "v"(y[K - I - 2]),
          "v"(x[I + 3]), "v"(y[K - I - 3]));
    vv_run<K, I + 4, CNT - 4>(acc, x, y);
  } else if constexpr (CNT == 3) {
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %4, %5, %0\n\t"
        "v_mad_u64_u32 %0, %1, %6, %7, %0"
        : "+v"(acc), "=&s"(cc)
        : "v"(x[I]), "v"(y[K - I]), "v"(x[I + 1]), "v"(y[K - I - 1]), "v"(x[I + 2]), "v"(y[K - I - 2]));
  } else if constexpr (CNT == 2) {
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %4, %5, %0"
        : "+v"(acc), "=&s"(cc)
        : "v"(x[I]), "v"(y[K - I]), "v"(x[I + 1]), "v"(y[K - I - 1]));
  } else if constexpr (CNT == 1) {
    mad29(acc, x[I], y[K - I]);
  }
  (void)cc;
}
// m_i MOD_{K-i}, i = I .. I+CNT-1 (MOD limbs: uniform, in SGPRs)
template <class Q, int K, int I, int CNT>
KZ_DEV void vs_run(uint64_t& acc, const uint32_t (&m)[Q::N]) {
  uint64_t cc;
  if constexpr (CNT >= 4) {
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %4, %5, %0\n\t"
        "v_mad_u64_u32 %0, %1, %6, %7, %0\n\tv_mad_u64_u32 %0, %1, %8, %9, %0"
        : "+v"(acc), "=&s"(cc)
        : "v"(m[I]), "s"(Q::MOD[K - I]), "v"(m[I + 1]), "s"(Q::MOD[K - I - 1]), "v"(m[I + 2]),
          "s"(Q::MOD[K - I - 2]), "v"(m[I + 3]), "s"(Q::MOD[K - I - 3]));
    vs_run<Q, K, I + 4, CNT - 4>(acc, m);
  } else if constexpr (CNT == 3) {
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %4, %5, %0\n\t"
        "v_mad_u64_u32 %0, %1, %6, %7, %0"
        : "+v"(acc), "=&s"(cc)
        : "v"(m[I]), "s"(Q::MOD[K - I]), "v"(m[I + 1]), "s"(Q::MOD[K - I - 1]), "v"(m[I + 2]),
          "s"(Q::MOD[K - I - 2]));
  } else if constexpr (CNT == 2) {
    asm("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %4, %5, %0"
        : "+v"(acc), "=&s"(cc)
        : "v"(m[I]), "s"(Q::MOD[K - I]), "v"(m[I + 1]), "s"(Q::MOD[K - I - 1]));
  } else if constexpr (CNT == 1) {
    mad29s(acc, m[I], Q::MOD[K - I]);
  }
  (void)cc;
}

// column K of (a b [+ c d] + m p): low columns produce m_K, high ones the result limbs
template <class Q, bool TWO, int K>
KZ_DEV void mont29_cols(uint64_t& acc, uint32_t (&m)[Q::N], F29<Q>& t, const F29<Q>& a, const F29<Q>& b,
                        const F29<Q>& c, const F29<Q>& d) {
  constexpr int N = Q::N;
  if constexpr (K < N) {
    if constexpr (K == 0) acc = (uint64_t)a.v[0] * b.v[0];  // compiler's mad with a 0 addend: no zeroed pair
    else vv_run<K, 0, K + 1>(acc, a.v, b.v);
    if constexpr (TWO) vv_run<K, 0, K + 1>(acc, c.v, d.v);
    vs_run<Q, K, 0, K>(acc, m);
    m[K] = ((uint32_t)acc * Q::INV) & M29;
    mad29s(acc, m[K], Q::MOD[0]);  // low 29 bits become 0
    acc >>= 29;
    mont29_cols<Q, TWO, K + 1>(acc, m, t, a, b, c, d);
  } else if constexpr (K < 2 * N - 1) {
    vv_run<K, K - N + 1, 2 * N - 1 - K>(acc, a.v, b.v);
    if constexpr (TWO) vv_run<K, K - N + 1, 2 * N - 1 - K>(acc, c.v, d.v);
    vs_run<Q, K, K - N + 1, 2 * N - 1 - K>(acc, m);
    t.v[K - N] = (uint32_t)acc & M29;
    acc >>= 29;
    mont29_cols<Q, TWO, K + 1>(acc, m, t, a, b, c, d);
  }
}

// column K of a^2 + m p: off-diagonal a2_i a_{K-i} (i < K - i), the diagonal, m p
template <class Q, int K>
KZ_DEV void sqr29_cols(uint64_t& acc, uint32_t (&m)[Q::N], F29<Q>& t, const uint32_t (&a2)[Q::N], const F29<Q>& a) {
  constexpr int N = Q::N;
  if constexpr (K < 2 * N - 1) {
    constexpr int lo = K < N ? 0 : K - N + 1;
    constexpr int hi = (K - 1) / 2;  // last i with i < K - i
    if constexpr (K >= 1 && hi >= lo) vv_run<K, lo, hi - lo + 1>(acc, a2, a.v);
    if constexpr (K == 0) acc = (uint64_t)a.v[0] * a.v[0];
    else if constexpr ((K & 1) == 0) mad29(acc, a.v[K / 2], a.v[K / 2]);
    if constexpr (K < N) {
      vs_run<Q, K, 0, K>(acc, m);
      m[K] = ((uint32_t)acc * Q::INV) & M29;
      mad29s(acc, m[K], Q::MOD[0]);
    } else {
      vs_run<Q, K, K - N + 1, 2 * N - 1 - K>(acc, m);
      t.v[K - N] = (uint32_t)acc & M29;
    }
    acc >>= 29;
    sqr29_cols<Q, K + 1>(acc, m, t, a2, a);
  }
}

// (a b [+ c d] + m p) / R29 -- product scanning, one 64-bit accumulator per column
template <class Q, bool TWO>
KZ_DEV F29<Q> mont29(const F29<Q>& a, const F29<Q>& b, const F29<Q>& c, const F29<Q>& d) {
  uint32_t m[Q::N];
  F29<Q> t;
  uint64_t acc = 0;
  mont29_cols<Q, TWO, 0>(acc, m, t, a, b, c, d);
  t.v[Q::N - 1] = (uint32_t)acc;
  return t;
}
template <class Q>
KZ_DEV F29<Q> mul29(const F29<Q>& a, const F29<Q>& b) { return mont29<Q, false>(a, b, a, b); }
// a^2 / R29: the off-diagonal limb products once, against a pre-doubled operand (2 a_i < 2^30),
// plus the squares on the diagonal -- 91 + 14 + 196 (m p) = 301 mads instead of 392.  Column
// bound: 7 x 2^59 + 2^58 + 14 x 2^58 + carry < 2^63 (limbs < 2^29, top limb < 2^16).
template <class Q>
KZ_DEV F29<Q> sqr29(const F29<Q>& a) {
  constexpr int N = Q::N;
  uint32_t a2[N];
  _Pragma("unroll") for (int i = 0; i < N; ++i) a2[i] = a.v[i] + a.v[i];
  uint32_t m[N];
  F29<Q> t;
  uint64_t acc = 0;
  sqr29_cols<Q, 0>(acc, m, t, a2, a);
  t.v[N - 1] = (uint32_t)acc;
  return t;
}

template <class Q>
KZ_DEV F29<Q> mul2_29(const F29<Q>& a, const F29<Q>& b, const F29<Q>& c, const F29<Q>& d) {
  return mont29<Q, true>(a, b, c, d);
}

// a + B - b, normalised (B: biased k p, k p >= b)
template <class Q>
KZ_DEV F29<Q> sub29(const F29<Q>& a, const F29<Q>& b, const uint32_t (&B)[Q::N]) {
  F29<Q> r;
  uint32_t c = 0;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) {
    const uint32_t x = a.v[i] + B[i] + c - b.v[i];
    if (i < Q::N - 1) {
      r.v[i] = x & M29;
      c = x >> 29;
    } else {
      r.v[i] = x;
    }
  }
  return r;
}

// a + C - s - 2t in one carry pass (C: a multiple of p with limbs in [3 (2^29 - 1), 2^31),
// params29_gen.hpp C4/C8; s, t normalised, so no limb goes negative): the accumulation's
// X3 = R^2 - (PPP + 2 Q2), which took an add3_29 pass and a sub29 pass (5 VALU per limb instead of 8)
template <class Q>
KZ_DEV F29<Q> sub3_29(const F29<Q>& a, const F29<Q>& s, const F29<Q>& t, const uint32_t (&C)[Q::N]) {
  F29<Q> r;
  uint32_t c = 0;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) {
    const uint32_t x = (a.v[i] + C[i] + c) - (s.v[i] + t.v[i] + t.v[i]);
    if (i < Q::N - 1) {
      r.v[i] = x & M29;
      c = x >> 29;
    } else {
      r.v[i] = x;
    }
  }
  return r;
}

// B - b limb by limb, no carry pass (B biased, b normalised): limbs in (0, 2^30), NOT normalised.
// Only as one operand of a product whose column sums keep their headroom -- in the accumulation,
// the y PPP pair of mul2_29: 14 x 2^59 + (14 + 14) x 2^58 < 2^64 (BLS12-381; BN254 9 limbs)
template <class Q>
KZ_DEV F29<Q> neg_lazy29(const F29<Q>& b, const uint32_t (&B)[Q::N]) {
  F29<Q> r;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) r.v[i] = B[i] - b.v[i];
  return r;
}

// a + b + e, normalised
template <class Q>
KZ_DEV F29<Q> add3_29(const F29<Q>& a, const F29<Q>& b, const F29<Q>& e) {
  F29<Q> r;
  uint32_t c = 0;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) {
    const uint32_t x = a.v[i] + b.v[i] + e.v[i] + c;
    if (i < Q::N - 1) {
      r.v[i] = x & M29;
      c = x >> 29;
    } else {
      r.v[i] = x;
    }
  }
  return r;
}

// a == 0 mod p for a < NKP p.  a = k p forces k = low limb x p^-1 mod 2^29 (p is odd), so one
// multiply filters; only k < NKP is compared limb by limb (no table of multiples stays live in
// registers across the accumulation loop)
template <class Q>
KZ_DEV bool is_zero29(const F29<Q>& a) {
  bool hit = false;
  _Pragma("unroll") for (int k = 0; k < Q::NKP; ++k) hit |= a.v[0] == Q::KP_LO[k];
  if (!hit) return false;
  for (int k = 0; k < Q::NKP; ++k) {
    uint32_t d = 0;
    for (int i = 0; i < Q::N; ++i) d |= a.v[i] ^ Q::KP[k][i];
    if (d == 0) return true;
  }
  return false;
}
// The same test with the multiply filter itself (k = a_0 p^-1 mod 2^29, then one table row
// compared): 3 VALU instead of ~40 on the common path, for the accumulation loop.  Elsewhere
// (the reduction's out-of-line addition) its divergent table load raised the register peak.
template <class Q>
KZ_DEV bool is_zero29_mf(const F29<Q>& a) {
  constexpr uint32_t PINV = 0u - Q::INV;  // p^-1 mod 2^32
  const uint32_t k = (a.v[0] * PINV) & M29;
  if (k >= (uint32_t)Q::NKP) return false;
  uint32_t d = 0;
  for (int i = 0; i < Q::N; ++i) d |= a.v[i] ^ Q::KP[k][i];
  return d == 0;
}

// a < 2p -> a mod p
template <class Q>
KZ_DEV F29<Q> canon29(const F29<Q>& a) {
  F29<Q> d;
  int32_t c = 0;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) {
    const int32_t x = (int32_t)a.v[i] - (int32_t)Q::MOD[i] + c;
    if (i < Q::N - 1) {
      d.v[i] = (uint32_t)x & M29;
      c = x >> 29;
    } else {
      d.v[i] = (uint32_t)x;
    }
  }
  const bool neg = (int32_t)d.v[Q::N - 1] < 0;
  F29<Q> r;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) r.v[i] = neg ? a.v[i] : d.v[i];
  return r;
}

// 32-bit words (value < 2^(32 NW)) <-> 29-bit limbs of the same integer
template <class Q, int NW>
KZ_DEV F29<Q> limbs29(const uint32_t (&w)[NW]) {
  F29<Q> r;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    const uint64_t lo = (wi < NW ? (uint64_t)w[wi] : 0) | (wi + 1 < NW ? (uint64_t)w[wi + 1] << 32 : 0);
    r.v[i] = (uint32_t)(lo >> sh) & (i < Q::N - 1 ? M29 : 0xffffffffu);
  }
  return r;
}
template <class Q, int NW>
KZ_DEV void words32(const F29<Q>& a, uint32_t (&w)[NW]) {  // a normalised, < 2^(32 NW)
  _Pragma("unroll") for (int j = 0; j < NW; ++j) {
    const int bit = 32 * j, li = bit / 29, sh = bit % 29;
    uint64_t x = (uint64_t)a.v[li] >> sh;
    if (li + 1 < Q::N) x |= (uint64_t)a.v[li + 1] << (29 - sh);
    if (li + 2 < Q::N && 58 - sh < 32) x |= (uint64_t)a.v[li + 2] << (58 - sh);
    w[j] = (uint32_t)x;
  }
}

// 32-bit Montgomery (x 2^384, canonical) -> radix-29 Montgomery (x R29), and back (canonical)
template <class Q, class P>
KZ_DEV F29<Q> fp_to29(const Fp<P>& a) {
  return mul29(limbs29<Q>(a.v), F29<Q>::from_const(Q::TO29));
}
template <class Q, class P>
KZ_DEV Fp<P> fp_from29(const F29<Q>& a) {  // a < 2^12 p
  Fp<P> r;
  words32<Q>(canon29(mul29(a, F29<Q>::from_const(Q::TO32))), r.v);
  return r;
}

}  // namespace kzgmi
