// Lane-parallel Montgomery arithmetic and G1 formulas for the latency-bound MSM tail
// (window combination, window-sum Horner): one dependent chain of point operations per wave.
//
// Why: a lone wave running the serial 32-bit product (field.hpp, ~650 VALU instructions) needs
// ~2 us per Fp product, so the 240 serial doublings of a 16-window Horner took ~3.9 ms of the
// single-batch latency.  Here a field element is spread over a 16-lane row, one signed 29-bit
// limb per lane (BLS12-381 14 limbs, R = 2^406; BN254 10 limbs, R = 2^290).  A Montgomery
// product is N systolic steps of ~11 instructions:
//     acc_j += a_i b_j      (a_i broadcast from lane i with DPP row_newbcast, v_mad_i64_i32)
//     m = (acc_0 p') mod 2^29 (broadcast from lane 0);  acc_j += m p_j
//     acc_j <- (acc_j >> 29) + (acc_{j+1} mod 2^29)   (divide the row's number by 2^29: DPP row_shl)
// so a product is ~160 instructions on the critical path instead of ~650.  The 4 rows of a wave
// compute up to 4 independent products at once (operands selected per row, results shared with
// ds_bpermute): an XYZZ doubling is 3 product steps (9 products), an XYZZ addition 4.
//
// Representation: limbs are SIGNED and redundant (|limb| < 2^29 + 4 after lp_norm); values are
// integers congruent to the element, never reduced: a - b is a limb-wise subtraction, no bias.
// Bound rule (params_lp_gen.hpp HEAD): |a|, |b| < 2^HEAD p  =>  |lp_mul(a, b)| < 1.5 p
// (|a b + m p| / R with m < R); the formulas below keep every product input below 64 p.
// Zero tests are row-local (lp_row_is_zero: reduce below p, carry passes, ballot); outputs
// canonicalise in uniform scalar code (lp_canon: quotient estimate in double precision from the
// top limbs, exact multi-limb correction).
// Reference: none (LICENSE only); checked through every MSM / batch parity test (the window
// combination of every MSM runs here) and kzgmi_selftest_lp.
#pragma once
#include <type_traits>
#include <utility>
#include "g1.hpp"
#include "params_lp_gen.hpp"

namespace kzgmi {

template <class Cv>
using LpQ = std::conditional_t<Cv::ID == 0, LpBls12_381, LpBn254>;

constexpr int32_t LP_M29 = (1 << 29) - 1;

// ---- DPP inside a 16-lane row
template <int I>
KZ_DEV int32_t lp_bcast(int32_t x) { return __builtin_amdgcn_mov_dpp(x, 0x150 + I, 0xF, 0xF, false); }  // row_newbcast:I
KZ_DEV int32_t lp_next(int32_t x) { return __builtin_amdgcn_update_dpp(0, x, 0x101, 0xF, 0xF, true); }  // row_shl:1: lane j <- j+1, lane 15 <- 0
KZ_DEV int32_t lp_prev(int32_t x) { return __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true); }  // row_shr:1: lane j <- j-1, lane 0 <- 0

// acc += a b, signed 32 x 32 -> 64: one v_mad_i64_i32.  ROCm 7.2's hipcc selects it from the C++
// form for gfx950 (earlier compilers lowered it to two unsigned mads plus sign fix-ups, hence the
// inline asm of rounds 1-2); the C++ form also spares the s_nop hipcc pads after
// every VGPR-writing asm statement -- 14 per lane-parallel product (lp_mul_iter).
KZ_DEV void lp_mad_i64(int64_t& acc, int32_t a, int32_t b) { acc += (int64_t)a * (int64_t)b; }
// acc += a b for 0 <= a, b < 2^31 (two's complement acc: the unsigned sum wraps correctly)
KZ_DEV void lp_mad_u64(int64_t& acc, int32_t a, int32_t b) {
  acc = (int64_t)((uint64_t)acc + (uint64_t)(uint32_t)a * (uint64_t)(uint32_t)b);
}

// per-lane constants of a lane-parallel kernel (lane j = threadIdx.x % 16 of row threadIdx.x / 16 % 4)
template <class Cv>
struct LpCtx {
  int32_t pj;      // limb j of p (0 for j >= N)
  int32_t lomask;  // 2^29 - 1 below the top limb, all ones from the top limb on
  int32_t cmask;   // all ones below the top limb: carries leave lanes 0..N-2 only
  int32_t tolp, to32;
  int row;
  int src[4];      // ds_bpermute byte address of this lane's limb in row r
};

template <class Cv>
KZ_DEV LpCtx<Cv> lp_ctx() {
  using Q = LpQ<Cv>;
  const int j = threadIdx.x & 15;
  LpCtx<Cv> c;
  c.pj = c.tolp = c.to32 = 0;
#pragma unroll
  for (int k = 0; k < Q::N; ++k) {
    if (j == k) {
      c.pj = (int32_t)Q::MOD[k];
      c.tolp = (int32_t)Q::TO_LP[k];
      c.to32 = (int32_t)Q::TO32[k];
    }
  }
  c.lomask = j < Q::N - 1 ? LP_M29 : -1;
  c.cmask = j < Q::N - 1 ? -1 : 0;
  c.row = (threadIdx.x >> 4) & 3;
#pragma unroll
  for (int r = 0; r < 4; ++r) c.src[r] = (16 * r + j) * 4;
  return c;
}

// one carry pass: limbs back into [-2, 2^29 + 2) for inputs |v| < 2^30.6
template <class Cv>
KZ_DEV int32_t lp_norm(const LpCtx<Cv>& c, int32_t v) {
  const int32_t carry = (v >> 29) & c.cmask;
  return (v & c.lomask) + lp_prev(carry);
}

template <class Cv, int I>
KZ_DEV void lp_mul_iter(int64_t& acc, int32_t ai, int32_t b, int32_t pj) {  // ai: limb I of a, broadcast
  lp_mad_i64(acc, ai, b);
  const int32_t mloc = (int32_t)(((uint32_t)acc * LpQ<Cv>::INV) & (uint32_t)LP_M29);
  const int32_t m = lp_bcast<0>(mloc);
  lp_mad_u64(acc, m, pj);  // lane 0: low 29 bits now zero
  const int32_t lo = (int32_t)((uint32_t)acc & (uint32_t)LP_M29);
  const int32_t hi = (int32_t)(acc >> 29);
  acc = (int64_t)(hi + lp_next(lo));
}
// every limb of a broadcast up front (independent DPP moves): the scheduler can place them in the
// systolic chain's wait states instead of an s_nop before each step's dependent DPP
template <class Cv, int... I>
KZ_DEV int32_t lp_mul_raw(int32_t a, int32_t b, int32_t pj, std::integer_sequence<int, I...>) {
  const int32_t ai[] = {lp_bcast<I>(a)...};
  int64_t acc = 0;
  (lp_mul_iter<Cv, I>(acc, ai[I], b, pj), ...);
  return (int32_t)acc;
}
// a b / R (mod p), each row independently
template <class Cv>
KZ_DEV int32_t lp_mul(const LpCtx<Cv>& c, int32_t a, int32_t b) {
  return lp_norm(c, lp_mul_raw<Cv>(a, b, c.pj, std::make_integer_sequence<int, LpQ<Cv>::N>{}));
}

// 64-bit per-lane accumulator (|acc| < 2^58; the top lane's own value must fit 32 bits, which the
// value bound guarantees) -> normalised limbs
template <class Cv>
KZ_DEV int32_t lp_norm64(const LpCtx<Cv>& c, int64_t acc) {
  const bool top = c.cmask == 0;  // lanes >= N - 1 keep their value and emit no carry
  const int32_t keep = top ? (int32_t)acc : (int32_t)((uint32_t)acc & (uint32_t)LP_M29);
  const int32_t carry = top ? 0 : (int32_t)(acc >> 29);
  return lp_norm(c, keep + lp_prev(carry));
}

// v - q p with q = round(v / p) from the row's two top limbs: |result| < 0.51 p, congruent to v.
// Row-local (each row its own value); ~15 instructions instead of a Montgomery product by 1.
template <class Cv>
KZ_DEV int32_t lp_reduce(const LpCtx<Cv>& c, int32_t v) {
  using Q = LpQ<Cv>;
  const double t = (double)lp_bcast<Q::N - 1>(v) * Q::RED_C1 + (double)lp_bcast<Q::N - 2>(v) * Q::RED_C2;
  const int32_t q = (int32_t)__builtin_rint(t);
  int64_t acc = (int64_t)v;
  lp_mad_i64(acc, -q, c.pj);
  return lp_norm64(c, acc);
}

// v == 0 (mod p), row-local: reduce below p, then resolve every carry (value 0 <=> all limbs 0)
template <class Cv>
KZ_DEV bool lp_row_is_zero(const LpCtx<Cv>& c, int32_t v) {
  int32_t r = lp_reduce(c, v);
#pragma unroll
  for (int k = 0; k < LpQ<Cv>::N; ++k) r = lp_norm(c, r);
  const uint64_t nz = __builtin_amdgcn_ballot_w64(r != 0);
  return ((nz >> (16 * c.row)) & 0xFFFFull) == 0;
}

template <class Cv> KZ_DEV int32_t lp_add(const LpCtx<Cv>& c, int32_t a, int32_t b) { return lp_norm(c, a + b); }
template <class Cv> KZ_DEV int32_t lp_sub(const LpCtx<Cv>& c, int32_t a, int32_t b) { return lp_norm(c, a - b); }
template <class Cv> KZ_DEV int32_t lp_dbl(const LpCtx<Cv>& c, int32_t a) { return lp_norm(c, a + a); }
template <class Cv> KZ_DEV int32_t lp_mul3(const LpCtx<Cv>& c, int32_t a) { return lp_norm(c, a + a + a); }
template <class Cv> KZ_DEV int32_t lp_mul8(const LpCtx<Cv>& c, int32_t a) { return lp_dbl(c, lp_dbl(c, lp_dbl(c, a))); }
template <class Cv> KZ_DEV int32_t lp_mul9(const LpCtx<Cv>& c, int32_t a) { return lp_mul3(c, lp_mul3(c, a)); }

// ---- row-parallel product steps: row r computes a_r b_r; every row receives every result
template <class Cv>
KZ_DEV int32_t lp_sel(const LpCtx<Cv>& c, int32_t v0, int32_t v1, int32_t v2, int32_t v3) {
  return c.row == 0 ? v0 : c.row == 1 ? v1 : c.row == 2 ? v2 : v3;
}
template <class Cv>
KZ_DEV int32_t lp_row(const LpCtx<Cv>& c, int32_t v, int r) { return __builtin_amdgcn_ds_bpermute(c.src[r], v); }

template <class Cv>
KZ_DEV void lp_step2(const LpCtx<Cv>& c, int32_t& r0, int32_t a0, int32_t b0, int32_t& r1, int32_t a1, int32_t b1) {
  const int32_t p = lp_mul(c, lp_sel(c, a0, a1, a0, a1), lp_sel(c, b0, b1, b0, b1));
  r0 = lp_row(c, p, 0);
  r1 = lp_row(c, p, 1);
}
template <class Cv>
KZ_DEV void lp_step3(const LpCtx<Cv>& c, int32_t& r0, int32_t a0, int32_t b0, int32_t& r1, int32_t a1, int32_t b1,
                     int32_t& r2, int32_t a2, int32_t b2) {
  const int32_t p = lp_mul(c, lp_sel(c, a0, a1, a2, a2), lp_sel(c, b0, b1, b2, b2));
  r0 = lp_row(c, p, 0);
  r1 = lp_row(c, p, 1);
  r2 = lp_row(c, p, 2);
}
template <class Cv>
KZ_DEV void lp_step4(const LpCtx<Cv>& c, int32_t& r0, int32_t a0, int32_t b0, int32_t& r1, int32_t a1, int32_t b1,
                     int32_t& r2, int32_t a2, int32_t b2, int32_t& r3, int32_t a3, int32_t b3) {
  const int32_t p = lp_mul(c, lp_sel(c, a0, a1, a2, a3), lp_sel(c, b0, b1, b2, b3));
  r0 = lp_row(c, p, 0);
  r1 = lp_row(c, p, 1);
  r2 = lp_row(c, p, 2);
  r3 = lp_row(c, p, 3);
}

// ---- canonical value (uniform scalar code on row 0's limbs)
// x = (the element) mod p in 29-bit limbs l[0..N-1], each in [0, 2^29)
template <class Cv>
KZ_DEV void lp_canon(int32_t v, int64_t (&l)[LpQ<Cv>::N]) {
  using Q = LpQ<Cv>;
  constexpr int N = Q::N;
  int64_t carry = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {  // exact signed carry propagation: l[N-1] keeps the sign
    const int64_t t = (int64_t)__builtin_amdgcn_readlane(v, j) + carry;
    if (j < N - 1) {
      l[j] = t & LP_M29;
      carry = t >> 29;
    } else {
      l[j] = t;
    }
  }
  // quotient estimate from the top limbs (|value| < 2^13 p: exact to well below 1/2)
  constexpr int S = 32 * (Q::W - 1);
  const double vt = (double)l[N - 1] * __builtin_ldexp(1.0, 29 * (N - 1) - S) +
                    (double)l[N - 2] * __builtin_ldexp(1.0, 29 * (N - 2) - S) +
                    (double)l[N - 3] * __builtin_ldexp(1.0, 29 * (N - 3) - S);
  const int64_t q = (int64_t)__builtin_floor(vt / Q::P_TOP);
  // l -= q p; then at most one +p and one -p fix-up
  auto addmul = [&](int64_t k) {
    int64_t cy = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int64_t t = l[j] + k * (int64_t)Q::MOD[j] + cy;
      if (j < N - 1) {
        l[j] = t & LP_M29;
        cy = t >> 29;
      } else {
        l[j] = t;
      }
    }
  };
  addmul(-q);
  if (l[N - 1] < 0) addmul(1);
  // value >= p ?  (compare via value - p: non-negative top means >= p)
  int64_t cy = 0, top = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const int64_t t = l[j] - (int64_t)Q::MOD[j] + cy;
    if (j < N - 1) cy = t >> 29;
    else top = t;
  }
  if (top >= 0) addmul(-1);
}

// canonical limbs -> the 32-bit-limb words of field.hpp
template <class Cv>
KZ_DEV Fp<typename Cv::FpP> lp_pack(const int64_t (&l)[LpQ<Cv>::N]) {
  using Q = LpQ<Cv>;
  Fp<typename Cv::FpP> r;
  uint64_t buf = 0;
  int nb = 0, k = 0;
#pragma unroll
  for (int j = 0; j < Q::N; ++j) {
    buf |= (uint64_t)l[j] << nb;
    nb += 29;
    if (nb >= 32) {
      if (k < Q::W) r.v[k] = (uint32_t)buf;
      ++k;
      buf >>= 32;
      nb -= 32;
    }
  }
  if (k < Q::W) r.v[k] = (uint32_t)buf;
  return r;
}

// element (lp Montgomery form, x R) -> canonical field.hpp Montgomery form (x R32)
template <class Cv>
KZ_DEV Fp<typename Cv::FpP> lp_to_fp(const LpCtx<Cv>& c, int32_t v) {
  int64_t l[LpQ<Cv>::N];
  lp_canon<Cv>(lp_mul(c, v, c.to32), l);
  return lp_pack<Cv>(l);
}

// canonical field.hpp words in memory (x R32) -> this lane's raw limb of the same integer
template <class Cv>
KZ_DEV int32_t lp_raw_from_words(const uint32_t* w) {
  using Q = LpQ<Cv>;
  const int j = threadIdx.x & 15;
  if (j >= Q::N) return 0;
  const int bit = 29 * j, wi = bit >> 5, sh = bit & 31;
  const uint32_t lo = wi < Q::W ? w[wi] : 0u;
  const uint32_t hi = wi + 1 < Q::W ? w[wi + 1] : 0u;
  return (int32_t)(__builtin_amdgcn_alignbit(hi, lo, sh) & (uint32_t)LP_M29);
}

// ---------------------------------------------------------------------------- G1 (a = 0)
template <class Cv>
struct LpXyzz {  // x = X / ZZ, y = Y / ZZZ
  int32_t x, y, zz, zzz;
  bool inf;
};

// XYZZ record of field.hpp words (canonical; infinity = ZZ 0) -> lp form
template <class Cv>
KZ_DEV LpXyzz<Cv> lp_load_xyzz(const LpCtx<Cv>& c, const Xyzz<Cv>* src) {
  constexpr int N32 = Cv::FpP::N;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(src);
  const int32_t x = lp_raw_from_words<Cv>(w), y = lp_raw_from_words<Cv>(w + N32);
  const int32_t zz = lp_raw_from_words<Cv>(w + 2 * N32), zzz = lp_raw_from_words<Cv>(w + 3 * N32);
  LpXyzz<Cv> p;
  p.inf = __builtin_amdgcn_ballot_w64(zz != 0) == 0;
  lp_step4(c, p.x, x, c.tolp, p.y, y, c.tolp, p.zz, zz, c.tolp, p.zzz, zzz, c.tolp);
  return p;
}

template <class Cv>
KZ_DEV void lp_store_xyzz(const LpCtx<Cv>& c, Xyzz<Cv>* dst, const LpXyzz<Cv>& p) {
  Xyzz<Cv> o = Xyzz<Cv>::inf();
  if (!p.inf) {
    int32_t x, y, zz, zzz;
    lp_step4(c, x, p.x, c.to32, y, p.y, c.to32, zz, p.zz, c.to32, zzz, p.zzz, c.to32);
    int64_t l[LpQ<Cv>::N];
    lp_canon<Cv>(x, l);
    o.x = lp_pack<Cv>(l);
    lp_canon<Cv>(y, l);
    o.y = lp_pack<Cv>(l);
    lp_canon<Cv>(zz, l);
    o.zz = lp_pack<Cv>(l);
    lp_canon<Cv>(zzz, l);
    o.zzz = lp_pack<Cv>(l);
  }
  if (threadIdx.x == 0) *dst = o;
}

// 2P in XYZZ (dbl-2008-s-1), 3 product steps
template <class Cv>
KZ_DEV LpXyzz<Cv> lp_xyzz_dbl(const LpCtx<Cv>& c, const LpXyzz<Cv>& p) {
  const int32_t U = lp_dbl(c, p.y);
  int32_t V, XX, W, S, MM, ZZ3, Y3a, WY, ZZZ3;
  lp_step2(c, V, U, U, XX, p.x, p.x);
  const int32_t M = lp_mul3(c, XX);
  lp_step4(c, W, U, V, S, p.x, V, MM, M, M, ZZ3, V, p.zz);
  LpXyzz<Cv> r;
  r.x = lp_sub(c, MM, lp_dbl(c, S));
  lp_step3(c, Y3a, M, lp_sub(c, S, r.x), WY, W, p.y, ZZZ3, W, p.zzz);
  r.y = lp_sub(c, Y3a, WY);
  r.zz = ZZ3;
  r.zzz = ZZZ3;
  r.inf = p.inf;
  return r;
}

// P + Q in XYZZ (add-2008-s) with the exceptional cases, 4 product steps
template <class Cv>
KZ_DEV LpXyzz<Cv> lp_xyzz_add(const LpCtx<Cv>& c, const LpXyzz<Cv>& p, const LpXyzz<Cv>& q) {
  if (p.inf) return q;
  if (q.inf) return p;
  int32_t U1, U2, S1, S2;
  lp_step4(c, U1, p.x, q.zz, U2, q.x, p.zz, S1, p.y, q.zzz, S2, q.y, p.zzz);
  const int32_t P = lp_sub(c, U2, U1), R = lp_sub(c, S2, S1);
  // row-local zero tests (|P|, |R| < 3 p; every row holds the same value): a reduction and carry
  // passes on the row, not a serial readlane canonicalisation (lp_canon): with the XYZZ running
  // sum, k_window_combine 0.436 -> 0.369 ms (profiles/r05/ab_window_combine.txt)
  if (lp_row_is_zero(c, P)) {
    if (lp_row_is_zero(c, R)) return lp_xyzz_dbl(c, p);
    LpXyzz<Cv> o = p;
    o.inf = true;
    return o;
  }
  int32_t PP, ZZ12, ZZZ12, RR, PPP, Q, ZZ3, ZZZ3, T, Y3a;
  lp_step4(c, PP, P, P, ZZ12, p.zz, q.zz, ZZZ12, p.zzz, q.zzz, RR, R, R);
  lp_step3(c, PPP, P, PP, Q, U1, PP, ZZ3, ZZ12, PP);
  LpXyzz<Cv> r;
  r.x = lp_sub(c, lp_sub(c, RR, PPP), lp_dbl(c, Q));
  lp_step3(c, ZZZ3, ZZZ12, PPP, T, S1, PPP, Y3a, R, lp_sub(c, Q, r.x));
  r.y = lp_sub(c, Y3a, T);
  r.zz = ZZ3;
  r.zzz = ZZZ3;
  r.inf = false;
  return r;
}

}  // namespace kzgmi
