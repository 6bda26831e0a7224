// Modular inversion for the single-lane tails (MSM result -> affine, the pairing's Fp inversion):
// the optimised binary GCD of T. Pornin ("Optimized Binary GCD for Modular Inversion", IACR
// ePrint 2020/972, Algorithm 2), with K = 30 inner steps per outer step.
//
// The classic binary extended Euclid (field.hpp fp_inv before round 3) halves one N-limb
// cofactor modulo p for every bit it strips: ~760 steps of four N-limb passes, ~566 K cycles
// for BLS12-381 on one lane.  Here each outer step runs K = 30 binary-GCD steps on 64-bit
// approximations of a and b (their low K bits and their top K + 2 bits), collecting the steps
// in a 2 x 2 matrix of signed factors (|f| + |g| <= 2^K), then applies it once to the N-limb
// a, b and to the cofactors u, v (the cofactor update divides by 2^K modulo m with one
// Montgomery-style correction t m).  ceil((2 len(m) - 1) / K) outer steps (26 for a 381-bit
// modulus, 17 for 254 bits) leave b = gcd = 1 and v = y^-1 mod m; the loop leaves as soon as a
// reaches 0.
//
// Variable time (the inputs of a verifier are public).  Host + device: tests/test_bingcd.py
// runs the host build (tools/bingcd_check.cpp) against Python's pow(y, -1, m).
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace kzgmi {

#define KZ_HD __host__ __device__ __forceinline__

template <int N>
struct BinGcd {
  static constexpr int K = 30;
  static constexpr uint32_t MASK = (1u << K) - 1;

  static KZ_HD int bitlen(const uint32_t (&x)[N]) {
    int len = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (x[i]) len = 32 * i + 32 - __builtin_clz(x[i]);
    return len;
  }
  // the 32 bits of x from bit pos (0 <= pos < 32 N); no dynamic register indexing
  static KZ_HD uint32_t bits32(const uint32_t (&x)[N], int pos) {
    const int w = pos >> 5, s = pos & 31;
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      lo = i == w ? x[i] : lo;
      hi = i == w + 1 ? x[i] : hi;
    }
    return (uint32_t)((((uint64_t)hi << 32) | lo) >> s);
  }
  // x = (a f + b g) / 2^K (exact); returns true and stores |x| if x < 0
  static KZ_HD bool lin(const uint32_t (&a)[N], const uint32_t (&b)[N], int64_t f, int64_t g, uint32_t (&x)[N]) {
    uint32_t lo[N + 1];
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int64_t t = (int64_t)a[i] * f + (int64_t)b[i] * g + c;  // |t| < 2^62 + 2^31
      lo[i] = (uint32_t)t;
      c = t >> 32;
    }
    lo[N] = (uint32_t)c;
    return shift_abs(lo, x);
  }
  // lo (N + 1 limbs, two's complement) >> K into x as a magnitude; true if negative
  static KZ_HD bool shift_abs(const uint32_t (&lo)[N + 1], uint32_t (&x)[N]) {
    const bool neg = (int32_t)lo[N] < 0;
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = (lo[i] >> K) | (lo[i + 1] << (32 - K));
    if (neg) {  // |x| < 2^(32 N - 1): the N-limb two's complement negation is exact
      uint32_t cy = 1;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const uint64_t t = (uint64_t)(~x[i]) + cy;
        x[i] = (uint32_t)t;
        cy = (uint32_t)(t >> 32);
      }
    }
    return neg;
  }
  // x = (u f + v g) / 2^K mod m, in [0, m) (u, v in [0, m); nmi = -m^-1 mod 2^K)
  static KZ_HD void linmod(const uint32_t (&u)[N], const uint32_t (&v)[N], int64_t f, int64_t g,
                           const uint32_t (&m)[N], uint32_t nmi, uint32_t (&x)[N]) {
    const int64_t x0 = (int64_t)u[0] * f + (int64_t)v[0] * g;
    const int64_t t = (int64_t)(((uint32_t)x0 * nmi) & MASK);  // x + t m = 0 mod 2^K
    uint32_t lo[N + 1];
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int64_t s = (int64_t)u[i] * f + (int64_t)v[i] * g + t * (int64_t)m[i] + c;  // |s| < 2^63
      lo[i] = (uint32_t)s;
      c = s >> 32;
    }
    lo[N] = (uint32_t)c;
    // (x + t m) / 2^K lies in (-m, 2m): bring it into [0, m)
    const bool neg = (int32_t)lo[N] < 0;
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = (lo[i] >> K) | (lo[i + 1] << (32 - K));
    if (neg) {  // x + m (two's complement wraps to the value in [0, m))
      uint32_t cy = 0;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const uint64_t s = (uint64_t)x[i] + m[i] + cy;
        x[i] = (uint32_t)s;
        cy = (uint32_t)(s >> 32);
      }
    } else {  // x >= m ? x - m
      uint32_t d[N], bw = 0;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const uint64_t s = (uint64_t)x[i] - m[i] - bw;
        d[i] = (uint32_t)s;
        bw = (uint32_t)(s >> 63);
      }
      if (!bw) {
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] = d[i];
      }
    }
  }

  // out = y^-1 mod m for odd m of len_m bits, 0 < y < m (y = 0 gives 0)
  static KZ_HD void inv(const uint32_t (&y)[N], const uint32_t (&m)[N], int len_m, uint32_t (&out)[N]) {
    uint32_t a[N], b[N], u[N], v[N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      a[i] = y[i];
      b[i] = m[i];
      u[i] = 0;
      v[i] = 0;
    }
    u[0] = 1;
    uint32_t mi = m[0];  // m^-1 mod 2^32 by Newton steps (m odd: 5 doublings of precision)
#pragma unroll
    for (int k = 0; k < 5; ++k) mi *= 2u - m[0] * mi;
    const uint32_t nmi = (0u - mi) & MASK;
    const int steps = (2 * len_m - 1 + K - 1) / K;
    for (int it = 0; it < steps; ++it) {
      const int la = bitlen(a), lb = bitlen(b);
      // a = 0: b = gcd = 1 and every further step keeps v (f0 = 1, g0 = 0, f1 = g1 = 2^K:
      // u <- u / 2^K, v <- v).  Random 381-bit inputs get there after 17-20 of the 26 steps
      // (variable time: a verifier's inputs are public)
      if (la == 0) break;
      int n = la > lb ? la : lb;
      n = n > 2 * K + 2 ? n : 2 * K + 2;
      uint64_t aa = (uint64_t)(a[0] & MASK) | ((uint64_t)bits32(a, n - (K + 2)) << K);
      uint64_t bb = (uint64_t)(b[0] & MASK) | ((uint64_t)bits32(b, n - (K + 2)) << K);
      int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
      for (int j = 0; j < K; ++j) {
        if (aa & 1) {
          if (aa < bb) {
            const uint64_t t = aa;
            aa = bb;
            bb = t;
            int64_t s = f0;
            f0 = f1;
            f1 = s;
            s = g0;
            g0 = g1;
            g1 = s;
          }
          aa = (aa - bb) >> 1;
          f0 -= f1;
          g0 -= g1;
        } else {
          aa >>= 1;
        }
        f1 *= 2;
        g1 *= 2;
      }
      uint32_t na[N], nb[N];
      if (lin(a, b, f0, g0, na)) {
        f0 = -f0;
        g0 = -g0;
      }
      if (lin(a, b, f1, g1, nb)) {
        f1 = -f1;
        g1 = -g1;
      }
      uint32_t nu[N], nv[N];
      linmod(u, v, f0, g0, m, nmi, nu);
      linmod(u, v, f1, g1, m, nmi, nv);
#pragma unroll
      for (int i = 0; i < N; ++i) {
        a[i] = na[i];
        b[i] = nb[i];
        u[i] = nu[i];
        v[i] = nv[i];
      }
    }
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = v[i];
  }
};

#undef KZ_HD

}  // namespace kzgmi
