// GLV endomorphism for the G1 MSMs.
//
// phi(x, y) = (beta x, y) acts on G1 as [lambda] with lambda^2 + lambda + 1 = 0 mod r, so a
// full Fr scalar k splits into two half-size ones: k P = k0 P + k1 phi(P) with |k0|, |k1| <
// 2^127 (Babai rounding in the reduced lattice basis v1, v2 of {(a, b): a + b lambda = 0};
// constants and bounds generated and checked by tools/gen_params.py, restated in
// tests/test_glv.py).  A 255-bit MSM then needs 8 signed 16-bit windows per point over twice
// the points instead of 16: the same number of bucket additions, half the bucket sets to
// reduce and half the serial window-combination doublings.
//
// Half-scalar format (what k_bin_count/k_bin_scatter read with scal_words = 4): |k_i| in
// bits 0..126 of 4 LE words, bit 127 = "negative" (the term uses -P; msm.hpp folds it into
// the entry's sign bit).  127-bit randomisers r_i have bit 127 clear, so both share a path.
// Reference: none (LICENSE only); results are bit-identical to the unsplit MSM and checked
// against the C oracle (tests/test_gpu_parity.py, test_gpu_glv.py).
#pragma once
#include "g1.hpp"

namespace kzgmi {

// c = round(k g / r) for k < r (8 LE words) and g < 2^128, i.e. floor((k g + (r-1)/2) / r);
// Barrett reduction with mu = floor(2^512 / r) (HAC 14.42, b = 2^32, k = 8 words).  The
// quotient is < 2^128 because g < 2^128 and k < r.
template <class Cv>
KZ_DEV void glv_round_div(const uint32_t (&k)[8], const uint32_t (&g)[4], uint32_t (&c)[4]) {
  using K = typename Cv::K;
  const uint32_t* R = Cv::FrP::MOD;
  uint32_t N[12];
#pragma unroll
  for (int i = 0; i < 12; ++i) N[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint64_t t = (uint64_t)k[i] * g[j] + N[i + j] + carry;
      N[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    N[i + 4] = (uint32_t)carry;
  }
  {
    uint32_t cy = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) N[i] = __builtin_addc(N[i], K::GLV_HALF_R[i], cy, &cy);
#pragma unroll
    for (int i = 8; i < 12; ++i) N[i] = __builtin_addc(N[i], 0u, cy, &cy);
  }
  // q3 = ((N >> 224) * mu) >> 288
  uint32_t q2[14];
#pragma unroll
  for (int i = 0; i < 14; ++i) q2[i] = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      uint64_t t = (uint64_t)N[7 + i] * K::GLV_MU[j] + q2[i + j] + carry;
      q2[i + j] = (uint32_t)t;
      carry = t >> 32;
    }
    q2[i + 9] = (uint32_t)carry;
  }
  uint32_t q[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) q[i] = q2[9 + i];
  // rem = N - q r (low 9 words suffice: rem < 3r < 2^288)
  uint32_t qr[9];
#pragma unroll
  for (int i = 0; i < 9; ++i) qr[i] = 0;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (i + j < 9) {
        uint64_t t = (uint64_t)q[i] * R[j] + qr[i + j] + carry;
        qr[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
    }
    if (i + 8 < 9) qr[i + 8] = (uint32_t)carry;
  }
  uint32_t rem[9];
  {
    uint32_t bw = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) rem[i] = __builtin_subc(N[i], qr[i], bw, &bw);
  }
#pragma unroll
  for (int it = 0; it < 2; ++it) {  // Barrett: at most two corrections
    uint32_t d[9], bw = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = __builtin_subc(rem[i], R[i], bw, &bw);
    d[8] = __builtin_subc(rem[8], 0u, bw, &bw);
    if (!bw) {
#pragma unroll
      for (int i = 0; i < 9; ++i) rem[i] = d[i];
      uint32_t cy = 1;
#pragma unroll
      for (int i = 0; i < 5; ++i) q[i] = __builtin_addc(q[i], 0u, cy, &cy);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) c[i] = q[i];
}

// low 128 bits of a * b (4-word operands)
KZ_DEV void mul_lo128(const uint32_t (&a)[4], const uint32_t* b, uint32_t (&out)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint64_t carry = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (i + j < 4) {
        uint64_t t = (uint64_t)a[i] * b[j] + out[i + j] + carry;
        out[i + j] = (uint32_t)t;
        carry = t >> 32;
      }
    }
  }
}

KZ_DEV void sub128(uint32_t (&a)[4], const uint32_t (&b)[4]) {
  uint32_t bw = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) a[i] = __builtin_subc(a[i], b[i], bw, &bw);
}

// two's-complement 128-bit value (|v| < 2^127) -> magnitude with bit 127 = sign
KZ_DEV void to_sign_magnitude(uint32_t (&v)[4]) {
  const bool neg = (v[3] >> 31) != 0;
  if (neg) {
    uint32_t bw = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __builtin_subc(0u, v[i], bw, &bw);
    v[3] |= 0x80000000u;
  }
}

// k (< r, 8 LE words) -> half scalars h0, h1 with k = h0 + h1 lambda (mod r)
template <class Cv>
KZ_DEV void glv_split(const uint32_t (&k)[8], uint32_t (&h0)[4], uint32_t (&h1)[4]) {
  using K = typename Cv::K;
  uint32_t g1[4], g2[4], c1[4], c2[4], t[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) { g1[i] = K::GLV_G1[i]; g2[i] = K::GLV_G2[i]; }
  glv_round_div<Cv>(k, g1, c1);
  glv_round_div<Cv>(k, g2, c2);
  // k0 = k - c1 a1 - c2 a2,  k1 = -c1 b1 - c2 b2   (mod 2^128; the true values fit)
#pragma unroll
  for (int i = 0; i < 4; ++i) { h0[i] = k[i]; h1[i] = 0; }
  mul_lo128(c1, K::GLV_A1, t);
  sub128(h0, t);
  mul_lo128(c2, K::GLV_A2, t);
  sub128(h0, t);
  mul_lo128(c1, K::GLV_B1, t);
  sub128(h1, t);
  mul_lo128(c2, K::GLV_B2, t);
  sub128(h1, t);
  to_sign_magnitude(h0);
  to_sign_magnitude(h1);
}

// scal: n scalars of 8 LE words at `stride` words apart -> h0[4 i..], h1[4 i..]
template <class Cv>
__global__ void __launch_bounds__(256) k_glv_split(const uint32_t* __restrict__ scal, uint32_t stride, uint32_t n,
                                                   uint32_t* __restrict__ h0, uint32_t* __restrict__ h1) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t k[8], a[4], b[4];
  const uint4* s = reinterpret_cast<const uint4*>(scal + (size_t)i * stride);
  uint4 q0 = s[0], q1 = s[1];
  k[0] = q0.x; k[1] = q0.y; k[2] = q0.z; k[3] = q0.w;
  k[4] = q1.x; k[5] = q1.y; k[6] = q1.z; k[7] = q1.w;
  glv_split<Cv>(k, a, b);
  reinterpret_cast<uint4*>(h0)[i] = make_uint4(a[0], a[1], a[2], a[3]);
  reinterpret_cast<uint4*>(h1)[i] = make_uint4(b[0], b[1], b[2], b[3]);
}

// dst[i] = phi(src[i]) = (beta x, y); infinity flags copied
template <class Cv>
__global__ void __launch_bounds__(256) k_endo_points(const Affine<Cv>* __restrict__ src, const uint8_t* __restrict__ src_inf,
                                                     uint32_t n, Affine<Cv>* __restrict__ dst,
                                                     uint8_t* __restrict__ dst_inf) {
  using F = Fp<typename Cv::FpP>;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<Cv> a = src[i];
  a.x = fp_mul(F::from_const(Cv::K::GLV_BETA_M), a.x);
  dst[i] = a;
  dst_inf[i] = src_inf[i];
}

}  // namespace kzgmi
