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
// additions, one thread per point; beta is chosen in tools/gen_params.py by checking the
// identity on the generator.
#pragma once
#include <type_traits>

#include "kernels.hpp"

namespace kzgmi {

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
      F y = fp_pow_words(rhs, P::SQRT_EXP);
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

// [|x|] q by the fixed bit pattern of the BLS parameter (uniform control flow)
template <class Cv, class Base>
KZ_DEV Xyzz<Cv> mul_by_x_abs(const Base& q, const Xyzz<Cv>& q_xyzz) {
  constexpr uint64_t X = Cv::K::X_ABS;
  Xyzz<Cv> acc = q_xyzz;  // top bit
  for (int b = 62; b >= 0; --b) {
    acc = xyzz_dbl(acc);
    if ((X >> b) & 1) {
      if constexpr (std::is_same_v<Base, Affine<Cv>>) acc = xyzz_add_affine(acc, q);
      else acc = xyzz_add(acc, q);
    }
  }
  return acc;
}

template <class Cv>
__global__ void __launch_bounds__(256) k_subgroup_check(const Affine<Cv>* __restrict__ pts,
                                                        const uint8_t* __restrict__ inf, uint32_t n,
                                                        uint32_t* __restrict__ err) {
  static_assert(Cv::ID == 0, "BN254 G1 has cofactor 1: no subgroup check");
  using P = typename Cv::FpP;
  using F = Fp<P>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || inf[i]) return;
  const Affine<Cv> p = pts[i];
  const Xyzz<Cv> q1 = mul_by_x_abs<Cv>(p, xyzz_from_affine(p));
  const Xyzz<Cv> q2 = mul_by_x_abs<Cv>(q1, q1);  // [x^2] p
  // p in G1 <=> q2 == -phi(p) = (beta x, -y): X2 == beta x ZZ2 and Y2 == -y ZZZ2, q2 finite
  const F bx = fp_mul(F::from_const(Cv::K::BETA_M), p.x);
  const bool ok = !q2.is_inf() && q2.x == fp_mul(bx, q2.zz) && q2.y == fp_mul(fp_neg(p.y), q2.zzz);
  if (!ok) raise_err(err, DERR_NOT_IN_SUBGROUP);
}

}  // namespace kzgmi
