// Non-MSM device kernels: input decoding/validation, scalar preparation (randomisers,
// s_i = r_i z_i, t = sum r_i y_i), pairing check, output encoding, partial sums (multi-GPU),
// and the synthetic-input generators.  Reference: none (LICENSE only); semantics of every
// kernel are those of oracle/pyspec/kzg.py, checked bit-exactly against the C oracle.
#pragma once
#include "msm.hpp"
#include "glv.hpp"
#include "pairing.hpp"

namespace kzgmi {

struct Seed {
  uint32_t w[8];  // big-endian words of the 32-byte seed
};

// ------------------------------------------------------------------------------ decoding
template <int NW>
KZ_DEV void load_words(const uint8_t* src, uint32_t (&w)[NW]) {
  static_assert(NW % 4 == 0, "16-byte granules");
  const uint4* s = reinterpret_cast<const uint4*>(src);
#pragma unroll
  for (int k = 0; k < NW / 4; ++k) {
    uint4 q = s[k];
    w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
  }
}
template <int NW>
KZ_DEV void store_words(uint8_t* dst, const uint32_t (&w)[NW]) {
  uint4* d = reinterpret_cast<uint4*>(dst);
#pragma unroll
  for (int k = 0; k < NW / 4; ++k) d[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}

// bytes (as loaded little-endian words) big-endian field element at word offset `o`
template <class P, int NW>
KZ_DEV Fp<P> fp_from_be_words(const uint32_t (&w)[NW], int o) {
  Fp<P> r;
#pragma unroll
  for (int k = 0; k < P::N; ++k) r.v[k] = __builtin_bswap32(w[o + P::N - 1 - k]);
  return r;
}
template <class P, int NW>
KZ_DEV void fp_to_be_words(const Fp<P>& a, uint32_t (&w)[NW], int o) {
#pragma unroll
  for (int k = 0; k < P::N; ++k) w[o + P::N - 1 - k] = __builtin_bswap32(a.v[k]);
}

// G1 encoding -> affine Montgomery point + infinity flag (errors into *err)
// To29: the validated point is stored directly in the accumulation's radix-29
// format (what k_pts_to29 would make of it), saving that kernel's pass over the points.
// img != nullptr (To29, GLV batches): phi(P) = (beta x, y) is stored at img[i] too -- what
// k_endo_points29 would compute from pts[i] after a second pass over the points.
template <class Cv, bool To29 = false>
__global__ void __launch_bounds__(256) k_convert_points(const uint8_t* __restrict__ bytes, uint32_t n,
                                                        Affine<Cv>* __restrict__ pts, uint8_t* __restrict__ inf,
                                                        uint32_t* __restrict__ err, Affine<Cv>* __restrict__ img = nullptr,
                                                        uint8_t* __restrict__ img_inf = nullptr) {
  using P = typename Cv::FpP;
  constexpr int NW = 2 * P::N;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[NW];
  load_words(bytes + (size_t)i * 4 * NW, w);
  uint32_t any = 0;
#pragma unroll
  for (int k = 1; k < NW; ++k) any |= w[k];
  bool is_inf = false;
  if constexpr (Cv::ID == 0) {
    uint32_t flags = w[0] & 0xe0u;  // byte 0 = low byte of the little-endian word
    if (flags & 0x80u) { raise_err(err, DERR_ENCODING); is_inf = true; }
    else if (flags & 0x40u) {
      if (w[0] != 0x40u || any) raise_err(err, DERR_ENCODING);  // exactly 0x40 || zeros
      is_inf = true;
    } else if (flags & 0x20u) { raise_err(err, DERR_ENCODING); is_inf = true; }
  } else {
    is_inf = (any | w[0]) == 0;
  }
  if constexpr (To29) {  // x R29 = mont29(x, R29^2); on-curve test y^2 - x^3 - b == 0 in radix 29
    using Q = Fp29Of<Cv>;
    F29<Q> x29 = F29<Q>::zero(), y29 = F29<Q>::zero();
    if (!is_inf) {
      const Fp<P> x = fp_from_be_words<P>(w, 0), y = fp_from_be_words<P>(w, P::N);
      if (!fp_raw_lt_mod(x) || !fp_raw_lt_mod(y)) {
        raise_err(err, DERR_ENCODING);
        is_inf = true;
      } else {
        const F29<Q> r2 = F29<Q>::from_const(Q::R2);
        x29 = mul29(limbs29<Q>(x.v), r2);  // < p (1 + 2^-24): inputs < p
        y29 = mul29(limbs29<Q>(y.v), r2);
        const F29<Q> rhs = add3_29(mul29(sqr29(x29), x29), F29<Q>::from_const(Q::BCURVE), F29<Q>::zero());  // < 2.1 p
        if (!is_zero29(sub29(sqr29(y29), rhs, Q::B4))) {  // < 5.1 p, within is_zero29's range
          raise_err(err, DERR_NOT_ON_CURVE);
          is_inf = true;
        }
      }
      if (is_inf) x29 = y29 = F29<Q>::zero();
    }
    store_pt29<Cv>(pts + i, x29, y29);
    if (img) {  // x29 < (p / R29 + 1) p; beta R29 likewise: the product stays below it (k_endo_points29)
      store_pt29<Cv>(img + i, mul29(x29, fp_to29<Q>(Fp<P>::from_const(Cv::K::GLV_BETA_M))), y29);
      img_inf[i] = is_inf ? 1 : 0;
    }
  } else {
    Affine<Cv> a;
    if (is_inf) {
      a.x = Fp<P>::zero();
      a.y = Fp<P>::zero();
    } else {
      Fp<P> x = fp_from_be_words<P>(w, 0), y = fp_from_be_words<P>(w, P::N);
      if (!fp_raw_lt_mod(x) || !fp_raw_lt_mod(y)) { raise_err(err, DERR_ENCODING); is_inf = true; }
      a.x = fp_to_mont(x);
      a.y = fp_to_mont(y);
      if (!is_inf && !affine_on_curve(a)) { raise_err(err, DERR_NOT_ON_CURVE); is_inf = true; }
    }
    uint32_t o[NW];
#pragma unroll
    for (int k = 0; k < P::N; ++k) { o[k] = a.x.v[k]; o[P::N + k] = a.y.v[k]; }
    store_words(reinterpret_cast<uint8_t*>(pts + i), o);
  }
  inf[i] = is_inf ? 1 : 0;
}

template <class Cv>
__global__ void k_set_generator(Affine<Cv>* pts, uint8_t* inf) {
  using P = typename Cv::FpP;
  pts->x = Fp<P>::from_const(Cv::K::G1X_M);
  pts->y = Fp<P>::from_const(Cv::K::G1Y_M);
  *inf = 0;
}

// Fr scalar (32 B BE) -> 8 LE words, canonical check
template <class Cv>
__global__ void __launch_bounds__(256) k_convert_scalars(const uint8_t* __restrict__ bytes, uint32_t n,
                                                         uint32_t* __restrict__ out, uint32_t* __restrict__ err) {
  using R = typename Cv::FrP;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  load_words(bytes + (size_t)i * 32, w);
  Fp<R> s = fp_from_be_words<R>(w, 0);
  if (!fp_raw_lt_mod(s)) { raise_err(err, DERR_SCALAR); s = Fp<R>::zero(); }
  store_words(reinterpret_cast<uint8_t*>(out + 8 * (size_t)i), s.v);
}

// G2 encoding (x.c1, x.c0, y.c1, y.c0) -> affine Montgomery twist point
template <class Cv>
__global__ void k_convert_g2(const uint8_t* __restrict__ bytes, uint32_t n, G2Aff<Cv>* __restrict__ out,
                             uint8_t* __restrict__ inf, uint32_t* __restrict__ err) {
  using P = typename Cv::FpP;
  constexpr int NW = 4 * P::N;
  uint32_t i = threadIdx.x;
  if (i >= n) return;
  uint32_t w[NW];
  load_words(bytes + (size_t)i * 4 * NW, w);
  uint32_t any = 0;
#pragma unroll
  for (int k = 1; k < NW; ++k) any |= w[k];
  bool is_inf = false;
  if constexpr (Cv::ID == 0) {
    if (w[0] & 0x80u) { raise_err(err, DERR_ENCODING); is_inf = true; }
    else if (w[0] & 0x40u) is_inf = true;
  } else {
    is_inf = (any | w[0]) == 0;
  }
  G2Aff<Cv> q;
  q.x = Fp2<Cv>::zero();
  q.y = Fp2<Cv>::zero();
  if (!is_inf) {
    Fp<P> v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k] = fp_from_be_words<P>(w, k * P::N);
      if (!fp_raw_lt_mod(v[k])) { raise_err(err, DERR_ENCODING); is_inf = true; }
      v[k] = fp_to_mont(v[k]);
    }
    q.x = {v[1], v[0]};
    q.y = {v[3], v[2]};
    auto lhs = f2_sqr(q.y);
    auto rhs = f2_add(f2_mul(f2_sqr(q.x), q.x), f2_const<Cv>(Cv::K::B2_M));
    if (!is_inf && !(lhs == rhs)) { raise_err(err, DERR_NOT_ON_CURVE); is_inf = true; }
  }
  out[i] = q;
  inf[i] = is_inf ? 1 : 0;
}

// ------------------------------------------------------------------------------ scalar prep
// r_i (127-bit, 4 words), s_i = r_i z_i mod r (8 words), per-block partial sum of r_i y_i.
// seed_dev != null: the seed's 8 big-endian words are read from device memory (the
// Fiat-Shamir challenge r computed on the GPU by k_fs_challenge) instead of `seed`.
// h0 != null (GLV batches): s_i leaves as its GLV half scalars (h0[i], h1[i], k_glv_split's
// output) instead of 8 words -- no second kernel reading s back.
constexpr int PREP_BLOCK = 256;

template <class Cv>
__global__ void __launch_bounds__(PREP_BLOCK) k_scalar_prep(Seed seed, const uint32_t* __restrict__ seed_dev,
                                                            uint64_t index_offset,
                                                            const uint8_t* __restrict__ zs, const uint8_t* __restrict__ ys,
                                                            uint32_t n, uint32_t* __restrict__ r_out,
                                                            uint32_t* __restrict__ s_out, Fp<typename Cv::FrP>* __restrict__ tpart,
                                                            uint32_t* __restrict__ err, uint32_t* __restrict__ h0 = nullptr,
                                                            uint32_t* __restrict__ h1 = nullptr) {
  using R = typename Cv::FrP;
  using F = Fp<R>;
  __shared__ F lds[PREP_BLOCK];
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (seed_dev) {
#pragma unroll
    for (int k = 0; k < 8; ++k) seed.w[k] = seed_dev[k];
  }
  F acc = F::zero();
  if (i < n) {
    uint32_t wz[8], wy[8];
    load_words(zs + (size_t)i * 32, wz);
    load_words(ys + (size_t)i * 32, wy);
    F z = fp_from_be_words<R>(wz, 0), y = fp_from_be_words<R>(wy, 0);
    if (!fp_raw_lt_mod(z) || !fp_raw_lt_mod(y)) { raise_err(err, DERR_SCALAR); z = F::zero(); y = F::zero(); }
    uint32_t r4[4];
    randomizer127(seed.w, index_offset + i, r4);
    F r = F::zero();
#pragma unroll
    for (int k = 0; k < 4; ++k) r.v[k] = r4[k];
    F rm = fp_to_mont(r);
    F s = fp_mul(rm, z);  // r z (standard form)
    acc = fp_mul(rm, y);  // r y (standard form)
    *reinterpret_cast<uint4*>(r_out + 4 * (size_t)i) = make_uint4(r4[0], r4[1], r4[2], r4[3]);
    if (h0) {
      uint32_t k[8], a[4], b[4];
#pragma unroll
      for (int j = 0; j < 8; ++j) k[j] = s.v[j];
      glv_split<Cv>(k, a, b);
      reinterpret_cast<uint4*>(h0)[i] = make_uint4(a[0], a[1], a[2], a[3]);
      reinterpret_cast<uint4*>(h1)[i] = make_uint4(b[0], b[1], b[2], b[3]);
    } else {
      store_words(reinterpret_cast<uint8_t*>(s_out + 8 * (size_t)i), s.v);
    }
  }
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (int st = PREP_BLOCK / 2; st >= 1; st >>= 1) {
    if ((int)threadIdx.x < st) lds[threadIdx.x] = fp_add(lds[threadIdx.x], lds[threadIdx.x + st]);
    __syncthreads();
  }
  if (threadIdx.x == 0) tpart[blockIdx.x] = lds[0];
}

// negt = -(sum of partials) mod r, as 8 LE words
template <class Cv>
__global__ void __launch_bounds__(256) k_tsum(const Fp<typename Cv::FrP>* __restrict__ tpart, uint32_t nblocks,
                                              uint32_t* __restrict__ negt) {
  using F = Fp<typename Cv::FrP>;
  __shared__ F lds[256];
  F acc = F::zero();
  for (uint32_t b = threadIdx.x; b < nblocks; b += 256) acc = fp_add(acc, tpart[b]);
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (int st = 128; st >= 1; st >>= 1) {
    if ((int)threadIdx.x < st) lds[threadIdx.x] = fp_add(lds[threadIdx.x], lds[threadIdx.x + st]);
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    F t = fp_neg(lds[0]);
#pragma unroll
    for (int k = 0; k < 8; ++k) negt[k] = t.v[k];
  }
}

// ------------------------------------------------------------------------------ pairing check
// res[0] = A, res[1] = B (XYZZ).  lines: [tau]_2 lines then [1]_2 lines.  q_inf: G2 flags.
template <class Cv>
__global__ void k_pairing_check(const Xyzz<Cv>* __restrict__ res, const Line<Cv>* __restrict__ lines,
                                const uint8_t* __restrict__ q_inf, int* __restrict__ ok) {
  if (threadIdx.x != 0) return;
  Xyzz<Cv> A = load_xyzz(&res[0]);
  Xyzz<Cv> B = load_xyzz(&res[1]);
  Homog<Cv> P[2] = {homog_from_xyzz(A, false), homog_from_xyzz(B, true)};
  bool skip[2] = {A.is_inf() || q_inf[0] != 0, B.is_inf() || q_inf[1] != 0};
  Fp12<Cv> f = miller2(lines, P, skip);
  f = final_exp(f);
  *ok = f12_is_one(f) ? 1 : 0;
}

// e(P, Q) for one pair (diagnostic API): lines for Q at slot 0
template <class Cv>
__global__ void k_pairing_one(const Affine<Cv>* __restrict__ p, const uint8_t* __restrict__ p_inf,
                              const Line<Cv>* __restrict__ lines, const uint8_t* __restrict__ q_inf,
                              uint8_t* __restrict__ out) {
  using P = typename Cv::FpP;
  if (threadIdx.x != 0) return;
  Xyzz<Cv> X = xyzz_from_affine(*p);
  Homog<Cv> H[2] = {homog_from_xyzz(X, false), homog_from_xyzz(X, false)};
  bool skip[2] = {p_inf[0] != 0 || q_inf[0] != 0, true};
  Fp12<Cv> f = final_exp(miller2(lines, H, skip));
  const Fp<P>* c[12] = {&f.c0.c0.c0, &f.c0.c0.c1, &f.c0.c1.c0, &f.c0.c1.c1, &f.c0.c2.c0, &f.c0.c2.c1,
                        &f.c1.c0.c0, &f.c1.c0.c1, &f.c1.c1.c0, &f.c1.c1.c1, &f.c1.c2.c0, &f.c1.c2.c1};
  for (int k = 0; k < 12; ++k) {
    Fp<P> v = fp_from_mont(*c[k]);
    uint32_t w[P::N];
#pragma unroll
    for (int j = 0; j < P::N; ++j) w[P::N - 1 - j] = __builtin_bswap32(v.v[j]);
    uint32_t* o = reinterpret_cast<uint32_t*>(out + k * 4 * P::N);
#pragma unroll
    for (int j = 0; j < P::N; ++j) o[j] = w[j];
  }
}

// XYZZ -> G1 encoding, one wave per point: the record's words are made wave-uniform
// (readfirstlane), so the conversion's inversion compiles to scalar code instead of one lane's
// vector code under an exec mask (the same change took the pairing's inversion round 245 K -> ~140 K
// cycles, profiles/r05/ab_pairing_inv_uniform.txt); lane 0 stores.
template <class Cv>
KZ_DEV void fp_uniform(Fp<typename Cv::FpP>& a) {
#pragma unroll
  for (int k = 0; k < Cv::FpP::N; ++k) a.v[k] = (uint32_t)__builtin_amdgcn_readfirstlane((int)a.v[k]);
}
template <class Cv>
__global__ void __launch_bounds__(64) k_encode_points(const Xyzz<Cv>* __restrict__ res, uint32_t count,
                                                      uint8_t* __restrict__ out) {
  using P = typename Cv::FpP;
  constexpr int NW = 2 * P::N;
  const uint32_t i = blockIdx.x;
  if (i >= count) return;
  Xyzz<Cv> p = load_xyzz(&res[i]);
  fp_uniform<Cv>(p.x);
  fp_uniform<Cv>(p.y);
  fp_uniform<Cv>(p.zz);
  fp_uniform<Cv>(p.zzz);
  Affine<Cv> a;
  uint32_t w[NW];
  const bool finite = !p.is_inf();
  if (finite) {  // xyzz_to_affine with the inversion inlined (its out-of-line form takes VGPR arguments)
    const auto I = fp_inv(fp_mul(p.zz, p.zzz));
    a.x = fp_mul(p.x, fp_mul(p.zzz, I));
    a.y = fp_mul(p.y, fp_mul(p.zz, I));
  }
  if (!finite) {
#pragma unroll
    for (int k = 0; k < NW; ++k) w[k] = 0;
    if constexpr (Cv::ID == 0) w[0] = 0x40u;
  } else {
    fp_to_be_words(fp_from_mont(a.x), w, 0);
    fp_to_be_words(fp_from_mont(a.y), w, P::N);
  }
  if (threadIdx.x == 0) store_words(out + (size_t)i * 4 * NW, w);
}

// A shard partial record that failed on its own device (or rank) is marked, not dropped: its x
// words are all ones (no Montgomery value < p has that top limb) and y.v[0] holds the device
// error code.  Records the caller marks by filling every byte with 0xFF read as DERR_SHARD.
// Every combine that reads the record then fails too, so no rank can accept a batch one of
// whose shards was rejected (include/kzgmi.h, multi-GPU section).
template <class Cv>
KZ_DEV uint32_t partial_mark(const Xyzz<Cv>& p) {
  if (p.x.v[Cv::FpP::N - 1] != 0xffffffffu) return DERR_NONE;
  const uint32_t code = p.y.v[0];
  return code >= DERR_ENCODING && code < DERR_SHARD ? code : DERR_SHARD;
}

// partial records out (count of them) = res, or marked records when *err != 0
template <class Cv>
__global__ void k_partial_out(const Xyzz<Cv>* __restrict__ res, uint32_t count, const uint32_t* __restrict__ err,
                              Xyzz<Cv>* __restrict__ out) {
  const uint32_t k = threadIdx.x;
  if (k >= count) return;
  const uint32_t e = *err;
  Xyzz<Cv> p = load_xyzz(&res[k]);
  if (e) {
    using F = typename Xyzz<Cv>::F;
    p.y = F::zero();
    p.zz = F::zero();
    p.zzz = F::zero();
#pragma unroll
    for (int i = 0; i < F::N; ++i) p.x.v[i] = 0xffffffffu;
    p.y.v[0] = e;
  }
  store_xyzz(&out[k], p);
}

// sum of partial records: out[k] = sum_j parts[j * stride + k] for k < nout; a marked record
// raises its error code into *err (and is left out of the sum)
template <class Cv>
__global__ void k_sum_partials(const Xyzz<Cv>* __restrict__ parts, uint32_t nparts, uint32_t stride,
                               uint32_t nout, Xyzz<Cv>* __restrict__ out, uint32_t* __restrict__ err) {
  uint32_t k = threadIdx.x;
  if (k >= nout) return;
  Xyzz<Cv> acc = Xyzz<Cv>::inf();
  for (uint32_t j = 0; j < nparts; ++j) {
    const Xyzz<Cv> p = load_xyzz(&parts[j * stride + k]);
    if (const uint32_t m = partial_mark(p)) {
      raise_err(err, m);
      continue;
    }
    acc = xyzz_add_c(acc, p);
  }
  store_xyzz(&out[k], acc);
}

// ------------------------------------------------------------------------------ generators
// Fixed-base comb for G1: table[j*256 + d] = d * 2^(8j) * G1 (affine Montgomery), j < 32.
template <class Cv>
__global__ void k_gen_table_base(Xyzz<Cv>* __restrict__ base) {
  uint32_t j = threadIdx.x;
  if (j >= 32) return;
  using P = typename Cv::FpP;
  Affine<Cv> g = {Fp<P>::from_const(Cv::K::G1X_M), Fp<P>::from_const(Cv::K::G1Y_M)};
  Xyzz<Cv> b = xyzz_from_affine(g);
  for (uint32_t i = 0; i < 8 * j; ++i) b = xyzz_dbl_c(b);
  store_xyzz(&base[j], b);
}
template <class Cv>
__global__ void __launch_bounds__(256) k_gen_table(const Xyzz<Cv>* __restrict__ base, Affine<Cv>* __restrict__ table) {
  uint32_t j = blockIdx.x, d = threadIdx.x;
  if (d == 0) return;
  Xyzz<Cv> b = load_xyzz(&base[j]);
  Xyzz<Cv> acc = Xyzz<Cv>::inf();
  for (int bit = 7; bit >= 0; --bit) {
    acc = xyzz_dbl_c(acc);
    if ((d >> bit) & 1) acc = xyzz_add_c(acc, b);
  }
  Affine<Cv> a;
  xyzz_to_affine(acc, a);
  table[j * 256 + d] = a;
}

template <class Cv>
KZ_DEV Xyzz<Cv> comb_mul(const Affine<Cv>* __restrict__ table, const Fp<typename Cv::FrP>& k) {
  Xyzz<Cv> acc = Xyzz<Cv>::inf();
#pragma unroll 4
  for (int j = 0; j < 32; ++j) {
    uint32_t byte = (k.v[j >> 2] >> (8 * (j & 3))) & 0xffu;
    if (byte) acc = xyzz_add_affine_c(acc, load_affine(table, j * 256 + byte));
  }
  return acc;
}

template <class Cv>
KZ_DEV void encode_xyzz_to(const Xyzz<Cv>& p, uint8_t* dst) {
  using P = typename Cv::FpP;
  constexpr int NW = 2 * P::N;
  uint32_t w[NW];
  Affine<Cv> a;
  if (!xyzz_to_affine(p, a)) {
#pragma unroll
    for (int k = 0; k < NW; ++k) w[k] = 0;
    if constexpr (Cv::ID == 0) w[0] = 0x40u;
  } else {
    fp_to_be_words(fp_from_mont(a.x), w, 0);
    fp_to_be_words(fp_from_mont(a.y), w, P::N);
  }
  store_words(dst, w);
}

template <class Cv>
__global__ void __launch_bounds__(256) k_gen_g1(const uint8_t* __restrict__ scalars, uint32_t n,
                                                const Affine<Cv>* __restrict__ table, uint8_t* __restrict__ out,
                                                uint32_t* __restrict__ err) {
  using R = typename Cv::FrP;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t w[8];
  load_words(scalars + (size_t)i * 32, w);
  Fp<R> k = fp_from_be_words<R>(w, 0);
  if (!fp_raw_lt_mod(k)) { raise_err(err, DERR_SCALAR); k = Fp<R>::zero(); }
  encode_xyzz_to(comb_mul(table, k), out + (size_t)i * 8 * Cv::FpP::N);
}

// 253-bit value from SHA256(seed || le64(i) || tag), as Fr limbs
template <class Cv>
KZ_DEV Fp<typename Cv::FrP> hash_scalar(const Seed& seed, uint64_t i, int tag) {
  uint32_t h[8];
  sha256_seed_index(seed.w, i, tag, h);
  h[0] &= 0x1fffffffu;
  Fp<typename Cv::FrP> r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = h[7 - k];
  return r;
}

template <class Cv>
__global__ void __launch_bounds__(256) k_gen_tuples(Seed seed, Fp<typename Cv::FrP> tau, uint32_t n,
                                                    const Affine<Cv>* __restrict__ table,
                                                    uint8_t* __restrict__ cm, uint8_t* __restrict__ zs,
                                                    uint8_t* __restrict__ ys, uint8_t* __restrict__ pf) {
  using R = typename Cv::FrP;
  using F = Fp<R>;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  F c = hash_scalar<Cv>(seed, i, 'c');
  F z = hash_scalar<Cv>(seed, i, 'z');
  F y = hash_scalar<Cv>(seed, i, 'y');
  // q = (c - y) / (tau - z) mod r   (Montgomery domain for the product)
  F num = fp_sub(c, y);
  F den = fp_sub(tau, z);
  F q = fp_from_mont(fp_mul(fp_to_mont(num), fp_inv_c(fp_to_mont(den))));
  uint32_t wz[8], wy[8];
  fp_to_be_words(z, wz, 0);
  fp_to_be_words(y, wy, 0);
  store_words(zs + (size_t)i * 32, wz);
  store_words(ys + (size_t)i * 32, wy);
  encode_xyzz_to(comb_mul(table, c), cm + (size_t)i * 8 * Cv::FpP::N);
  encode_xyzz_to(comb_mul(table, q), pf + (size_t)i * 8 * Cv::FpP::N);
}

}  // namespace kzgmi

namespace kzgmi {

// [k]_2 = k * Q on the twist by affine double-and-add (toy-SRS generation: one thread).
template <class Cv>
__global__ void k_g2_mul(const G2Aff<Cv>* __restrict__ q_in, const uint8_t* __restrict__ q_inf,
                         Fp<typename Cv::FrP> k, uint8_t* __restrict__ out) {
  using P = typename Cv::FpP;
  if (threadIdx.x != 0) return;
  G2Aff<Cv> Q = q_in[0], T = Q;
  bool t_inf = true;
  Line<Cv> dummy;
  for (int i = 255; i >= 0; --i) {
    if (!t_inf) {
      if (T.y.is_zero()) t_inf = true;  // 2-torsion (not in the prime-order subgroup)
      else line_dbl(T, dummy);
    }
    if ((k.v[i >> 5] >> (i & 31)) & 1) {
      if (t_inf) { T = Q; t_inf = false; }
      else if (T.x == Q.x) {
        if (T.y == Q.y) line_dbl(T, dummy);
        else t_inf = true;
      } else line_add(T, Q, dummy);
    }
  }
  constexpr int NW = 4 * P::N;
  uint32_t w[NW];
  if (t_inf || q_inf[0]) {
    for (int j = 0; j < NW; ++j) w[j] = 0;
    if constexpr (Cv::ID == 0) w[0] = 0x40u;
  } else {
    fp_to_be_words(fp_from_mont(T.x.c1), w, 0);
    fp_to_be_words(fp_from_mont(T.x.c0), w, P::N);
    fp_to_be_words(fp_from_mont(T.y.c1), w, 2 * P::N);
    fp_to_be_words(fp_from_mont(T.y.c0), w, 3 * P::N);
  }
  store_words(out, w);
}

// Fp-multiplication throughput probe (compute roofline of the MSM): every thread runs
// `iters` rounds of 8 independent Montgomery products.  out[] keeps the results live.
template <class Cv>
__global__ void __launch_bounds__(256) k_fpmul_probe(uint32_t iters, uint32_t* __restrict__ out) {
  using P = typename Cv::FpP;
  using F = Fp<P>;
  F a[8];
  F b = F::one();
  b.v[0] ^= threadIdx.x;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = F::one();
    a[j].v[1] ^= (blockIdx.x * 8 + j);
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = fp_mul(a[j], b);
  }
  uint32_t x = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) x ^= a[j].v[0] ^ a[j].v[P::N - 1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

}  // namespace kzgmi
