// Fiat-Shamir randomisers ("deterministic r from a hash of all inputs,
// c-kzg-style powers of r ... a GPU-friendly hash or tree-hash").  Reference: none (LICENSE
// only); the transcript is defined here and restated in oracle/pyspec/kzg.py (fs_challenge).
//
//   leaf_i = SHA256("KZGMI_FS_LEAF_V1" || be64(i) || C_i || pi_i || z_i || y_i)
//            (C_i, pi_i in COMPRESSED form whatever the input format; i the global index)
//   root   = binary Merkle root over L = max(4096, next_pow2(n)) leaf slots, slot i >= n
//            holding 32 zero bytes, node = SHA256(left || right)
//   r      = int_be(SHA256("KZGMI_FS_ROOT_V1" || be64(n) || root)) mod r  (1 if 0)
//   r_i    = r^i
// Every leaf and every tree level is hashed in parallel (a single sequential SHA-256 over
// the 160-256 MiB transcript would run on one lane for seconds).  Shards whose offsets are
// multiples of 4096 own whole 4096-leaf subtrees, so ranks exchange only subtree roots.
// KZGMI_FLAG_POWERS takes r from the caller instead (e.g. the EIP-4844 transcript).
#pragma once
#include "points.hpp"

namespace kzgmi {


// "KZGMI_FS_LEAF_V1" / "KZGMI_FS_ROOT_V1" as big-endian words
__constant__ static const uint32_t kFsLeafTag[4] = {0x4b5a474du, 0x495f4653u, 0x5f4c4541u, 0x465f5631u};
__constant__ static const uint32_t kFsRootTag[4] = {0x4b5a474du, 0x495f4653u, 0x5f524f4fu, 0x545f5631u};
// root of an all-zero-slot 4096-leaf subtree (12 levels of SHA256(z || z) from z = 0^32):
// pads the chunk-digest level up to a power of two
__constant__ static const uint32_t kFsZeroChunk[8] = {0xb7d05f87u, 0x5f140027u, 0xef5118a2u, 0x247bbb84u, 0xce8f2f0fu, 0x11236230u, 0x85daf796u, 0x0c329f5fu};

template <class Cv>
__global__ void __launch_bounds__(256) k_fs_leaves(const uint8_t* __restrict__ dC, const uint8_t* __restrict__ dpi,
                                                   const uint8_t* __restrict__ dz, const uint8_t* __restrict__ dy,
                                                   uint32_t n, uint64_t offset, int compressed,
                                                   uint32_t* __restrict__ leaves) {
  constexpr int N = Cv::FpP::N;
  constexpr int NW = 4 + 2 + 2 * N + 16;  // tag, index, C, pi, z, y
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t m[NW];
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = kFsLeafTag[k];
  const uint64_t gi = offset + i;
  m[4] = (uint32_t)(gi >> 32);
  m[5] = (uint32_t)gi;
  uint32_t c[N], p[N];
  if (compressed) {
    load_words(dC + (size_t)i * 4 * N, c);
    load_words(dpi + (size_t)i * 4 * N, p);
  } else {
    uint32_t w[2 * N];
    load_words(dC + (size_t)i * 8 * N, w);
    compress_encoding<Cv>(w, c);
    load_words(dpi + (size_t)i * 8 * N, w);
    compress_encoding<Cv>(w, p);
  }
  uint32_t z[8], y[8];
  load_words(dz + (size_t)i * 32, z);
  load_words(dy + (size_t)i * 32, y);
#pragma unroll
  for (int k = 0; k < N; ++k) { m[6 + k] = __builtin_bswap32(c[k]); m[6 + N + k] = __builtin_bswap32(p[k]); }
#pragma unroll
  for (int k = 0; k < 8; ++k) { m[6 + 2 * N + k] = __builtin_bswap32(z[k]); m[14 + 2 * N + k] = __builtin_bswap32(y[k]); }
  uint32_t h[8];
  sha256_words(m, h);
  uint4* d = reinterpret_cast<uint4*>(leaves + 8 * (size_t)i);
  d[0] = make_uint4(h[0], h[1], h[2], h[3]);
  d[1] = make_uint4(h[4], h[5], h[6], h[7]);
}

KZ_DEV void fs_node(const uint32_t* l, const uint32_t* r, uint32_t (&h)[8]) {
  uint32_t m[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) { m[k] = l[k]; m[8 + k] = r[k]; }
  sha256_words(m, h);
}

// Each workgroup reduces `group` (a power of two <= 512) consecutive nodes to one.
static __global__ void __launch_bounds__(256) k_fs_merkle(const uint32_t* __restrict__ in, uint32_t group,
                                                          uint32_t* __restrict__ out) {
  __shared__ uint32_t lds[256 * 8];
  const uint32_t* base = in + (size_t)blockIdx.x * group * 8;
  uint32_t h[8];
  const uint32_t half = group / 2;
  if (threadIdx.x < half) {
    fs_node(base + 16 * threadIdx.x, base + 16 * threadIdx.x + 8, h);
#pragma unroll
    for (int k = 0; k < 8; ++k) lds[8 * threadIdx.x + k] = h[k];
  }
  __syncthreads();
  for (uint32_t width = half / 2; width >= 1; width >>= 1) {
    if (threadIdx.x < width) fs_node(&lds[16 * threadIdx.x], &lds[16 * threadIdx.x + 8], h);
    __syncthreads();
    if (threadIdx.x < width) {
#pragma unroll
      for (int k = 0; k < 8; ++k) lds[8 * threadIdx.x + k] = h[k];
    }
    __syncthreads();
  }
  if (threadIdx.x < 8) out[8 * blockIdx.x + threadIdx.x] = lds[threadIdx.x];
}

// digests[nchunks .. p2) = kFsZeroChunk
static __global__ void k_fs_pad(uint32_t* __restrict__ digests, uint32_t nchunks, uint32_t p2) {
  const uint32_t i = nchunks + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p2) return;
#pragma unroll
  for (int k = 0; k < 8; ++k) digests[8 * (size_t)i + k] = kFsZeroChunk[k];
}

// r = H(root tag || be64(n) || root) mod r; pow[k] = r^(2^k) (Montgomery) for k < FS_POW_BITS;
// chal_out = r as 32 big-endian bytes (8 words, for the caller / tests)
template <class Cv>
__global__ void k_fs_challenge(const uint32_t* __restrict__ root, uint64_t n, Fp<typename Cv::FrP>* __restrict__ pow,
                               uint32_t* __restrict__ chal_out) {
  using R = typename Cv::FrP;
  using F = Fp<R>;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint32_t m[14];
#pragma unroll
  for (int k = 0; k < 4; ++k) m[k] = kFsRootTag[k];
  m[4] = (uint32_t)(n >> 32);
  m[5] = (uint32_t)n;
#pragma unroll
  for (int k = 0; k < 8; ++k) m[6 + k] = root[k];
  uint32_t h[8];
  sha256_words(m, h);
  F r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = h[7 - k];
  for (int t = 0; t < 8 && !fp_raw_lt_mod(r); ++t) {  // h < 2^256 < 8r for both curves
    uint32_t bw = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) r.v[k] = __builtin_subc(r.v[k], R::MOD[k], bw, &bw);
  }
  if (r.is_zero()) r.v[0] = 1;
#pragma unroll
  for (int k = 0; k < 8; ++k) chal_out[k] = r.v[7 - k];
  F x = fp_to_mont(r);
  for (int k = 0; k < FS_POW_BITS; ++k) {
    pow[k] = x;
    x = fp_sqr(x);
  }
}

// caller-supplied challenge (KZGMI_FLAG_POWERS): r = int_be(r32) mod r -> pow table
template <class Cv>
__global__ void k_pow_table(Seed r_be, Fp<typename Cv::FrP>* __restrict__ pow, uint32_t* __restrict__ err) {
  using R = typename Cv::FrP;
  using F = Fp<R>;
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  F r;
#pragma unroll
  for (int k = 0; k < 8; ++k) r.v[k] = r_be.w[7 - k];
  if (!fp_raw_lt_mod(r)) { raise_err(err, DERR_SCALAR); r = F::zero(); }
  F x = fp_to_mont(r);
  for (int k = 0; k < FS_POW_BITS; ++k) {
    pow[k] = x;
    x = fp_sqr(x);
  }
}

// r_i = r^(offset + i) from the pow table; s_i = r_i z_i; block partials of sum r_i y_i.
// r_out / s_out: 8 LE words per tuple (standard form), as the MSM digit extraction wants.
template <class Cv, int BLOCK>
__global__ void __launch_bounds__(BLOCK) k_scalar_prep_pow(const Fp<typename Cv::FrP>* __restrict__ pow,
                                                           uint64_t index_offset, const uint8_t* __restrict__ zs,
                                                           const uint8_t* __restrict__ ys, uint32_t n,
                                                           uint32_t* __restrict__ r_out, uint32_t* __restrict__ s_out,
                                                           Fp<typename Cv::FrP>* __restrict__ tpart,
                                                           uint32_t* __restrict__ err) {
  using R = typename Cv::FrP;
  using F = Fp<R>;
  __shared__ F lds[BLOCK];
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  F acc = F::zero();
  if (i < n) {
    uint32_t wz[8], wy[8];
    load_words(zs + (size_t)i * 32, wz);
    load_words(ys + (size_t)i * 32, wy);
    F z = fp_from_be_words<R>(wz, 0), y = fp_from_be_words<R>(wy, 0);
    if (!fp_raw_lt_mod(z) || !fp_raw_lt_mod(y)) { raise_err(err, DERR_SCALAR); z = F::zero(); y = F::zero(); }
    const uint64_t gi = index_offset + i;
    F rm = F::one();
    for (int k = 0; k < FS_POW_BITS; ++k)
      if ((gi >> k) & 1) rm = fp_mul(rm, pow[k]);
    const F r = fp_from_mont(rm);
    const F s = fp_mul(rm, z);  // r z (standard form)
    acc = fp_mul(rm, y);
    store_words(reinterpret_cast<uint8_t*>(r_out + 8 * (size_t)i), r.v);
    store_words(reinterpret_cast<uint8_t*>(s_out + 8 * (size_t)i), s.v);
  }
  lds[threadIdx.x] = acc;
  __syncthreads();
  for (int st = BLOCK / 2; st >= 1; st >>= 1) {
    if ((int)threadIdx.x < st) lds[threadIdx.x] = fp_add(lds[threadIdx.x], lds[threadIdx.x + st]);
    __syncthreads();
  }
  if (threadIdx.x == 0) tpart[blockIdx.x] = lds[0];
}

}  // namespace kzgmi
