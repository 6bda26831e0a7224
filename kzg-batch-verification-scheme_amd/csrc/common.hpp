// Shared device utilities: error words, SHA-256 (randomiser derivation), byte codecs.
// Reference: none (LICENSE only); randomiser rule fixed by oracle/pyspec/kzg.py and
// declared in include/kzgmi.h.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include "g1.hpp"

namespace kzgmi {

// device-side error codes (atomicMax into the context's error word; host maps to KZGMI_ERR_*)
// DERR_SHARD: a gathered partial record was marked failed without a code of its own (k_sum_partials)
enum : uint32_t { DERR_NONE = 0, DERR_ENCODING = 1, DERR_NOT_ON_CURVE = 2, DERR_SCALAR = 3, DERR_NOT_IN_SUBGROUP = 4,
                  DERR_SHARD = 5 };

KZ_DEV void raise_err(uint32_t* err, uint32_t code) { atomicMax(err, code); }

// Latency-critical tail kernels (bucket-sum reduction, window combination, pairing, fix-ups)
// run one to a few waves per CU beside the accumulation of other pipelined batches (4 waves
// per SIMD).  Raising their wave priority lets the SIMD's issue arbiter pick them first, so a
// batch's tail is not stretched ~4x while full-chip work shares its SIMDs.
#define KZ_TAIL_PRIO() __builtin_amdgcn_s_setprio(3)

// Fiat-Shamir transcript geometry (fs.hpp)
constexpr uint32_t FS_CHUNK = 4096;  // leaves per shard-alignment subtree
constexpr int FS_POW_BITS = 32;      // r^(2^k), k < 32: any global index < 2^32

// ---------------------------------------------------------------------------- SHA-256
__constant__ static const uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

KZ_DEV uint32_t ror32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); hipcc emits two v_xor_b32 for it
KZ_DEV uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }

KZ_DEV void sha256_init(uint32_t (&h)[8]) {
  h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
  h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
}

// One compression of a block given as 16 big-endian words into the chaining state h.
KZ_DEV void sha256_compress(const uint32_t (&blk)[16], uint32_t (&h)[8]) {
  uint32_t w[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) w[i] = blk[i];
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
  uint32_t e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i];
    } else {
      uint32_t w15 = w[(i - 15) & 15], w2 = w[(i - 2) & 15];
      uint32_t s0 = xor3(ror32(w15, 7), ror32(w15, 18), w15 >> 3);
      uint32_t s1 = xor3(ror32(w2, 17), ror32(w2, 19), w2 >> 10);
      wi = w[i & 15] + s0 + w[(i - 7) & 15] + s1;
      w[i & 15] = wi;
    }
    uint32_t S1 = xor3(ror32(e, 6), ror32(e, 11), ror32(e, 25));
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + kSha256K[i] + wi;
    uint32_t S0 = xor3(ror32(a, 2), ror32(a, 13), ror32(a, 22));
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d;
  h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// One compression of a single padded block (the whole message fits one block).
KZ_DEV void sha256_one_block(const uint32_t (&blk)[16], uint32_t (&h)[8]) {
  sha256_init(h);
  sha256_compress(blk, h);
}

// SHA-256 of a message given as NW big-endian words (4 NW bytes), padding included.
template <int NW>
KZ_DEV void sha256_words(const uint32_t (&m)[NW], uint32_t (&h)[8]) {
  constexpr int BYTES = 4 * NW;
  constexpr int NB = (BYTES + 9 + 63) / 64;  // padded blocks
  sha256_init(h);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    uint32_t blk[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int wi = 16 * b + k;
      blk[k] = wi < NW ? m[wi] : wi == NW ? 0x80000000u : 0u;
    }
    if (b == NB - 1) blk[15] = (uint32_t)(BYTES * 8);  // length < 2^32 bits
    sha256_compress(blk, h);
  }
}

// SHA256(seed[32] || le64(i) [|| tag]) for messages of 40 or 41 bytes (one block).
KZ_DEV void sha256_seed_index(const uint32_t (&seed_be)[8], uint64_t i, int tag, uint32_t (&h)[8]) {
  uint32_t blk[16];
#pragma unroll
  for (int k = 0; k < 8; ++k) blk[k] = seed_be[k];
  // bytes 32..39 = little-endian i, then optional tag byte, then 0x80 padding
  uint32_t lo = (uint32_t)i, hi = (uint32_t)(i >> 32);
  blk[8] = __builtin_bswap32(lo);
  blk[9] = __builtin_bswap32(hi);
  uint32_t len_bits;
  if (tag < 0) {
    blk[10] = 0x80000000u;
    len_bits = 40 * 8;
  } else {
    blk[10] = ((uint32_t)(tag & 0xff) << 24) | 0x00800000u;
    len_bits = 41 * 8;
  }
#pragma unroll
  for (int k = 11; k < 15; ++k) blk[k] = 0;
  blk[15] = len_bits;
  sha256_one_block(blk, h);
}

// r_i = int_be(SHA256(seed || le64(i))[0:16]) >> 1, 1 if zero.  Returned as 4 LE words.
KZ_DEV void randomizer127(const uint32_t (&seed_be)[8], uint64_t i, uint32_t (&r)[4]) {
  uint32_t h[8];
  sha256_seed_index(seed_be, i, -1, h);
  // 128-bit big-endian value h[0..3] (h[0] most significant) >> 1
  r[3] = h[0] >> 1;
  r[2] = (h[1] >> 1) | (h[0] << 31);
  r[1] = (h[2] >> 1) | (h[1] << 31);
  r[0] = (h[3] >> 1) | (h[2] << 31);
  if ((r[0] | r[1] | r[2] | r[3]) == 0) r[0] = 1;
}

// ---------------------------------------------------------------------------- byte codecs
// Big-endian byte string of N*4 bytes (given as aligned 32-bit words w[0..N)) -> LE limbs.
template <int N>
KZ_DEV void be_words_to_limbs(const uint32_t* w, uint32_t (&limb)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) limb[k] = __builtin_bswap32(w[N - 1 - k]);
}
template <int N>
KZ_DEV void limbs_to_be_words(const uint32_t (&limb)[N], uint32_t* w) {
#pragma unroll
  for (int k = 0; k < N; ++k) w[N - 1 - k] = __builtin_bswap32(limb[k]);
}

}  // namespace kzgmi
