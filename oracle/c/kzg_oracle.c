/* C oracle for the MI355X KZG batch verifier -- TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library (liboracle.so).  It is the CPU restatement that the HIP product path is checked
 * against bit for bit, and it is the timed CPU baseline ("kind": "port").
 *
 * PARITY UNPINNED BY THE REFERENCE: /root/reference holds only LICENSE (LICENSE:1-201);
 * there is no reference algorithm, test or golden vector.  This
 * file restates the semantics fixed by BASELINE.json:5 (north_star: batch_verify with two G1
 * MSMs + a 2-pairing check) and oracle/pyspec/kzg.py, and is pinned against the golden
 * fixtures that the independent Python spec generates (tests/golden/).
 *
 * Instantiates BLS12-381 (6x64 limbs) and BN254 (4x64 limbs) from the include-templates.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "consts_gen.h"
#include "tmul_x86_gen.h"
#include "fexp_gen.h"

#define KZGO_OK 0
#define KZGO_ERR_ARG (-1)
#define KZGO_ERR_ENCODING (-2)
#define KZGO_ERR_NOT_ON_CURVE (-3)
#define KZGO_ERR_SCALAR (-4)

static int g_threads = 0;
static int kzgo_threads(void) {
#ifdef _OPENMP
  return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
  return 1;
#endif
}

/* ------------------------------------------------------------------ SHA-256 (FIPS 180-4) */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_block(uint32_t* h, const uint8_t* blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; ++i)
    w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 | (uint32_t)blk[4 * i + 2] << 8 | blk[4 * i + 3];
  for (int i = 16; i < 64; ++i) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; ++i) {
    uint32_t S1 = ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25);
    uint32_t ch = (e & f) ^ (~e & g);
    uint32_t t1 = hh + S1 + ch + K256[i] + w[i];
    uint32_t S0 = ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22);
    uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}
void kzgo_sha256(uint8_t out[32], const uint8_t* msg, size_t len) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  size_t i = 0;
  for (; i + 64 <= len; i += 64) sha256_block(h, msg + i);
  uint8_t blk[128]; memset(blk, 0, sizeof(blk));
  size_t rem = len - i; memcpy(blk, msg + i, rem); blk[rem] = 0x80;
  size_t tot = (rem + 9 <= 64) ? 64 : 128;
  uint64_t bits = (uint64_t)len * 8;
  for (int k = 0; k < 8; ++k) blk[tot - 1 - k] = (uint8_t)(bits >> (8 * k));
  sha256_block(h, blk);
  if (tot == 128) sha256_block(h, blk + 64);
  for (int k = 0; k < 8; ++k) { out[4*k] = h[k] >> 24; out[4*k+1] = h[k] >> 16; out[4*k+2] = h[k] >> 8; out[4*k+3] = h[k]; }
}

/* r_i = int_be(SHA256(seed || le64(i))[0:16]) >> 1, or 1 if zero (oracle/pyspec/kzg.py) */
static void kzgo_randomizer(const uint8_t* seed, uint64_t i, uint64_t out[4]) {
  uint8_t msg[40], h[32];
  memcpy(msg, seed, 32);
  for (int k = 0; k < 8; ++k) msg[32 + k] = (uint8_t)(i >> (8 * k));
  kzgo_sha256(h, msg, 40);
  uint64_t hi = 0, lo = 0;
  for (int k = 0; k < 8; ++k) { hi = hi << 8 | h[k]; lo = lo << 8 | h[8 + k]; }
  lo = (lo >> 1) | (hi << 63); hi >>= 1;
  if (!hi && !lo) lo = 1;
  out[0] = lo; out[1] = hi; out[2] = 0; out[3] = 0;
}

/* ================================================================== BLS12-381 */
#define F fp_bls
#define F_(x) fp_bls_##x
#define FN 6
#define FMOD BLS_P_MOD
#define FRR BLS_P_R
#define FR2 BLS_P_R2
#define FINV BLS_P_INV
#include "field_tmpl.h"
#undef F
#undef F_
#undef FN
#undef FMOD
#undef FRR
#undef FR2
#undef FINV

#define F fr_bls
#define F_(x) fr_bls_##x
#define FN 4
#define FMOD BLS_FR_MOD
#define FRR BLS_FR_R
#define FR2 BLS_FR_R2
#define FINV BLS_FR_INV
#include "field_tmpl.h"
#undef F
#undef F_
#undef FN
#undef FMOD
#undef FRR
#undef FR2
#undef FINV

#define FP fp_bls
#define FP_(x) fp_bls_##x
#define FR fr_bls
#define FR_(x) fr_bls_##x
#define T_(x) bls_##x
#define XI_A 1
#include "tower_tmpl.h"
static const uint64_t BLS_LOOPW[2] = {BLS_LOOP, 0};
#define C_(x) bls_##x
#define FPB 48
#define IS_BLS 1
#define B_SMALL 4
#define G1X BLS_G1X
#define G1Y BLS_G1Y
#define FEXP BLS_FEXP
#define FEXP_BITS BLS_FEXP_BITS
#define LOOP_WORDS BLS_LOOPW
#define LOOP_BITS 64
#define FROB_GX0 BLS_FROB_GX0
#define FROB_GX1 BLS_FROB_GX1
#define FROB_GY0 BLS_FROB_GY0
#define FROB_GY1 BLS_FROB_GY1
#define B2_0 BLS_B2_0
#define B2_1 BLS_B2_1
#define PRAW BLS_P_MOD
#define RRAW BLS_FR_MOD
#include "curve_tmpl.h"
#define PINV_T BLS_P_INV
#define HARD_L BLS_HARD_L
#define HARD_NEG BLS_HARD_NEG
#define HARD_BITS BLS_HARD_BITS
#include "pippenger_tuned_tmpl.h"
#undef PINV_T
#undef HARD_L
#undef HARD_NEG
#undef HARD_BITS
#undef PRAW
#undef RRAW
#undef FP
#undef FP_
#undef FR
#undef FR_
#undef T_
#undef XI_A
#undef C_
#undef FPB
#undef IS_BLS
#undef B_SMALL
#undef G1X
#undef G1Y
#undef FEXP
#undef FEXP_BITS
#undef LOOP_WORDS
#undef LOOP_BITS
#undef FROB_GX0
#undef FROB_GX1
#undef FROB_GY0
#undef FROB_GY1
#undef B2_0
#undef B2_1

/* ================================================================== BN254 */
#define F fp_bn
#define F_(x) fp_bn_##x
#define FN 4
#define FMOD BN_P_MOD
#define FRR BN_P_R
#define FR2 BN_P_R2
#define FINV BN_P_INV
#include "field_tmpl.h"
#undef F
#undef F_
#undef FN
#undef FMOD
#undef FRR
#undef FR2
#undef FINV

#define F fr_bn
#define F_(x) fr_bn_##x
#define FN 4
#define FMOD BN_FR_MOD
#define FRR BN_FR_R
#define FR2 BN_FR_R2
#define FINV BN_FR_INV
#include "field_tmpl.h"
#undef F
#undef F_
#undef FN
#undef FMOD
#undef FRR
#undef FR2
#undef FINV

#define FP fp_bn
#define FP_(x) fp_bn_##x
#define FR fr_bn
#define FR_(x) fr_bn_##x
#define T_(x) bn_##x
#define XI_A 9
#include "tower_tmpl.h"
#define C_(x) bn_##x
#define FPB 32
#define IS_BLS 0
#define B_SMALL 3
#define G1X BN_G1X
#define G1Y BN_G1Y
#define FEXP BN_FEXP
#define FEXP_BITS BN_FEXP_BITS
#define LOOP_WORDS BN_LOOP_BIG
#define LOOP_BITS BN_LOOP_BITS
#define FROB_GX0 BN_FROB_GX0
#define FROB_GX1 BN_FROB_GX1
#define FROB_GY0 BN_FROB_GY0
#define FROB_GY1 BN_FROB_GY1
#define B2_0 BN_B2_0
#define B2_1 BN_B2_1
#define PRAW BN_P_MOD
#define RRAW BN_FR_MOD
#include "curve_tmpl.h"
#define PINV_T BN_P_INV
#define HARD_L BN_HARD_L
#define HARD_NEG BN_HARD_NEG
#define HARD_BITS BN_HARD_BITS
#include "pippenger_tuned_tmpl.h"
#undef PINV_T
#undef HARD_L
#undef HARD_NEG
#undef HARD_BITS

/* ================================================================== C API (ctypes) */
#define CURVE_DISPATCH(curve, call_bls, call_bn) \
  ((curve) == 0 ? (call_bls) : (curve) == 1 ? (call_bn) : KZGO_ERR_ARG)

void kzgo_set_threads(int n) { g_threads = n; }
int kzgo_get_threads(void) { return kzgo_threads(); }

void kzgo_randomizer_bytes(const uint8_t* seed, uint64_t i, uint8_t out[32]) {
  uint64_t r[4];
  kzgo_randomizer(seed, i, r);
  for (int k = 0; k < 32; ++k) out[31 - k] = (uint8_t)(r[k / 8] >> (8 * (k % 8)));
}

int kzgo_batch_verify(int curve, const uint8_t* cm, const uint8_t* zs, const uint8_t* ys, const uint8_t* pf,
                      size_t n, const uint8_t* g2, const uint8_t* tau_g2, const uint8_t* seed, int* ok,
                      uint8_t* a_out, uint8_t* b_out) {
  if (!ok || !seed || !g2 || !tau_g2 || (n && (!cm || !zs || !ys || !pf))) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_batch_verify(cm, zs, ys, pf, n, g2, tau_g2, seed, ok, a_out, b_out, 0, 1, NULL, NULL),
                        bn_batch_verify(cm, zs, ys, pf, n, g2, tau_g2, seed, ok, a_out, b_out, 0, 1, NULL, NULL));
}

/* The tuned CPU verifier (pippenger_tuned_tmpl.h): same A, B and verdict as kzgo_batch_verify
 * (seeded randomisers), signed c-bit windows, XYZZ buckets, tasks of `chunk` points (0 = 2^19).
 * do_pairing = 0 computes A, B only (ok untouched). */
int kzgo_batch_verify_tuned(int curve, const uint8_t* cm, const uint8_t* zs, const uint8_t* ys, const uint8_t* pf,
                            size_t n, const uint8_t* g2, const uint8_t* tau_g2, const uint8_t* seed, int wbits,
                            size_t chunk, int do_pairing, int* ok, uint8_t* a_out, uint8_t* b_out) {
  if (!ok || !seed || !g2 || !tau_g2 || (n && (!cm || !zs || !ys || !pf))) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(
      curve, bls_batch_verify_tuned(cm, zs, ys, pf, n, g2, tau_g2, seed, ok, a_out, b_out, 0, do_pairing, wbits, chunk),
      bn_batch_verify_tuned(cm, zs, ys, pf, n, g2, tau_g2, seed, ok, a_out, b_out, 0, do_pairing, wbits, chunk));
}

/* e(P, Q) by the tuned verifier's pairing (precomputed Miller program, easy part + Frobenius
 * multi-exponent hard part): the same 12 Fp values as kzgo_pairing */
#define DEF_PFAST(C)                                                                           \
  static int C##_pairing_fast_api(const uint8_t* g1, const uint8_t* g2, uint8_t* out) {        \
    C##_aff P; C##_aff2 Q; int e;                                                              \
    if ((e = C##_g1_decode(&P, g1)) || (e = C##_g2_decode(&Q, g2))) return e;                  \
    C##_fp12 f; C##_pairing_fast(&f, &P, &Q); C##_fp12_encode(out, &f);                        \
    return 0;                                                                                  \
  }
DEF_PFAST(bls)
DEF_PFAST(bn)
int kzgo_pairing_fast(int curve, const uint8_t* g1, const uint8_t* g2, uint8_t* out) {
  if (!g1 || !g2 || !out) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_pairing_fast_api(g1, g2, out), bn_pairing_fast_api(g1, g2, out));
}

/* Powers mode (Fiat-Shamir / caller-supplied challenge): r_i = r^(offset + i), r = int_be(r32) < r.
 * do_pairing = 0 gives the shard partials (ok untouched). */
int kzgo_batch_verify_powers(int curve, const uint8_t* cm, const uint8_t* zs, const uint8_t* ys, const uint8_t* pf,
                             size_t n, uint64_t offset, const uint8_t* g2, const uint8_t* tau_g2, const uint8_t* r32,
                             int do_pairing, int* ok, uint8_t* a_out, uint8_t* b_out) {
  if (!ok || !r32 || !g2 || !tau_g2 || (n && (!cm || !zs || !ys || !pf))) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(
      curve, bls_batch_verify(cm, zs, ys, pf, n, g2, tau_g2, NULL, ok, a_out, b_out, offset, do_pairing, r32, NULL),
      bn_batch_verify(cm, zs, ys, pf, n, g2, tau_g2, NULL, ok, a_out, b_out, offset, do_pairing, r32, NULL));
}

/* A, B of tuples [offset, offset+n) of a global batch (no pairing): the shard partials */
int kzgo_batch_combination(int curve, const uint8_t* cm, const uint8_t* zs, const uint8_t* ys, const uint8_t* pf,
                           size_t n, uint64_t offset, const uint8_t* g2, const uint8_t* tau_g2, const uint8_t* seed,
                           uint8_t* a_out, uint8_t* b_out) {
  int ok = -1;
  if (!seed || !g2 || !tau_g2 || !a_out || !b_out || (n && (!cm || !zs || !ys || !pf))) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_batch_verify(cm, zs, ys, pf, n, g2, tau_g2, seed, &ok, a_out, b_out, offset, 0, NULL, NULL),
                        bn_batch_verify(cm, zs, ys, pf, n, g2, tau_g2, seed, &ok, a_out, b_out, offset, 0, NULL, NULL));
}

/* Batch verification / shard partials against an SRS whose G1 element is g1 (NULL = the
 * standard generator): the -t [1]_1 term uses it.  do_pairing = 0 gives A, B only. */
int kzgo_batch_verify_g1(int curve, const uint8_t* cm, const uint8_t* zs, const uint8_t* ys, const uint8_t* pf,
                         size_t n, uint64_t offset, const uint8_t* g1, const uint8_t* g2, const uint8_t* tau_g2,
                         const uint8_t* seed, int do_pairing, int* ok, uint8_t* a_out, uint8_t* b_out) {
  if (!ok || !seed || !g2 || !tau_g2 || (n && (!cm || !zs || !ys || !pf))) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(
      curve, bls_batch_verify(cm, zs, ys, pf, n, g2, tau_g2, seed, ok, a_out, b_out, offset, do_pairing, NULL, g1),
      bn_batch_verify(cm, zs, ys, pf, n, g2, tau_g2, seed, ok, a_out, b_out, offset, do_pairing, NULL, g1));
}

/* sum_i a_i b_i mod r for canonical big-endian Fr values (the discrete-log side of the MSM
 * identity sum_i b_i [a_i] G = [sum_i a_i b_i] G).  Non-canonical input -> error. */
#define DEF_FRDOT(C, FRT)                                                                      \
  static int C##_fr_dot_api(const uint8_t* a, const uint8_t* b, size_t n, uint8_t* out) {      \
    FRT acc; FRT##_zero(&acc);                                                                 \
    int err = 0;                                                                               \
    _Pragma("omp parallel num_threads(kzgo_threads())")                                        \
    {                                                                                          \
      FRT loc; FRT##_zero(&loc);                                                               \
      _Pragma("omp for schedule(static)")                                                      \
      for (size_t i = 0; i < n; ++i) {                                                         \
        uint64_t x[4], y[4];                                                                   \
        FRT##_raw_from_be(x, a + 32 * i, 32); FRT##_raw_from_be(y, b + 32 * i, 32);            \
        if (FRT##_geq_mod(x) || FRT##_geq_mod(y)) { err = KZGO_ERR_SCALAR; continue; }        \
        FRT xm, ym, p; FRT##_to_mont(&xm, x); FRT##_to_mont(&ym, y);                           \
        FRT##_mul(&p, &xm, &ym); FRT##_add(&loc, &loc, &p);                                    \
      }                                                                                        \
      _Pragma("omp critical")                                                                  \
      FRT##_add(&acc, &acc, &loc);                                                             \
    }                                                                                          \
    uint64_t raw[4]; FRT##_from_mont(raw, &acc); FRT##_raw_to_be(out, raw, 32);                \
    return err;                                                                                \
  }
DEF_FRDOT(bls, fr_bls)
DEF_FRDOT(bn, fr_bn)

int kzgo_fr_dot(int curve, const uint8_t* a, const uint8_t* b, size_t n, uint8_t* out) {
  if (!out || (n && (!a || !b))) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_fr_dot_api(a, b, n, out), bn_fr_dot_api(a, b, n, out));
}

int kzgo_pairing_check(int curve, const uint8_t* a, const uint8_t* b, const uint8_t* g2, const uint8_t* tau_g2, int* ok) {
  if (!a || !b || !g2 || !tau_g2 || !ok) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_pairing_check_api(a, b, g2, tau_g2, ok), bn_pairing_check_api(a, b, g2, tau_g2, ok));
}

#define DEF_MSM(C)                                                                         \
  static int C##_msm_api(const uint8_t* pts, const uint8_t* scs, size_t n, uint8_t* out) { \
    int pb = 2 * (C##_FPB_);                                                                \
    C##_aff* P = (C##_aff*)malloc((n ? n : 1) * sizeof(C##_aff));                          \
    uint64_t* S = (uint64_t*)malloc((n ? n : 1) * 32);                                     \
    int err = 0;                                                                           \
    for (size_t i = 0; i < n && !err; ++i) {                                               \
      err = C##_g1_decode(&P[i], pts + i * pb);                                            \
      if (!err) err = C##_fr_decode_raw(S + 4 * i, scs + 32 * i);                          \
    }                                                                                      \
    if (!err) {                                                                            \
      C##_jac r; C##_msm(&r, P, S, n);                                                     \
      C##_aff a; C##_jac_to_aff(&a, &r); C##_g1_encode(out, &a);                           \
    }                                                                                      \
    free(P); free(S);                                                                      \
    return err;                                                                            \
  }
#define bls_FPB_ 48
#define bn_FPB_ 32
DEF_MSM(bls)
DEF_MSM(bn)

int kzgo_msm_g1(int curve, const uint8_t* pts, const uint8_t* scalars, size_t n, uint8_t* out) {
  if (!out || (n && (!pts || !scalars))) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_msm_api(pts, scalars, n, out), bn_msm_api(pts, scalars, n, out));
}

/* k_i * G1 for each i (fixture / test-input generation).  Scalars are reduced mod r. */
#define DEF_MULGEN(C, FRT)                                                                  \
  static int C##_mul_gen_api(const uint8_t* scs, size_t n, uint8_t* out) {                  \
    C##_aff g; C##_generator(&g);                                                           \
    int err = 0;                                                                            \
    _Pragma("omp parallel for num_threads(kzgo_threads()) schedule(dynamic, 16)")          \
    for (size_t i = 0; i < n; ++i) {                                                        \
      uint64_t k[4]; FRT##_raw_from_be(k, scs + 32 * i, 32);                                \
      if (FRT##_geq_mod(k)) { err = KZGO_ERR_SCALAR; continue; }                           \
      C##_jac r; C##_mul_raw(&r, &g, k);                                                    \
      C##_aff a; C##_jac_to_aff(&a, &r); C##_g1_encode(out + i * 2 * (C##_FPB_), &a);       \
    }                                                                                       \
    return err;                                                                             \
  }
DEF_MULGEN(bls, fr_bls)
DEF_MULGEN(bn, fr_bn)

/* Compressed encodings and the subgroup definition (SURVEY.md 8f item 1 oracle). */
#define DEF_COMPRESSED(C)                                                                    \
  static int C##_decompress_api(const uint8_t* in, size_t n, uint8_t* out) {                \
    int err = 0;                                                                             \
    for (size_t i = 0; i < n; ++i) {                                                         \
      C##_aff a; int e = C##_g1_decode_compressed(&a, in + i * (C##_FPB_));                  \
      if (e) { if (!err) err = e; memset(&a, 0, sizeof(a)); a.inf = 1; }                     \
      C##_g1_encode(out + i * 2 * (C##_FPB_), &a);                                           \
    }                                                                                        \
    return err;                                                                              \
  }                                                                                          \
  static int C##_compress_api(const uint8_t* in, size_t n, uint8_t* out) {                  \
    for (size_t i = 0; i < n; ++i) {                                                         \
      C##_aff a; int e = C##_g1_decode(&a, in + i * 2 * (C##_FPB_));                         \
      if (e) return e;                                                                       \
      C##_g1_encode_compressed(out + i * (C##_FPB_), &a);                                    \
    }                                                                                        \
    return 0;                                                                                \
  }                                                                                          \
  static int C##_subgroup_api(const uint8_t* in, size_t n, int* ok) {                       \
    int err = 0, good = 1;                                                                   \
    _Pragma("omp parallel for num_threads(kzgo_threads()) schedule(dynamic, 4) reduction(&:good)") \
    for (size_t i = 0; i < n; ++i) {                                                         \
      C##_aff a; int e = C##_g1_decode(&a, in + i * 2 * (C##_FPB_));                         \
      if (e) { err = e; continue; }                                                          \
      good &= C##_in_subgroup(&a);                                                           \
    }                                                                                        \
    *ok = good;                                                                              \
    return err;                                                                              \
  }
DEF_COMPRESSED(bls)
DEF_COMPRESSED(bn)

int kzgo_g1_decompress(int curve, const uint8_t* in, size_t n, uint8_t* out) {
  if (n && (!in || !out)) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_decompress_api(in, n, out), bn_decompress_api(in, n, out));
}
int kzgo_g1_compress(int curve, const uint8_t* in, size_t n, uint8_t* out) {
  if (n && (!in || !out)) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_compress_api(in, n, out), bn_compress_api(in, n, out));
}
int kzgo_g1_subgroup_check(int curve, const uint8_t* in, size_t n, int* ok) {
  if (!ok || (n && !in)) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_subgroup_api(in, n, ok), bn_subgroup_api(in, n, ok));
}

int kzgo_g1_mul_gen(int curve, const uint8_t* scalars, size_t n, uint8_t* out) {
  if (n && (!scalars || !out)) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_mul_gen_api(scalars, n, out), bn_mul_gen_api(scalars, n, out));
}

#define DEF_PAIR(C)                                                                          \
  static int C##_pairing_api(const uint8_t* p, const uint8_t* q, uint8_t* out) {             \
    C##_aff P; C##_aff2 Q; int e;                                                            \
    if ((e = C##_g1_decode(&P, p))) return e;                                                \
    if ((e = C##_g2_decode(&Q, q))) return e;                                                \
    C##_fp12 f; C##_miller(&f, &P, &Q); C##_final_exp(&f, &f); C##_fp12_encode(out, &f);    \
    return 0;                                                                                \
  }
DEF_PAIR(bls)
DEF_PAIR(bn)

int kzgo_pairing(int curve, const uint8_t* g1, const uint8_t* g2, uint8_t* out) {
  if (!g1 || !g2 || !out) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_pairing_api(g1, g2, out), bn_pairing_api(g1, g2, out));
}

/* tau * G2 (toy SRS for tests) */
#define DEF_G2MUL(C, FRT)                                                                    \
  static int C##_g2_mul_api(const uint8_t* q, const uint8_t* k, uint8_t* out) {              \
    C##_aff2 Q; int e; if ((e = C##_g2_decode(&Q, q))) return e;                             \
    uint64_t s[4]; FRT##_raw_from_be(s, k, 32);                                              \
    C##_aff2 R; memset(&R, 0, sizeof(R)); R.inf = 1;                                         \
    for (int i = 255; i >= 0; --i) {                                                         \
      if (!R.inf) { C##_fp12 dummy; C##_aff P; C##_generator(&P); C##_fp12_one(&dummy);      \
        C##_aff2 Rc = R; C##_step(&dummy, &R, &Rc, &P); }                                    \
      if ((s[i / 64] >> (i % 64)) & 1) {                                                     \
        if (R.inf) R = Q; else { C##_fp12 dummy; C##_aff P; C##_generator(&P);               \
          C##_fp12_one(&dummy); C##_step(&dummy, &R, &Q, &P); }                              \
      }                                                                                      \
    }                                                                                        \
    C##_g2_encode(out, &R);                                                                  \
    return 0;                                                                                \
  }
DEF_G2MUL(bls, fr_bls)
DEF_G2MUL(bn, fr_bn)

int kzgo_g2_mul(int curve, const uint8_t* q, const uint8_t* k, uint8_t* out) {
  if (!q || !k || !out) return KZGO_ERR_ARG;
  return CURVE_DISPATCH(curve, bls_g2_mul_api(q, k, out), bn_g2_mul_api(q, k, out));
}
