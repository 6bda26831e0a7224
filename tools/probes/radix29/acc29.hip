// Probe: bucket-accumulation mixed addition in carry-free radix 2^29 (14 limbs, R29 = 2^406)
// vs the production 32-bit-limb lazy loop, same harness (4 waves/SIMD, ZZ/ZZZ in LDS, random
// gathers from a 2^20-point table).  In radix 2^29 every column of a Montgomery product fits
// a 64-bit accumulator (<= 42 products < 2^58), so a limb product is ONE v_mad_u64_u32 with no
// carry fold; additions/subtractions pay a carry-normalisation pass instead.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I kzg-batch-verification-scheme_amd/csrc \
//     -I include tools/probes/radix29/acc29.hip -o tools/probes/radix29/acc29
#include "field.hpp"
#include "params_gen.hpp"
#include "consts29.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace kzgmi;
using P32 = Bls12_381FpParams;
using F32 = Fp<P32>;

constexpr int L = 14;
constexpr uint32_t M29 = (1u << 29) - 1;
struct F29 { uint32_t v[L]; };

KZ_DEV void mad29(uint64_t& acc, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b));
}
KZ_DEV void mad29s(uint64_t& acc, uint32_t a, uint32_t b_uniform) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "s"(b_uniform));
}

// (a b [+ c d] + m p) / 2^406, inputs with normalised limbs (< 2^29), values < 2^12 p:
// result < 2p with normalised limbs
template <bool TWO>
KZ_DEV F29 mont29(const F29& a, const F29& b, const F29& c, const F29& d) {
  uint32_t m[L];
  F29 t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < L; ++k) {
#pragma unroll
    for (int i = 0; i < k; ++i) {
      mad29(acc, a.v[i], b.v[k - i]);
      if constexpr (TWO) mad29(acc, c.v[i], d.v[k - i]);
      mad29s(acc, m[i], C29::P[k - i]);
    }
    mad29(acc, a.v[k], b.v[0]);
    if constexpr (TWO) mad29(acc, c.v[k], d.v[0]);
    m[k] = ((uint32_t)acc * C29::INV) & M29;
    mad29s(acc, m[k], C29::P[0]);
    acc >>= 29;
  }
#pragma unroll
  for (int k = L; k < 2 * L - 1; ++k) {
#pragma unroll
    for (int i = k - L + 1; i < L; ++i) {
      mad29(acc, a.v[i], b.v[k - i]);
      if constexpr (TWO) mad29(acc, c.v[i], d.v[k - i]);
      mad29s(acc, m[i], C29::P[k - i]);
    }
    t.v[k - L] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  t.v[L - 1] = (uint32_t)acc;
  return t;
}
KZ_DEV F29 mul29(const F29& a, const F29& b) { return mont29<false>(a, b, a, b); }
KZ_DEV F29 mul2_29(const F29& a, const F29& b, const F29& c, const F29& d) { return mont29<true>(a, b, c, d); }

// a + B - b (B = k p with limbs biased into [2^29, 2^30) >= b's limbs), normalised
KZ_DEV F29 sub29(const F29& a, const F29& b, const uint32_t (&B)[L]) {
  F29 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t x = a.v[i] + B[i] + c - b.v[i];
    if (i < L - 1) { r.v[i] = x & M29; c = x >> 29; } else r.v[i] = x;
  }
  return r;
}
// a + b + e, normalised
KZ_DEV F29 add3_29(const F29& a, const F29& b, const F29& e) {
  F29 r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const uint32_t x = a.v[i] + b.v[i] + e.v[i] + c;
    if (i < L - 1) { r.v[i] = x & M29; c = x >> 29; } else r.v[i] = x;
  }
  return r;
}
// a == 0 mod p for a < 20 p (normalised): low-limb filter, then the full comparison
KZ_DEV bool is_zero29(const F29& a) {
  bool hit = false;
#pragma unroll
  for (int k = 0; k < 20; ++k) hit |= a.v[0] == C29::KP_LO[k];
  if (!hit) return false;
  for (int k = 0; k < 20; ++k) {
    uint32_t d = 0;
    for (int i = 0; i < L; ++i) d |= a.v[i] ^ C29::KP[k][i];
    if (d == 0) return true;
  }
  return false;
}

// ---- conversions (probe checks only)
KZ_DEV F29 from_plain32(const F32& w) {  // plain 32-bit words -> 29-bit limbs
  F29 r;
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    uint64_t lo = (wi < 12 ? (uint64_t)w.v[wi] : 0) | (wi + 1 < 12 ? (uint64_t)w.v[wi + 1] << 32 : 0);
    r.v[i] = (uint32_t)(lo >> sh) & (i < L - 1 ? M29 : 0xffffffffu);
  }
  return r;
}
KZ_DEV F32 to_plain32(const F29& a) {  // a normalised, < 2^384
  F32 w;
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    const int bit = 32 * j, li = bit / 29, sh = bit % 29;
    uint64_t x = (uint64_t)a.v[li] >> sh;
    if (li + 1 < L) x |= (uint64_t)a.v[li + 1] << (29 - sh);
    if (li + 2 < L && 29 * 2 - sh < 64) x |= (uint64_t)a.v[li + 2] << (58 - sh);
    w.v[j] = (uint32_t)x;
  }
  return w;
}
KZ_DEV F29 canon29(const F29& a) {  // a < 2p -> a mod p
  F29 d;
  int32_t c = 0;
  for (int i = 0; i < L; ++i) {
    int32_t x = (int32_t)a.v[i] - (int32_t)C29::P[i] + c;
    if (i < L - 1) { d.v[i] = (uint32_t)x & M29; c = x >> 29; } else d.v[i] = (uint32_t)x;
  }
  return ((int32_t)d.v[L - 1] < 0) ? a : d;
}
KZ_DEV F29 c29(const uint32_t (&k)[L]) { F29 r; for (int i = 0; i < L; ++i) r.v[i] = k[i]; return r; }

// check: random a,b,c,d < p: (a b + c d) and a - b and the mixed-add pieces vs the 32-bit field
__global__ void k_check(uint32_t seed, int* bad) {
  uint32_t s = seed ^ (threadIdx.x * 2654435761u + blockIdx.x * 40503u);
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return s; };
  F32 pa[4];
  for (int j = 0; j < 4; ++j) {
    for (int i = 0; i < 12; ++i) pa[j].v[i] = rnd();
    pa[j].v[11] &= 0x0fffffffu;  // < 2^380 < p
  }
  const F29 R2 = c29(C29::R2);
  F29 q[4];
  for (int j = 0; j < 4; ++j) q[j] = mul29(from_plain32(pa[j]), R2);  // Montgomery radix-29
  F32 m[4];
  for (int j = 0; j < 4; ++j) m[j] = fp_to_mont(pa[j]);
  // (a b + c d), via TWO; then - (a - b) * d ; result plain
  F29 t = mul2_29(q[0], q[1], q[2], q[3]);
  F29 u = sub29(t, sub29(q[0], q[1], C29::B2), C29::B4);  // t - (a - b), < 6p
  F29 v = mul29(u, q[3]);
  F29 one{};
  one.v[0] = 1;
  F29 vp = canon29(mul29(v, one));  // plain value
  F32 t32 = fp_add(fp_mul(m[0], m[1]), fp_mul(m[2], m[3]));
  F32 u32 = fp_sub(t32, fp_sub(m[0], m[1]));
  F32 v32 = fp_from_mont(fp_mul(u32, m[3]));
  F32 got = to_plain32(vp);
  if (!(got == v32)) atomicAdd(bad, 1);
}

// production 32-bit lazy loop body (msm.hpp k_accumulate), ZZ/ZZZ in LDS
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_loop32(const F32* __restrict__ pts, uint32_t npts, int iters, F32* out) {
  __shared__ uint32_t s_zz[12][256], s_zzz[12][256];
  const uint32_t tx = threadIdx.x;
  auto ld = [tx](uint32_t (&a)[12][256]) { asm volatile("" ::: "memory"); F32 r; for (int k = 0; k < 12; ++k) r.v[k] = a[k][tx]; return r; };
  auto st = [tx](uint32_t (&a)[12][256], const F32& v) { for (int k = 0; k < 12; ++k) a[k][tx] = v.v[k]; asm volatile("" ::: "memory"); };
  uint32_t s = blockIdx.x * 256 + tx;
  F32 x = pts[(s * 7) % npts], y = pts[(s * 13) % npts];
  st(s_zz, F32::one()); st(s_zzz, F32::one());
  for (int it = 0; it < iters; ++it) {
    s = s * 1664525u + 1013904223u;
    const uint32_t i = s % npts;
    F32 qx = pts[2 * (i / 2)], qy = pts[2 * (i / 2) + 1];
    qy = fp_select((s >> 31) != 0, fp_rsub_mod(qy), qy);
    const F32 U2 = fp_mul_lazy(qx, ld(s_zz));
    const F32 S2 = fp_mul_lazy(qy, ld(s_zzz));
    const F32 P = fp_sub_lazy(U2, x);
    const F32 R = fp_sub_lazy(S2, y);
    if (fp_is_zero_lazy(P)) continue;
    const F32 PP = fp_mul_lazy(P, P);
    const F32 PPP = fp_mul_lazy(P, PP);
    st(s_zz, fp_mul_lazy(ld(s_zz), PP));
    st(s_zzz, fp_mul_lazy(ld(s_zzz), PPP));
    const F32 Q = fp_mul_lazy(x, PP);
    const F32 X3 = fp_sub_lazy(fp_sub_lazy(fp_mul_lazy(R, R), PPP), fp_add_lazy(Q, Q));
    y = fp_mul2_lazy(R, fp_sub_lazy(Q, X3), y, fp_neg_lazy(PPP));
    x = X3;
  }
  out[blockIdx.x * 256 + tx] = fp_add(x, fp_add(y, fp_add(ld(s_zz), ld(s_zzz))));
}

// radix-29 loop body: bounds (values): x < 10p, y/zz/zzz < 2p, q < p
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4)))
k_loop29(const F29* __restrict__ pts, uint32_t npts, int iters, F29* out) {
  __shared__ uint32_t s_zz[L][256], s_zzz[L][256];
  const uint32_t tx = threadIdx.x;
  auto ld = [tx](uint32_t (&a)[L][256]) { asm volatile("" ::: "memory"); F29 r; for (int k = 0; k < L; ++k) r.v[k] = a[k][tx]; return r; };
  auto st = [tx](uint32_t (&a)[L][256], const F29& v) { for (int k = 0; k < L; ++k) a[k][tx] = v.v[k]; asm volatile("" ::: "memory"); };
  uint32_t s = blockIdx.x * 256 + tx;
  F29 x = pts[(s * 7) % npts], y = pts[(s * 13) % npts];
  st(s_zz, c29(C29::ONE)); st(s_zzz, c29(C29::ONE));
  for (int it = 0; it < iters; ++it) {
    s = s * 1664525u + 1013904223u;
    const uint32_t i = s % npts;
    F29 qx = pts[2 * (i / 2)], qy = pts[2 * (i / 2) + 1];
    {
      const F29 ny = sub29(F29{}, qy, C29::B1);  // p - y
      const bool neg = (s >> 31) != 0;
      for (int k = 0; k < L; ++k) qy.v[k] = neg ? ny.v[k] : qy.v[k];
    }
    const F29 U2 = mul29(qx, ld(s_zz));
    const F29 S2 = mul29(qy, ld(s_zzz));
    const F29 P = sub29(U2, x, C29::B16);  // < 18p
    const F29 R = sub29(S2, y, C29::B2);   // < 4p
    if (is_zero29(P)) continue;
    const F29 PP = mul29(P, P);
    const F29 PPP = mul29(P, PP);
    st(s_zz, mul29(ld(s_zz), PP));
    st(s_zzz, mul29(ld(s_zzz), PPP));
    const F29 Q = mul29(x, PP);
    const F29 X3 = sub29(mul29(R, R), add3_29(PPP, Q, Q), C29::B8);  // < 10p
    y = mul2_29(R, sub29(Q, X3, C29::B16), y, sub29(F29{}, PPP, C29::B2));
    x = X3;
  }
  F29 r = add3_29(x, y, add3_29(ld(s_zz), ld(s_zzz), F29{}));
  out[blockIdx.x * 256 + tx] = r;
}

int main() {
  int* bad;
  (void)hipMalloc(&bad, 4);
  (void)hipMemset(bad, 0, 4);
  k_check<<<64, 256>>>(12345u, bad);
  int hbad = -1;
  (void)hipMemcpy(&hbad, bad, 4, hipMemcpyDeviceToHost);
  printf("radix-29 vs 32-bit field: %d mismatches of %d\n", hbad, 64 * 256);

  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint32_t npts = 1u << 21;  // x and y words of 2^20 points
  std::vector<uint32_t> h(npts * 16);
  uint32_t s = 7;
  for (auto& w : h) { s = s * 1664525u + 1013904223u; w = s; }
  // 32-bit values < 2^380 (< p); radix-29: limbs < 2^29, top limb < 2^3
  for (uint32_t i = 0; i < npts; ++i) h[i * 12 + 11] &= 0x0fffffffu;
  F32* p32; F29* p29; F32* o32; F29* o29;
  (void)hipMalloc(&p32, npts * sizeof(F32));
  (void)hipMalloc(&p29, npts * sizeof(F29));
  (void)hipMemcpy(p32, h.data(), npts * sizeof(F32), hipMemcpyHostToDevice);
  for (uint32_t i = 0; i < npts; ++i)
    for (int k = 0; k < L; ++k) h[i * L + k] = (h[i * L + k] & M29) >> (k == L - 1 ? 26 : 0);
  (void)hipMemcpy(p29, h.data(), npts * sizeof(F29), hipMemcpyHostToDevice);
  const int blocks = cus * 4;  // 4 workgroups of 4 waves per CU: 4 waves per SIMD
  (void)hipMalloc(&o32, blocks * 256 * sizeof(F32));
  (void)hipMalloc(&o29, blocks * 256 * sizeof(F29));
  const int iters = 256;
  for (int rep = 0; rep < 2; ++rep) {
    float ms[2];
    for (int v = 0; v < 2; ++v) {
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0);
      (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      if (v == 0) k_loop32<<<blocks, 256>>>(p32, npts, iters, o32);
      else k_loop29<<<blocks, 256>>>(p29, npts, iters, o29);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      (void)hipEventElapsedTime(&ms[v], e0, e1);
    }
    const double adds = (double)blocks * 256 * iters;
    printf("mixed additions: 32-bit %.3f ms (%.2f G/s), radix-29 %.3f ms (%.2f G/s): %.3fx\n", ms[0],
           adds / ms[0] / 1e6, ms[1], adds / ms[1] / 1e6, ms[0] / ms[1]);
  }
  return 0;
}
