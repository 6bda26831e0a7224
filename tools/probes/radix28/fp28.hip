// Probe: carry-free radix-2^28 Montgomery multiplication (14 x 28-bit limbs in 32-bit words,
// R = 2^392) vs the production 32-bit product-scanning multiply: equality and throughput.
// Column sums stay below 2^63 (28 products < 2^56 plus carry), so each limb product is one
// v_mad_u64_u32 with no carry-out handling.
#include "field.hpp"
#include "params_gen.hpp"
#include "fp28_consts.h"
#include <cstdio>
#include <cstdlib>
using namespace kzgmi;
using P32 = Bls12_381FpParams;

struct F28 { uint32_t v[14]; };
constexpr uint32_t MASK = (1u << 28) - 1;

__device__ __forceinline__ F28 mul28(const F28& a, const F28& b) {
  uint32_t m[14];
  F28 t;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 14; ++k) {
#pragma unroll
    for (int i = 0; i < k; ++i) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)m[i] * C28::P[k - i];
    }
    acc += (uint64_t)a.v[k] * b.v[0];
    m[k] = ((uint32_t)acc * C28::INV) & MASK;
    acc += (uint64_t)m[k] * C28::P[0];
    acc >>= 28;
  }
#pragma unroll
  for (int k = 14; k < 27; ++k) {
#pragma unroll
    for (int i = k - 13; i < 14; ++i) {
      acc += (uint64_t)a.v[i] * b.v[k - i];
      acc += (uint64_t)m[i] * C28::P[k - i];
    }
    t.v[k - 14] = (uint32_t)acc & MASK;
    acc >>= 28;
  }
  t.v[13] = (uint32_t)acc;
  return t;  // value < 2p (inputs < 4p, 16p < R): lazily reduced
}

__device__ F28 pack28(const uint32_t (&w)[12]) {  // raw 32-bit words -> 28-bit limbs
  F28 r;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    int bit = 28 * i, wi = bit >> 5, sh = bit & 31;
    uint64_t lo = w[wi] | ((wi + 1 < 12) ? (uint64_t)w[wi + 1] << 32 : 0);
    r.v[i] = (uint32_t)(lo >> sh) & MASK;
  }
  return r;
}
__device__ void unpack28(const F28& a, uint32_t (&w)[12]) {  // canonical (< p) raw words
  uint32_t x[13] = {0};
  uint64_t acc = 0;
  int filled = 0, o = 0;
#pragma unroll
  for (int i = 0; i < 14; ++i) {
    acc |= (uint64_t)a.v[i] << filled;
    filled += 28;
    while (filled >= 32) { x[o++] = (uint32_t)acc; acc >>= 32; filled -= 32; }
  }
  if (o < 13) x[o] = (uint32_t)acc;
  uint32_t d[12], bw = 0;
  for (int i = 0; i < 12; ++i) d[i] = __builtin_subc(x[i], P32::MOD[i], bw, &bw);
  for (int i = 0; i < 12; ++i) w[i] = bw ? x[i] : d[i];
}

__global__ void k_check(const uint32_t* in, uint32_t* out32, uint32_t* out28, uint32_t n) {
  uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  uint32_t x[12], y[12];
  for (int i = 0; i < 12; ++i) { x[i] = in[t * 24 + i]; y[i] = in[t * 24 + 12 + i]; }
  Fp<P32> a, b;
  for (int i = 0; i < 12; ++i) { a.v[i] = x[i]; b.v[i] = y[i]; }
  Fp<P32> am32 = fp_to_mont(a), bm32 = fp_to_mont(b);
  Fp<P32> zm32 = fp_mul(am32, bm32);
  for (int rep = 0; rep < 50; ++rep) zm32 = fp_mul(fp_mul(zm32, am32), bm32);
  Fp<P32> z = fp_from_mont(zm32);
  for (int i = 0; i < 12; ++i) out32[t * 12 + i] = z.v[i];
  F28 r2, one;
  for (int i = 0; i < 14; ++i) { r2.v[i] = C28::R2[i]; one.v[i] = i == 0; }
  F28 am = mul28(pack28(x), r2), bm = mul28(pack28(y), r2);
  F28 zm = mul28(am, bm);
  for (int rep = 0; rep < 50; ++rep) zm = mul28(mul28(zm, am), bm);  // longer lazy chains
  F28 zr = mul28(zm, one);
  uint32_t w[12];
  unpack28(zr, w);
  for (int i = 0; i < 12; ++i) out28[t * 12 + i] = w[i];
}

template <int CH, bool R28>
__global__ void __launch_bounds__(256) k_tp(uint32_t iters, uint32_t* out) {
  extern __shared__ uint32_t pad[];
  if (iters == 0xffffffffu) pad[threadIdx.x] = 0;
  if constexpr (R28) {
    F28 a[CH], b;
    for (int i = 0; i < 14; ++i) b.v[i] = (threadIdx.x * 2654435761u + i) & MASK;
    for (int j = 0; j < CH; ++j) for (int i = 0; i < 14; ++i) a[j].v[i] = (blockIdx.x * 40503u + i * 7 + j) & MASK;
    for (uint32_t it = 0; it < iters; ++it)
#pragma unroll
      for (int j = 0; j < CH; ++j) a[j] = mul28(a[j], b);
    uint32_t x = 0;
    for (int j = 0; j < CH; ++j) for (int k = 0; k < 14; ++k) x = x * 31 + a[j].v[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  } else {
    using F = Fp<P32>;
    F a[CH], b = F::one();
    b.v[0] ^= threadIdx.x * 2654435761u;
    for (int j = 0; j < CH; ++j) { a[j] = F::one(); a[j].v[1] ^= (blockIdx.x * 8 + j) * 40503u; }
    for (uint32_t it = 0; it < iters; ++it)
#pragma unroll
      for (int j = 0; j < CH; ++j) a[j] = fp_mul(a[j], b);
    uint32_t x = 0;
    for (int j = 0; j < CH; ++j) for (int k = 0; k < 12; ++k) x = x * 31 + a[j].v[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  }
}

template <int CH, bool R28>
void tp(uint32_t* o, int waves) {
  const uint32_t blocks = 256 * 16, iters = 2048 / CH;
  const size_t lds = waves >= 6 ? 26 * 1024 : waves == 4 ? 40 * 1024 : waves == 3 ? 48 * 1024 : 64 * 1024;
  hipFuncSetAttribute((const void*)k_tp<CH, R28>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k_tp<CH, R28><<<blocks, 256, lds>>>(4, o);
  hipEventRecord(e0);
  k_tp<CH, R28><<<blocks, 256, lds>>>(iters, o);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("%s chains=%d waves<=%d: %.2f G mul/s\n", R28 ? "radix-2^28" : "32-bit ps ", CH, waves,
         (double)blocks * 256 * iters * CH / ms / 1e6);
}

int main() {
  const uint32_t n = 1 << 16;
  uint32_t* h = (uint32_t*)malloc(n * 24 * 4);
  srand(7);
  for (uint32_t t = 0; t < n; ++t)
    for (int k = 0; k < 2; ++k) {
      for (int i = 0; i < 12; ++i) h[t * 24 + k * 12 + i] = ((uint32_t)rand() << 17) ^ (uint32_t)rand() ^ (t % 5 == 0 ? 0xffffffffu : 0);
      h[t * 24 + k * 12 + 11] &= 0x0fffffffu;  // < 2^380 < p
      if (t % 97 == 0) for (int i = 0; i < 12; ++i) h[t * 24 + k * 12 + i] = P32::MOD[i] - (i == 0 ? 1 : 0);  // p - 1
    }
  uint32_t *din, *o32, *o28;
  hipMalloc(&din, n * 24 * 4); hipMalloc(&o32, n * 12 * 4); hipMalloc(&o28, n * 12 * 4);
  hipMemcpy(din, h, n * 24 * 4, hipMemcpyHostToDevice);
  k_check<<<n / 256, 256>>>(din, o32, o28, n);
  uint32_t* a = (uint32_t*)malloc(n * 48); uint32_t* b = (uint32_t*)malloc(n * 48);
  hipMemcpy(a, o32, n * 48, hipMemcpyDeviceToHost);
  hipMemcpy(b, o28, n * 48, hipMemcpyDeviceToHost);
  size_t bad = 0;
  for (size_t i = 0; i < (size_t)n * 12; ++i) bad += a[i] != b[i];
  printf("check: %s, mismatching words %zu of %zu\n", hipGetErrorString(hipGetLastError()), bad, (size_t)n * 12);
  free(h);
  uint32_t* o; hipMalloc(&o, 256 * 16 * 256 * 4);
  tp<2, false>(o, 3);
  tp<2, true>(o, 3);
  tp<2, true>(o, 4);
  tp<1, true>(o, 6);
  return 0;
}
