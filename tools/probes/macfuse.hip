// Which fused v_mad_u64_u32/v_addc carry pattern is hazard-free on gfx950, and how fast?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#define MAD_A(A, B) "v_mad_u64_u32 %0, %1, " A ", " B ", %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1\n\t"
#define MAD_B(A, B) "v_mad_u64_u32 %0, %1, " A ", " B ", %0\n\tv_addc_co_u32_e64 %2, %3, %2, 0, %1\n\t"
#define MAD_D(A, B) "v_mad_u64_u32 %0, %1, " A ", " B ", %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1\n\ts_nop 0\n\t"
#define MAD_E(A, B) "v_mad_u64_u32 %0, %1, " A ", " B ", %0\n\ts_nop 0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1\n\t"
#define MAD_F(A, B) "v_mad_u64_u32 %0, %1, " A ", " B ", %0\n\ts_nop 1\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1\n\t"

template <int V>
__device__ void mac4(uint64_t& acc, uint32_t& top, uint32_t a0, uint32_t b0, uint32_t a1, uint32_t b1, uint32_t a2,
                     uint32_t b2, uint32_t a3, uint32_t b3) {
  uint64_t cc, dd;
  if constexpr (V == 0) {  // one pair per asm (current production form)
    asm(MAD_A("%3", "%4") : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a0), "v"(b0));
    asm(MAD_A("%3", "%4") : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a1), "v"(b1));
    asm(MAD_A("%3", "%4") : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a2), "v"(b2));
    asm(MAD_A("%3", "%4") : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a3), "v"(b3));
  } else if constexpr (V == 1) {
    asm(MAD_A("%3", "%4") MAD_A("%5", "%6") MAD_A("%7", "%8") MAD_A("%9", "%10")
        : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3));
  } else if constexpr (V == 2) {
    asm(MAD_B("%4", "%5") MAD_B("%6", "%7") MAD_B("%8", "%9") MAD_B("%10", "%11")
        : "+v"(acc), "=&s"(cc), "+v"(top), "=&s"(dd)
        : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3));
  } else if constexpr (V == 3) {
    asm(MAD_D("%3", "%4") MAD_D("%5", "%6") MAD_D("%7", "%8") MAD_D("%9", "%10")
        : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3));
  } else if constexpr (V == 4) {
    asm(MAD_E("%3", "%4") MAD_E("%5", "%6") MAD_E("%7", "%8") MAD_E("%9", "%10")
        : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3));
  } else if constexpr (V == 5) {
    asm(MAD_F("%3", "%4") MAD_F("%5", "%6") MAD_F("%7", "%8") MAD_F("%9", "%10")
        : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a0), "v"(b0), "v"(a1), "v"(b1), "v"(a2), "v"(b2), "v"(a3), "v"(b3));
  } else if constexpr (V == 7) {  // odd products read an SGPR (uniform) operand, fused
    uint32_t s1 = __builtin_amdgcn_readfirstlane(b1), s3 = __builtin_amdgcn_readfirstlane(b3);
    asm(MAD_A("%3", "%4") MAD_A("%5", "%6") MAD_A("%7", "%8") MAD_A("%9", "%10")
        : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a0), "v"(b0), "v"(a1), "s"(s1), "v"(a2), "v"(b2), "v"(a3), "s"(s3));
  } else if constexpr (V == 8) {  // same with a nop after each addc
    uint32_t s1 = __builtin_amdgcn_readfirstlane(b1), s3 = __builtin_amdgcn_readfirstlane(b3);
    asm(MAD_D("%3", "%4") MAD_D("%5", "%6") MAD_D("%7", "%8") MAD_D("%9", "%10")
        : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a0), "v"(b0), "v"(a1), "s"(s1), "v"(a2), "v"(b2), "v"(a3), "s"(s3));
  } else if constexpr (V == 9) {  // same, separate carry-out SGPR for the addc
    uint32_t s1 = __builtin_amdgcn_readfirstlane(b1), s3 = __builtin_amdgcn_readfirstlane(b3);
    asm(MAD_B("%4", "%5") MAD_B("%6", "%7") MAD_B("%8", "%9") MAD_B("%10", "%11")
        : "+v"(acc), "=&s"(cc), "+v"(top), "=&s"(dd) : "v"(a0), "v"(b0), "v"(a1), "s"(s1), "v"(a2), "v"(b2), "v"(a3), "s"(s3));
  } else if constexpr (V == 10) {  // one pair per asm with SGPR operand (production form)
    uint32_t s1 = __builtin_amdgcn_readfirstlane(b1), s3 = __builtin_amdgcn_readfirstlane(b3);
    asm(MAD_A("%3", "%4") : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a0), "v"(b0));
    asm(MAD_A("%3", "%4") : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a1), "s"(s1));
    asm(MAD_A("%3", "%4") : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a2), "v"(b2));
    asm(MAD_A("%3", "%4") : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a3), "s"(s3));
  } else {  // plain C: compiler's own carry handling
    uint64_t p[4] = {(uint64_t)a0 * b0, (uint64_t)a1 * b1, (uint64_t)a2 * b2, (uint64_t)a3 * b3};
    for (int i = 0; i < 4; ++i) { uint64_t s = acc + p[i]; top += s < acc; acc = s; }
  }
}

// 12x12 schoolbook product scanning of x*y, 24 output words
template <int V>
__global__ void k(const uint32_t* in, uint32_t* out, int iters) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[12], y[12];
  for (int i = 0; i < 12; ++i) { x[i] = in[t * 24 + i]; y[i] = in[t * 24 + 12 + i]; }
  uint32_t r[24];
  for (int it = 0; it < iters; ++it) {
    uint64_t acc = 0;
    uint32_t top = 0;
#pragma unroll
    for (int k = 0; k < 23; ++k) {
      int lo = k < 12 ? 0 : k - 11, hi = k < 12 ? k : 11;  // inclusive
      int i = lo;
#pragma unroll
      for (; i + 3 <= hi; i += 4) mac4<V>(acc, top, x[i], y[k - i], x[i + 1], y[k - i - 1], x[i + 2], y[k - i - 2], x[i + 3], y[k - i - 3]);
#pragma unroll
      for (; i <= hi; ++i) mac4<V>(acc, top, x[i], y[k - i], 0, 0, 0, 0, 0, 0);
      r[k] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)top << 32);
      top = 0;
    }
    r[23] = (uint32_t)acc;
    // feed back to keep it live
    for (int i = 0; i < 12; ++i) { x[i] ^= r[i] & 0; }
  }
  for (int i = 0; i < 24; ++i) out[t * 24 + i] = r[i];
}

static void host_ref(const uint32_t* x, const uint32_t* y, uint32_t* r) {
  unsigned __int128 acc = 0;
  for (int k = 0; k < 23; ++k) {
    for (int i = 0; i < 12; ++i) { int j = k - i; if (j < 0 || j > 11) continue; acc += (unsigned __int128)x[i] * y[j]; }
    r[k] = (uint32_t)acc;
    acc >>= 32;
  }
  r[23] = (uint32_t)acc;
}

int main() {
  const int T = 256 * 2048;
  size_t nin = (size_t)T * 24;
  uint32_t* h = (uint32_t*)malloc(nin * 4);
  uint32_t* o = (uint32_t*)malloc(nin * 4);
  srand(1);
  for (size_t i = 0; i < nin; ++i) h[i] = ((uint32_t)rand() << 16) ^ (uint32_t)rand() ^ ((i % 7 == 0) ? 0xffff0000u : 0);
  // y words identical across each wavefront (so readfirstlane of y is exact)
  for (int t = 0; t < T; ++t) for (int i = 12; i < 24; ++i) h[(size_t)t * 24 + i] = h[(size_t)(t & ~63) * 24 + i];
  uint32_t *din, *dout;
  hipMalloc(&din, nin * 4); hipMalloc(&dout, nin * 4);
  hipMemcpy(din, h, nin * 4, hipMemcpyHostToDevice);
  void (*ks[11])(const uint32_t*, uint32_t*, int) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>, k<9>, k<10>};
  const char* names[11] = {"pair-per-asm", "fused", "fused-sep-carryout", "fused-nop-after", "fused-nop-mid", "fused-nop1-mid", "plainC", "fused-sgpr", "fused-sgpr-nop", "fused-sgpr-sepco", "pair-per-asm-sgpr"};
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int v = 0; v < 11; ++v) {
    hipLaunchKernelGGL(ks[v], dim3(T / 256), dim3(256), 0, 0, din, dout, 1);
    hipMemcpy(o, dout, nin * 4, hipMemcpyDeviceToHost);
    long bad = 0;
    for (int t = 0; t < T; ++t) {
      uint32_t r[24];
      host_ref(h + t * 24, h + t * 24 + 12, r);
      for (int i = 0; i < 24; ++i) bad += r[i] != o[t * 24 + i];
    }
    int iters = 200;
    hipEventRecord(e0);
    hipLaunchKernelGGL(ks[v], dim3(T / 256), dim3(256), 0, 0, din, dout, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-20s bad=%ld  %.3f ms  %.1f G 12x12-products/s\n", names[v], bad, ms, (double)T * iters / ms / 1e6);
  }
  return 0;
}
