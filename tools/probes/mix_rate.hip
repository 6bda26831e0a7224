// Marginal issue cost of the accumulation loop's non-mad instructions when they are interleaved
// with v_mad_u64_u32 (the mix of k_accumulate: ~3544 mads + ~995 other VALU + ~1078 s_nop per
// addition, tools/asm_census.py).  Each iteration issues 8 independent mads (4 per statement,
// as field29.hpp does) plus K instructions of one kind on independent registers; the time per
// iteration minus the mads-only time, divided by K, is what one instruction of that kind costs
// beside mads at the kernel's 4 waves per SIMD.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/mix_rate.hip -o tools/probes/mix_rate
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define MAD4(c0, c1, c2, c3, a, b)                                                                        \
  asm volatile("v_mad_u64_u32 %0, %4, %5, %6, %0\n\tv_mad_u64_u32 %1, %4, %5, %6, %1\n\t"                 \
               "v_mad_u64_u32 %2, %4, %5, %6, %2\n\tv_mad_u64_u32 %3, %4, %5, %6, %3"                     \
               : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "=&s"(cc)                                          \
               : "v"(a), "v"(b))

template <int MODE>
__device__ __forceinline__ void filler(uint32_t (&t)[8], uint64_t (&q)[4], uint32_t a) {
  // 8 instructions of one kind per call, on independent registers
  if constexpr (MODE == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_and_b32 %0, 0x1fffffff, %0" : "+v"(t[i]));
  } else if constexpr (MODE == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("v_lshrrev_b64 %0, 29, %0\n\tv_lshrrev_b64 %0, 3, %0" : "+v"(q[i]));
  } else if constexpr (MODE == 3) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(t[i]) : "v"(a));
  } else if constexpr (MODE == 4) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(t[i]) : "v"(a));
  } else if constexpr (MODE == 5) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(t[i]) : "v"(a));
  } else if constexpr (MODE == 6) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("s_nop 0" ::: "memory");
  } else if constexpr (MODE == 7) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshrrev_b32 %0, 29, %0" : "+v"(t[i]));
  } else if constexpr (MODE == 8) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_alignbit_b32 %0, %0, %1, 29" : "+v"(t[i]) : "v"(a));
  } else if constexpr (MODE == 9) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_mov_b32 %0, %1" : "=v"(t[i]) : "v"(a));
  } else if constexpr (MODE == 10) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(t[i]) : "v"(a));
  } else if constexpr (MODE == 11) {
#pragma unroll
    for (int i = 0; i < 8; ++i) asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(t[i]) : "v"(a));
  } else if constexpr (MODE == 12) {  // mad_u64_u32 as a filler (reference: a 9th..16th mad)
    uint64_t cc;
    asm volatile("v_mad_u64_u32 %0, %2, %3, %3, %0\n\tv_mad_u64_u32 %1, %2, %3, %3, %1" : "+v"(q[0]), "+v"(q[1]), "=&s"(cc) : "v"(a));
    asm volatile("v_mad_u64_u32 %0, %2, %3, %3, %0\n\tv_mad_u64_u32 %1, %2, %3, %3, %1" : "+v"(q[2]), "+v"(q[3]), "=&s"(cc) : "v"(a));
    asm volatile("v_mad_u64_u32 %0, %2, %3, %3, %0\n\tv_mad_u64_u32 %1, %2, %3, %3, %1" : "+v"(q[0]), "+v"(q[1]), "=&s"(cc) : "v"(a));
    asm volatile("v_mad_u64_u32 %0, %2, %3, %3, %0\n\tv_mad_u64_u32 %1, %2, %3, %3, %1" : "+v"(q[2]), "+v"(q[3]), "=&s"(cc) : "v"(a));
  } else if constexpr (MODE == 13) {  // v_mad_i64_i32 (the signed form lpfield.hpp uses)
    uint64_t cc;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      asm volatile("v_mad_i64_i32 %0, %1, %2, %2, %0\n\tv_mad_i64_i32 %0, %1, %2, %2, %0" : "+v"(q[i]), "=&s"(cc) : "v"(a));
  } else if constexpr (MODE == 14) {  // v_fma_f64
    double d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = __builtin_bit_cast(double, q[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("v_fma_f64 %0, %0, %0, %0\n\tv_fma_f64 %0, %0, %0, %0" : "+v"(d[i]));
#pragma unroll
    for (int i = 0; i < 4; ++i) q[i] = __builtin_bit_cast(uint64_t, d[i]);
  } else if constexpr (MODE == 15) {  // v_lshl_add_u64 (64-bit integer add, gfx950)
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("v_lshl_add_u64 %0, %0, 0, %0\n\tv_lshl_add_u64 %0, %0, 0, %0" : "+v"(q[i]));
  }
}

template <int MODE>
__global__ void __launch_bounds__(256) k_mix(uint32_t* out, int iters, uint32_t seed) {
  uint64_t cc;
  const uint32_t a = seed ^ threadIdx.x, b = seed * 3 + blockIdx.x;
  uint64_t c0 = a, c1 = b, c2 = a ^ 1, c3 = b ^ 1, c4 = a ^ 2, c5 = b ^ 2, c6 = a ^ 3, c7 = b ^ 3;
  uint32_t t[8];
  uint64_t q[4];
#pragma unroll
  for (int i = 0; i < 8; ++i) t[i] = a + i;
#pragma unroll
  for (int i = 0; i < 4; ++i) q[i] = (uint64_t)b * (i + 1);
  for (int it = 0; it < iters; ++it) {
    MAD4(c0, c1, c2, c3, a, b);
    if constexpr (MODE > 0) filler<MODE>(t, q, a);
    MAD4(c4, c5, c6, c7, a, b);
  }
  uint64_t s = c0 ^ c1 ^ c2 ^ c3 ^ c4 ^ c5 ^ c6 ^ c7;
  uint32_t u = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) u ^= t[i];
#pragma unroll
  for (int i = 0; i < 4; ++i) s ^= q[i];
  if (s == 0x1234567 && u == 7) out[0] = 1;  // keep everything live
}

template <int MODE>
static double run(int waves_per_simd) {
  int cus = 0;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  uint32_t* out;
  (void)hipMalloc(&out, 4);
  const int iters = 8192, blocks = cus * waves_per_simd;
  hipLaunchKernelGGL(k_mix<MODE>, dim3(blocks), dim3(256), 0, 0, out, 16, 1u);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int r = 0; r < 3; ++r) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_mix<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  (void)hipFree(out);
  // ns per iteration per wave-slot: each SIMD runs waves_per_simd waves of `iters` iterations
  return best * 1e6 / ((double)iters * waves_per_simd);
}

int main() {
  const char* names[] = {"8 mads alone", "+8 v_and_b32", "+8 v_lshrrev_b64", "+8 v_mul_lo_u32", "+8 v_sub_u32",
                         "+8 v_add3_u32", "+8 s_nop 0", "+8 v_lshrrev_b32", "+8 v_alignbit_b32", "+8 v_mov_b32",
                         "+8 v_cndmask_b32", "+8 v_lshl_add_u32", "+8 v_mad_u64_u32", "+8 v_mad_i64_i32",
                         "+8 v_fma_f64", "+8 v_lshl_add_u64"};
  for (int w : {4}) {
    double t[16];
    t[0] = run<0>(w); t[1] = run<1>(w); t[2] = run<2>(w); t[3] = run<3>(w); t[4] = run<4>(w); t[5] = run<5>(w);
    t[6] = run<6>(w); t[7] = run<7>(w); t[8] = run<8>(w); t[9] = run<9>(w); t[10] = run<10>(w); t[11] = run<11>(w);
    t[12] = run<12>(w); t[13] = run<13>(w); t[14] = run<14>(w); t[15] = run<15>(w);
    printf("# waves/SIMD %d: ns per iteration per wave (SIMD time / waves); marginal = (t - t_mads) / 8\n", w);
    for (int m = 0; m < 16; ++m)
      printf("%-22s %7.3f ns/iter   marginal %6.3f ns per instruction (mad alone: %.3f)\n", names[m], t[m],
             m ? (t[m] - t[0]) / 8 : 0.0, t[0] / 8);
  }
  return 0;
}
