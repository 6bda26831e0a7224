// Issue-rate probe: v_mad_u64_u32 vs plain 32-bit VALU on gfx950, alone and mixed.
// Each thread runs 8 independent chains so dependency latency is hidden; reports wave64
// instructions per SIMD per ns for each mix.  Decides the cost model of the field layer:
// if the 64-bit multiply-add has its own (slower) rate and the 32-bit carry/move ops issue in
// its shadow, only the multiply-add count matters.
//   hipcc -O3 --offload-arch=gfx950 tools/probes/mad_rate.hip -o tools/probes/mad_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define MAD(acc, a, b) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc), "=s"(cc) : "v"(a), "v"(b))
#define MAC(acc, top, a, b) asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1" : "+v"(acc), "=&s"(cc), "+v"(top) : "v"(a), "v"(b))
#define ADDC(x, y) asm volatile("v_add_co_u32_e64 %0, %1, %0, %2" : "+v"(x), "=s"(cc) : "v"(y))
#define MOV(x, y) asm volatile("v_mov_b32 %0, %1" : "=v"(x) : "v"(y))
#define MULLO(x, y) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(y))
#define U24(x, y) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(x) : "v"(y))
// 4 mads per statement: independent accumulators (MAD4I) or one dependent chain (MAD4D)
#define MAD4I(c0, c1, c2, c3, a, b) asm volatile("v_mad_u64_u32 %0, %4, %5, %6, %0\n\tv_mad_u64_u32 %1, %4, %5, %6, %1\n\t" \
    "v_mad_u64_u32 %2, %4, %5, %6, %2\n\tv_mad_u64_u32 %3, %4, %5, %6, %3" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "=&s"(cc) : "v"(a), "v"(b))
#define MAD4D(c0, a, b) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %3, %2, %0\n\t" \
    "v_mad_u64_u32 %0, %1, %2, %3, %0\n\tv_mad_u64_u32 %0, %1, %3, %2, %0" : "+v"(c0), "=&s"(cc) : "v"(a), "v"(b))
#define SHR64(x) asm volatile("v_lshrrev_b64 %0, 29, %0" : "+v"(x))
#define ALIGN(lo, hi) asm volatile("v_alignbit_b32 %0, %1, %0, 29" : "+v"(lo) : "v"(hi))
#define MULLO_AND(m, x, y) asm volatile("v_mul_lo_u32 %0, %1, %2\n\tv_and_b32 %0, 0x1fffffff, %0" : "=&v"(m) : "v"(x), "v"(y))
#define FMA64(x, y) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(y))

template <int MODE>
__global__ void __launch_bounds__(256) k_probe(uint32_t* out, int iters, uint32_t seed) {
  uint64_t cc;
  uint32_t a = seed ^ threadIdx.x, b = seed * 3 + blockIdx.x;
  uint64_t acc0 = a, acc1 = b, acc2 = a ^ 1, acc3 = b ^ 1, acc4 = a ^ 2, acc5 = b ^ 2, acc6 = a ^ 3, acc7 = b ^ 3;
  uint32_t t0 = 0, t1 = 1, t2 = 2, t3 = 3, t4 = 4, t5 = 5, t6 = 6, t7 = 7;
  uint32_t m0, m1, m2, m3, m4, m5, m6, m7;
  double d0 = a, d1 = b, d2 = a + 1.0, d3 = b + 1.0, d4 = a + 2.0, d5 = b + 2.0, d6 = a + 3.0, d7 = b + 3.0, dy = 1.0000001;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {  // 8 v_mad_u64_u32
      MAD(acc0, a, b); MAD(acc1, a, b); MAD(acc2, a, b); MAD(acc3, a, b);
      MAD(acc4, a, b); MAD(acc5, a, b); MAD(acc6, a, b); MAD(acc7, a, b);
    } else if constexpr (MODE == 1) {  // 8 x (mad + addc) = the field layer's mac32
      MAC(acc0, t0, a, b); MAC(acc1, t1, a, b); MAC(acc2, t2, a, b); MAC(acc3, t3, a, b);
      MAC(acc4, t4, a, b); MAC(acc5, t5, a, b); MAC(acc6, t6, a, b); MAC(acc7, t7, a, b);
    } else if constexpr (MODE == 2) {  // 8 v_add_co_u32
      ADDC(t0, a); ADDC(t1, a); ADDC(t2, a); ADDC(t3, a); ADDC(t4, a); ADDC(t5, a); ADDC(t6, a); ADDC(t7, a);
    } else if constexpr (MODE == 3) {  // 8 mad + 8 mov
      MAD(acc0, a, b); MOV(m0, t0); MAD(acc1, a, b); MOV(m1, t1); MAD(acc2, a, b); MOV(m2, t2); MAD(acc3, a, b); MOV(m3, t3);
      MAD(acc4, a, b); MOV(m4, t4); MAD(acc5, a, b); MOV(m5, t5); MAD(acc6, a, b); MOV(m6, t6); MAD(acc7, a, b); MOV(m7, t7);
      t0 += m0; t1 += m1; t2 += m2; t3 += m3; t4 += m4; t5 += m5; t6 += m6; t7 += m7;
    } else if constexpr (MODE == 4) {  // 8 v_mul_lo_u32
      MULLO(t0, a); MULLO(t1, a); MULLO(t2, a); MULLO(t3, a); MULLO(t4, a); MULLO(t5, a); MULLO(t6, a); MULLO(t7, a);
    } else if constexpr (MODE == 5) {  // 8 v_mad_u32_u24
      U24(t0, a); U24(t1, a); U24(t2, a); U24(t3, a); U24(t4, a); U24(t5, a); U24(t6, a); U24(t7, a);
    } else if constexpr (MODE == 6) {  // 8 v_fma_f64
      FMA64(d0, dy); FMA64(d1, dy); FMA64(d2, dy); FMA64(d3, dy); FMA64(d4, dy); FMA64(d5, dy); FMA64(d6, dy); FMA64(d7, dy);
    } else if constexpr (MODE == 8) {  // 8 independent mads, 4 per statement
      MAD4I(acc0, acc1, acc2, acc3, a, b); MAD4I(acc4, acc5, acc6, acc7, a, b);
    } else if constexpr (MODE == 9) {  // one dependent chain of 8 mads, 4 per statement
      MAD4D(acc0, a, b); MAD4D(acc0, a, b);
    } else if constexpr (MODE == 10) {  // one dependent chain of 8 mads, 1 per statement
      MAD(acc0, a, b); MAD(acc0, a, b); MAD(acc0, a, b); MAD(acc0, a, b);
      MAD(acc0, a, b); MAD(acc0, a, b); MAD(acc0, a, b); MAD(acc0, a, b);
    } else if constexpr (MODE == 11) {  // two dependent chains, 4 per statement, alternating
      MAD4D(acc0, a, b); MAD4D(acc1, a, b);
    } else if constexpr (MODE == 12) {  // 8 v_lshrrev_b64 (the column shift of the radix-29 products)
      SHR64(acc0); SHR64(acc1); SHR64(acc2); SHR64(acc3); SHR64(acc4); SHR64(acc5); SHR64(acc6); SHR64(acc7);
    } else if constexpr (MODE == 13) {  // 8 v_alignbit_b32
      ALIGN(t0, t1); ALIGN(t1, t2); ALIGN(t2, t3); ALIGN(t3, t4); ALIGN(t4, t5); ALIGN(t5, t6); ALIGN(t6, t7); ALIGN(t7, t0);
    } else if constexpr (MODE == 7) {  // 8 mad + 8 add_co
      MAD(acc0, a, b); ADDC(t0, a); MAD(acc1, a, b); ADDC(t1, a); MAD(acc2, a, b); ADDC(t2, a); MAD(acc3, a, b); ADDC(t3, a);
      MAD(acc4, a, b); ADDC(t4, a); MAD(acc5, a, b); ADDC(t5, a); MAD(acc6, a, b); ADDC(t6, a); MAD(acc7, a, b); ADDC(t7, a);
    }
  }
  uint64_t s = acc0 ^ acc1 ^ acc2 ^ acc3 ^ acc4 ^ acc5 ^ acc6 ^ acc7;
  uint32_t u = t0 ^ t1 ^ t2 ^ t3 ^ t4 ^ t5 ^ t6 ^ t7;
  double d = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7;
  if (s == 0x1234567 && u == 7 && d == 1.0) out[0] = 1;  // keep the chains live
}

template <int MODE>
static void run(const char* name, int instr_per_iter, int waves_per_simd) {
  int dev = 0, cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  uint32_t* out;
  hipMalloc(&out, 4);
  const int iters = 4096;
  const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
  hipLaunchKernelGGL(k_probe<MODE>, dim3(blocks), dim3(256), 0, 0, out, 16, 1u);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(k_probe<MODE>, dim3(blocks), dim3(256), 0, 0, out, iters, 1u);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  double wave_instr = (double)blocks * 4 * iters * instr_per_iter;  // wave64 instructions
  double per_simd_ns = wave_instr / (cus * 4.0) / (ms * 1e6);
  printf("%-28s waves/SIMD %2d  %8.3f ms  %.4f wave-instr/SIMD/ns  (%.2f ns each)\n", name, waves_per_simd, ms,
         per_simd_ns, 1.0 / per_simd_ns);
  hipFree(out);
}

int main() {
  for (int w : {4, 8}) {
    run<0>("mad_u64_u32 x8", 8, w);
    run<1>("mad+addc (mac32) x8", 16, w);
    run<2>("add_co_u32 x8", 8, w);
    run<3>("mad x8 + mov x8 (+8 add)", 24, w);
    run<7>("mad x8 + add_co x8", 16, w);
    run<4>("mul_lo_u32 x8", 8, w);
    run<5>("mad_u32_u24 x8", 8, w);
    run<6>("fma_f64 x8", 8, w);
    run<8>("mad x8 indep, 4/statement", 8, w);
    run<9>("mad chain x8, 4/statement", 8, w);
    run<10>("mad chain x8, 1/statement", 8, w);
    run<11>("2 mad chains, 4/statement", 8, w);
    run<12>("lshrrev_b64 x8", 8, w);
    run<13>("alignbit_b32 x8", 8, w);
  }
  return 0;
}
