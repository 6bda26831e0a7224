// Latency of the lane-parallel arithmetic (csrc/lpfield.hpp) that every latency-bound tail kernel
// runs on: the window combination, the reduction's upper levels, the small-call path and the
// pairing interpreter.  One workgroup; each wave runs a dependent chain (x <- lp_mul(x, y), or
// an XYZZ doubling chain); cycles per operation from s_memtime on thread 0.  Waves 1, 2, 4, 8 per
// workgroup show what a second wave on the same SIMD costs (the pairing runs 8 waves, 2 per SIMD).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I kzg-batch-verification-scheme_amd/csrc \
//     tools/probes/lp_latency.hip -o tools/probes/lp_latency
#include <hip/hip_runtime.h>
#include <cstdio>

#include "lpfield.hpp"
#include "params_gen.hpp"

using namespace kzgmi;
using Cv = Bls12_381;

template <int MODE>
__global__ void k_lp(int iters, uint64_t* out, int* sink) {
  const LpCtx<Cv> c = lp_ctx<Cv>();
  const int lane = threadIdx.x & 15;
  int32_t x = lane < 13 ? (int32_t)(0x1234567u * (lane + 1) & LP_M29) : 0;
  int32_t y = lane < 13 ? (int32_t)(0x7654321u * (lane + 3) & LP_M29) : 0;
  LpXyzz<Cv> p;
  p.x = x; p.y = y; p.zz = c.pj == 0 ? 0 : 1; p.zzz = p.zz; p.inf = false;
  __syncthreads();
  asm volatile("" ::"v"(x), "v"(y), "v"(p.x));
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 0) {
      x = lp_mul(c, x, y);
      asm volatile("" : "+v"(x));
    } else if constexpr (MODE == 1) {
      x = lp_reduce(c, lp_mul(c, x, y));
    } else if constexpr (MODE == 2) {
      p = lp_xyzz_dbl(c, p);
    } else if constexpr (MODE == 3) {
      __syncthreads();
    }
  }
  // the chains must be complete before the second stamp (a volatile use orders them before it)
  asm volatile("" ::"v"(x), "v"(p.x), "v"(p.y), "v"(p.zz), "v"(p.zzz));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[0] = t1 - t0;
  if (x == 0x12345 && p.x == 7) sink[0] = 1;
}

template <int MODE>
static double cycles(int waves, int iters) {
  uint64_t* out;
  int* sink;
  (void)hipMalloc(&out, 8);
  (void)hipMalloc(&sink, 4);
  k_lp<MODE><<<1, 64 * waves>>>(4, out, sink);
  k_lp<MODE><<<1, 64 * waves>>>(iters, out, sink);
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, out, 8, hipMemcpyDeviceToHost);
  (void)hipFree(out);
  (void)hipFree(sink);
  return (double)cyc / iters;
}

int main() {
  // s_memtime ticks: compare with wall time once
  const char* names[] = {"lp_mul (dependent)", "lp_mul + lp_reduce", "lp_xyzz_dbl", "__syncthreads"};
  for (int w : {1, 2, 4, 8, 16}) {
    printf("waves %2d:  %s %8.0f   %s %8.0f   %s %8.0f   %s %6.0f  (s_memtime ticks per op, thread 0)\n", w, names[0],
           cycles<0>(w, 2000), names[1], cycles<1>(w, 2000), names[2], cycles<2>(w, 200), names[3], cycles<3>(w, 20000));
  }
  // clock calibration: one long lp_mul chain timed by events and by s_memtime
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  uint64_t* out;
  int* sink;
  (void)hipMalloc(&out, 8);
  (void)hipMalloc(&sink, 4);
  (void)hipEventRecord(e0);
  k_lp<0><<<1, 64>>>(200000, out, sink);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, out, 8, hipMemcpyDeviceToHost);
  printf("calibration: 200000 lp_mul in %.3f ms = %.1f ns each; s_memtime %.3f GHz\n", ms, ms * 1e6 / 200000,
         cyc / (ms * 1e6));
  return 0;
}
