// Fp-product throughput vs independent dependency chains per thread (ILP) and occupancy.
// Each thread runs CH independent chains a_j <- a_j * b; the accumulation kernel has ~1-2.
#include "field.hpp"
#include "params_gen.hpp"
#include <cstdio>
using namespace kzgmi;

template <class P, int CH, int UNR = 1>
__global__ void __launch_bounds__(256) k_chain(uint32_t iters, uint32_t* out) {
  extern __shared__ uint32_t pad[];  // dynamic LDS only to cap workgroups per CU
  if (iters == 0xffffffffu) pad[threadIdx.x] = 0;
  using F = Fp<P>;
  F a[CH];
  F b = F::one();
  b.v[0] ^= threadIdx.x * 2654435761u;
  for (int j = 0; j < CH; ++j) { a[j] = F::one(); a[j].v[1] ^= (blockIdx.x * 8 + j) * 40503u; }
  for (uint32_t it = 0; it < iters; it += UNR) {
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
#pragma unroll
      for (int j = 0; j < CH; ++j) a[j] = fp_mul(a[j], b);
    }
  }
  uint32_t x = 0;
  for (int j = 0; j < CH; ++j) for (int k = 0; k < P::N; ++k) x = x * 31 + a[j].v[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <class P, int CH, int UNR = 1>
void run(uint32_t* o, const char* name, int waves) {
  const uint32_t blocks = 256 * 16, iters = 4096 / CH;
  const size_t lds = waves >= 6 ? 26 * 1024 : waves == 4 ? 40 * 1024 : waves == 3 ? 48 * 1024 : waves == 2 ? 64 * 1024 : 96 * 1024;
  hipFuncSetAttribute((const void*)k_chain<P, CH, UNR>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k_chain<P, CH, UNR><<<blocks, 256, lds>>>(8, o);
  hipEventRecord(e0);
  k_chain<P, CH, UNR><<<blocks, 256, lds>>>(iters, o);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double nm = (double)blocks * 256 * iters * CH;
  printf("%s unroll=%d chains=%d waves/SIMD<=%d: %.2f G mul/s  (%s)\n", name, UNR, CH, waves, nm / ms / 1e6, hipGetErrorString(hipGetLastError()));
}

int main() {
  uint32_t* o; hipMalloc(&o, 256 * 16 * 256 * 4);
  run<Bls12_381FpParams, 2, 1>(o, "BLS", 3);
  run<Bls12_381FpParams, 2, 2>(o, "BLS", 3);
  run<Bls12_381FpParams, 2, 4>(o, "BLS", 3);
  run<Bls12_381FpParams, 2, 8>(o, "BLS", 3);
  run<Bls12_381FpParams, 2, 16>(o, "BLS", 3);
  run<Bls12_381FpParams, 1, 16>(o, "BLS", 3);
  return 0;
}
