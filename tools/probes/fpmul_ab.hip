// A/B probe: CIOS vs product-scanning Montgomery multiplication (throughput + equality).
#include "field.hpp"
#include "params_gen.hpp"
#include <cstdio>
using namespace kzgmi;

template <class P, int V>
__global__ void __launch_bounds__(256) k_probe(uint32_t iters, uint32_t* out) {
  using F = Fp<P>;
  F a[8];
  F b = F::one();
  b.v[0] ^= threadIdx.x * 2654435761u;
  for (int j = 0; j < 8; ++j) { a[j] = F::one(); a[j].v[1] ^= (blockIdx.x * 8 + j) * 40503u; }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = V ? fp_mul_ps(a[j], b) : fp_mul_cios(a[j], b);
  }
  uint32_t x = 0;
  for (int j = 0; j < 8; ++j) for (int k = 0; k < P::N; ++k) x = x * 31 + a[j].v[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <class P>
void run(const char* name) {
  const uint32_t blocks = 256 * 16, iters = 512;
  uint32_t *o0, *o1;
  hipMalloc(&o0, blocks * 256 * 4); hipMalloc(&o1, blocks * 256 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float t[2];
  for (int v = 0; v < 2; ++v) {
    auto k = v ? k_probe<P, 1> : k_probe<P, 0>;
    uint32_t* o = v ? o1 : o0;
    k<<<blocks, 256>>>(8, o);
    hipEventRecord(e0);
    k<<<blocks, 256>>>(iters, o);
    hipEventRecord(e1); hipEventSynchronize(e1);
    hipEventElapsedTime(&t[v], e0, e1);
  }
  uint32_t *h0 = new uint32_t[blocks * 256], *h1 = new uint32_t[blocks * 256];
  hipMemcpy(h0, o0, blocks * 256 * 4, hipMemcpyDeviceToHost); hipMemcpy(h1, o1, blocks * 256 * 4, hipMemcpyDeviceToHost);
  size_t diff = 0; for (size_t i = 0; i < (size_t)blocks * 256; ++i) diff += h0[i] != h1[i];
  double nm = (double)blocks * 256 * iters * 8;
  printf("%s: cios %.2f G mul/s   ps %.2f G mul/s   speedup %.2fx   mismatches %zu\n", name, nm / t[0] / 1e6, nm / t[1] / 1e6, t[0] / t[1], diff);
}

int main() {
  run<Bls12_381FpParams>("BLS12-381 Fp (12 limbs)");
  run<Bn254FpParams>("BN254 Fp (8 limbs)");
  run<Bls12_381FrParams>("BLS12-381 Fr (8 limbs)");
  return 0;
}
