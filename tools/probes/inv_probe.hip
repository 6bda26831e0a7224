// Cost of the pairing's one Fp inversion (pairing_par.hpp K_INV: field.hpp fp_inv -> bingcd.hpp
// BinGcd<12>::inv on wave 0, uniform operands), split into its parts: the whole inversion, the
// 26 x 30 inner binary-GCD steps on the 64-bit approximations alone, and one outer step's four
// N-limb updates (lin, linmod).  Cycles from s_memtime on thread 0.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I kzg-batch-verification-scheme_amd/csrc \
//     tools/probes/inv_probe.hip -o tools/probes/inv_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#include "field.hpp"
#include "params_gen.hpp"

using namespace kzgmi;
using P = Bls12_381FpParams;
constexpr int N = P::N;
using G = BinGcd<N>;

template <int MODE>
__global__ void k_inv(int iters, const uint32_t* __restrict__ in, uint64_t* out, uint32_t* sink) {
  uint32_t y[N];
#pragma unroll
  for (int i = 0; i < N; ++i) y[i] = __builtin_amdgcn_readfirstlane(in[i]);
  uint32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
      Fp<P> a;
#pragma unroll
      for (int i = 0; i < N; ++i) a.v[i] = y[i];
      const Fp<P> r = fp_inv(a);
      y[0] ^= r.v[0] & 1;  // keeps the chain dependent
      acc += r.v[1];
    } else if constexpr (MODE == 1) {  // the inner steps only
      uint64_t aa = ((uint64_t)y[1] << 32) | y[0], bb = ((uint64_t)y[3] << 32) | y[2] | 1;
      int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
      for (int s = 0; s < 26; ++s) {
        for (int j = 0; j < G::K; ++j) {
          if (aa & 1) {
            if (aa < bb) {
              const uint64_t t = aa;
              aa = bb;
              bb = t;
              int64_t q = f0;
              f0 = f1;
              f1 = q;
              q = g0;
              g0 = g1;
              g1 = q;
            }
            aa = (aa - bb) >> 1;
            f0 -= f1;
            g0 -= g1;
          } else {
            aa >>= 1;
          }
          f1 *= 2;
          g1 *= 2;
        }
        aa ^= (uint64_t)y[4 + (s & 3)] << 20;
        bb |= 1;
      }
      acc += (uint32_t)(f0 ^ g0 ^ f1 ^ g1 ^ aa);
      y[0] += acc & 1;
    } else {  // 26 outer steps' updates only (lin x 2, linmod x 2)
      uint32_t a[N], b[N], u[N], v[N], m[N];
#pragma unroll
      for (int i = 0; i < N; ++i) {
        a[i] = y[i];
        b[i] = y[(i + 3) % N] ^ 0x5555;
        u[i] = y[(i + 5) % N] >> 2;
        v[i] = y[(i + 7) % N] >> 2;
        m[i] = P::MOD[i];
      }
      for (int s = 0; s < 26; ++s) {
        const int64_t f0 = (int64_t)(y[s % N] & 0x1fffffff) - (1 << 28), g0 = (int64_t)(y[(s + 1) % N] >> 3) - (1 << 28);
        const int64_t f1 = -g0 / 2, g1 = f0 / 2;
        uint32_t na[N], nb[N], nu[N], nv[N];
        G::lin(a, b, f0, g0, na);
        G::lin(a, b, f1, g1, nb);
        G::linmod(u, v, f0, g0, m, 0x1234567u, nu);
        G::linmod(u, v, f1, g1, m, 0x1234567u, nv);
#pragma unroll
        for (int i = 0; i < N; ++i) {
          a[i] = na[i] | 1;
          b[i] = nb[i];
          u[i] = nu[i] >> 1;
          v[i] = nv[i] >> 1;
        }
      }
      acc += a[0] ^ b[1] ^ u[2] ^ v[3];
      y[0] += acc & 1;
    }
  }
  asm volatile("" ::"s"(acc));
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    sink[0] = acc;
  }
}

template <int MODE>
static double run(const uint32_t* d_in, int iters) {
  uint64_t* out;
  uint32_t* sink;
  (void)hipMalloc(&out, 8);
  (void)hipMalloc(&sink, 4);
  k_inv<MODE><<<1, 64>>>(2, d_in, out, sink);
  k_inv<MODE><<<1, 64>>>(iters, d_in, out, sink);
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, out, 8, hipMemcpyDeviceToHost);
  (void)hipFree(out);
  (void)hipFree(sink);
  return (double)cyc / iters;
}

int main() {
  uint32_t h[N];
  for (int i = 0; i < N; ++i) h[i] = 0x9E3779B9u * (i + 1);
  h[N - 1] &= 0x0fffffff;
  uint32_t* d;
  (void)hipMalloc(&d, sizeof h);
  (void)hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  printf("fp_inv (BLS12-381, wave 0, uniform):        %8.0f s_memtime ticks\n", run<0>(d, 50));
  printf("26 x 30 inner steps alone:                  %8.0f\n", run<1>(d, 50));
  printf("26 outer updates alone (2 lin + 2 linmod):  %8.0f\n", run<2>(d, 50));
  return 0;
}
