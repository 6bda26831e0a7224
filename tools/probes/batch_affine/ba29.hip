// Probe: batch-affine bucket additions with a per-thread Montgomery-trick
// inversion, radix 2^29 (csrc/field29.hpp), against the production XYZZ accumulation rate.
//
// Idealised first level of a batch-affine Pippenger (pairs of points of one bucket added in
// affine coordinates, one shared inversion per thread of S additions):
//   pass 1: d_e = x2 - x1, prefix products P_e = d_0 ... d_e (stored, S per thread)
//   one inversion of P_{S-1} (Fermat, ~570 products)
//   pass 2, e = S-1..0: 1/d_e = inv P_{e-1}; inv *= d_e; lambda = (y2 - y1)/d_e;
//           x3 = lambda^2 - x1 - x2; y3 = lambda (x1 - x3) - y1
// = 6 products per addition + 570 / S, against 10 (8M + 2S) for the XYZZ mixed addition, but
// ~560 B of HBM traffic per addition (inputs 224 B, prefix 2 x 56 B, outputs 112 B, re-reads).
// Inputs are contiguous here (the real first level gathers them through the sorted bucket
// entries, and later levels re-read the sums), so the measured rate is an upper bound.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I kzg-batch-verification-scheme_amd/csrc -I include \
//     tools/probes/batch_affine/ba29.hip -o tools/probes/batch_affine/ba29
#include "field29.hpp"
#include "params_gen.hpp"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace kzgmi;
using Q = Bls12_381Fp29;
using F = F29<Q>;
using P32 = Bls12_381FpParams;

KZ_DEV F ld(const F* a, size_t i) { return a[i]; }
KZ_DEV void st(F* a, size_t i, const F& v) { a[i] = v; }

// a^(p-2) (Montgomery radix 29): square-and-multiply over the 381 bits of p - 2
KZ_DEV F inv29(const F& a) {
  F r = F::from_const(Q::ONE);
  for (int w = P32::N - 1; w >= 0; --w) {
    const uint32_t e = P32::PM2[w];
    for (int b = 31; b >= 0; --b) {
      r = mul29(r, r);
      if ((e >> b) & 1) r = mul29(r, a);
    }
  }
  return r;
}

// bounds: inputs < 2p (canonical random values here); B_k biases as csrc/msm.hpp uses them
__global__ void __launch_bounds__(256) k_batch_affine(const F* X1, const F* Y1, const F* X2, const F* Y2, F* pre,
                                                      F* X3, F* Y3, int S, size_t T) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T) return;
  F acc;
  for (int e = 0; e < S; ++e) {
    const size_t i = (size_t)e * T + t;
    const F d = sub29(ld(X2, i), ld(X1, i), Q::B4);
    acc = e == 0 ? d : mul29(acc, d);
    st(pre, i, acc);
  }
  F inv = inv29(acc);
  for (int e = S - 1; e >= 0; --e) {
    const size_t i = (size_t)e * T + t;
    const F x1 = ld(X1, i), x2 = ld(X2, i);
    const F d = sub29(x2, x1, Q::B4);
    const F ie = e > 0 ? mul29(inv, ld(pre, i - T)) : inv;
    inv = mul29(inv, d);
    const F lam = mul29(sub29(ld(Y2, i), ld(Y1, i), Q::B4), ie);
    const F x3 = sub29(sub29(mul29(lam, lam), x1, Q::B4), x2, Q::B4);
    const F y3 = sub29(mul29(lam, sub29(x1, x3, Q::B16)), ld(Y1, i), Q::B4);
    st(X3, i, x3);
    st(Y3, i, y3);
  }
}

// reference for a few elements: one Fermat inversion per addition
__global__ void k_check(const F* X1, const F* Y1, const F* X2, const F* Y2, const F* X3, const F* Y3, size_t T,
                        int S, uint32_t* bad) {
  const size_t i = ((size_t)blockIdx.x * 7919u + threadIdx.x * 104729u) % ((size_t)S * T);
  const F x1 = X1[i], x2 = X2[i];
  const F lam = mul29(sub29(Y2[i], Y1[i], Q::B4), inv29(sub29(x2, x1, Q::B4)));
  const F x3 = sub29(sub29(mul29(lam, lam), x1, Q::B4), x2, Q::B4);
  const F y3 = sub29(mul29(lam, sub29(x1, x3, Q::B16)), Y1[i], Q::B4);
  // compare canonically: multiply both by 1 (Montgomery) -> < 2p, then canon
  const F one = F::from_const(Q::ONE);
  const F a = canon29(mul29(x3, one)), b = canon29(mul29(X3[i], one));
  const F c = canon29(mul29(y3, one)), d = canon29(mul29(Y3[i], one));
  uint32_t diff = 0;
  for (int k = 0; k < Q::N; ++k) diff |= (a.v[k] ^ b.v[k]) | (c.v[k] ^ d.v[k]);
  if (diff) atomicAdd(bad, 1u);
}

__global__ void k_fill(F* a, size_t n, uint32_t seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)(i * 2654435761u) ^ seed;
  F v;
  for (int k = 0; k < Q::N; ++k) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    v.v[k] = x & M29;
  }
  v.v[Q::N - 1] &= 0x7;  // < 2^380 < p
  a[i] = v;
}

int main() {
  const size_t total = (size_t)1 << 24;  // 2^24 additions = the first level at n = 2^20 (32 n / 2)
  std::vector<F*> buf(7);
  for (auto& b : buf) (void)hipMalloc(&b, total * sizeof(F));
  for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_fill, dim3((total + 255) / 256), dim3(256), 0, 0, buf[k], total, 77u + k);
  uint32_t* bad;
  (void)hipMalloc(&bad, 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int S : {16, 32, 64, 128, 256}) {
    const size_t T = total / S;
    auto run = [&]() {
      hipLaunchKernelGGL(k_batch_affine, dim3((T + 255) / 256), dim3(256), 0, 0, buf[0], buf[1], buf[2], buf[3], buf[4],
                         buf[5], buf[6], S, T);
    };
    run();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) run();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 3;
    (void)hipMemset(bad, 0, 4);
    hipLaunchKernelGGL(k_check, dim3(64), dim3(64), 0, 0, buf[0], buf[1], buf[2], buf[3], buf[5], buf[6], T, S, bad);
    uint32_t nbad = 0;
    (void)hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost);
    printf("S %3d  threads %8zu  %.3f ms per 2^24 additions  %.2f G additions/s  check mismatches %u/4096\n", S, T, ms,
           total / (ms * 1e6), nbad);
  }
  printf("production XYZZ accumulation (k_accumulate, n = 2^20): 32 n = 33.5 M additions in ~6.45 ms = 5.2 G additions/s\n");
  return 0;
}
