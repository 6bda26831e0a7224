// Probe: batch-affine bucket additions with the inversion amortised across
// the WAVE instead of per thread, radix 2^29 (csrc/field29.hpp), against the production XYZZ
// accumulation (k_accumulate: 33.55 M additions in 5.19 ms = 6.46 G additions/s at n = 2^20).
//
// Round 2's probe (ba29.hip) paid a per-thread Fermat inversion (~570 products) per S additions
// and stored the prefix products in HBM.  Here, for S independent additions per lane:
//   forward, per lane:  d_e = x2 - x1, prefix products q_e = d_0 ... d_e           S - 1 products
//   across the wave:    exclusive prefix E and suffix U of the lane totals q_{S-1}
//                       (Hillis-Steele over 64 lanes: 2 x 6 full-wave products, 14-limb shuffles)
//   one inversion per wave: lane 0 inverts the wave product (word-level binary GCD, bingcd.hpp),
//                       broadcast; inv(q_{S-1}) = inv(W) E U                              2 products
//   backward, per lane: e = S-1..0: 1/d_e = inv q_{e-1}; inv *= d_e; lambda = (y2 - y1)/d_e;
//                       x3 = lambda^2 - x1 - x2; y3 = lambda (x1 - x3) - y1               5 products
// = 6 products per addition + (14 products + one inversion) / (64 S), against 10 (8M + 2S) of
// the XYZZ mixed addition.  PREFIX_REGS: the S prefix products stay in VGPRs (S <= 4); else in
// HBM as in round 2.  Inputs are contiguous (the real first level gathers them through the
// sorted bucket entries; later levels re-read the sums), so the rate is an upper bound.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I kzg-batch-verification-scheme_amd/csrc -I include \
//     tools/probes/batch_affine/ba_wave.hip -o tools/probes/batch_affine/ba_wave
#include "field29.hpp"
#include "params_gen.hpp"
#include <cstdio>
#include <cstdlib>
#include <vector>
using namespace kzgmi;
using Q = Bls12_381Fp29;
using F = F29<Q>;
using P32 = Bls12_381FpParams;

KZ_DEV F shfl_f(const F& a, int src) {
  F r;
#pragma unroll
  for (int k = 0; k < Q::N; ++k) r.v[k] = (uint32_t)__shfl((int)a.v[k], src);
  return r;
}

// canonical x^-1 (Montgomery radix 29) on one lane: radix-29 -> 32-bit Montgomery, bingcd, back
KZ_DEV F inv_one_lane(const F& a) {
  const Fp<P32> w = fp_from29<Q, P32>(a);
  return fp_to29<Q, P32>(fp_inv(w));
}

template <int S, bool PREFIX_REGS>
__global__ void __launch_bounds__(256) k_batch_affine_wave(const F* X1, const F* Y1, const F* X2, const F* Y2,
                                                           F* pre, F* X3, F* Y3, size_t T) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // T is a multiple of 256
  const int lane = threadIdx.x & 63;
  const F one = F::from_const(Q::ONE);
  F q[PREFIX_REGS ? S : 1];
  F acc;
  // ---- forward: prefix products of this lane's S differences
#pragma unroll
  for (int e = 0; e < S; ++e) {
    const size_t i = (size_t)e * T + t;
    const F d = sub29(X2[i], X1[i], Q::B4);
    acc = e == 0 ? d : mul29(acc, d);
    if constexpr (PREFIX_REGS) q[e] = acc;
    else pre[i] = acc;
  }
  // ---- across the wave: exclusive prefix E and suffix U of the lane totals (Hillis-Steele)
  F inc = acc, suf = acc;
#pragma unroll
  for (int k = 1; k < 64; k <<= 1) {
    const F a = shfl_f(inc, lane - k >= 0 ? lane - k : lane);
    const F b = shfl_f(suf, lane + k < 64 ? lane + k : lane);
    if (lane >= k) inc = mul29(inc, a);
    if (lane + k < 64) suf = mul29(suf, b);
  }
  const F E = lane > 0 ? shfl_f(inc, lane - 1) : one;   // d-products of lanes 0 .. lane-1
  const F U = lane < 63 ? shfl_f(suf, lane + 1) : one;  // lanes lane+1 .. 63
  // ---- one inversion per wave (lane 0: the wave product), broadcast
  F winv = one;
  const F wprod = shfl_f(inc, 63);
  if (lane == 0) winv = inv_one_lane(wprod);
  winv = shfl_f(winv, 0);
  F inv = mul29(mul29(winv, E), U);  // 1 / (this lane's total)
  // ---- backward
#pragma unroll
  for (int e = S - 1; e >= 0; --e) {
    const size_t i = (size_t)e * T + t;
    const F x1 = X1[i], x2 = X2[i];
    const F d = sub29(x2, x1, Q::B4);
    F ie = inv;
    if (e > 0) {
      if constexpr (PREFIX_REGS) ie = mul29(inv, q[e - 1]);
      else ie = mul29(inv, pre[i - T]);
      inv = mul29(inv, d);
    }
    const F lam = mul29(sub29(Y2[i], Y1[i], Q::B4), ie);
    const F x3 = sub29(sub29(sqr29(lam), x1, Q::B4), x2, Q::B4);
    const F y3 = sub29(mul29(lam, sub29(x1, x3, Q::B16)), Y1[i], Q::B4);
    X3[i] = x3;
    Y3[i] = y3;
  }
}

// reference for a few elements: one inversion per addition
__global__ void k_check(const F* X1, const F* Y1, const F* X2, const F* Y2, const F* X3, const F* Y3, size_t n,
                        uint32_t* bad) {
  const size_t i = ((size_t)blockIdx.x * 7919u + threadIdx.x * 104729u) % n;
  const F x1 = X1[i], x2 = X2[i];
  const F lam = mul29(sub29(Y2[i], Y1[i], Q::B4), inv_one_lane(sub29(x2, x1, Q::B4)));
  const F x3 = sub29(sub29(mul29(lam, lam), x1, Q::B4), x2, Q::B4);
  const F y3 = sub29(mul29(lam, sub29(x1, x3, Q::B16)), Y1[i], Q::B4);
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

template <int S, bool REGS>
void run_case(std::vector<F*>& buf, size_t total, uint32_t* bad, hipEvent_t e0, hipEvent_t e1) {
  const size_t T = total / S;
  auto run = [&]() {
    hipLaunchKernelGGL((k_batch_affine_wave<S, REGS>), dim3(T / 256), dim3(256), 0, 0, buf[0], buf[1], buf[2],
                       buf[3], buf[4], buf[5], buf[6], T);
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
  hipLaunchKernelGGL(k_check, dim3(64), dim3(64), 0, 0, buf[0], buf[1], buf[2], buf[3], buf[5], buf[6], total, bad);
  uint32_t nbad = 0;
  (void)hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost);
  printf("S %3d  prefix %s  lanes %8zu  %.3f ms per 2^24 additions  %.2f G additions/s  check mismatches %u/4096\n",
         S, REGS ? "VGPR" : "HBM ", T, ms, total / (ms * 1e6), nbad);
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
  run_case<2, true>(buf, total, bad, e0, e1);
  run_case<4, true>(buf, total, bad, e0, e1);
  run_case<8, false>(buf, total, bad, e0, e1);
  run_case<16, false>(buf, total, bad, e0, e1);
  run_case<32, false>(buf, total, bad, e0, e1);
  run_case<64, false>(buf, total, bad, e0, e1);
  printf("production XYZZ accumulation (k_accumulate, n = 2^20, round 4): 32 n = 33.55 M additions in 5.19 ms = "
         "6.46 G additions/s\n");
  return 0;
}
