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

// the production point table's slot: radix-29 x, y of one affine point in a 128-B line
struct PtSlot {
  F x, y;
  uint32_t pad[4];
};
// level-1 form: the operands of addition i are points idx[2i], idx[2i+1] of a 2^21-point table (the
// real first level pairs sorted entries, whose point indices are scattered like these)
struct Gather {
  const PtSlot* pts;
  const uint32_t* idx;
  KZ_DEV F x1(size_t i) const { return pts[idx[2 * i]].x; }
  KZ_DEV F y1(size_t i) const { return pts[idx[2 * i]].y; }
  KZ_DEV F x2(size_t i) const { return pts[idx[2 * i + 1]].x; }
  KZ_DEV F y2(size_t i) const { return pts[idx[2 * i + 1]].y; }
};
struct Contig {
  const F *X1, *Y1, *X2, *Y2;
  KZ_DEV F x1(size_t i) const { return X1[i]; }
  KZ_DEV F y1(size_t i) const { return Y1[i]; }
  KZ_DEV F x2(size_t i) const { return X2[i]; }
  KZ_DEV F y2(size_t i) const { return Y2[i]; }
};

template <int S, bool PREFIX_REGS, class In>
__global__ void __launch_bounds__(256) k_batch_affine_wave(In in, F* pre, F* X3, F* Y3, size_t T) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // T is a multiple of 256
  const int lane = threadIdx.x & 63;
  const F one = F::from_const(Q::ONE);
  F q[PREFIX_REGS ? S : 1];
  F acc;
  // ---- forward: prefix products of this lane's S differences
#pragma unroll
  for (int e = 0; e < S; ++e) {
    const size_t i = (size_t)e * T + t;
    const F d = sub29(in.x2(i), in.x1(i), Q::B4);
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
  // every lane takes part in the shuffles (a shuffle under a lane mask may read a register the
  // compiler has already reused in the masked-off source lane: lanes 1 and 62 read garbage)
  const F Es = shfl_f(inc, lane > 0 ? lane - 1 : 0), Us = shfl_f(suf, lane < 63 ? lane + 1 : 63);
  const F E = lane > 0 ? Es : one;   // d-products of lanes 0 .. lane-1
  const F U = lane < 63 ? Us : one;  // lanes lane+1 .. 63
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
    const F x1 = in.x1(i), x2 = in.x2(i);
    const F d = sub29(x2, x1, Q::B4);
    F ie = inv;
    if (e > 0) {
      if constexpr (PREFIX_REGS) ie = mul29(inv, q[e - 1]);
      else ie = mul29(inv, pre[i - T]);
      inv = mul29(inv, d);
    }
    const F y1 = in.y1(i);
    const F lam = mul29(sub29(in.y2(i), y1, Q::B4), ie);
    const F x3 = sub29(sub29(sqr29(lam), x1, Q::B4), x2, Q::B4);
    const F y3 = sub29(mul29(lam, sub29(x1, x3, Q::B16)), y1, Q::B4);
    X3[i] = x3;
    Y3[i] = y3;
  }
}

// reference for a few elements: one inversion per addition
template <class In>
__global__ void k_check(In in, const F* X3, const F* Y3, size_t n, uint32_t* bad) {
  const size_t i = ((size_t)blockIdx.x * 7919u + threadIdx.x * 104729u) % n;
  const F x1 = in.x1(i), x2 = in.x2(i), y1 = in.y1(i);
  const F lam = mul29(sub29(in.y2(i), y1, Q::B4), inv_one_lane(sub29(x2, x1, Q::B4)));
  const F x3 = sub29(sub29(mul29(lam, lam), x1, Q::B4), x2, Q::B4);
  const F y3 = sub29(mul29(lam, sub29(x1, x3, Q::B16)), y1, Q::B4);
  const F one = F::from_const(Q::ONE);
  const F a = canon29(mul29(x3, one)), b = canon29(mul29(X3[i], one));
  const F c = canon29(mul29(y3, one)), d = canon29(mul29(Y3[i], one));
  uint32_t diff = 0;
  for (int k = 0; k < Q::N; ++k) diff |= (a.v[k] ^ b.v[k]) | (c.v[k] ^ d.v[k]);
  if (diff) {
    const uint32_t k = atomicAdd(bad, 1u);
    if (k < 8) bad[1 + k] = (uint32_t)i;
  }
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

__global__ void k_fill_pts(PtSlot* p, size_t n, uint32_t seed) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t x = (uint32_t)(i * 2654435761u) ^ seed;
  PtSlot v;
  for (int k = 0; k < Q::N; ++k) {
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    v.x.v[k] = x & M29;
    x ^= x << 13; x ^= x >> 17; x ^= x << 5;
    v.y.v[k] = x & M29;
  }
  v.x.v[Q::N - 1] &= 0x7;
  v.y.v[Q::N - 1] &= 0x7;
  for (int k = 0; k < 4; ++k) v.pad[k] = 0;
  p[i] = v;
}
// operand pairs of distinct scattered points (a pair of equal points would zero its wave's product)
__global__ void k_fill_idx(uint32_t* idx, size_t pairs, uint32_t npts_log2) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= pairs) return;
  const uint32_t m = (1u << npts_log2) - 1;
  uint32_t h = (uint32_t)(i * 2246822519u) ^ 0x9e3779b9u;
  h ^= h >> 15; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  const uint32_t a = h & m;
  uint32_t g = h * 0x27d4eb2fu + 0x165667b1u;
  g ^= g >> 15;
  idx[2 * i] = a;
  idx[2 * i + 1] = (a + 1 + g % m) & m;
}

template <int S, bool REGS, class In>
void run_case(const In& in, std::vector<F*>& buf, size_t total, uint32_t* bad, hipEvent_t e0, hipEvent_t e1,
              const char* form) {
  const size_t T = total / S;
  auto run = [&]() {
    hipLaunchKernelGGL((k_batch_affine_wave<S, REGS, In>), dim3(T / 256), dim3(256), 0, 0, in, buf[4], buf[5],
                       buf[6], T);
  };
  run();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) run();
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 3;
  (void)hipMemset(bad, 0, 36);
  hipLaunchKernelGGL(k_check<In>, dim3(64), dim3(64), 0, 0, in, buf[5], buf[6], total, bad);
  uint32_t hb[9] = {};
  (void)hipMemcpy(hb, bad, 36, hipMemcpyDeviceToHost);
  const uint32_t nbad = hb[0];
  for (uint32_t k = 0; k < nbad && k < 8; ++k)
    printf("  mismatch i %u: e %zu lane-index %zu (lane %zu of wave %zu)\n", hb[1 + k], hb[1 + k] / T, hb[1 + k] % T,
           (hb[1 + k] % T) % 64, (hb[1 + k] % T) / 64);
  printf("%s  S %3d  prefix %s  lanes %8zu  %.3f ms per 2^24 additions  %.2f G additions/s  check mismatches %u/4096\n",
         form, S, REGS ? "VGPR" : "HBM ", T, ms, total / (ms * 1e6), nbad);
}

int main() {
  const size_t total = (size_t)1 << 24;  // 2^24 additions = the first level at n = 2^20 (32 n / 2)
  std::vector<F*> buf(7);
  for (auto& b : buf) (void)hipMalloc(&b, total * sizeof(F));
  for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_fill, dim3((total + 255) / 256), dim3(256), 0, 0, buf[k], total, 77u + k);
  uint32_t* bad;
  (void)hipMalloc(&bad, 36);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const Contig c{buf[0], buf[1], buf[2], buf[3]};
  run_case<2, true>(c, buf, total, bad, e0, e1, "contiguous");
  run_case<4, true>(c, buf, total, bad, e0, e1, "contiguous");
  run_case<8, false>(c, buf, total, bad, e0, e1, "contiguous");
  run_case<16, false>(c, buf, total, bad, e0, e1, "contiguous");
  run_case<32, false>(c, buf, total, bad, e0, e1, "contiguous");
  run_case<64, false>(c, buf, total, bad, e0, e1, "contiguous");
  // level 1 through scattered point indices: 2^21 points (2n at n = 2^20) in 128-B slots
  constexpr uint32_t NPTS_LOG2 = 21;
  PtSlot* pts;
  uint32_t* idx;
  (void)hipMalloc(&pts, sizeof(PtSlot) << NPTS_LOG2);
  (void)hipMalloc(&idx, total * 8);
  hipLaunchKernelGGL(k_fill_pts, dim3((1u << NPTS_LOG2) / 256), dim3(256), 0, 0, pts, (size_t)1 << NPTS_LOG2, 99u);
  hipLaunchKernelGGL(k_fill_idx, dim3(total / 256), dim3(256), 0, 0, idx, total, NPTS_LOG2);
  const Gather g{pts, idx};
  run_case<16, false>(g, buf, total, bad, e0, e1, "gathered  ");
  run_case<32, false>(g, buf, total, bad, e0, e1, "gathered  ");
  run_case<64, false>(g, buf, total, bad, e0, e1, "gathered  ");
  printf("production XYZZ accumulation (k_accumulate, n = 2^20, round 4): 32 n = 33.55 M additions in 5.19 ms = "
         "6.46 G additions/s\n");
  return 0;
}
