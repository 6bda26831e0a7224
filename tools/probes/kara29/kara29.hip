// Probe: a one-level limb Karatsuba for the a b half of the radix-2^29
// Montgomery product (csrc/field29.hpp mont29) against the shipped product-scanning form.
//
// Shipped: column K of (a b + m p) is one 64-bit accumulator fed by v_mad_u64_u32 -- the
// multiply AND the 64-bit accumulate are one instruction, 392 of them per BLS12-381 product.
// Karatsuba (14 = 7 + 7 limbs): L = a0 b0, H = a1 b1, M = (a0 + a1)(b0 + b1) as 3 x 49 mads into
// 3 x 13 column sums, then T_k = L_k + (M - L - H)_{k-7} + H_{k-14}: 49 mads fewer, but the
// recombination needs explicit 64-bit adds / subtracts (v_lshl_add_u64, v_sub_co + v_subb_co)
// that the schoolbook form gets for free inside its mads, plus the 13 + 13 + 13 column sums live
// at once (78 VGPRs).  Both forms then run the same interleaved reduction (m_K per low column).
// The probe runs CH independent product chains per thread over the whole chip and reports G
// products/s of each form, with a bit-exact cross-check of the results.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I kzg-batch-verification-scheme_amd/csrc -I include \
//     tools/probes/kara29/kara29.hip -o tools/probes/kara29/kara29
#include "field29.hpp"
#include <cstdio>
#include <vector>
using namespace kzgmi;
using Q = Bls12_381Fp29;
using F = F29<Q>;
constexpr int N = Q::N, H = N / 2;  // 14 = 7 + 7

// (a b + m p) / R29 with a b by one-level Karatsuba
KZ_DEV F kara29(const F& a, const F& b) {
  uint32_t sa[H], sb[H];
#pragma unroll
  for (int i = 0; i < H; ++i) { sa[i] = a.v[i] + a.v[i + H]; sb[i] = b.v[i] + b.v[i + H]; }  // < 2^30
  uint64_t L[2 * H - 1], Hh[2 * H - 1], M[2 * H - 1];
#pragma unroll
  for (int k = 0; k < 2 * H - 1; ++k) {
    uint64_t l = 0, h = 0, m = 0;
#pragma unroll
    for (int i = 0; i < H; ++i) {
      const int j = k - i;
      if (j < 0 || j >= H) continue;
      l += (uint64_t)a.v[i] * b.v[j];
      h += (uint64_t)a.v[i + H] * b.v[j + H];
      m += (uint64_t)sa[i] * sb[j];  // 7 x 2^60 < 2^63
    }
    L[k] = l; Hh[k] = h; M[k] = m;
  }
  // T_k, k = 0 .. 2N - 2: every column sum < 14 x 2^58 (the schoolbook column bound)
  uint64_t T[2 * N - 1];
#pragma unroll
  for (int k = 0; k < 2 * N - 1; ++k) T[k] = 0;
#pragma unroll
  for (int k = 0; k < 2 * H - 1; ++k) {
    T[k] += L[k];
    T[k + H] += M[k] - L[k] - Hh[k];
    T[k + 2 * H] += Hh[k];
  }
  // interleaved Montgomery reduction, as mont29_cols
  uint32_t m[N];
  F t;
  uint64_t acc = 0;
#pragma unroll
  for (int K = 0; K < 2 * N - 1; ++K) {
    acc += T[K];
    const int lo = K < N ? 0 : K - N + 1, hi = K < N ? K - 1 : N - 1;
#pragma unroll
    for (int i = lo; i <= hi; ++i) acc += (uint64_t)m[i] * Q::MOD[K - i];
    if (K < N) {
      m[K] = ((uint32_t)acc * Q::INV) & M29;
      acc += (uint64_t)m[K] * Q::MOD[0];
    } else {
      t.v[K - N] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  t.v[N - 1] = (uint32_t)acc;
  return t;
}

// the shipped column recursion written as plain C++ (the compiler's own mads, no asm s_nop pads):
// separates the Karatsuba effect from the asm-vs-C++ effect
KZ_DEV F school29_plain(const F& a, const F& b) {
  uint32_t m[N];
  F t;
  uint64_t acc = 0;
#pragma unroll
  for (int K = 0; K < 2 * N - 1; ++K) {
    const int lo = K < N ? 0 : K - N + 1, hi = K < N ? K : N - 1;
#pragma unroll
    for (int i = lo; i <= hi; ++i) acc += (uint64_t)a.v[i] * b.v[K - i];
#pragma unroll
    for (int i = lo; i <= (K < N ? K - 1 : N - 1); ++i) acc += (uint64_t)m[i] * Q::MOD[K - i];
    if (K < N) {
      m[K] = ((uint32_t)acc * Q::INV) & M29;
      acc += (uint64_t)m[K] * Q::MOD[0];
    } else {
      t.v[K - N] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  t.v[N - 1] = (uint32_t)acc;
  return t;
}

template <int FORM, int CH>
__global__ void __launch_bounds__(256) k_chain(uint32_t iters, uint32_t* out) {
  F a[CH];
  F b = F::from_const(Q::ONE);
  b.v[0] ^= threadIdx.x * 2654435u & M29;
  for (int j = 0; j < CH; ++j) {
    a[j] = F::from_const(Q::ONE);
    a[j].v[1] ^= ((blockIdx.x * 8 + j) * 40503u) & M29;
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < CH; ++j) a[j] = FORM == 0 ? mul29(a[j], b) : FORM == 1 ? kara29(a[j], b) : school29_plain(a[j], b);
  }
  uint32_t x = 0;
  for (int j = 0; j < CH; ++j)
    for (int k = 0; k < N; ++k) x = x * 31 + a[j].v[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}

template <int FORM, int CH>
double run(uint32_t* o, uint32_t blocks, uint32_t iters) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k_chain<FORM, CH><<<blocks, 256>>>(4, o);
  hipEventRecord(e0);
  k_chain<FORM, CH><<<blocks, 256>>>(iters, o);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return (double)blocks * 256 * iters * CH / (ms * 1e-3) / 1e9;
}

int main() {
  const uint32_t blocks = 256 * 16, iters = 1024;
  uint32_t *o0, *o1;
  hipMalloc(&o0, blocks * 256 * 4);
  hipMalloc(&o1, blocks * 256 * 4);
  // bit-exact: the same chains through both forms
  k_chain<0, 2><<<blocks, 256>>>(64, o0);
  k_chain<1, 2><<<blocks, 256>>>(64, o1);
  std::vector<uint32_t> h0(blocks * 256), h1(blocks * 256);
  hipMemcpy(h0.data(), o0, h0.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(h1.data(), o1, h1.size() * 4, hipMemcpyDeviceToHost);
  size_t diff = 0;
  for (size_t i = 0; i < h0.size(); ++i) diff += h0[i] != h1[i];
  k_chain<2, 2><<<blocks, 256>>>(64, o1);
  hipMemcpy(h1.data(), o1, h1.size() * 4, hipMemcpyDeviceToHost);
  size_t diff2 = 0;
  for (size_t i = 0; i < h0.size(); ++i) diff2 += h0[i] != h1[i];
  printf("karatsuba results differ in %zu of %zu threads, plain schoolbook in %zu\n", diff, h0.size(), diff2);
  for (int rep = 0; rep < 3; ++rep) {
    printf("rep %d  shipped (asm) CH=1 %.2f  CH=2 %.2f  |  karatsuba CH=1 %.2f  CH=2 %.2f  |  plain schoolbook "
           "CH=1 %.2f  CH=2 %.2f  G products/s\n", rep,
           run<0, 1>(o0, blocks, iters), run<0, 2>(o0, blocks, iters / 2), run<1, 1>(o0, blocks, iters),
           run<1, 2>(o0, blocks, iters / 2), run<2, 1>(o0, blocks, iters), run<2, 2>(o0, blocks, iters / 2));
  }
  printf("%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}
