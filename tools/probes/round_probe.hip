// A CYC-shaped round of the pairing interpreter (csrc/pairing_par.hpp par_round_fast<CYC>) in
// isolation: 8 waves (32 rows of 16 lanes), register file and products in LDS, every product row
// evaluates two 4-term factor forms, one lane-parallel product (lpfield.hpp lp_mul) and stores
// it; barrier; 12 output rows evaluate 8-term forms, lp_reduce, store; barrier.  No bytecode
// decode, no dispatch: what the round's arithmetic, LDS traffic and barriers cost by themselves,
// against the 4661 cycles per CYC round the interpreter spends (profiles/r05/pairing/).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include -I kzg-batch-verification-scheme_amd/csrc \
//     tools/probes/round_probe.hip -o tools/probes/round_probe
#include <hip/hip_runtime.h>
#include <cstdio>

#include "lpfield.hpp"
#include "params_gen.hpp"

using namespace kzgmi;
using Cv = Bls12_381;

constexpr int NR = 96;  // register rows
template <int NP, int NO>
__global__ void __launch_bounds__(512) k_round(int iters, uint64_t* out, int* sink) {
  __shared__ int32_t R[NR + 32][16];  // registers, then the round's products (rows NR..)
  const LpCtx<Cv> c = lp_ctx<Cv>();
  const int tid = threadIdx.x, row = tid >> 4, lane = tid & 15;
  for (int r = row; r < NR + 32; r += 32) R[r][lane] = lane < 13 ? (int32_t)((0x9E3779B9u * (r * 16 + lane + 1)) & LP_M29) : 0;
  // per-row term lists in registers (register rows + coefficients), as the CYC rows keep theirs
  int wl[4], wr[4], wo[8], cl[4], co[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    wl[k] = (row * 7 + k * 13) % 48;
    wr[k] = 48 + (row * 5 + k * 11) % 48;
    cl[k] = (k & 1) ? -1 : 1;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    wo[k] = NR + (row * 3 + k * 5) % NP;
    co[k] = (k % 3) - 1;
  }
  __syncthreads();
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (row < NP) {
      int64_t aL = 0, aR = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        lp_mad_i64(aL, R[wl[k]][lane], cl[k]);
        lp_mad_i64(aR, R[wr[k]][lane], cl[k]);
      }
      R[NR + row][lane] = lp_mul(c, lp_norm64(c, aL), lp_norm64(c, aR));
    }
    __syncthreads();
    if (row < NO) {
      int64_t a = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) lp_mad_i64(a, R[wo[k]][lane], co[k]);
      R[(row * 8) % 48][lane] = lp_reduce(c, lp_norm64(c, a));  // outputs feed the next round's forms
    }
    __syncthreads();
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[0] = t1 - t0;
  if (R[0][lane] == 0x12345) sink[0] = 1;
}

// MUL-shaped (par_round_fast<MUL>: 54 products on 32 rows, 8-term factor forms and 36-term
// output forms read from LDS term tables each round, 12 outputs)
template <int NP, int NO, int WF, int WO, int NT = 512, int NACC = 1>
__global__ void __launch_bounds__(NT) k_round_lds(int iters, uint64_t* out, int* sink) {
  constexpr int ROWS = NT / 16;
  __shared__ int32_t R[NR + 64][16];
  __shared__ uint32_t fp[NP][2 * WF];
  __shared__ uint32_t fo[NO][WO];
  const LpCtx<Cv> c = lp_ctx<Cv>();
  const int tid = threadIdx.x, row = tid >> 4, lane = tid & 15;
  for (int r = row; r < NR + 64; r += ROWS) R[r][lane] = lane < 13 ? (int32_t)((0x9E3779B9u * (r * 16 + lane + 1)) & LP_M29) : 0;
  for (int i = tid; i < NP * 2 * WF; i += NT) fp[i / (2 * WF)][i % (2 * WF)] = (uint32_t)((i * 7) % NR) | (uint32_t)(((i % 3) - 1) & 0xff) << 24;
  for (int i = tid; i < NO * WO; i += NT) fo[i / WO][i % WO] = (uint32_t)(NR + (i * 5) % NP) | (uint32_t)(((i % 3) - 1) & 0xff) << 24;
  __syncthreads();
  auto terms = [&](const uint32_t* t, int W) {
    int64_t a[NACC] = {};
#pragma unroll
    for (int q = 0; q < W; q += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(t + q);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) lp_mad_i64(a[(q + k) % NACC], R[w[k] & 0xffff][lane], (int32_t)w[k] >> 24);
    }
    int64_t r = a[0];
#pragma unroll
    for (int k = 1; k < NACC; ++k) r += a[k];
    return r;
  };
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    for (int pp = row; pp < NP; pp += ROWS)
      R[NR + pp][lane] = lp_mul(c, lp_norm64(c, terms(fp[pp], WF)), lp_norm64(c, terms(fp[pp] + WF, WF)));
    __syncthreads();
    if (row < NO) R[(row * 8) % 48][lane] = lp_reduce(c, lp_norm64(c, terms(fo[row], WO)));
    __syncthreads();
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[0] = t1 - t0;
  if (R[0][lane] == 0x12345) sink[0] = 1;
}

// A CYC chain with the output phase of squaring k run beside the products of squaring k + 1 (rows
// 32.. vs rows 0..NP-1): the factor forms of k + 1 composed through k's output forms (WF terms over
// k's products and inputs, reduced before the product), one barrier per squaring
template <int NP, int NO, int WF, int WO, int NT = 1024>
__global__ void __launch_bounds__(NT) k_round_comp(int iters, uint64_t* out, int* sink) {
  constexpr int ROWS = NT / 16;
  __shared__ int32_t R[NR + 128][16];
  __shared__ uint32_t fp[NP][2 * WF];
  __shared__ uint32_t fo[NO][WO];
  const LpCtx<Cv> c = lp_ctx<Cv>();
  const int tid = threadIdx.x, row = tid >> 4, lane = tid & 15;
  for (int r = row; r < NR + 128; r += ROWS) R[r][lane] = lane < 13 ? (int32_t)((0x9E3779B9u * (r * 16 + lane + 1)) & LP_M29) : 0;
  // factor terms: half products of the previous squaring (rows NR + buf * 64 + u), half inputs
  for (int i = tid; i < NP * 2 * WF; i += NT)
    fp[i / (2 * WF)][i % (2 * WF)] = (i & 1 ? (uint32_t)(NR + (i * 5) % NP) | 1u << 16 : (uint32_t)((i * 7) % 48)) |
                                     (uint32_t)(((i % 3) - 1) & 0xff) << 24;
  for (int i = tid; i < NO * WO; i += NT)
    fo[i / WO][i % WO] = (uint32_t)(NR + (i * 5) % NP) | 1u << 16 | (uint32_t)(((i % 3) - 1) & 0xff) << 24;
  __syncthreads();
  auto terms = [&](const uint32_t* t, int W, int pb) {
    int64_t a = 0;
#pragma unroll
    for (int q = 0; q < W; q += 4) {
      const uint4 v = *reinterpret_cast<const uint4*>(t + q);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) lp_mad_i64(a, R[(w[k] & 0xffff) + (w[k] >> 16 & 1) * pb][lane], (int32_t)w[k] >> 24);
    }
    return a;
  };
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const int pb = (it & 1) * 64, nb = 64 - pb;  // previous products at +pb, this squaring's at +nb
    if (row < NP) {
      const int32_t L = lp_reduce(c, lp_norm64(c, terms(fp[row], WF, pb)));
      const int32_t Rr = lp_reduce(c, lp_norm64(c, terms(fp[row] + WF, WF, pb)));
      R[NR + nb + row][lane] = lp_mul(c, L, Rr);
    } else if (row >= 32 && row < 32 + NO) {
      const int o = row - 32;
      R[48 + (o * 8 + (it & 1) * 4) % 48][lane] = lp_reduce(c, lp_norm64(c, terms(fo[o], WO, pb)));
    }
    __syncthreads();
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) out[0] = t1 - t0;
  if (R[0][lane] == 0x12345) sink[0] = 1;
}

template <int NP, int NO, int WF, int WO>
static double run_comp(int iters) {
  uint64_t* out;
  int* sink;
  (void)hipMalloc(&out, 8);
  (void)hipMalloc(&sink, 4);
  k_round_comp<NP, NO, WF, WO><<<1, 1024>>>(4, out, sink);
  k_round_comp<NP, NO, WF, WO><<<1, 1024>>>(iters, out, sink);
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, out, 8, hipMemcpyDeviceToHost);
  (void)hipFree(out);
  (void)hipFree(sink);
  return (double)cyc / iters;
}

template <int NP, int NO, int WF, int WO, int NT = 512, int NACC = 1>
static double run_lds(int iters) {
  uint64_t* out;
  int* sink;
  (void)hipMalloc(&out, 8);
  (void)hipMalloc(&sink, 4);
  k_round_lds<NP, NO, WF, WO, NT, NACC><<<1, NT>>>(4, out, sink);
  k_round_lds<NP, NO, WF, WO, NT, NACC><<<1, NT>>>(iters, out, sink);
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, out, 8, hipMemcpyDeviceToHost);
  (void)hipFree(out);
  (void)hipFree(sink);
  return (double)cyc / iters;
}

template <int NP, int NO>
static double run(int iters) {
  uint64_t* out;
  int* sink;
  (void)hipMalloc(&out, 8);
  (void)hipMalloc(&sink, 4);
  k_round<NP, NO><<<1, 512>>>(4, out, sink);
  k_round<NP, NO><<<1, 512>>>(iters, out, sink);
  uint64_t cyc = 0;
  (void)hipMemcpy(&cyc, out, 8, hipMemcpyDeviceToHost);
  (void)hipFree(out);
  (void)hipFree(sink);
  return (double)cyc / iters;
}

int main() {
  printf("CYC-shaped round (18 products, 12 outputs): %.0f s_memtime ticks per round\n", run<18, 12>(2000));
  printf("16 products, 12 outputs:                    %.0f\n", run<16, 12>(2000));
  printf("4 products, 4 outputs:                      %.0f\n", run<4, 4>(2000));
  printf("32 products, 12 outputs:                    %.0f\n", run<32, 12>(2000));
  printf("MUL-shaped, LDS term tables (54 products, 8-term forms, 12 outputs of 36 terms): %.0f\n",
         run_lds<54, 12, 8, 36>(1000));
  printf("CYC-shaped, LDS term tables (18 products, 4-term forms, 12 outputs of 8 terms):  %.0f\n",
         run_lds<18, 12, 4, 8>(1000));
  // round 6: 16 waves (64 rows, the shipped pairing workgroup) and independent accumulators
  for (int pass = 0; pass < 2; ++pass) {
    printf("MUL-shaped 1024 threads, 1 accumulator:  %.0f\n", run_lds<54, 12, 8, 36, 1024, 1>(1000));
    printf("MUL-shaped 1024 threads, 2 accumulators: %.0f\n", run_lds<54, 12, 8, 36, 1024, 2>(1000));
    printf("MUL-shaped 1024 threads, 4 accumulators: %.0f\n", run_lds<54, 12, 8, 36, 1024, 4>(1000));
    printf("MUL-shaped 1024 threads, outputs of 18 terms: %.0f\n", run_lds<54, 12, 8, 18, 1024, 1>(1000));
    printf("MUL-shaped 1024 threads, outputs of 4 terms:  %.0f\n", run_lds<54, 12, 8, 4, 1024, 1>(1000));
    printf("MUL-shaped 1024 threads, factor forms of 4 terms: %.0f\n", run_lds<54, 12, 4, 36, 1024, 1>(1000));
    printf("CYC-shaped LDS 1024 threads, 1 / 2 accumulators: %.0f / %.0f\n", run_lds<18, 12, 4, 8, 1024, 1>(1000),
           run_lds<18, 12, 4, 8, 1024, 2>(1000));
    printf("CYC chain, composed factor forms (16 / 24 / 32 terms), outputs beside the next products, one barrier: %.0f / %.0f / %.0f\n",
           run_comp<18, 12, 16, 8>(1000), run_comp<18, 12, 24, 8>(1000), run_comp<18, 12, 32, 8>(1000));
  }
  return 0;
}
