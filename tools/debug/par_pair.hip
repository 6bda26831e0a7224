// Debug harness: parallel pairing vs serial pairing with checkpoints (dev tool, not product).
#include "pairing_par.hpp"
#include <cstdio>
using namespace kzgmi;
using Cv = Bls12_381;
using F = Fp<Cv::FpP>;
constexpr int NL = num_lines<Cv>();

__global__ void k_setup(G2Aff<Cv>* q) {
  // G2 generator (Montgomery) from raw constants
  const uint32_t xs[2][12] = {{0xc121bdb8u,0xd48056c8u,0xa805bbefu,0x0bac0326u,0x7ae3d177u,0xb4510b64u,0xfa403b02u,0xc6e47ad4u,0x2dc51051u,0x26080527u,0xf08f0a91u,0x024aa2b2u},
                              {0x5d042b7eu,0xe5ac7d05u,0x13945d57u,0x334cf112u,0xdc7f5049u,0xb5da61bbu,0x9920b61au,0x596bd0d0u,0x88274f65u,0x7dacd3a0u,0x52719f60u,0x13e02b60u}};
  const uint32_t ys[2][12] = {{0x08b82801u,0xe1935486u,0x3baca289u,0x923ac9ccu,0x5160d12cu,0x6d429a69u,0x8cbdd3a7u,0xadfd9baau,0xda2e351au,0x8cc9cdc6u,0x727d6e11u,0x0ce5d527u},
                              {0xf05f79beu,0xaaa9075fu,0x5cec1da1u,0x3f370d27u,0x572e99abu,0x267492abu,0x85a763afu,0xcb3e287eu,0x2bc28b99u,0x32acd2b0u,0x2ea734ccu,0x0606c4a0u}};
  F a, b, c, d;
  for (int i = 0; i < 12; ++i) { a.v[i] = xs[0][i]; b.v[i] = xs[1][i]; c.v[i] = ys[0][i]; d.v[i] = ys[1][i]; }
  q[0] = {{fp_to_mont(a), fp_to_mont(b)}, {fp_to_mont(c), fp_to_mont(d)}};
  q[1] = q[0];
}

__global__ void k_serial(const Line<Cv>* lines, F* out) {
  Affine<Cv> p = {F::from_const(Cv::K::G1X_M), F::from_const(Cv::K::G1Y_M)};
  Xyzz<Cv> X = xyzz_from_affine(p);
  Homog<Cv> H[2] = {homog_from_xyzz(X, false), homog_from_xyzz(X, false)};
  bool skip[2] = {false, true};
  Fp12<Cv> f = miller2(lines, H, skip);
  const F* ff = &f.c0.c0.c0;
  for (int k = 0; k < 12; ++k) out[k] = ff[k];
  // easy part
  Fp12<Cv> g = f12_mul(f12_conj(f), f12_inv(f));
  g = f12_mul(f12_frob<Cv, 2>(g), g);
  const F* gg = &g.c0.c0.c0;
  for (int k = 0; k < 12; ++k) out[12 + k] = gg[k];
  Fp12<Cv> e = final_exp(f);
  const F* ee = &e.c0.c0.c0;
  for (int k = 0; k < 12; ++k) out[24 + k] = ee[k];
}

__global__ void __launch_bounds__(PAR_THREADS) k_par(const Line<Cv>* lines, F* out) {
  __shared__ ParShared<Cv> S;
  par_load_consts(S);
  int tid = threadIdx.x;
  if (tid < 2) { S.P[tid][0] = F::from_const(Cv::K::G1X_M); S.P[tid][1] = F::from_const(Cv::K::G1Y_M); S.P[tid][2] = F::one(); }
  __syncthreads();
  bool skip[2] = {false, true};
  par_pairing_is_one(S, lines, skip, out);
  if (tid < 12) out[24 + tid] = S.reg[7][tid];
}

int main() {
  G2Aff<Cv>* q; Line<Cv>* lines; F *o1, *o2;
  hipMalloc(&q, 2 * sizeof(G2Aff<Cv>)); hipMalloc(&lines, 2 * NL * sizeof(Line<Cv>));
  hipMalloc(&o1, 64 * sizeof(F)); hipMalloc(&o2, 64 * sizeof(F));
  hipMemset(o1, 0, 64 * sizeof(F)); hipMemset(o2, 0, 64 * sizeof(F));
  k_setup<<<1, 1>>>(q);
  k_precompute_lines<Cv><<<1, 64>>>(q, lines);
  k_serial<<<1, 1>>>(lines, o1);
  k_par<<<1, PAR_THREADS>>>(lines, o2);
  hipError_t e = hipDeviceSynchronize();
  F h1[64], h2[64];
  hipMemcpy(h1, o1, 64 * sizeof(F), hipMemcpyDeviceToHost); hipMemcpy(h2, o2, 64 * sizeof(F), hipMemcpyDeviceToHost);
  printf("err=%s\n", hipGetErrorString(e));
  const char* names[3] = {"miller", "easy", "final"};
  for (int s = 0; s < 3; ++s) {
    int same = 1;
    for (int k = 0; k < 12; ++k) for (int j = 0; j < 12; ++j) if (h1[12 * s + k].v[j] != h2[12 * s + k].v[j]) same = 0;
    printf("%s: %s   serial[0]=%08x par[0]=%08x\n", names[s], same ? "MATCH" : "DIFF", h1[12 * s].v[0], h2[12 * s].v[0]);
  }
  printf("E[0][0][*].v0: "); for (int k = 0; k < 6; ++k) printf("%08x ", h2[36 + k].v[0]); printf("\n");
  return 0;
}
