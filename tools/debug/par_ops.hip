// Debug harness: every parallel op vs its serial tower counterpart (dev tool, not product).
#include "pairing_par.hpp"
#include <cstdio>
using namespace kzgmi;
using Cv = Bls12_381;
using F = Fp<Cv::FpP>;

KZ_DEV void ld12(const F* s, Fp12<Cv>& t) {
  t.c0.c0 = {s[0], s[1]}; t.c0.c1 = {s[2], s[3]}; t.c0.c2 = {s[4], s[5]};
  t.c1.c0 = {s[6], s[7]}; t.c1.c1 = {s[8], s[9]}; t.c1.c2 = {s[10], s[11]};
}
KZ_DEV bool eq12(const Fp12<Cv>& z, const F* o) {
  const F* zz = &z.c0.c0.c0;
  for (int k = 0; k < 12; ++k) if (!(zz[k] == o[k])) return false;
  return true;
}

__device__ __noinline__ void run(ParShared<Cv>& S, int op, const F* A, const F* B, F* out) {
  ParEngine<Cv> E{S.prod, S.K};
  E.op(op, A, B, out);
}

__global__ void __launch_bounds__(PAR_THREADS) k_dbg(int* res) {
  __shared__ ParShared<Cv> S;
  par_load_consts(S);
  int tid = threadIdx.x;
  if (tid < 12) {
    F a = F::one(), b = F::one();
    a.v[0] += 7 * tid + 1; a.v[5] ^= 0x1234567u * tid; b.v[1] += 3 * tid + 5; b.v[7] ^= 0x7654321u * tid;
    S.reg[0][tid] = a; S.reg[1][tid] = b;
  }
  __syncthreads();
  F* A = S.reg[0]; F* B = S.reg[1]; F* O = S.reg[2];
  Fp12<Cv> x, y;
  int r = 0;
  // SQR
  run(S, OP_SQR, A, nullptr, O);
  if (tid == 0) { ld12(A, x); r |= eq12(f12_sqr(x), O) ? 0 : 1; }
  __syncthreads();
  run(S, OP_CYC, A, nullptr, O);
  if (tid == 0) { ld12(A, x); r |= eq12(f12_cyclo_sqr(x), O) ? 0 : 2; }
  __syncthreads();
  run(S, OP_FROB1, A, nullptr, O);
  if (tid == 0) { ld12(A, x); r |= eq12(f12_frob<Cv, 1>(x), O) ? 0 : 4; }
  __syncthreads();
  run(S, OP_FROB2, A, nullptr, O);
  if (tid == 0) { ld12(A, x); r |= eq12(f12_frob<Cv, 2>(x), O) ? 0 : 8; }
  __syncthreads();
  run(S, OP_FROB3, A, nullptr, O);
  if (tid == 0) { ld12(A, x); r |= eq12(f12_frob<Cv, 3>(x), O) ? 0 : 16; }
  __syncthreads();
  // LINE: f * line(B[0..6))
  run(S, OP_LINE, A, B, O);
  if (tid == 0) { ld12(A, x); r |= eq12(f12_mul_line(x, Fp2<Cv>{B[0], B[1]}, Fp2<Cv>{B[2], B[3]}, Fp2<Cv>{B[4], B[5]}), O) ? 0 : 32; }
  __syncthreads();
  // LL: line(A) * line(B)
  run(S, OP_LL, A, B, O);
  if (tid == 0) {
    Fp12<Cv> la; for (int k = 0; k < 12; ++k) (&la.c0.c0.c0)[k] = F::zero();
    la.c0.c0 = {A[0], A[1]}; la.c0.c1 = {A[2], A[3]}; la.c1.c1 = {A[4], A[5]};
    r |= eq12(f12_mul_line(la, Fp2<Cv>{B[0], B[1]}, Fp2<Cv>{B[2], B[3]}, Fp2<Cv>{B[4], B[5]}), O) ? 0 : 64;
  }
  __syncthreads();
  // inverse pipeline
  {
    F* r3 = S.reg[3]; F* r4 = S.reg[4]; F* r5 = S.reg[5]; F* r6 = S.reg[6];
    run(S, OP_INV_NORM, A, nullptr, r3);
    run(S, OP_INV6_T, r3, nullptr, r4);
    run(S, OP_INV6_D, r3, r4, r5);
    run(S, OP_INV2_N, r5, nullptr, S.scal);
    if (tid == 0) S.scal[1] = fp_inv(S.scal[0]);
    __syncthreads();
    run(S, OP_INV2_FIN, r5, S.scal + 1, r6);
    run(S, OP_INV6_FIN, r4, r6, r3);
    run(S, OP_INV12_FIN, A, r3, O);
    if (tid == 0) { ld12(A, x); r |= eq12(f12_inv(x), O) ? 0 : 128; }
    __syncthreads();
  }
  if (tid == 0) res[0] = r;
}

int main() {
  int* r; hipMalloc(&r, 4); hipMemset(r, 0xff, 4);
  k_dbg<<<1, PAR_THREADS>>>(r);
  hipError_t e = hipDeviceSynchronize();
  int hr; hipMemcpy(&hr, r, 4, hipMemcpyDeviceToHost);
  printf("err=%s failmask=0x%x (1 SQR,2 CYC,4 F1,8 F2,16 F3,32 LINE,64 LL,128 INV)\n", hipGetErrorString(e), hr);
  return 0;
}
