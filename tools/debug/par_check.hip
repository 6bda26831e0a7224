// Debug harness: one parallel-engine round vs the serial tower formula (dev tool, not product).
#include "pairing_par.hpp"
#include <cstdio>
using namespace kzgmi;
using Cv = Bls12_381;
using F = Fp<Cv::FpP>;

__device__ __noinline__ void run_mul(ParShared<Cv>& S) {
  ParEngine<Cv> E{S.prod, S.K};
  E.op(OP_MUL, S.reg[0], S.reg[1], S.reg[2]);
}

__global__ void __launch_bounds__(PAR_THREADS) k_dbg(int* res, uint32_t* dump) {
  __shared__ ParShared<Cv> S;
  par_load_consts(S);
  int tid = threadIdx.x;
  if (tid < 12) {
    F a = F::one(), b = F::one();
    a.v[0] += 7 * tid + 1; b.v[1] += 3 * tid + 5;
    S.reg[0][tid] = a; S.reg[1][tid] = b;
  }
  __syncthreads();
  run_mul(S);
  if (tid == 0) {
    Fp12<Cv> x, y;
    const F* A = S.reg[0]; const F* B = S.reg[1];
    auto ld = [](const F* s, Fp12<Cv>& t) {
      t.c0.c0 = {s[0], s[1]}; t.c0.c1 = {s[2], s[3]}; t.c0.c2 = {s[4], s[5]};
      t.c1.c0 = {s[6], s[7]}; t.c1.c1 = {s[8], s[9]}; t.c1.c2 = {s[10], s[11]};
    };
    ld(A, x); ld(B, y);
    Fp12<Cv> z = f12_mul(x, y);
    const F* zz = &z.c0.c0.c0;
    int ok = 1;
    for (int k = 0; k < 12; ++k) if (!(zz[k] == S.reg[2][k])) ok = 0;
    res[0] = ok;
    for (int k = 0; k < 12; ++k) dump[k] = S.reg[2][k].v[0];
    for (int k = 0; k < 12; ++k) dump[12 + k] = zz[k].v[0];
    dump[24] = S.prod[0].v[0]; dump[25] = S.prod[1].v[0]; dump[26] = S.K[2].v[0];
    dump[27] = OpTables<Cv>::code()[0]; dump[28] = OpTables<Cv>::get(OP_MUL).np; dump[29] = OpTables<Cv>::get(OP_MUL).P[0];
  }
}

int main() {
  int* r; uint32_t* d;
  hipMalloc(&r, 4); hipMalloc(&d, 64 * 4);
  hipMemset(r, 0xff, 4); hipMemset(d, 0, 256);
  k_dbg<<<1, PAR_THREADS>>>(r, d);
  hipError_t e = hipDeviceSynchronize();
  int hr; uint32_t hd[64];
  hipMemcpy(&hr, r, 4, hipMemcpyDeviceToHost); hipMemcpy(hd, d, 256, hipMemcpyDeviceToHost);
  printf("err=%s ok=%d\n", hipGetErrorString(e), hr);
  for (int k = 0; k < 30; ++k) printf("%08x%s", hd[k], (k % 12 == 11) ? "\n" : " ");
  printf("\n");
  return 0;
}
