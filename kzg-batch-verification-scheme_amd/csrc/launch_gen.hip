// Synthetic-input generator launchers (compiled once per curve).  Kernels: kernels.hpp.
#include "launch.hpp"

namespace kzgmi {

// prover commit key: out_i = 2^16 in_i as an affine point; one thread
// per point (one-time precomputation at key load: 16 doublings + one inversion per point)
template <class Cv>
__global__ void __launch_bounds__(256) k_shift_points(const Affine<Cv>* __restrict__ in,
                                                      const uint8_t* __restrict__ inf_in, uint32_t n,
                                                      Affine<Cv>* __restrict__ out, uint8_t* __restrict__ inf_out) {
  using F = Fp<typename Cv::FpP>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Affine<Cv> a;
  bool finite = false;
  if (!inf_in[i]) {
    Xyzz<Cv> acc = xyzz_from_affine(in[i]);
    for (int k = 0; k < WBITS; ++k) acc = xyzz_dbl_c(acc);
    finite = xyzz_to_affine(acc, a);
  }
  if (!finite) { a.x = F::zero(); a.y = F::zero(); }
  out[i] = a;
  inf_out[i] = finite ? 0 : 1;
}

template <class Cv>
void Launch<Cv>::shift_points(hipStream_t st, const AF* in, const uint8_t* inf_in, uint32_t n, AF* out,
                              uint8_t* inf_out) {
  if (n) k_shift_points<Cv><<<grid_for(n, 256), 256, 0, st>>>(in, inf_in, n, out, inf_out);
}

template <class Cv>
void Launch<Cv>::gen_table(hipStream_t st, XY* base, AF* table) {
  k_gen_table_base<Cv><<<1, 64, 0, st>>>(base);
  k_gen_table<Cv><<<32, 256, 0, st>>>(base, table);
}
template <class Cv>
void Launch<Cv>::gen_g1(hipStream_t st, const uint8_t* scalars, uint32_t n, const AF* table, uint8_t* out, uint32_t* err) {
  if (n) k_gen_g1<Cv><<<grid_for(n, 256), 256, 0, st>>>(scalars, n, table, out, err);
}
template <class Cv>
void Launch<Cv>::gen_tuples(hipStream_t st, const Seed& seed, const uint32_t (&tau_le)[8], uint32_t n, const AF* table,
                            uint8_t* cm, uint8_t* zs, uint8_t* ys, uint8_t* pf) {
  Fp<typename Cv::FrP> tau;
  for (int k = 0; k < 8; ++k) tau.v[k] = tau_le[k];
  if (n) k_gen_tuples<Cv><<<grid_for(n, 256), 256, 0, st>>>(seed, tau, n, table, cm, zs, ys, pf);
}

template <class Cv>
void Launch<Cv>::g2_mul(hipStream_t st, const G2Aff<Cv>* q, const uint8_t* q_inf, const uint32_t (&k_le)[8], uint8_t* out) {
  Fp<typename Cv::FrP> k;
  for (int j = 0; j < 8; ++j) k.v[j] = k_le[j];
  k_g2_mul<Cv><<<1, 64, 0, st>>>(q, q_inf, k, out);
}
template <class Cv>
void Launch<Cv>::fpmul_probe(hipStream_t st, uint32_t blocks, uint32_t iters, uint32_t* out) {
  k_fpmul_probe<Cv><<<blocks, 256, 0, st>>>(iters, out);
}

using C_ = KZ_CURVE_T;
template void Launch<KZ_CURVE_T>::shift_points(hipStream_t, const Affine<KZ_CURVE_T>*, const uint8_t*, uint32_t,
                                               Affine<KZ_CURVE_T>*, uint8_t*);
template void Launch<C_>::g2_mul(hipStream_t, const G2Aff<C_>*, const uint8_t*, const uint32_t (&)[8], uint8_t*);
template void Launch<C_>::fpmul_probe(hipStream_t, uint32_t, uint32_t, uint32_t*);
template void Launch<C_>::gen_table(hipStream_t, Xyzz<C_>*, Affine<C_>*);
template void Launch<C_>::gen_g1(hipStream_t, const uint8_t*, uint32_t, const Affine<C_>*, uint8_t*, uint32_t*);
template void Launch<C_>::gen_tuples(hipStream_t, const Seed&, const uint32_t (&)[8], uint32_t, const Affine<C_>*,
                                     uint8_t*, uint8_t*, uint8_t*, uint8_t*);

}  // namespace kzgmi
