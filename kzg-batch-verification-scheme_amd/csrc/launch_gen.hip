// Synthetic-input generator launchers (compiled once per curve).  Kernels: kernels.hpp.
#include "launch.hpp"

namespace kzgmi {

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
template void Launch<C_>::g2_mul(hipStream_t, const G2Aff<C_>*, const uint8_t*, const uint32_t (&)[8], uint8_t*);
template void Launch<C_>::fpmul_probe(hipStream_t, uint32_t, uint32_t, uint32_t*);
template void Launch<C_>::gen_table(hipStream_t, Xyzz<C_>*, Affine<C_>*);
template void Launch<C_>::gen_g1(hipStream_t, const uint8_t*, uint32_t, const Affine<C_>*, uint8_t*, uint32_t*);
template void Launch<C_>::gen_tuples(hipStream_t, const Seed&, const uint32_t (&)[8], uint32_t, const Affine<C_>*,
                                     uint8_t*, uint8_t*, uint8_t*, uint8_t*);

}  // namespace kzgmi
