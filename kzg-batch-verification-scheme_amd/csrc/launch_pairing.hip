// Pairing launchers (compiled once per curve).  Kernels: pairing.hpp / kernels.hpp.
#include "launch.hpp"
#include "pairing_par.hpp"

namespace kzgmi {

template <class Cv>
int Launch<Cv>::num_lines() { return kzgmi::num_lines<Cv>(); }
template <class Cv>
void Launch<Cv>::precompute_lines(hipStream_t st, const G2Aff<Cv>* q, Line<Cv>* lines) {
  k_precompute_lines<Cv><<<1, 64, 0, st>>>(q, lines);
}
template <class Cv>
void Launch<Cv>::pairing_check(hipStream_t st, const XY* res, const Line<Cv>* lines, const uint8_t* q_inf, int* ok) {
  k_pairing_check_par<Cv><<<1, PAR_THREADS, 0, st>>>(res, lines, q_inf, ok);
}
template <class Cv>
void Launch<Cv>::pairing_one(hipStream_t st, const AF* p, const uint8_t* p_inf, const Line<Cv>* lines,
                             const uint8_t* q_inf, uint8_t* out) {
  k_pairing_one_par<Cv><<<1, PAR_THREADS, 0, st>>>(p, p_inf, lines, q_inf, out);
}

using C_ = KZ_CURVE_T;
template int Launch<C_>::num_lines();
template void Launch<C_>::precompute_lines(hipStream_t, const G2Aff<C_>*, Line<C_>*);
template void Launch<C_>::pairing_check(hipStream_t, const Xyzz<C_>*, const Line<C_>*, const uint8_t*, int*);
template void Launch<C_>::pairing_one(hipStream_t, const Affine<C_>*, const uint8_t*, const Line<C_>*, const uint8_t*,
                                      uint8_t*);

}  // namespace kzgmi
