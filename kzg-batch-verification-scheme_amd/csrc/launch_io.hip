// Decoding / scalar-prep / encoding launchers (compiled once per curve).  Kernels: kernels.hpp.
#include "launch.hpp"
#include "points.hpp"

namespace kzgmi {

template <class Cv>
void Launch<Cv>::convert_points(hipStream_t st, const uint8_t* bytes, uint32_t n, AF* pts, uint8_t* inf, uint32_t* err) {
  if (n) k_convert_points<Cv><<<grid_for(n, 256), 256, 0, st>>>(bytes, n, pts, inf, err);
}
template <class Cv>
void Launch<Cv>::set_generator(hipStream_t st, AF* pt, uint8_t* inf) {
  k_set_generator<Cv><<<1, 1, 0, st>>>(pt, inf);
}
template <class Cv>
void Launch<Cv>::decompress_points(hipStream_t st, const uint8_t* bytes, uint32_t n, AF* pts, uint8_t* inf,
                                   uint32_t* err) {
  if (n) k_decompress_points<Cv><<<grid_for(n, 256), 256, 0, st>>>(bytes, n, pts, inf, err);
}
template <class Cv>
void Launch<Cv>::compress_points(hipStream_t st, const uint8_t* in, uint32_t n, uint8_t* out) {
  if (n) k_compress_points<Cv><<<grid_for(n, 256), 256, 0, st>>>(in, n, out);
}
template <class Cv>
void Launch<Cv>::subgroup_check(hipStream_t st, const AF* pts, const uint8_t* inf, uint32_t n, uint32_t* err) {
  if constexpr (Cv::ID == 0) {  // BN254: cofactor 1, every curve point is in G1
    if (n) k_subgroup_check<Cv><<<grid_for(n, 256), 256, 0, st>>>(pts, inf, n, err);
  }
}
template <class Cv>
void Launch<Cv>::convert_scalars(hipStream_t st, const uint8_t* bytes, uint32_t n, uint32_t* out, uint32_t* err) {
  if (n) k_convert_scalars<Cv><<<grid_for(n, 256), 256, 0, st>>>(bytes, n, out, err);
}
template <class Cv>
void Launch<Cv>::convert_g2(hipStream_t st, const uint8_t* bytes, uint32_t n, G2Aff<Cv>* out, uint8_t* inf,
                            uint32_t* err) {
  k_convert_g2<Cv><<<1, 64, 0, st>>>(bytes, n, out, inf, err);
}
template <class Cv>
size_t Launch<Cv>::tpart_bytes(uint32_t n) {
  return (size_t)grid_for(n, PREP_BLOCK) * sizeof(Fp<typename Cv::FrP>);
}
template <class Cv>
void Launch<Cv>::scalar_prep(hipStream_t st, const Seed& seed, uint64_t index_offset, const uint8_t* zs,
                             const uint8_t* ys, uint32_t n, uint32_t* r_out, uint32_t* s_out, void* tpart,
                             uint32_t* negt, uint32_t* err) {
  using FrF = Fp<typename Cv::FrP>;
  const uint32_t nblk = grid_for(n, PREP_BLOCK);
  k_scalar_prep<Cv><<<nblk, PREP_BLOCK, 0, st>>>(seed, index_offset, zs, ys, n, r_out, s_out, (FrF*)tpart, err);
  k_tsum<Cv><<<1, 256, 0, st>>>((const FrF*)tpart, nblk, negt);
}
template <class Cv>
void Launch<Cv>::encode_points(hipStream_t st, const XY* res, uint32_t count, uint8_t* out) {
  k_encode_points<Cv><<<grid_for(count, 64), 64, 0, st>>>(res, count, out);
}
template <class Cv>
void Launch<Cv>::sum_partials(hipStream_t st, const XY* parts, uint32_t nparts, uint32_t stride, uint32_t nout, XY* out) {
  k_sum_partials<Cv><<<1, 64, 0, st>>>(parts, nparts, stride, nout, out);
}

using C_ = KZ_CURVE_T;
template void Launch<C_>::convert_points(hipStream_t, const uint8_t*, uint32_t, Affine<C_>*, uint8_t*, uint32_t*);
template void Launch<C_>::set_generator(hipStream_t, Affine<C_>*, uint8_t*);
template void Launch<C_>::decompress_points(hipStream_t, const uint8_t*, uint32_t, Affine<C_>*, uint8_t*, uint32_t*);
template void Launch<C_>::compress_points(hipStream_t, const uint8_t*, uint32_t, uint8_t*);
template void Launch<C_>::subgroup_check(hipStream_t, const Affine<C_>*, const uint8_t*, uint32_t, uint32_t*);
template void Launch<C_>::convert_scalars(hipStream_t, const uint8_t*, uint32_t, uint32_t*, uint32_t*);
template void Launch<C_>::convert_g2(hipStream_t, const uint8_t*, uint32_t, G2Aff<C_>*, uint8_t*, uint32_t*);
template size_t Launch<C_>::tpart_bytes(uint32_t);
template void Launch<C_>::scalar_prep(hipStream_t, const Seed&, uint64_t, const uint8_t*, const uint8_t*, uint32_t,
                                      uint32_t*, uint32_t*, void*, uint32_t*, uint32_t*);
template void Launch<C_>::encode_points(hipStream_t, const Xyzz<C_>*, uint32_t, uint8_t*);
template void Launch<C_>::sum_partials(hipStream_t, const Xyzz<C_>*, uint32_t, uint32_t, uint32_t, Xyzz<C_>*);

}  // namespace kzgmi
