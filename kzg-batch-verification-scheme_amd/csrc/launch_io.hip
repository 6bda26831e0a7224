// Decoding / scalar-prep / encoding launchers (compiled once per curve).  Kernels: kernels.hpp.
#include "launch.hpp"
#include "points.hpp"
#include "fs.hpp"

namespace kzgmi {

template <class Cv>
void Launch<Cv>::convert_points(hipStream_t st, const uint8_t* bytes, uint32_t n, AF* pts, uint8_t* inf, uint32_t* err,
                                bool to29, AF* img, uint8_t* img_inf) {
  if (!n) return;
  if (to29) {
    k_convert_points<Cv, true><<<grid_for(n, 256), 256, 0, st>>>(bytes, n, pts, inf, err, img, img_inf);
    return;
  }
  k_convert_points<Cv><<<grid_for(n, 256), 256, 0, st>>>(bytes, n, pts, inf, err);
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
void Launch<Cv>::glv_split(hipStream_t st, const uint32_t* scal, uint32_t stride, uint32_t n, uint32_t* h0,
                           uint32_t* h1) {
  if (n) k_glv_split<Cv><<<grid_for(n, 256), 256, 0, st>>>(scal, stride, n, h0, h1);
}
template <class Cv>
void Launch<Cv>::endo_points(hipStream_t st, const AF* src, const uint8_t* src_inf, uint32_t n, AF* dst,
                             uint8_t* dst_inf, bool in29) {
  if (!n) return;
  if (in29) {
    k_endo_points29<Cv><<<grid_for(n, 256), 256, 0, st>>>(src, src_inf, n, dst, dst_inf);
    return;
  }
  k_endo_points<Cv><<<grid_for(n, 256), 256, 0, st>>>(src, src_inf, n, dst, dst_inf);
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
void Launch<Cv>::tsum(hipStream_t st, const void* tpart, uint32_t nblocks, uint32_t* negt) {
  k_tsum<Cv><<<1, 256, 0, st>>>((const Fp<typename Cv::FrP>*)tpart, nblocks, negt);
}
template <class Cv>
void Launch<Cv>::scalar_prep(hipStream_t st, const Seed& seed, const uint32_t* seed_dev, uint64_t index_offset,
                             const uint8_t* zs,
                             const uint8_t* ys, uint32_t n, uint32_t* r_out, uint32_t* s_out, void* tpart,
                             uint32_t* negt, uint32_t* err, uint32_t* h0, uint32_t* h1) {
  using FrF = Fp<typename Cv::FrP>;
  const uint32_t nblk = grid_for(n, PREP_BLOCK);
  k_scalar_prep<Cv><<<nblk, PREP_BLOCK, 0, st>>>(seed, seed_dev, index_offset, zs, ys, n, r_out, s_out, (FrF*)tpart, err,
                                                 h0, h1);
  k_tsum<Cv><<<1, 256, 0, st>>>((const FrF*)tpart, nblk, negt);
}
template <class Cv>
void Launch<Cv>::fs_leaves(hipStream_t st, const uint8_t* dC, const uint8_t* dpi, const uint8_t* dz, const uint8_t* dy,
                           uint32_t n, uint64_t offset, bool compressed, uint32_t* leaves) {
  if (n) k_fs_leaves<Cv><<<grid_for(n, 256), 256, 0, st>>>(dC, dpi, dz, dy, n, offset, compressed ? 1 : 0, leaves);
}
template <class Cv>
const uint32_t* Launch<Cv>::fs_reduce(hipStream_t st, const uint32_t* in, uint32_t count, uint32_t target,
                                      uint32_t* tmp) {
  // ping-pong inside tmp (3 count / 4 nodes): pass outputs alternate between
  // [0, count/2) and [count/2, 3 count/4)
  uint32_t* bufs[2] = {tmp, tmp + 8 * (size_t)(count / 2)};
  int which = 0;
  while (count > target) {
    uint32_t group = count / target < 512 ? count / target : 512;
    uint32_t out_n = count / group;
    uint32_t* out = bufs[which];
    k_fs_merkle<<<out_n, 256, 0, st>>>(in, group, out);
    in = out;
    count = out_n;
    which ^= 1;
  }
  return in;
}
template <class Cv>
void Launch<Cv>::fs_pad(hipStream_t st, uint32_t* digests, uint32_t nchunks, uint32_t p2) {
  if (p2 > nchunks) k_fs_pad<<<grid_for(p2 - nchunks, 256), 256, 0, st>>>(digests, nchunks, p2);
}
template <class Cv>
void Launch<Cv>::fs_challenge(hipStream_t st, const uint32_t* root, uint64_t n, void* pow, uint32_t* chal_out) {
  k_fs_challenge<Cv><<<1, 64, 0, st>>>(root, n, (Fp<typename Cv::FrP>*)pow, chal_out);
}
template <class Cv>
void Launch<Cv>::pow_table(hipStream_t st, const Seed& r_be, void* pow, uint32_t* err) {
  k_pow_table<Cv><<<1, 64, 0, st>>>(r_be, (Fp<typename Cv::FrP>*)pow, err);
}
template <class Cv>
void Launch<Cv>::scalar_prep_pow(hipStream_t st, const void* pow, uint64_t index_offset, const uint8_t* zs,
                                 const uint8_t* ys, uint32_t n, uint32_t* r_out, uint32_t* s_out, void* tpart,
                                 uint32_t* negt, uint32_t* err) {
  using FrF = Fp<typename Cv::FrP>;
  const uint32_t nblk = grid_for(n, PREP_BLOCK);
  k_scalar_prep_pow<Cv, PREP_BLOCK><<<nblk, PREP_BLOCK, 0, st>>>((const FrF*)pow, index_offset, zs, ys, n, r_out,
                                                                  s_out, (FrF*)tpart, err);
  k_tsum<Cv><<<1, 256, 0, st>>>((const FrF*)tpart, nblk, negt);
}
template <class Cv>
void Launch<Cv>::encode_points(hipStream_t st, const XY* res, uint32_t count, uint8_t* out) {
  if (count) k_encode_points<Cv><<<count, 64, 0, st>>>(res, count, out);
}
template <class Cv>
void Launch<Cv>::sum_partials(hipStream_t st, const XY* parts, uint32_t nparts, uint32_t stride, uint32_t nout, XY* out,
                               uint32_t* err) {
  k_sum_partials<Cv><<<1, 64, 0, st>>>(parts, nparts, stride, nout, out, err);
}
template <class Cv>
void Launch<Cv>::partial_out(hipStream_t st, const XY* res, uint32_t count, const uint32_t* err, XY* out) {
  k_partial_out<Cv><<<1, 64, 0, st>>>(res, count, err, out);
}

using C_ = KZ_CURVE_T;
template void Launch<C_>::convert_points(hipStream_t, const uint8_t*, uint32_t, Affine<C_>*, uint8_t*, uint32_t*, bool, Affine<C_>*,
                                         uint8_t*);
template void Launch<C_>::set_generator(hipStream_t, Affine<C_>*, uint8_t*);
template void Launch<C_>::decompress_points(hipStream_t, const uint8_t*, uint32_t, Affine<C_>*, uint8_t*, uint32_t*);
template void Launch<C_>::compress_points(hipStream_t, const uint8_t*, uint32_t, uint8_t*);
template void Launch<C_>::subgroup_check(hipStream_t, const Affine<C_>*, const uint8_t*, uint32_t, uint32_t*);
template void Launch<C_>::convert_scalars(hipStream_t, const uint8_t*, uint32_t, uint32_t*, uint32_t*);
template void Launch<C_>::convert_g2(hipStream_t, const uint8_t*, uint32_t, G2Aff<C_>*, uint8_t*, uint32_t*);
template size_t Launch<C_>::tpart_bytes(uint32_t);
template void Launch<C_>::tsum(hipStream_t, const void*, uint32_t, uint32_t*);
template void Launch<C_>::scalar_prep(hipStream_t, const Seed&, const uint32_t*, uint64_t, const uint8_t*, const uint8_t*, uint32_t,
                                      uint32_t*, uint32_t*, void*, uint32_t*, uint32_t*, uint32_t*, uint32_t*);
template void Launch<C_>::fs_leaves(hipStream_t, const uint8_t*, const uint8_t*, const uint8_t*, const uint8_t*,
                                     uint32_t, uint64_t, bool, uint32_t*);
template const uint32_t* Launch<C_>::fs_reduce(hipStream_t, const uint32_t*, uint32_t, uint32_t, uint32_t*);
template void Launch<C_>::fs_pad(hipStream_t, uint32_t*, uint32_t, uint32_t);
template void Launch<C_>::fs_challenge(hipStream_t, const uint32_t*, uint64_t, void*, uint32_t*);
template void Launch<C_>::pow_table(hipStream_t, const Seed&, void*, uint32_t*);
template void Launch<C_>::scalar_prep_pow(hipStream_t, const void*, uint64_t, const uint8_t*, const uint8_t*, uint32_t,
                                          uint32_t*, uint32_t*, void*, uint32_t*, uint32_t*);
template void Launch<C_>::encode_points(hipStream_t, const Xyzz<C_>*, uint32_t, uint8_t*);
template void Launch<C_>::glv_split(hipStream_t, const uint32_t*, uint32_t, uint32_t, uint32_t*, uint32_t*);
template void Launch<C_>::endo_points(hipStream_t, const Affine<C_>*, const uint8_t*, uint32_t, Affine<C_>*, uint8_t*, bool);
template void Launch<C_>::sum_partials(hipStream_t, const Xyzz<C_>*, uint32_t, uint32_t, uint32_t, Xyzz<C_>*, uint32_t*);
template void Launch<C_>::partial_out(hipStream_t, const Xyzz<C_>*, uint32_t, const uint32_t*, Xyzz<C_>*);

}  // namespace kzgmi
