// MSM launchers (compiled once per curve, -DKZ_CURVE=0/1).  See msm.hpp for the kernels.
#include "launch.hpp"

namespace kzgmi {

template <class Cv>
void Launch<Cv>::digits(hipStream_t st, bool scatter, const TermList& tl, const uint8_t* inf, uint32_t* cnt_or_cursor,
                        uint32_t* sval, uint32_t* skey) {
  if (!tl.total) return;
  if (scatter)
    k_digits<true><<<grid_for(tl.total, 256), 256, 0, st>>>(tl, inf, cnt_or_cursor, sval, skey);
  else
    k_digits<false><<<grid_for(tl.total, 256), 256, 0, st>>>(tl, inf, cnt_or_cursor, nullptr, nullptr);
}

template <class Cv>
void Launch<Cv>::scan(hipStream_t st, const uint32_t* cnt, uint32_t nb, uint32_t* off, uint32_t* blk, uint32_t* total,
                      uint32_t* cursor) {
  const uint32_t nscan = nb / (SCAN_BLOCK * SCAN_ITEMS);
  k_scan_blocks<<<nscan, SCAN_BLOCK, 0, st>>>(cnt, nb, off, blk);
  k_scan_totals<<<1, 1024, 0, st>>>(blk, nscan, total);
  k_scan_add<<<grid_for(nb, 256), 256, 0, st>>>(off, nb, blk, cursor);
}

template <class Cv>
void Launch<Cv>::accumulate(hipStream_t st, size_t nchunks, const uint32_t* total, const uint32_t* sval,
                            const uint32_t* skey, const uint32_t* off, const uint32_t* cnt, const AF* pts, XY* buckets,
                            XY* pfirst, XY* plast) {
  k_accumulate<Cv><<<grid_for(nchunks, 256), 256, 0, st>>>(total, sval, skey, off, cnt, pts, buckets, pfirst, plast);
  k_fixup<Cv><<<grid_for(nchunks, 256), 256, 0, st>>>(total, skey, off, cnt, pfirst, plast, buckets);
}

template <class Cv>
void Launch<Cv>::reduce(hipStream_t st, uint32_t nsets, const uint32_t* cnt, const XY* buckets, XY* R, XY* U,
                        XY* scratch, XY* winsum) {
  const uint32_t nseg = nsets * (NBUCKETS / SEG);
  k_reduce_segments<Cv><<<grid_for(nseg, 256), 256, 0, st>>>(nseg, cnt, buckets, R, U);
  k_reduce_finish<Cv><<<nsets, 256, 0, st>>>(R, U, scratch, winsum);
}

template <class Cv>
void Launch<Cv>::window_combine(hipStream_t st, const MsmWindows& mw, const XY* winsum, XY* res) {
  k_window_combine<Cv><<<1, 64, 0, st>>>(mw, winsum, res);
}

template void Launch<KZ_CURVE_T>::digits(hipStream_t, bool, const TermList&, const uint8_t*, uint32_t*, uint32_t*, uint32_t*);
template void Launch<KZ_CURVE_T>::scan(hipStream_t, const uint32_t*, uint32_t, uint32_t*, uint32_t*, uint32_t*, uint32_t*);
template void Launch<KZ_CURVE_T>::accumulate(hipStream_t, size_t, const uint32_t*, const uint32_t*, const uint32_t*,
                                             const uint32_t*, const uint32_t*, const Affine<KZ_CURVE_T>*,
                                             Xyzz<KZ_CURVE_T>*, Xyzz<KZ_CURVE_T>*, Xyzz<KZ_CURVE_T>*);
template void Launch<KZ_CURVE_T>::reduce(hipStream_t, uint32_t, const uint32_t*, const Xyzz<KZ_CURVE_T>*,
                                         Xyzz<KZ_CURVE_T>*, Xyzz<KZ_CURVE_T>*, Xyzz<KZ_CURVE_T>*, Xyzz<KZ_CURVE_T>*);
template void Launch<KZ_CURVE_T>::window_combine(hipStream_t, const MsmWindows&, const Xyzz<KZ_CURVE_T>*,
                                                 Xyzz<KZ_CURVE_T>*);

}  // namespace kzgmi
