// MSM launchers (compiled once per curve, -DKZ_CURVE=0/1).  See msm.hpp for the kernels.
#include "launch.hpp"

namespace kzgmi {

// the window widths a call may use (msm.hpp Win): c = 16, and c = 13 for small calls
template <class F>
void with_wbits(int wbits, F&& f) {
  if (wbits == 13) f(std::integral_constant<int, 13>{});
  else f(std::integral_constant<int, WBITS>{});
}

template <class Cv>
void Launch<Cv>::sort(hipStream_t st, const TermList& tl, uint32_t nsets, const uint8_t* inf, uint32_t* digits,
                      uint32_t* coarse, uint64_t* ent, size_t emax, int sort_flags, uint32_t* off, uint32_t* cnt, uint32_t* total, uint32_t* sval,
                      uint32_t* skey, int wbits) {
  const bool force_split = (sort_flags & SORT_SPLIT) != 0;
  with_wbits(wbits, [&](auto wb) {
    constexpr int WB = decltype(wb)::value;
    const uint32_t nbins = nsets * Win<WB>::BINS;
    SetShift ss;
    // more sets than the table holds: every set at the full 128-bucket bins (always correct;
    // SORT_FULL_BINS forces it, tests)
    const bool table = !(sort_flags & SORT_FULL_BINS) && set_shifts_host<WB>(tl, nsets, ss);
    uint32_t* ccnt = coarse;
    uint32_t* coff = coarse + nbins;
    uint32_t* ccur = coarse + 2 * nbins;
    (void)hipMemsetAsync(ccnt, 0, (size_t)nbins * 4, st);
    const uint32_t tiles = num_tiles_host(tl);
    bool uniform = true;
    for (uint32_t s = 0; table && s < nsets; ++s) uniform &= ss.s[s] == COARSE_SHIFT;
    if (tl.total && uniform) k_digits_count<WB, true><<<num_digit_groups_host(tl), 256, 0, st>>>(tl, ss, inf, digits, ccnt);
    else if (tl.total) k_digits_count<WB, false><<<num_digit_groups_host(tl), 256, 0, st>>>(tl, ss, inf, digits, ccnt);
    k_bin_scan<<<1, 1024, 0, st>>>(ccnt, nbins, coff, ccur, total);
    // coarse-pass entries (msm.hpp EntPacked / EntSplit): packed 4 B when every sorted value (point
    // index << 1 | sign) fits CV_BITS, else 4 B values + 1 B fine indices (ent holds emax x 8 B)
    uint64_t npts = 0;
    for (uint32_t k = 0; k < tl.nclass; ++k)
      if (tl.c[k].count) npts = std::max<uint64_t>(npts, (uint64_t)tl.c[k].pt_base + tl.c[k].count);
    auto scatter_and_sort = [&](auto e, auto uni) {
      using E = decltype(e);
      constexpr bool U = decltype(uni)::value;
      if (tiles) k_bin_scatter<E, WB, U><<<tiles, 256, 0, st>>>(tl, ss, digits, ccur, e);
      k_fine_sort<E, WB, U><<<nbins, 256, 0, st>>>(coff, ccnt, e, off, cnt, sval, skey, ss);
    };
    auto with_uniform = [&](auto e) {
      if (uniform) scatter_and_sort(e, std::true_type{});
      else scatter_and_sort(e, std::false_type{});
    };
    if (!force_split && 2 * npts < (1ull << CV_BITS)) with_uniform(EntPacked{reinterpret_cast<uint32_t*>(ent)});
    else with_uniform(EntSplit{reinterpret_cast<uint32_t*>(ent), reinterpret_cast<uint8_t*>(ent) + 4 * emax});
  });
}

template <class Cv>
void Launch<Cv>::accumulate(hipStream_t st, size_t nchunks, const uint32_t* total, const uint32_t* sval,
                            const uint32_t* skey, const uint32_t* off, const uint32_t* cnt, const AF* pts,
                            uint32_t* acc29, uint32_t nb, size_t acc_threads, uint32_t* next_chunk,
                            uint32_t* crowd, const uint32_t* lo, hipStream_t fix_st) {
  // nchunks threads (rounded up to whole 256-thread blocks); both kernels derive the chunk
  // length from the same grid -- except the radix-29 work-queue form: acc_threads (< nchunks,
  // whole blocks) threads take the nchunks chunks from the counter next_chunk, zeroed here
  const unsigned blocks = grid_for(nchunks, 256);
  if (next_chunk && acc_threads && acc_threads < nchunks) {
    (void)hipMemsetAsync(next_chunk, 0, 4, st);
    k_accumulate<Cv><<<grid_for(acc_threads, 256), 256, 0, st>>>(total, sval, skey, off, cnt, pts, acc29, nb,
                                                                  (uint32_t)(blocks * 256u), next_chunk, lo, crowd);
  } else {
    k_accumulate<Cv><<<blocks, 256, 0, st>>>(total, sval, skey, off, cnt, pts, acc29, nb, 0u, nullptr, lo, crowd);
  }
  if (fix_st) fixup(fix_st, nchunks, total, skey, off, cnt, acc29, nb, crowd, lo);
}

template <class Cv>
void Launch<Cv>::fixup(hipStream_t st, size_t nchunks, const uint32_t* total, const uint32_t* skey, const uint32_t* off,
                       const uint32_t* cnt, uint32_t* acc29, uint32_t nb, uint32_t* crowd, const uint32_t* lo) {
  const unsigned blocks = grid_for(nchunks, 256);
  // crowd: zeroed by the accumulation launch this one follows (k_accumulate)
  k_fixup<Cv><<<blocks, 256, 0, st>>>(total, skey, off, cnt, acc29, nb, crowd, lo);
  // crowded buckets: at most one per FIX_LP_FROM + 1 chunks; 1024 waves stride over the list
  k_fixup_crowded<Cv><<<256, 256, 0, st>>>(crowd, acc29, nb, blocks * 256u);
}

template <class Cv>
void Launch<Cv>::pts_to29(hipStream_t st, AF* pts, uint32_t n) {
  if (n) k_pts_to29<Cv><<<grid_for(n, 256), 256, 0, st>>>(pts, n);
}

template <class Cv>
void Launch<Cv>::reduce(hipStream_t st, uint32_t nsets, const uint32_t* cnt, const uint32_t* acc29, XY* R, XY* U,
                        XY* scratch, XY* winsum, int wbits, bool low_prio, int seg4_waves, int simds) {
  with_wbits(wbits, [&](auto wb) {
    constexpr int WB = decltype(wb)::value;
    const uint32_t nseg = nsets * Win<WB>::NSEG;
    // 4 threads per segment while that grid stays within seg4_waves waves per SIMD (few sets: the
    // segments' serial chains set the time); 2 otherwise (k_reduce_segments4 above)
    const bool four = seg4_waves > 0 && (size_t)nseg * 4 <= (size_t)seg4_waves * simds * 64;
    auto go = [&](auto lp) {
      constexpr bool LP = decltype(lp)::value;
      if (four) k_reduce_segments4<Cv, LP><<<grid_for(4 * (size_t)nseg, 256), 256, 0, st>>>(nseg, cnt, acc29, R, U);
      else k_reduce_segments<Cv, LP><<<grid_for(2 * (size_t)nseg, 256), 256, 0, st>>>(nseg, cnt, acc29, R, U);
      // scratch: nsets * RB_PARTS partial sums
      k_reduce_bits<Cv, WB, LP><<<nsets * Win<WB>::RB_PARTS, 256, 0, st>>>(R, U, scratch);
      if (four) k_reduce_bits_finish<Cv, WB, LP, 4><<<nsets, 64, 0, st>>>(scratch, winsum);
      else k_reduce_bits_finish<Cv, WB, LP, 2><<<nsets, 64, 0, st>>>(scratch, winsum);
    };
    if (low_prio) go(std::true_type{});
    else go(std::false_type{});
  });
}

template <class Cv>
void Launch<Cv>::merge_buckets(hipStream_t st, uint32_t nb, uint32_t* acc29, uint32_t* cnt, const uint32_t* acc29b,
                               const uint32_t* cntb) {
  if (nb) k_merge_buckets<Cv><<<(nb + 255) / 256, 256, 0, st>>>(nb, acc29, cnt, acc29b, cntb);
}

template <class Cv>
void Launch<Cv>::small_msm(hipStream_t st, const TermList& tl, const SmallPlan& sp, uint32_t terms, const AF* pts,
                           const uint8_t* inf, uint32_t* nodes, uint32_t* flags, uint32_t flag_words, XY* res) {
  (void)hipMemsetAsync(res, 0, (size_t)sp.nmsm * sizeof(XY), st);  // zz = 0: an MSM without terms is O
  (void)hipMemsetAsync(flags, 0, (size_t)flag_words * 4, st);
  if (terms) k_small_msm<Cv><<<terms, 64, 0, st>>>(tl, sp, pts, inf, nodes, flags, res);
}

template <class Cv>
void Launch<Cv>::window_combine(hipStream_t st, const MsmWindows& mw, const XY* winsum, XY* res, int wbits,
                                bool low_prio) {
  with_wbits(wbits, [&](auto wb) {
    constexpr int WB = decltype(wb)::value;
    if (low_prio) k_window_combine<Cv, WB, true><<<mw.nmsm, 64, 0, st>>>(mw, winsum, res);
    else k_window_combine<Cv, WB><<<mw.nmsm, 64, 0, st>>>(mw, winsum, res);
  });
}

template void Launch<KZ_CURVE_T>::sort(hipStream_t, const TermList&, uint32_t, const uint8_t*, uint32_t*, uint32_t*,
                                       uint64_t*, size_t, int, uint32_t*, uint32_t*, uint32_t*, uint32_t*, uint32_t*, int);
template void Launch<KZ_CURVE_T>::accumulate(hipStream_t, size_t, const uint32_t*, const uint32_t*, const uint32_t*,
                                             const uint32_t*, const uint32_t*, const Affine<KZ_CURVE_T>*, uint32_t*,
                                             uint32_t, size_t, uint32_t*, uint32_t*, const uint32_t*, hipStream_t);
template void Launch<KZ_CURVE_T>::fixup(hipStream_t, size_t, const uint32_t*, const uint32_t*, const uint32_t*,
                                        const uint32_t*, uint32_t*, uint32_t, uint32_t*, const uint32_t*);
template void Launch<KZ_CURVE_T>::pts_to29(hipStream_t, Affine<KZ_CURVE_T>*, uint32_t);
template void Launch<KZ_CURVE_T>::reduce(hipStream_t, uint32_t, const uint32_t*, const uint32_t*, Xyzz<KZ_CURVE_T>*,
                                         Xyzz<KZ_CURVE_T>*, Xyzz<KZ_CURVE_T>*, Xyzz<KZ_CURVE_T>*, int, bool, int, int);
template void Launch<KZ_CURVE_T>::window_combine(hipStream_t, const MsmWindows&, const Xyzz<KZ_CURVE_T>*,
                                                 Xyzz<KZ_CURVE_T>*, int, bool);
template void Launch<KZ_CURVE_T>::merge_buckets(hipStream_t, uint32_t, uint32_t*, uint32_t*, const uint32_t*,
                                                const uint32_t*);
template void Launch<KZ_CURVE_T>::small_msm(hipStream_t, const TermList&, const SmallPlan&, uint32_t,
                                            const Affine<KZ_CURVE_T>*, const uint8_t*, uint32_t*, uint32_t*, uint32_t,
                                            Xyzz<KZ_CURVE_T>*);

}  // namespace kzgmi
