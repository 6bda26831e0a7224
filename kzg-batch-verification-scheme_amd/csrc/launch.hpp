// Host-side launchers for every kernel, one set per curve.  Each group of launchers is
// defined in its own translation unit (launch_*.hip) compiled once per curve (-DKZ_CURVE=0
// BLS12-381, 1 BN254), so the device code builds in parallel; api.hip only calls these.
#pragma once
#include "kernels.hpp"
#include "msm_small.hpp"

namespace kzgmi {

template <class Cv>
struct Launch {
  using XY = Xyzz<Cv>;
  using AF = Affine<Cv>;
  // ---- MSM (launch_msm.hip)
  // digits: sum_k count_k * nwin_k u32 (tl.c[k].dig_base set), coarse: 3 * nsets * 256 u32
  // (counts, offsets, cursors), ent: emax x 8 B (coarse-pass entries: msm.hpp EntPacked / EntSplit)
  // sort_flags: SORT_SPLIT (split coarse-pass entries at every size), SORT_FULL_BINS (every set at
  // full-width coarse bins, the fallback of a set table overflow) -- test knobs
  static constexpr int SORT_SPLIT = 1, SORT_FULL_BINS = 2;
  static void sort(hipStream_t st, const TermList& tl, uint32_t nsets, const uint8_t* inf, uint32_t* digits,
                   uint32_t* coarse, uint64_t* ent, size_t emax, int sort_flags, uint32_t* off, uint32_t* cnt, uint32_t* total, uint32_t* sval,
                   uint32_t* skey, int wbits = WBITS);
  // both curves accumulate in radix 2^29: pts in that format (convert_points(to29) or
  // pts_to29), acc29 = (nb + 2 x launched threads) records of W29 words that stay the bucket
  // store (k_fixup joins pieces into them; reduce reads them).  The sorted entries [*lo, *total)
  // (lo nullptr: from 0), whole buckets
  static void accumulate(hipStream_t st, size_t nchunks, const uint32_t* total, const uint32_t* sval,
                         const uint32_t* skey, const uint32_t* off, const uint32_t* cnt, const AF* pts,
                         uint32_t* acc29, uint32_t nb, size_t acc_threads, uint32_t* next_chunk, uint32_t* crowd,
                         const uint32_t* lo, hipStream_t fix_st);
  // the piece joins of an accumulation launch (k_fixup, k_fixup_crowded: same nchunks, nb, lo);
  // accumulate issues them itself on fix_st (nullptr: the caller does, e.g. on another stream,
  // always behind the accumulation launch with the same crowd list, which zeroes it).
  // nb: the record index of the launch's first piece (its pieces follow the nb bucket records)
  static void fixup(hipStream_t st, size_t nchunks, const uint32_t* total, const uint32_t* skey, const uint32_t* off,
                    const uint32_t* cnt, uint32_t* acc29, uint32_t nb, uint32_t* crowd, const uint32_t* lo);
  static void pts_to29(hipStream_t st, AF* pts, uint32_t n);  // in place
  // acc29[b] += acc29b[b] for the buckets with cntb[b] != 0, cnt[b] += cntb[b] (chunked batches)
  static void merge_buckets(hipStream_t st, uint32_t nb, uint32_t* acc29, uint32_t* cnt, const uint32_t* acc29b,
                            const uint32_t* cntb);
  // low_prio: the kernels run at normal issue priority instead of the tail's raised one (the
  // side stream of a split accumulation)
  // seg4_waves: 4 threads per reduction segment when that grid stays within seg4_waves waves per
  // SIMD of the device's `simds` (0: always 2 threads)
  static void reduce(hipStream_t st, uint32_t nsets, const uint32_t* cnt, const uint32_t* acc29, XY* R, XY* U,
                     XY* scratch, XY* winsum, int wbits = WBITS, bool low_prio = false, int seg4_waves = 0,
                     int simds = 1024);
  static void window_combine(hipStream_t st, const MsmWindows& mw, const XY* winsum, XY* res, int wbits = WBITS,
                             bool low_prio = false);
  // small calls (msm_small.hpp): one wave per term + a counter tree; res (nmsm records)
  // and flags are cleared here; nodes: small_node_words() words, flags: small_flag_words() words
  static void small_msm(hipStream_t st, const TermList& tl, const SmallPlan& sp, uint32_t terms, const AF* pts,
                        const uint8_t* inf, uint32_t* nodes, uint32_t* flags, uint32_t flag_words, XY* res);
  // ---- I/O and scalars (launch_io.hip)
  // to29: store in the accumulation's radix-29 format, for
  // points that go straight into run_msm_core(..., pts29 = true)
  static void convert_points(hipStream_t st, const uint8_t* bytes, uint32_t n, AF* pts, uint8_t* inf, uint32_t* err,
                             bool to29 = false, AF* img = nullptr, uint8_t* img_inf = nullptr);
  static void set_generator(hipStream_t st, AF* pt, uint8_t* inf);
  static void decompress_points(hipStream_t st, const uint8_t* bytes, uint32_t n, AF* pts, uint8_t* inf,
                                uint32_t* err);
  static void compress_points(hipStream_t st, const uint8_t* in, uint32_t n, uint8_t* out);
  static void subgroup_check(hipStream_t st, const AF* pts, const uint8_t* inf, uint32_t n, uint32_t* err);
  static void convert_scalars(hipStream_t st, const uint8_t* bytes, uint32_t n, uint32_t* out, uint32_t* err);
  // GLV (glv.hpp): n scalars of 8 words, `stride` words apart -> half scalars h0, h1 (4 words each)
  static void glv_split(hipStream_t st, const uint32_t* scal, uint32_t stride, uint32_t n, uint32_t* h0, uint32_t* h1);
  // in29: src is in the accumulation's radix-29 format (and dst is written in it)
  static void endo_points(hipStream_t st, const AF* src, const uint8_t* src_inf, uint32_t n, AF* dst, uint8_t* dst_inf,
                          bool in29 = false);
  static void convert_g2(hipStream_t st, const uint8_t* bytes, uint32_t n, G2Aff<Cv>* out, uint8_t* inf,
                         uint32_t* err);
  static void tsum(hipStream_t st, const void* tpart, uint32_t nblocks, uint32_t* negt);  // negt = -(sum) mod r
  static void scalar_prep(hipStream_t st, const Seed& seed, const uint32_t* seed_dev, uint64_t index_offset,
                          const uint8_t* zs,
                          const uint8_t* ys, uint32_t n, uint32_t* r_out, uint32_t* s_out, void* tpart,
                          uint32_t* negt, uint32_t* err, uint32_t* h0 = nullptr, uint32_t* h1 = nullptr);
  static size_t tpart_bytes(uint32_t n);
  // ---- Fiat-Shamir / powers-of-r randomisers (fs.hpp)
  static void fs_leaves(hipStream_t st, const uint8_t* dC, const uint8_t* dpi, const uint8_t* dz, const uint8_t* dy,
                        uint32_t n, uint64_t offset, bool compressed, uint32_t* leaves);
  // Merkle-reduce `count` 32-byte nodes to `target` (count / target a power of two; each
  // result node covers count / target consecutive inputs); tmp holds 3 count / 4 nodes;
  // returns the buffer holding the result
  static const uint32_t* fs_reduce(hipStream_t st, const uint32_t* in, uint32_t count, uint32_t target, uint32_t* tmp);
  static void fs_pad(hipStream_t st, uint32_t* digests, uint32_t nchunks, uint32_t p2);
  static void fs_challenge(hipStream_t st, const uint32_t* root, uint64_t n, void* pow, uint32_t* chal_out);
  static void pow_table(hipStream_t st, const Seed& r_be, void* pow, uint32_t* err);
  static void scalar_prep_pow(hipStream_t st, const void* pow, uint64_t index_offset, const uint8_t* zs,
                              const uint8_t* ys, uint32_t n, uint32_t* r_out, uint32_t* s_out, void* tpart,
                              uint32_t* negt, uint32_t* err);
  static void encode_points(hipStream_t st, const XY* res, uint32_t count, uint8_t* out);
  // sum of gathered partial records; a record marked failed raises its code into *err
  static void sum_partials(hipStream_t st, const XY* parts, uint32_t nparts, uint32_t stride, uint32_t nout, XY* out,
                           uint32_t* err);
  // count partial records out = res, marked failed (kernels.hpp partial_mark) when *err != 0
  static void partial_out(hipStream_t st, const XY* res, uint32_t count, const uint32_t* err, XY* out);
  // ---- pairing (launch_pairing.hip)
  static int num_lines();
  static void precompute_lines(hipStream_t st, const G2Aff<Cv>* q, Line<Cv>* lines);
  static void pairing_check(hipStream_t st, const XY* res, const Line<Cv>* lines, const uint8_t* q_inf, int* ok);
  static void pairing_one(hipStream_t st, const AF* p, const uint8_t* p_inf, const Line<Cv>* lines,
                          const uint8_t* q_inf, uint8_t* out);
  // ---- prover commit key (launch_gen.hip): row out = 2^16 * row in, affine
  static void shift_points(hipStream_t st, const AF* in, const uint8_t* inf_in, uint32_t n, AF* out, uint8_t* inf_out);
  // ---- generators (launch_gen.hip)
  static void gen_table(hipStream_t st, XY* base, AF* table);
  static void gen_g1(hipStream_t st, const uint8_t* scalars, uint32_t n, const AF* table, uint8_t* out, uint32_t* err);
  static void g2_mul(hipStream_t st, const G2Aff<Cv>* q, const uint8_t* q_inf, const uint32_t (&k_le)[8], uint8_t* out);
  static void fpmul_probe(hipStream_t st, uint32_t blocks, uint32_t iters, uint32_t* out);
  static void gen_tuples(hipStream_t st, const Seed& seed, const uint32_t (&tau_le)[8], uint32_t n, const AF* table,
                         uint8_t* cm, uint8_t* zs, uint8_t* ys, uint8_t* pf);
};

inline unsigned grid_for(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

}  // namespace kzgmi

#if defined(KZ_CURVE)
#if KZ_CURVE == 0
#define KZ_CURVE_T ::kzgmi::Bls12_381
#else
#define KZ_CURVE_T ::kzgmi::Bn254
#endif
#endif
