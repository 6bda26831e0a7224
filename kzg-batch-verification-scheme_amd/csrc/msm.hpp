// G1 Pippenger MSM kernels for gfx950 (hot-path rows a5/a6 of SURVEY.md 8a).
//
// Pipeline (all on one HIP stream; no host synchronisation inside):
//   k_digits_count .. k_fine_sort  signed 16-bit window digits of every term, grouped by
//                     bucket with a two-pass LDS-privatised MSD partition (see "sort")
//   k_accumulate      load-balanced bucket accumulation: every thread owns exactly
//                     ACC_CHUNK consecutive sorted entries (not a bucket), so Poisson bucket
//                     sizes do not diverge a wavefront; bucket pieces cut by a chunk
//                     boundary go to partial slots and are joined by k_fixup.
//   k_fixup           joins the pieces of buckets cut by chunk boundaries
//   k_reduce_segments sum_b b*S_b per window: 16-bucket segments (running sums) ...
//   k_reduce_bits     ... combined per window by bit decomposition of the segment index
//   k_window_combine  Horner over the 16-bit windows (2^16 * acc + W_w)
//
// A "term list" generalises the two MSMs of batch verification (BASELINE.json:5,
// SURVEY.md 3.1): MSM#0 = sum r_i pi_i (127-bit scalars, 8 windows) and MSM#1 = sum r_i C_i
// + sum s_i pi_i - t G1 (windows 8..23), sharing one sort and one accumulation launch.
// Reference: none (LICENSE only); parity vs the C oracle in tests/test_gpu_parity.py.
#pragma once
#include "common.hpp"
#include "field29.hpp"
#include "lpfield.hpp"

namespace kzgmi {

constexpr int WBITS = 16;                      // window width c
constexpr int NBUCKETS = 1 << (WBITS - 1);     // signed digits: |d| in [1, 2^15]
// Accumulation chunk (entries per thread) the host sizes the grid for (run_msm_core): ACC_CHUNK,
// or ACC_CHUNK_SMALL for calls of at most ACC_SMALL_ENTRIES entries.  The grid is capped at one
// resident round (CUs x 4 SIMDs x 4 waves), so from n ~ 2^18 on every chunk is longer anyway.
// Below that, shorter chunks mean more waves and shorter chains (a 256-tuple batch: 128 threads
// of 64 sequential additions, 0.43 ms, vs 768 of 12, 0.15 ms) but more flushed pieces: at 2^17
// the pipelined rate was 869/s with 64-entry chunks, 850 with 16 and 830 with 8
// (profiles/r03/misc_ab_r03.txt) -- so only small calls take the short chunks.
constexpr int ACC_CHUNK = 64;
constexpr int ACC_CHUNK_SMALL = 16;
constexpr size_t ACC_SMALL_ENTRIES = size_t(1) << 20;
constexpr int SEG = 16;                        // buckets per reduction segment
constexpr int MAX_CLASSES = 16;

struct TermClass {
  uint32_t count;       // number of terms in the class
  uint32_t pt_base;     // index of the first point in the point array
  uint32_t scal_words;  // 4 (127-bit randomisers) or 8 (full Fr)
  uint32_t nwin;        // windows to emit
  uint32_t set_base;    // bucket set (= msm window) of window 0
  uint32_t scal_stride; // 0: one shared scalar for the whole class, else = scal_words
  const uint32_t* scal; // LE words, standard (non-Montgomery) form
  uint32_t win_off;     // window of the scalar that local window 0 reads (fixed-base tables:
                        // row w of 2^(16w)-shifted points reads digit w into one bucket set)
  uint32_t dig_base;    // first digit code of this class in the digit array (set by the host:
                        // digit (w, i) at dig_base + w * count + i)
};
struct TermList {
  TermClass c[MAX_CLASSES];
  uint32_t nclass;
  uint32_t total;
};

// Coarse-bin width per bucket set: bin = (|d| - 1) >> s[set].  A full window spreads over every
// bucket (s = COARSE_SHIFT: 128 buckets per bin); a window cut short by the top of its scalars
// does not: 13-bit windows keep 8 bits of a 255-bit scalar in the top one, and with 128-bucket
// bins its 2^17 terms fell into 2 bins of 64 K entries, each sorted by one workgroup in 16 chunks
// (k_fine_sort 0.18 ms of a 2^17 batch).  Narrower bins (s = top bits - log2(bins)) spread such a
// window over every bin; k_fine_sort writes the counts of the buckets no bin covers as 0.
constexpr int MAX_SETS = 64;
struct SetShift {
  uint8_t s[MAX_SETS];
};

// ------------------------------------------------------------------------------ sort
// Entries (one per nonzero signed window digit) are grouped by global bucket id
// key = set * 2^15 + (|d| - 1) with a two-pass MSD partition that keeps the atomics in LDS:
//   k_digits_count every signed digit of every term, once, counted per (class, 4096 terms) into
//                 LDS histograms of each window's 256 coarse bins (key >> 7), then one global
//                 atomic per non-empty (window, bin)
//   k_bin_scan    exclusive scan of the nsets*256 coarse counts (+ total entries)
//   k_bin_scatter the stored digits; LDS ranks, one global atomic per bin reserves the tile's run,
//                 entries (fine index, value: EntPacked / EntSplit) written into their coarse bin
//   k_fine_sort   one workgroup per coarse bin (128 buckets): LDS counting sort, writes the
//                 sorted (value, key) arrays and every bucket's offset/count; the value of
//                 a bucket's first entry carries SV_FIRST (bit 31), so the accumulation
//                 streams the values alone and reads a key only where a bucket starts
// Sorting is unstable inside a bucket; bucket sums (and the final affine result) do not
// depend on the order.
constexpr int COARSE_SHIFT = 7;
constexpr int FINE = 1 << COARSE_SHIFT;                 // buckets per coarse bin
constexpr int BINS_PER_SET = NBUCKETS >> COARSE_SHIFT;  // 256
constexpr int TILE_TERMS = 4096;                        // terms per tile (16 per thread)
// Window width c of a call (WBITS, NBUCKETS, BINS_PER_SET above are c = 16's): large calls use
// c = 16; small ones (few entries per bucket) c = 13 -- 8x fewer buckets to reduce for 5/4 the
// terms (api.hip call_wbits).  The sort, the window-sum reduction and the combination are
// instantiated per c.
template <int C>
struct Win {
  static constexpr int WBITS = C;
  static constexpr int NBUCKETS = 1 << (C - 1);         // signed digits |d| in [1, 2^(c-1)]
  static constexpr int BINS = NBUCKETS >> COARSE_SHIFT;  // coarse bins per set (<= 256 = block)
  static constexpr int NSEG = NBUCKETS / SEG;            // reduction segments per set
  static constexpr int SEG_BITS = C - 1 - 4;             // log2(NSEG)
  static constexpr int MAXW = 256 / C + 1;               // windows of a 256-bit scalar (+ carry)
  static constexpr int RB_PARTS = SEG_BITS + 6;         // k_reduce_bits parts per set
  static_assert(NSEG == (1 << SEG_BITS) && BINS <= 256 && BINS >= 1, "window width");
  static constexpr int BINS_LOG2 = C - 1 - COARSE_SHIFT;
};

// SetShift of a call (host): per set, the widest bin any of its windows needs.  A window of a
// class reads raw bits [w c, w c + c) of scalars below 2^127 (4-word: randomisers, GLV halves)
// or 2^255 (8-word: Fr); a window with tb < c raw bits takes |d| <= 2^tb (its carry-in included,
// no carry out), so bins of 2^(tb - log2 BINS) buckets cover it.
template <int WB>
inline bool set_shifts_host(const TermList& tl, uint32_t nsets, SetShift& ss) {
  using W = Win<WB>;
  if (nsets > (uint32_t)MAX_SETS) return false;
  for (uint32_t s = 0; s < nsets; ++s) ss.s[s] = 0;
  for (uint32_t k = 0; k < tl.nclass; ++k) {
    const TermClass& C = tl.c[k];
    if (!C.count) continue;
    const int bits = C.scal_words == 4 ? 127 : 255;
    for (uint32_t w = 0; w < C.nwin; ++w) {
      const int tb = std::min(WB, std::max(0, bits - (int)(C.win_off + w) * WB));
      const int need = tb >= WB - 1 ? COARSE_SHIFT : std::max(0, tb - W::BINS_LOG2);
      const uint32_t s = C.set_base + w;
      if (s >= nsets) return false;
      ss.s[s] = (uint8_t)std::max<int>(ss.s[s], need);
    }
  }
  return true;
}
// sorted value = point index << 1 | sign, | SV_FIRST on the first entry of each bucket (point
// indices stay below 2^30: at most 16 x 2^26 commit-key points)
constexpr uint32_t SV_FIRST = 1u << 31;
KZ_DEV uint32_t sv_point(uint32_t v) { return (v & ~SV_FIRST) >> 1; }

// Entries of the coarse pass (k_bin_scatter -> k_fine_sort): the coarse bin fixes a key's upper
// bits, so an entry is its 7-bit fine index and its sorted value.  Packed: fine << CV_BITS |
// value in 4 B, when every value fits CV_BITS (fewer than 2^24 points: every BLS12-381 batch up to
// n = 2^23, every 2^21-point MSM shard).  Split: the value (4 B) and the fine index (1 B) in two
// arrays, for any size (BN254 2^22 with its GLV images, the 2^24-point MSM, the commit key) --
// the fine sort's histogram pass then reads 1 B per entry.  (The round-2 form, key << 32 |
// value in 8 B, moved 16 B per entry through the fine sort's two reads.)
constexpr int CV_BITS = 25;
struct EntPacked {
  uint32_t* p;
  using R = uint32_t;  // register form
  KZ_DEV R load(size_t i) const { return p[i]; }
  KZ_DEV uint32_t fine_at(size_t i) const { return p[i] >> CV_BITS; }
  KZ_DEV void store(size_t i, R r) const { p[i] = r; }
  KZ_DEV static uint32_t fine(R r) { return r >> CV_BITS; }
  KZ_DEV static uint32_t val(R r) { return r & ((1u << CV_BITS) - 1); }
  KZ_DEV static R make(uint32_t fine, uint32_t v) { return ((fine & (FINE - 1)) << CV_BITS) | v; }
};
struct EntSplit {
  uint32_t* p;
  uint8_t* f;
  using R = uint64_t;  // fine << 32 | value
  KZ_DEV R load(size_t i) const { return ((uint64_t)f[i] << 32) | p[i]; }
  KZ_DEV uint32_t fine_at(size_t i) const { return f[i]; }
  KZ_DEV void store(size_t i, R r) const {
    p[i] = (uint32_t)r;
    f[i] = (uint8_t)(r >> 32);
  }
  KZ_DEV static uint32_t fine(R r) { return (uint32_t)(r >> 32); }
  KZ_DEV static uint32_t val(R r) { return (uint32_t)r; }
  KZ_DEV static R make(uint32_t fine, uint32_t v) { return ((uint64_t)(fine & (FINE - 1)) << 32) | v; }
};
// empty register slot (never a real entry: packed values stay below 2^CV_BITS - 1, fine < 128)
template <class R>
constexpr R kNoEnt = ~(R)0;

struct TileRef {
  int k, w;
  uint32_t c;
};
KZ_DEV TileRef tile_decode(const TermList& tl, uint32_t t) {
  int k = 0;
  for (; k < (int)tl.nclass - 1; ++k) {
    uint32_t chunks = (tl.c[k].count + TILE_TERMS - 1) / TILE_TERMS;
    uint32_t nt = chunks * tl.c[k].nwin;
    if (t < nt) break;
    t -= nt;
  }
  uint32_t chunks = (tl.c[k].count + TILE_TERMS - 1) / TILE_TERMS;
  return {k, (int)(t / chunks), t % chunks};
}

// The signed window digits of term i of class C: the scalar read once, the carry chain walked
// over its windows; emit(local window, code) for windows win_off .. win_off + nwin - 1.  Code = 0
// for a zero digit or a point at infinity, else |d| | (entry sign << 31) with entry sign =
// (d < 0) xor the half-scalar's sign flag.
template <int WB, class Emit>
KZ_DEV void term_digits(const TermClass& C, uint32_t i, const uint8_t* __restrict__ inf, Emit&& emit) {
  using W = Win<WB>;
  const uint32_t* sp = C.scal + (size_t)i * C.scal_stride;
  uint32_t w8[8];
  bool neg = false;
  if (C.scal_words == 4) {
    const uint4 q = *reinterpret_cast<const uint4*>(sp);
    neg = (q.w >> 31) != 0;
    w8[0] = q.x; w8[1] = q.y; w8[2] = q.z; w8[3] = q.w & 0x7fffffffu;
    w8[4] = w8[5] = w8[6] = w8[7] = 0;
  } else {
    const uint4 q0 = *reinterpret_cast<const uint4*>(sp);
    const uint4 q1 = *reinterpret_cast<const uint4*>(sp + 4);
    w8[0] = q0.x; w8[1] = q0.y; w8[2] = q0.z; w8[3] = q0.w;
    w8[4] = q1.x; w8[5] = q1.y; w8[6] = q1.z; w8[7] = q1.w;
  }
  const bool is_inf = inf[C.pt_base + i] != 0;
  const int w0 = (int)C.win_off, w1 = (int)(C.win_off + C.nwin);
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < W::MAXW; ++w) {
    if (w >= w1) break;
    // bits [w c, w c + c) of the scalar (compile-time word index and shift)
    const int bit = w * WB, wi = bit >> 5, sh = bit & 31;
    uint32_t raw = wi < 8 ? w8[wi] >> sh : 0u;
    if (sh + WB > 32 && wi + 1 < 8) raw |= w8[wi + 1] << (32 - sh);
    raw &= (1u << WB) - 1;
    int d = (int)(raw + carry);
    if (d > W::NBUCKETS) { d -= (1 << WB); carry = 1; } else { carry = 0; }
    if (w >= w0) {
      uint32_t code = 0;
      if (d != 0 && !is_inf) code = (uint32_t)(d < 0 ? -d : d) | ((d < 0) != neg ? 0x80000000u : 0u);
      emit(w - w0, code);
    }
  }
}

// Every signed digit of every term, once, and the coarse counts, in one pass: workgroup = 4096
// terms of one class (16 per thread), every window's digits written (digit w of term i at
// dig_base + w * count + i) and counted into an LDS histogram per window, then one global atomic
// per non-empty (window, coarse bin); the scatter pass reads the digits back.
inline uint32_t num_digit_groups_host(const TermList& tl) {
  uint32_t g = 0;
  for (uint32_t k = 0; k < tl.nclass; ++k) g += (tl.c[k].count + TILE_TERMS - 1) / TILE_TERMS;
  return g;
}
// UNIFORM: every set at COARSE_SHIFT (16-bit windows: no window is cut short), the shift a constant
template <int WB, bool UNIFORM>
__global__ void __launch_bounds__(256) k_digits_count(TermList tl, SetShift ss, const uint8_t* __restrict__ inf,
                                                      uint32_t* __restrict__ digits,
                                                      uint32_t* __restrict__ coarse_cnt) {
  using W = Win<WB>;
  __shared__ uint32_t hist[W::MAXW][W::BINS];
  uint32_t b = blockIdx.x;
  int k = 0;
  for (; k < (int)tl.nclass - 1; ++k) {
    const uint32_t nb = (tl.c[k].count + TILE_TERMS - 1) / TILE_TERMS;
    if (b < nb) break;
    b -= nb;
  }
  const TermClass& C = tl.c[k];
  const uint32_t t = threadIdx.x;
  uint32_t shw[W::MAXW];  // each window's coarse-bin shift, read once (uniform)
#pragma unroll
  for (int w = 0; w < W::MAXW; ++w)
    shw[w] = UNIFORM ? (uint32_t)COARSE_SHIFT : ss.s[min(C.set_base + (uint32_t)w, (uint32_t)MAX_SETS - 1)];
  if (t < (uint32_t)W::BINS) {
#pragma unroll
    for (int w = 0; w < W::MAXW; ++w) hist[w][t] = 0;
  }
  __syncthreads();
#pragma unroll 1
  for (int j = 0; j < TILE_TERMS / 256; ++j) {
    const uint32_t i = b * TILE_TERMS + j * 256 + t;
    if (i >= C.count) break;
    term_digits<WB>(C, i, inf, [&](int w, uint32_t code) {
      if (code) atomicAdd(&hist[w][((code & 0x7fffffffu) - 1) >> shw[w]], 1u);
      digits[C.dig_base + (size_t)w * C.count + i] = code;
    });
  }
  __syncthreads();
  if (t >= (uint32_t)W::BINS) return;
  for (int w = 0; w < (int)C.nwin; ++w) {
    const uint32_t h = hist[w][t];
    if (h) atomicAdd(&coarse_cnt[(C.set_base + w) * W::BINS + t], h);
  }
}

// single block: exclusive scan of nbins (<= 8192) coarse counts; cursor copy; total
static __global__ void __launch_bounds__(1024) k_bin_scan(const uint32_t* __restrict__ cnt, uint32_t nbins,
                                                          uint32_t* __restrict__ off, uint32_t* __restrict__ cursor,
                                                          uint32_t* __restrict__ total) {
  __shared__ uint32_t s[1024];
  constexpr int PER = 8;
  uint32_t v[PER];
  uint32_t sum = 0;
  const uint32_t base = threadIdx.x * PER;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    v[i] = base + i < nbins ? cnt[base + i] : 0u;
    sum += v[i];
  }
  s[threadIdx.x] = sum;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    uint32_t x = threadIdx.x >= (unsigned)d ? s[threadIdx.x - d] : 0u;
    __syncthreads();
    s[threadIdx.x] += x;
    __syncthreads();
  }
  uint32_t run = s[threadIdx.x] - sum;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    if (base + i < nbins) { off[base + i] = run; cursor[base + i] = run; }
    run += v[i];
  }
  if (threadIdx.x == 1023) *total = s[1023];
}

// Entries are ranked per coarse bin in LDS, staged in bin order, and written out so that
// consecutive threads store consecutive addresses of a bin's run (the tile's run in each bin
// is contiguous in `tmp`); writing each entry from the thread that ranked it scattered every
// wavefront store over ~64 bins.
template <class E, int WB = WBITS, bool UNIFORM = true>
__global__ void __launch_bounds__(256) k_bin_scatter(TermList tl, SetShift ss, const uint32_t* __restrict__ digits,
                                                     uint32_t* __restrict__ coarse_cursor, E tmp) {
  using W = Win<WB>;
  constexpr uint32_t NBIN = W::BINS;        // coarse bins per set (threads >= NBIN only rank)
  __shared__ uint32_t hist[NBIN];
  __shared__ uint32_t base[NBIN];   // global start of this tile's run in bin b
  __shared__ uint32_t lstart[NBIN]; // local (staged) start of bin b
  __shared__ typename E::R stage[TILE_TERMS];
  __shared__ uint8_t stage_bin[TILE_TERMS];
  const TileRef T = tile_decode(tl, blockIdx.x);
  const TermClass& C = tl.c[T.k];
  const uint32_t set = C.set_base + T.w;
  const uint32_t sh = UNIFORM ? (uint32_t)COARSE_SHIFT : ss.s[set];  // coarse-bin width of the set (SetShift)
  const uint32_t* dg = digits + C.dig_base + (size_t)T.w * C.count;
  const uint32_t t = threadIdx.x;
  if (t < NBIN) hist[t] = 0;
  __syncthreads();
  uint32_t rank[TILE_TERMS / 256], key[TILE_TERMS / 256], ent[TILE_TERMS / 256];
#pragma unroll
  for (int j = 0; j < TILE_TERMS / 256; ++j) {
    key[j] = 0xffffffffu;
    const uint32_t local = T.c * TILE_TERMS + j * 256 + t;
    const uint32_t code = local < C.count ? dg[local] : 0u;
    if (!code) continue;
    const uint32_t mag = code & 0x7fffffffu;
    key[j] = set * W::NBUCKETS + (mag - 1);
    ent[j] = ((C.pt_base + local) << 1) | (code >> 31);
    rank[j] = atomicAdd(&hist[(mag - 1) >> sh], 1u);
  }
  __syncthreads();
  const uint32_t h = t < NBIN ? hist[t] : 0u;
  if (t < NBIN) {
    base[t] = h ? atomicAdd(&coarse_cursor[set * NBIN + t], h) : 0u;
    lstart[t] = h;
  }
  __syncthreads();
  for (uint32_t d = 1; d < NBIN; d <<= 1) {  // inclusive scan of the tile's bin counts
    const uint32_t x = (t < NBIN && t >= d) ? lstart[t - d] : 0u;
    __syncthreads();
    if (t < NBIN) lstart[t] += x;
    __syncthreads();
  }
  const uint32_t ntile = lstart[NBIN - 1];
  __syncthreads();
  if (t < NBIN) lstart[t] -= h;  // exclusive
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TILE_TERMS / 256; ++j) {
    if (key[j] == 0xffffffffu) continue;
    const uint32_t m1 = key[j] & (W::NBUCKETS - 1);  // |d| - 1
    const uint32_t bin = m1 >> sh;
    const uint32_t q = lstart[bin] + rank[j];
    stage[q] = E::make(m1 & ((1u << sh) - 1), ent[j]);  // the fine index within the bin
    stage_bin[q] = (uint8_t)bin;
  }
  __syncthreads();
  for (uint32_t q = t; q < ntile; q += 256) {
    const uint32_t bin = stage_bin[q];
    tmp.store(base[bin] + (q - lstart[bin]), stage[q]);
  }
}

// one workgroup per coarse bin g: LDS counting sort of its entries by the low 7 key bits.
// Packed entries of a staged bin (the common case: 2^20 BLS12-381 batches average ~4 K entries per
// bin) are read once, into registers, and the histogram atomics return each entry's rank in its
// bucket (sort phase 0.368 -> 0.329 ms, profiles/r05/ab_fine_sort_one_read.txt); the rest:
// Both passes over the bin's entries issue FINE_ILP independent loads per thread before
// using them (the loops are latency-bound otherwise).  Bins of up to FINE_STAGE entries are
// sorted into an LDS staging array and then written out contiguously (coalesced stores; the
// bucket of output slot p comes from a 7-step search of the inclusive bucket scan) instead
// of two scattered 4-byte stores per entry.  Larger bins (BN254 at n = 2^22: ~32 K entries,
// the 2^24-point MSM: ~65 K) go through the same staging array a chunk of FINE_STAGE / 2 entries
// at a time: the chunk is counting-sorted in LDS (the histogram atomics return the ranks), and each
// bucket's run of the chunk is written at that bucket's running cursor -- runs of ~32 entries
// instead of one scattered 4-byte store pair per entry.
constexpr int FINE_ILP = 4;
constexpr int FINE_STAGE = 8192;

// Bins above FINE_STAGE entries, a chunk at a time (k_fine_sort): cursor[b] holds bucket b's
// next free position in the bin, bstart[b] its first (SV_FIRST goes there); `stage` is the
// kernel's staging array.  A chunk's entries stay in registers between the ranking and the
// staging: chunks of FINE_STAGE / 2 keep the kernel within 128 VGPRs (4 workgroups per CU for
// the staged bins, whose LDS allows 4).
template <class E>
KZ_DEV void fine_sort_chunks(uint32_t kbase, uint32_t start, uint32_t count, const E tmp,
                             const uint32_t* bstart, uint32_t* cursor, uint32_t* stage,
                             uint32_t* __restrict__ sorted_val, uint32_t* __restrict__ sorted_key) {
  constexpr uint32_t CHUNK = FINE_STAGE / 2, PER = CHUNK / 256;  // 16 per thread: 147 -> <= 128 VGPRs
  __shared__ uint32_t ccnt[FINE];   // chunk histogram
  __shared__ uint32_t cscan[FINE];  // chunk inclusive scan
  const uint32_t t = threadIdx.x;
  for (uint32_t c0 = 0; c0 < count; c0 += CHUNK) {
    const uint32_t cn = min(CHUNK, count - c0);
    if (t < FINE) ccnt[t] = 0;
    __syncthreads();
    using R = typename E::R;
    R v[PER];
    uint32_t rank[PER];
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const uint32_t e = j * 256 + t;
      v[j] = e < cn ? tmp.load(start + c0 + e) : kNoEnt<R>;
    }
#pragma unroll
    for (int j = 0; j < PER; ++j)
      rank[j] = v[j] != kNoEnt<R> ? atomicAdd(&ccnt[E::fine(v[j])], 1u) : 0u;
    __syncthreads();
    const uint32_t tot = t < FINE ? ccnt[t] : 0u;
    if (t < FINE) cscan[t] = tot;
    __syncthreads();
    for (int d = 1; d < FINE; d <<= 1) {  // Hillis-Steele, threads 0..127
      const uint32_t x = (t < FINE && t >= (uint32_t)d) ? cscan[t - d] : 0u;
      __syncthreads();
      if (t < FINE) cscan[t] += x;
      __syncthreads();
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (v[j] == kNoEnt<R>) continue;
      const uint32_t b = E::fine(v[j]);
      const uint32_t q = cscan[b] - ccnt[b] + rank[j];
      stage[q] = E::val(v[j]);
    }
    __syncthreads();
    for (uint32_t q = t; q < cn; q += 256) {
      uint32_t b = 0;  // smallest b with cscan[b] > q
#pragma unroll
      for (int step = FINE / 2; step >= 1; step >>= 1)
        if (cscan[b + step - 1] <= q) b += step;
      const uint32_t p = cursor[b] + q - (cscan[b] - ccnt[b]);  // position in the bin
      sorted_val[start + p] = stage[q] | (p == bstart[b] ? SV_FIRST : 0u);
      sorted_key[start + p] = kbase + b;
    }
    __syncthreads();
    if (t < FINE) cursor[t] += ccnt[t];
    __syncthreads();
  }
}

template <class E, int WB, bool UNIFORM>
__global__ void __launch_bounds__(256) k_fine_sort(const uint32_t* __restrict__ coarse_off,
                                                   const uint32_t* __restrict__ coarse_cnt, const E tmp,
                                                   uint32_t* __restrict__ off, uint32_t* __restrict__ cnt,
                                                   uint32_t* __restrict__ sorted_val,
                                                   uint32_t* __restrict__ sorted_key, SetShift ss) {
  __shared__ uint32_t fine[FINE];
  __shared__ uint32_t cursor[FINE];
  __shared__ uint32_t scan[FINE];  // inclusive bucket scan
  __shared__ uint32_t stage[FINE_STAGE];
  const uint32_t g = blockIdx.x;
  const uint32_t start = coarse_off[g], count = coarse_cnt[g];
  const uint32_t t = threadIdx.x;
  const bool staged = count <= (uint32_t)FINE_STAGE;
  // bin g = bin gl of set s: buckets kbase + [0, 2^sh) of the set's bins * FINE (SetShift)
  constexpr uint32_t bins = Win<WB>::BINS;
  const uint32_t s = g / bins, gl = g % bins, sh = UNIFORM ? (uint32_t)COARSE_SHIFT : ss.s[s];
  const uint32_t kbase = s * bins * FINE + (gl << sh), nfine = 1u << sh;
  if (sh < COARSE_SHIFT) {  // the set's buckets no bin covers: empty (this bin's share of them)
    const uint32_t unc = FINE - nfine, ub = s * bins * FINE + (bins << sh) + gl * unc;
    for (uint32_t u = t; u < unc; u += 256) {
      off[ub + u] = start;
      cnt[ub + u] = 0;
    }
  }
  if (t < FINE) fine[t] = 0;
  __syncthreads();
  using R = typename E::R;
  if constexpr (sizeof(R) == 4) {
    if (staged) {  // packed entries of a staged bin: ONE read, the histogram atomics return the ranks
      constexpr int PER = FINE_STAGE / 256;
      R v[PER];
      uint32_t rank[PER];
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        const uint32_t e = j * 256 + t;
        v[j] = e < count ? tmp.load(start + e) : kNoEnt<R>;
      }
#pragma unroll
      for (int j = 0; j < PER; ++j) rank[j] = v[j] != kNoEnt<R> ? atomicAdd(&fine[E::fine(v[j])], 1u) : 0u;
      __syncthreads();
      const uint32_t tot = t < FINE ? fine[t] : 0u;
      if (t < FINE) scan[t] = tot;
      __syncthreads();
      for (int d = 1; d < FINE; d <<= 1) {  // Hillis-Steele, threads 0..127
        const uint32_t x = (t < FINE && t >= (uint32_t)d) ? scan[t - d] : 0u;
        __syncthreads();
        if (t < FINE) scan[t] += x;
        __syncthreads();
      }
      if (t < nfine) {
        const uint32_t key = kbase + t;
        off[key] = start + scan[t] - tot;
        cnt[key] = tot;
      }
#pragma unroll
      for (int j = 0; j < PER; ++j) {
        if (v[j] == kNoEnt<R>) continue;
        const uint32_t f = E::fine(v[j]);
        stage[scan[f] - fine[f] + rank[j]] = E::val(v[j]) | (rank[j] == 0 ? SV_FIRST : 0u);
      }
      __syncthreads();
      for (uint32_t p = t; p < count; p += 256) {
        uint32_t b = 0;  // smallest b with scan[b] > p
#pragma unroll
        for (int step = FINE / 2; step >= 1; step >>= 1)
          if (scan[b + step - 1] <= p) b += step;
        sorted_val[start + p] = stage[p];
        sorted_key[start + p] = kbase + b;
      }
      return;
    }
  }
  for (uint32_t e0 = t; e0 < count; e0 += 256 * FINE_ILP) {
    uint32_t k[FINE_ILP];  // fine index, FINE = none
#pragma unroll
    for (int j = 0; j < FINE_ILP; ++j) {
      const uint32_t e = e0 + 256 * j;
      k[j] = e < count ? tmp.fine_at(start + e) : (uint32_t)FINE;
    }
#pragma unroll
    for (int j = 0; j < FINE_ILP; ++j)
      if (k[j] < (uint32_t)FINE) atomicAdd(&fine[k[j]], 1u);
  }
  __syncthreads();
  const uint32_t tot = t < FINE ? fine[t] : 0u;
  if (t < FINE) scan[t] = tot;
  __syncthreads();
  for (int d = 1; d < FINE; d <<= 1) {  // Hillis-Steele, threads 0..127
    const uint32_t x = (t < FINE && t >= (uint32_t)d) ? scan[t - d] : 0u;
    __syncthreads();
    if (t < FINE) scan[t] += x;
    __syncthreads();
  }
  if (t < FINE) {
    const uint32_t base = scan[t] - tot;
    cursor[t] = base;
    if (t < nfine) {
      const uint32_t key = kbase + t;
      off[key] = start + base;
      cnt[key] = tot;
    }
  }
  __syncthreads();
  if (!staged) {
    if (t < FINE) scan[t] -= fine[t];  // bucket starts (exclusive scan); cursor[] is a copy
    __syncthreads();
    fine_sort_chunks(kbase, start, count, tmp, scan, cursor, stage, sorted_val, sorted_key);
    return;
  }
  for (uint32_t e0 = t; e0 < count; e0 += 256 * FINE_ILP) {
    using R = typename E::R;
    R v[FINE_ILP];
#pragma unroll
    for (int j = 0; j < FINE_ILP; ++j) {
      const uint32_t e = e0 + 256 * j;
      v[j] = e < count ? tmp.load(start + e) : kNoEnt<R>;
    }
#pragma unroll
    for (int j = 0; j < FINE_ILP; ++j) {
      if (v[j] == kNoEnt<R>) continue;
      const uint32_t f = E::fine(v[j]);
      const uint32_t p = atomicAdd(&cursor[f], 1u);
      const uint32_t first = p == scan[f] - fine[f] ? SV_FIRST : 0u;
      stage[p] = E::val(v[j]) | first;
    }
  }
  __syncthreads();
  for (uint32_t p = t; p < count; p += 256) {
    uint32_t b = 0;  // smallest b with scan[b] > p
#pragma unroll
    for (int step = FINE / 2; step >= 1; step >>= 1)
      if (scan[b + step - 1] <= p) b += step;
    sorted_val[start + p] = stage[p];
    sorted_key[start + p] = kbase + b;
  }
}

inline uint32_t num_tiles_host(const TermList& tl) {
  uint32_t t = 0;
  for (uint32_t k = 0; k < tl.nclass; ++k) t += ((tl.c[k].count + TILE_TERMS - 1) / TILE_TERMS) * tl.c[k].nwin;
  return t;
}

// ------------------------------------------------------------------------------ points I/O
template <class Cv>
KZ_DEV Affine<Cv> load_affine(const Affine<Cv>* pts, uint32_t i) {
  // 96 B (BLS) / 64 B (BN) per point: 16-byte vector loads
  Affine<Cv> a;
  constexpr int W = 2 * Cv::FpP::N;  // 32-bit words per point
  const uint4* src = reinterpret_cast<const uint4*>(pts + i);
  uint32_t w[W];
#pragma unroll
  for (int k = 0; k < W / 4; ++k) {
    uint4 q = src[k];
    w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
  }
#pragma unroll
  for (int k = 0; k < Cv::FpP::N; ++k) { a.x.v[k] = w[k]; a.y.v[k] = w[Cv::FpP::N + k]; }
  return a;
}

template <class Cv>
KZ_DEV void store_xyzz(Xyzz<Cv>* dst, const Xyzz<Cv>& p) {
  constexpr int N = Cv::FpP::N;
  uint4* d = reinterpret_cast<uint4*>(dst);
  uint32_t w[4 * N];
#pragma unroll
  for (int k = 0; k < N; ++k) { w[k] = p.x.v[k]; w[N + k] = p.y.v[k]; w[2 * N + k] = p.zz.v[k]; w[3 * N + k] = p.zzz.v[k]; }
#pragma unroll
  for (int k = 0; k < N; ++k) d[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}
template <class Cv>
KZ_DEV Xyzz<Cv> load_xyzz(const Xyzz<Cv>* src) {
  constexpr int N = Cv::FpP::N;
  const uint4* s = reinterpret_cast<const uint4*>(src);
  uint32_t w[4 * N];
#pragma unroll
  for (int k = 0; k < N; ++k) { uint4 q = s[k]; w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w; }
  Xyzz<Cv> p;
#pragma unroll
  for (int k = 0; k < N; ++k) { p.x.v[k] = w[k]; p.y.v[k] = w[N + k]; p.zz.v[k] = w[2 * N + k]; p.zzz.v[k] = w[3 * N + k]; }
  return p;
}

// ------------------------------------------------------------------------------ accumulation
// Chunk length: every accumulation thread owns `len` consecutive sorted entries, len =
// ceil(total / nthreads) rounded up to a multiple of 4 (chunks start on 16-B boundaries: the
// radix-29 loop reads its values 4 at a time) for the launched thread count nthreads (the same
// value in k_accumulate and k_fixup).  The host picks nthreads ~ (entry bound) / ACC_CHUNK(_SMALL),
// capped at one resident round: the capped grid gives longer, equal chunks (fewer pieces, no
// partial last round).
// Work-queue form for calls whose grid reaches the cap (api.hip run_msm_core): ACC_QUEUE_FACTOR
// chunks per launched thread, none shorter than ACC_QUEUE_MIN_LEN entries.
#ifndef KZ_ACC_QUEUE_FACTOR
#define KZ_ACC_QUEUE_FACTOR 2
#endif
constexpr int ACC_QUEUE_FACTOR = KZ_ACC_QUEUE_FACTOR;
constexpr size_t ACC_QUEUE_MIN_LEN = 64;
// ... and only for calls of at least ACC_QUEUE_FROM entries (window terms).  Since the loop stopped
// spilling (round 4) the static one-round grid is faster for 2^20-tuple batches (2^25 entries:
// 184.3 vs 181.9 batch-verifies/s) and 2^20-point MSMs (2^24: 378.7 vs 375.7 M pts/s), while the
// queue still pays for configs[3]'s 2^24-point MSMs (2^28 entries, two in flight: 42.6 vs 44.3
// ms; profiles/r04/ab_acc_queue.txt).
#ifndef KZ_ACC_QUEUE_FROM
#define KZ_ACC_QUEUE_FROM (size_t(1) << 26)
#endif
constexpr size_t ACC_QUEUE_FROM = KZ_ACC_QUEUE_FROM;
KZ_DEV uint32_t acc_chunk_len(uint32_t total, uint32_t nthreads) {
  const uint32_t per = ((total + nthreads - 1) / nthreads + 3) & ~3u;
  return per > 4u ? per : 4u;
}

// ---- radix-2^29 accumulation (BLS12-381; field29.hpp) ------------------------------------
// Points arrive in radix-29 form (x in words 0..13, y in 14..27 of each 128-B slot), written so
// by k_convert_points<To29> or converted in place by k_pts_to29.  Finished buckets and bucket
// pieces are radix-29 records of W29 words (x, y, zz, zzz; zz = 0 marks infinity) in `acc29` =
// [nb bucket records | nthreads first pieces | nthreads last pieces]; k_fixup joins pieces into
// the records and k_reduce_segments runs its running sums on them, both with the radix-29 XYZZ
// addition (x29_add below), writing R/U as records too; k_reduce_bits converts to 32-bit limbs
// as it reads them.  No conversion at the flushes: some lane of a wavefront changes bucket in
// almost every step, so per-flush work runs on most iterations.
// words of a radix-29 XYZZ record: BLS12-381 56 (224 B), BN254 36 (144 B)
template <class Q>
constexpr int kW29 = 4 * Q::N;

// A point slot in the accumulation's format.  Limbs (BLS12-381): x, y as 2 x 14 radix-29 limbs,
// 112 B of the 128-B slot -- packing would save no 64-B sector.  Packed (BN254): x R29 and y R29
// (both < 1.01 p < 2^254) as 2 x 8 little-endian 32-bit words, the 64-B slot of the 32-bit form:
// one 64-B sector per gather instead of the two that 9 + 9 limbs (72 B) span, unpacked into limbs
// with ~2 VALU per limb (limbs29); the BN254 accumulation was bound by that gather traffic.
template <class Cv>
constexpr bool kPackPts = sizeof(Affine<Cv>) < 2 * Fp29Of<Cv>::N * 4;

template <class Cv>
KZ_DEV void store_pt29(Affine<Cv>* slot, const F29<Fp29Of<Cv>>& x, const F29<Fp29Of<Cv>>& y) {
  using Q = Fp29Of<Cv>;
  uint4* d = reinterpret_cast<uint4*>(slot);
  if constexpr (kPackPts<Cv>) {
    constexpr int NW = Cv::FpP::N;
    uint32_t w[2 * NW];
    words32<Q>(x, *reinterpret_cast<uint32_t(*)[NW]>(w));
    words32<Q>(y, *reinterpret_cast<uint32_t(*)[NW]>(w + NW));
#pragma unroll
    for (int k = 0; k < NW / 2; ++k) d[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  } else {
    static_assert(Q::N % 2 == 0, "limb slots are stored as 16-B vectors");
    uint32_t w[2 * Q::N];
#pragma unroll
    for (int k = 0; k < Q::N; ++k) { w[k] = x.v[k]; w[Q::N + k] = y.v[k]; }
#pragma unroll
    for (int k = 0; k < Q::N / 2; ++k) d[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  }
}
template <class Cv>
KZ_DEV void load_pt29(const Affine<Cv>* slot, F29<Fp29Of<Cv>>& x, F29<Fp29Of<Cv>>& y) {
  using Q = Fp29Of<Cv>;
  const uint4* s4 = reinterpret_cast<const uint4*>(slot);
  if constexpr (kPackPts<Cv>) {
    constexpr int NW = Cv::FpP::N;
    uint32_t wx[NW], wy[NW];
#pragma unroll
    for (int k = 0; k < NW / 4; ++k) {
      const uint4 a = s4[k], b = s4[NW / 4 + k];
      wx[4 * k] = a.x; wx[4 * k + 1] = a.y; wx[4 * k + 2] = a.z; wx[4 * k + 3] = a.w;
      wy[4 * k] = b.x; wy[4 * k + 1] = b.y; wy[4 * k + 2] = b.z; wy[4 * k + 3] = b.w;
    }
    x = limbs29<Q>(wx);
    y = limbs29<Q>(wy);
  } else {
    uint32_t w[2 * Q::N];
#pragma unroll
    for (int k = 0; k < Q::N / 2; ++k) {
      const uint4 q = s4[k];
      w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
    }
#pragma unroll
    for (int k = 0; k < Q::N; ++k) { x.v[k] = w[k]; y.v[k] = w[Q::N + k]; }
  }
}

// dst[i] = phi(src[i]) = (beta x, y) on points already in the accumulation's format (GLV on
// points converted straight into it: no 32-bit pass and no k_pts_to29 over 2 x (2n + 1) points)
template <class Cv>
__global__ void __launch_bounds__(256) k_endo_points29(const Affine<Cv>* __restrict__ src,
                                                       const uint8_t* __restrict__ src_inf, uint32_t n,
                                                       Affine<Cv>* __restrict__ dst, uint8_t* __restrict__ dst_inf) {
  using Q = Fp29Of<Cv>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  F29<Q> x, y;
  load_pt29<Cv>(src + i, x, y);  // < (p / R29 + 1) p; beta R29 likewise: the product stays below it
  store_pt29<Cv>(dst + i, mul29(x, fp_to29<Q>(Fp<typename Cv::FpP>::from_const(Cv::K::GLV_BETA_M))), y);
  dst_inf[i] = src_inf[i];
}

template <class Cv>
__global__ void __launch_bounds__(256) k_pts_to29(Affine<Cv>* __restrict__ pts, uint32_t n) {
  using Q = Fp29Of<Cv>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Affine<Cv> a = pts[i];
  store_pt29<Cv>(pts + i, fp_to29<Q>(a.x), fp_to29<Q>(a.y));
}

// ------------------------------------------------------------------------------ radix-29 XYZZ
// A bucket record as loaded for the reduction: coordinates in radix 2^29 (record bounds:
// x < 10p, y < 16p, zz, zzz < 2p) and an explicit infinity flag.
template <class Q>
struct X29 {
  F29<Q> x, y, zz, zzz;
  bool inf;
};
template <class Q>
KZ_DEV X29<Q> load_x29(const uint32_t* __restrict__ acc29, size_t r) {
  constexpr int N = Q::N, W29 = kW29<Q>;
  const uint4* s4 = reinterpret_cast<const uint4*>(acc29 + r * W29);
  uint32_t w[W29];
#pragma unroll
  for (int k = 0; k < W29 / 4; ++k) {
    const uint4 q = s4[k];
    w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
  }
  X29<Q> o;
  uint32_t zz_or = 0;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    o.x.v[k] = w[k];
    o.y.v[k] = w[N + k];
    o.zz.v[k] = w[2 * N + k];
    o.zzz.v[k] = w[3 * N + k];
    zz_or |= w[2 * N + k];
  }
  o.inf = zz_or == 0;
  return o;
}
template <class Q>
KZ_DEV void store_x29(uint32_t* __restrict__ acc29, size_t r, const X29<Q>& a) {
  constexpr int N = Q::N, W29 = kW29<Q>;
  uint32_t w[W29];
#pragma unroll
  for (int k = 0; k < N; ++k) {
    w[k] = a.x.v[k];
    w[N + k] = a.y.v[k];
    w[2 * N + k] = a.inf ? 0u : a.zz.v[k];  // zz = 0 marks infinity
    w[3 * N + k] = a.zzz.v[k];
  }
  uint4* d4 = reinterpret_cast<uint4*>(acc29 + r * W29);
#pragma unroll
  for (int k = 0; k < W29 / 4; ++k) d4[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
}
// value of lane (this lane ^ 1), every lane of the wave taking part
template <class Q>
KZ_DEV X29<Q> x29_swap_pair(const X29<Q>& a) {
  X29<Q> o;
#pragma unroll
  for (int k = 0; k < Q::N; ++k) {
    o.x.v[k] = (uint32_t)__shfl_xor((int)a.x.v[k], 1);
    o.y.v[k] = (uint32_t)__shfl_xor((int)a.y.v[k], 1);
    o.zz.v[k] = (uint32_t)__shfl_xor((int)a.zz.v[k], 1);
    o.zzz.v[k] = (uint32_t)__shfl_xor((int)a.zzz.v[k], 1);
  }
  o.inf = __shfl_xor((int)a.inf, 1) != 0;
  return o;
}
template <class Cv, class Q>
KZ_DEV Xyzz<Cv> x29_to32(const X29<Q>& a) {
  using P = typename Cv::FpP;
  if (a.inf) return Xyzz<Cv>::inf();
  return {fp_from29<Q, P>(a.x), fp_from29<Q, P>(a.y), fp_from29<Q, P>(a.zz), fp_from29<Q, P>(a.zzz)};
}
// 2a (dbl-2008-s-1, a = 0).  Inputs within the record bounds; outputs x < 5.1p, y, zz, zzz <
// 1.01p.  BLS12-381 G1 has no 2-torsion (#E(Fp) is odd), so only O doubles to O.
template <class Q>
KZ_DEV X29<Q> x29_dbl(const X29<Q>& a) {
  using G = F29<Q>;
  if (a.inf) return a;
  const G U = add3_29(a.y, a.y, G::zero());  // < 32p
  const G V = sqr29(U);
  const G W = mul29(U, V);
  const G S = mul29(a.x, V);
  const G X2 = sqr29(a.x);
  const G M = add3_29(X2, X2, X2);           // < 3.03p
  X29<Q> o;
  o.x = sub29(sqr29(M), add3_29(S, S, G::zero()), Q::B4);                    // < 5.1p
  o.y = mul2_29(M, sub29(S, o.x, Q::B8), W, sub29(G::zero(), a.y, Q::B16));  // M (S - X3) - W Y
  o.zz = mul29(V, a.zz);
  o.zzz = mul29(W, a.zzz);
  o.inf = false;
  return o;
}

// a + b (add-2008-s, 12M + 2S with the Y3 pair sharing one reduction).  Inputs within the record
// bounds (x < 10p, y < 16p, zz, zzz < 2p); outputs x < 9.1p, y, zz, zzz < 1.01p -- inside them.
template <class Cv, class Q>
KZ_DEV X29<Q> x29_add(const X29<Q>& a, const X29<Q>& b) {
  using G = F29<Q>;
  if (a.inf) return b;
  if (b.inf) return a;
  const G U1 = mul29(a.x, b.zz), U2 = mul29(b.x, a.zz);    // < 1.01p
  const G S1 = mul29(a.y, b.zzz), S2 = mul29(b.y, a.zzz);
  const G P = sub29(U2, U1, Q::B2);                         // < 3.02p
  const G R = sub29(S2, S1, Q::B2);
  if (is_zero29(P)) {
    if (is_zero29(R)) return x29_dbl<Q>(a);  // equal points (rare)
    return {G::zero(), G::zero(), G::zero(), G::zero(), true};
  }
  const G PP = sqr29(P);
  const G PPP = mul29(P, PP);
  const G Q2 = mul29(U1, PP);
  X29<Q> o;
  o.x = sub29(sqr29(R), add3_29(PPP, Q2, Q2), Q::B8);                           // < 9.1p
  o.y = mul2_29(R, sub29(Q2, o.x, Q::B16), S1, sub29(G::zero(), PPP, Q::B8));  // R (Q - X3) - S1 PPP
  o.zz = mul29(mul29(a.zz, b.zz), PP);
  o.zzz = mul29(mul29(a.zzz, b.zzz), PPP);
  o.inf = false;
  return o;
}



// 2Q for an affine Q (rare path: the running sum equals the incoming point), bounds: qx < p,
// qy < ACC_NEG p in; out (BLS12-381) x < 10p, y < 10p, zz, zzz < 2p -- per curve in
// tools/gen_params29.py check_bounds, with the biases Q::DBL_*
// out of line: its temporaries would otherwise raise the loop's register peak.  ZZ, ZZZ go
// straight to the caller's LDS columns (stride 256 words) so that arguments and result fit the
// 32 argument/return VGPRs of a call -- a 56-word return travelled through scratch (304 B of
// private segment per lane for the whole accumulation grid).
template <class Q>
struct Xy29 {
  F29<Q> x, y;
};
template <class Q>
__device__ __noinline__ Xy29<Q> dbl_affine29(const F29<Q> qx, const F29<Q> qy, uint32_t* zz, uint32_t* zzz) {
  using G = F29<Q>;
  const G U = add3_29(qy, qy, G::zero());                             // BLS12-381 < 16p
  const G V = mul29(U, U);
  const G W = mul29(U, V);
  const G S = mul29(qx, V);
  const G X2 = mul29(qx, qx);
  const G M = add3_29(X2, X2, X2);                                    // < 6p
  Xy29<Q> o;
  o.x = sub29(mul29(M, M), add3_29(S, S, G::zero()), Q::DBL_X);         // BLS12-381 < 10p
  o.y = sub29(mul29(M, sub29(S, o.x, Q::DBL_QX)), mul29(W, qy), Q::DBL_Y);  // BLS12-381 < 10p
#pragma unroll
  for (int k = 0; k < Q::N; ++k) {
    zz[k * 256] = V.v[k];
    zzz[k * 256] = W.v[k];
  }
  return o;
}

// R29 mod p (Montgomery one) in registers from literal moves at the point of use: two limbs per
// asm statement (one s_nop pad each), nothing the compiler can hoist and keep live (or spill)
// across the accumulation loop.
template <class Q, int K>
KZ_DEV void one_pair(F29<Q>& r) {
  asm volatile("v_mov_b32 %0, %2\n\tv_mov_b32 %1, %3" : "=v"(r.v[2 * K]), "=v"(r.v[2 * K + 1])
               : "i"(Q::ONE[2 * K]), "i"(Q::ONE[2 * K + 1]));
}
template <class Q, int... K>
KZ_DEV F29<Q> one_literals(std::integer_sequence<int, K...>) {
  F29<Q> r;
  (one_pair<Q, K>(r), ...);
  if constexpr (Q::N % 2) asm volatile("v_mov_b32 %0, %1" : "=v"(r.v[Q::N - 1]) : "i"(Q::ONE[Q::N - 1]));
  return r;
}

// The mixed-addition loop.  Bounds (values, all normalised), BLS12-381: q.x < p, q.y < 8p;
// x < 10p; y < 16p; zz, zzz < 2p; products < 2p -- only two biased multiples of p (8p, 16p),
// so few constants stay live across the loop.  BN254 (R29 / p ~ 169, no such headroom): q.y <
// p, x < 5.2p, y < 3.2p, zz, zzz < 1.1p with the biases 1p..8p.  Each subtraction names its
// bias by role (Q::ACC_*), chosen and checked per curve by tools/gen_params29.py.  ZZ/ZZZ in
// LDS as in the 32-bit loop below.
template <class Cv>
KZ_DEV void acc_loop29(uint32_t start, uint32_t end, uint32_t total, uint32_t chunk, uint32_t cur,
                       const uint32_t* __restrict__ sorted_val, const uint32_t* __restrict__ sorted_key,
                       const uint32_t* __restrict__ pts29, uint32_t* __restrict__ acc29, uint32_t nb,
                       uint32_t nthreads) {
  using Q = Fp29Of<Cv>;
  using G = F29<Q>;
  constexpr int N = Q::N, W29 = kW29<Q>;
  __shared__ uint32_t s_zz[N][256], s_zzz[N][256];
  const uint32_t tx = threadIdx.x;
  auto ld = [tx](uint32_t (&a)[N][256]) {
    asm volatile("" ::: "memory");
    G r;
    _Pragma("unroll") for (int k = 0; k < N; ++k) r.v[k] = a[k][tx];
    return r;
  };
  auto st = [tx](uint32_t (&a)[N][256], const G& v) {
    _Pragma("unroll") for (int k = 0; k < N; ++k) a[k][tx] = v.v[k];
    asm volatile("" ::: "memory");
  };
  // one coordinate at a time (BLS12-381: 8-B stores, a coordinate is 14 words; BN254: 9 words,
  // 4-B aligned), zz = 0 marks infinity
  auto put = [](uint32_t* d, const G& a) {
    if constexpr (N % 2 == 0) {
      _Pragma("unroll") for (int k = 0; k < N / 2; ++k) reinterpret_cast<uint2*>(d)[k] = make_uint2(a.v[2 * k], a.v[2 * k + 1]);
    } else {
      _Pragma("unroll") for (int k = 0; k < N; ++k) d[k] = a.v[k];
    }
  };
  // Where a finished bucket goes: only the chunk's first bucket can have started in an earlier
  // chunk (first piece) and only its last can continue into a later one (last piece), so both
  // are decided from the neighbouring sorted keys at the chunk's ends -- no off/cnt loads in the
  // loop (a flush runs in most iterations of a wavefront: some lane changes bucket).
  const bool started_before = start > 0 && sorted_key[start - 1] == cur;
  bool first = true;
  auto flush = [&](const G& x, const G& y, uint32_t key, bool inf, bool ends_after) {
    const size_t rec = (first && started_before) ? (size_t)nb + chunk : ends_after ? (size_t)nb + nthreads + chunk : key;
    first = false;
    uint32_t* d = acc29 + rec * W29;
    put(d, x);
    put(d + N, y);
    put(d + 2 * N, inf ? G::zero() : ld(s_zz));
    put(d + 3 * N, ld(s_zzz));
  };
  G x = G::zero(), y = G::zero();
  bool inf = true;  // running sum = O: at every bucket start, and after P + (-P)
  // loads entry e's point (sign applied: -y as ACC_NEG - y; BLS12-381 8p - y)
  auto load_q = [&](uint32_t v, G& qx, G& qy) {
    load_pt29<Cv>(reinterpret_cast<const Affine<Cv>*>(pts29) + sv_point(v), qx, qy);
    if (v & 1) qy = sub29(G::zero(), qy, Q::ACC_NEG);
  };
  // The rare doubling (running sum == incoming point) leaves the hot loop: a call or the
  // doubling's temporaries inside it would raise the loop's register peak (a call there cost
  // ~48 spilled VGPRs at 4 waves); the outer loop does it and resumes at the next entry.
  uint32_t e = start;
  for (;;) {
    bool dbl = false;
    // The values stream 4 at a time (one 16-B load per 4 entries, issued an iteration ahead of
    // their use; chunks start 16-B aligned, acc_chunk_len): each lane walks its own run, so a
    // per-entry 4-B load re-fetched the run's sector from beyond L2 for most entries.  A bucket
    // change is the SV_FIRST bit of the value; the key is read only then (a flush).
    // (The 4 values in registers were spilled to scratch and back around the addition at 128
    // VGPRs: 177.1 vs 179.4 batch-verifies/s, profiles/r04/ab_acc_vq_lds.txt.)  The 4 values of a group land in LDS by an asynchronous global_load_lds_dwordx4, one group
    // ahead; no VGPR holds them across the addition.  With the lane slot from v_mbcnt and ONE
    // from literals (below) the loop has no scratch traffic at all and needs 123 VGPRs (180.4 vs
    // 179.4/s, profiles/r04/ab_acc_spill_free.txt).
    __shared__ uint4 s_vq[256];
    uint4* const vq_wave = &s_vq[tx & ~63u];  // each lane's 16 B land at vq_wave[lane]
    __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(sorted_val + (e & ~3u)), vq_wave, 16, 0, 0);
    for (; e < end; ++e) {
      const uint32_t j = e & 3u;
      // the lane's slot from v_mbcnt every iteration: a loop-invariant address VGPR was spilled
      // and reloaded from scratch around the addition
      uint32_t lane;
      asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
      const uint32_t v = reinterpret_cast<const uint32_t*>(&s_vq[(tx & ~63u) + lane])[j];
      if (j == 3) {
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): v is read before the next group lands over it
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const uint4*>(sorted_val + e + 1), vq_wave, 16, 0, 0);
      }
      if ((v & SV_FIRST) && e != start) {
        flush(x, y, cur, inf, false);
        inf = true;
        cur = sorted_key[e];
      }
      G qx, qy;
      load_q(v, qx, qy);
      if (inf) {
        x = qx;
        y = qy;
        {  // ONE from literal moves here: the constant held in VGPRs across the loop was spilled
          const G one = one_literals<Q>(std::make_integer_sequence<int, N / 2>{});
          st(s_zz, one);
          st(s_zzz, one);
        }
        inf = false;
        continue;
      }
      const G U2 = mul29(qx, ld(s_zz));
      const G S2 = mul29(qy, ld(s_zzz));
      const G P = sub29(U2, x, Q::ACC_P);  // BLS12-381 < 18p
      const G R = sub29(S2, y, Q::ACC_R);  // BLS12-381 < 18p
      if (is_zero29_mf(P)) {
        if (is_zero29_mf(R)) {
          dbl = true;
          break;
        }
        inf = true;
        continue;
      }
      const G PP = sqr29(P);
      const G PPP = mul29(P, PP);
      st(s_zz, mul29(ld(s_zz), PP));
      st(s_zzz, mul29(ld(s_zzz), PPP));
      const G Q2 = mul29(x, PP);
      const G X3 = sub3_29(sqr29(R), PPP, Q2, Q::ACC_X3);  // one carry pass; BLS12-381 < 10p
      // R (Q - X3) - Y1 PPP, with -PPP as ACC_PPP - PPP limb by limb (no carry pass; neg_lazy29)
      y = mul2_29(R, sub29(Q2, X3, Q::ACC_QX), y, neg_lazy29(PPP, Q::ACC_PPP));
      x = X3;
    }
    if (!dbl) break;
    G qx, qy;  // entry e: running sum := 2 q
    load_q(sorted_val[e], qx, qy);
    asm volatile("" ::: "memory");
    const Xy29<Q> d = dbl_affine29<Q>(qx, qy, &s_zz[0][tx], &s_zzz[0][tx]);
    asm volatile("" ::: "memory");
    x = d.x;
    y = d.y;
    ++e;
  }
  flush(x, y, cur, inf, end < total && sorted_key[end] == cur);
}

// Waves per SIMD the accumulation is compiled for (VGPR budget 512 / waves per lane); the host
// caps the grid at one resident round of CUs x 4 SIMDs x kAccWaves waves (api.hip).
// ZZ/ZZZ staged in LDS make 4 waves fit (the all-register 32-bit loop of round 1 needed 168
// VGPRs: 7.53 vs 7.28 ms, profiles/r01/acc_lds_ab.txt); radix 2^29: 4 waves at 128 VGPRs once the rare doubling left the hot loop (7 VGPRs spilled outside it);
// 3 waves / 167 VGPRs measured 6.94 vs 6.63 ms (profiles/r01/acc29_ab.txt).
#ifndef KZ_ACC29_WAVES
#define KZ_ACC29_WAVES 4
#endif
#ifndef KZ_ACC29_WAVES_BN  // BN254's 9-limb loop (A/B knob)
#define KZ_ACC29_WAVES_BN KZ_ACC29_WAVES
#endif
template <class Cv>
constexpr int kAccWaves = Cv::ID == 1 ? KZ_ACC29_WAVES_BN : KZ_ACC29_WAVES;

template <class Cv>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kAccWaves<Cv>))) k_accumulate(const uint32_t* __restrict__ total_p,
                                                    const uint32_t* __restrict__ sorted_val,
                                                    const uint32_t* __restrict__ sorted_key,
                                                    const uint32_t* __restrict__ off,
                                                    const uint32_t* __restrict__ cnt,
                                                    const Affine<Cv>* __restrict__ pts,
                                                    uint32_t* __restrict__ acc29, uint32_t nb,
                                                    uint32_t nchunks, uint32_t* __restrict__ next_chunk,
                                                    const uint32_t* __restrict__ lo_p,
                                                    uint32_t* __restrict__ crowd) {
  // the crowded-bucket list k_fixup appends to behind this launch starts empty (a store here
  // instead of a fill kernel between the two launches)
  if (crowd && blockIdx.x == 0 && threadIdx.x == 0) *crowd = 0u;
  // the entry range [lo, total) of this launch: the whole sorted list, or the sets of one MSM
  // (api.hip run_msm_core's split accumulation; no bucket crosses a set boundary, so the range
  // end is where the last bucket ends)
  const uint32_t total = *total_p;
  const uint32_t lo = lo_p ? *lo_p : 0u;
  {
    if (next_chunk) {
      // Work queue (large calls, Launch::accumulate): nchunks chunks, more than the launched
      // threads; every wavefront takes the next 64 consecutive chunks (one per lane, the same
      // layout as the static grid) until none is left.  Waves that start late -- behind another
      // slot's accumulation -- take fewer, so the last accumulation in flight ends on every CU
      // at about the same time instead of a whole chunk duration apart.  Every wave's loop ends
      // once the counter passes nchunks (a multiple of 64).
      const uint32_t len = acc_chunk_len(total - lo, nchunks);
      const uint32_t lane = threadIdx.x & 63u;
      for (;;) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(next_chunk, 64u);
        base = __shfl(base, 0);
        if (base >= nchunks) break;
        const uint32_t chunk = base + lane;
        const uint32_t start = lo + chunk * len;
        if (chunk * len < total - lo)
          acc_loop29<Cv>(start, min(start + len, total), total, chunk, sorted_key[start], sorted_val, sorted_key,
                         reinterpret_cast<const uint32_t*>(pts), acc29, nb, nchunks);
      }
      return;
    }
  }
  const uint32_t len = acc_chunk_len(total - lo, gridDim.x * blockDim.x);
  const uint32_t chunk = blockIdx.x * blockDim.x + threadIdx.x;
  if (chunk * len >= total - lo) return;
  const uint32_t start = lo + chunk * len;
  const uint32_t end = min(start + len, total);
  acc_loop29<Cv>(start, end, total, chunk, sorted_key[start], sorted_val, sorted_key,
                 reinterpret_cast<const uint32_t*>(pts), acc29, nb, gridDim.x * blockDim.x);
}

// A bucket cut into k + 1 pieces (its last piece in chunk c0, first pieces of chunks c0+1..c1,
// k = c1 - c0) is joined with k dependent additions.  Thread-serial, one costs ~25 us at the
// occupancy of these kernels; narrow top windows crowd hundreds of entries into a bucket (13-bit
// windows of a 255-bit scalar keep 8 bits in the top one: 2^17 terms in 257 buckets, k ~ 8), so
// buckets of k >= FIX_LP_FROM pieces are listed by k_fixup and joined by k_fixup_crowded, one wave
// per bucket in lane-parallel arithmetic (lpfield.hpp: ~1.5 us per addition).  (Before: a
// two-level thread-serial join, G - 1 + ceil(k / G) additions with G = ceil(sqrt k).)
constexpr uint32_t FIX_LP_FROM = 4;

// (bucket, continuation range) of chunk c when its first entry continues a bucket begun in an
// earlier chunk: false otherwise.  c0 = the bucket's first chunk, c1 = its last.
KZ_DEV bool fix_range(uint32_t c, uint32_t len, uint32_t lo, uint32_t total, const uint32_t* __restrict__ sorted_key,
                      const uint32_t* __restrict__ off, const uint32_t* __restrict__ cnt, uint32_t& key,
                      uint32_t& c0, uint32_t& c1) {
  if (c * len >= total - lo) return false;
  const uint32_t start = lo + c * len;
  key = sorted_key[start];
  const uint32_t o = off[key];  // >= lo: the launch's range holds whole buckets
  if (o >= start) return false;  // bucket starts inside this chunk
  c0 = (o - lo) / len;
  c1 = (o + cnt[key] - 1 - lo) / len;
  return true;
}

// joins the pieces of buckets that cross chunk boundaries (launched with the same grid as
// k_accumulate, so acc_chunk_len agrees).  The pieces and the bucket are radix-29 records of
// acc29 = [nb buckets | nthreads first pieces | nthreads last pieces], joined with the radix-29
// XYZZ addition and written back as the record k_reduce_segments reads.  Buckets of
// FIX_LP_FROM pieces or more go to the crowded list (crowd[0] = count, then (key, c0, c1)).
template <class Cv>
__global__ void __launch_bounds__(256) k_fixup(const uint32_t* __restrict__ total_p,
                                               const uint32_t* __restrict__ sorted_key,
                                               const uint32_t* __restrict__ off,
                                               const uint32_t* __restrict__ cnt, uint32_t* __restrict__ acc29,
                                               uint32_t nb, uint32_t* __restrict__ crowd,
                                               const uint32_t* __restrict__ lo_p) {
  KZ_TAIL_PRIO();
  const uint32_t total = *total_p;
  const uint32_t lo = lo_p ? *lo_p : 0u;  // the accumulation launch's range [lo, total)
  const uint32_t len = acc_chunk_len(total - lo, gridDim.x * blockDim.x);
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x + 1;
  uint32_t key, c0, c1;
  if (!fix_range(c, len, lo, total, sorted_key, off, cnt, key, c0, c1)) return;
  if (c0 != c - 1) return;  // a later continuation chunk: handled by c0+1
  if (c1 - c0 >= FIX_LP_FROM) {
    const uint32_t i = atomicAdd(&crowd[0], 1u);
    crowd[1 + 3 * i] = key;
    crowd[2 + 3 * i] = c0;
    crowd[3 + 3 * i] = c1;
    return;
  }
  const size_t nthreads = (size_t)gridDim.x * blockDim.x;
  using Q = Fp29Of<Cv>;
  X29<Q> acc = load_x29<Q>(acc29, nb + nthreads + c0);
  for (uint32_t cc = c; cc <= c1; ++cc) acc = x29_add<Cv, Q>(acc, load_x29<Q>(acc29, nb + cc));
  store_x29<Q>(acc29, key, acc);
}

// a radix-29 record (load_x29 layout) <-> lane-parallel form.  BLS12-381: the record limbs are
// the lane limbs (R29 = R); BN254: x R29 <-> x R by one row-parallel product each way
template <class Cv>
KZ_DEV LpXyzz<Cv> lp_load_x29(const LpCtx<Cv>& c, const uint32_t* rec) {
  using Q = Fp29Of<Cv>;
  using LQ = LpQ<Cv>;
  const int j = threadIdx.x & 15;
  LpXyzz<Cv> p;
  p.x = j < Q::N ? (int32_t)rec[j] : 0;
  p.y = j < Q::N ? (int32_t)rec[Q::N + j] : 0;
  p.zz = j < Q::N ? (int32_t)rec[2 * Q::N + j] : 0;
  p.zzz = j < Q::N ? (int32_t)rec[3 * Q::N + j] : 0;
  p.inf = __builtin_amdgcn_ballot_w64(p.zz != 0) == 0;  // zz = 0 marks infinity (store_x29)
  if constexpr (LQ::N != Q::N) {
    int32_t from29 = 0;
#pragma unroll
    for (int q = 0; q < LQ::N; ++q)
      if (j == q) from29 = (int32_t)LQ::FROM29[q];
    lp_step4(c, p.x, p.x, from29, p.y, p.y, from29, p.zz, p.zz, from29, p.zzz, p.zzz, from29);
  }
  return p;
}
template <class Cv>
KZ_DEV void lp_store_x29(const LpCtx<Cv>& c, uint32_t* rec, const LpXyzz<Cv>& p) {
  using Q = Fp29Of<Cv>;
  using LQ = LpQ<Cv>;
  int32_t v[4] = {p.x, p.y, p.zz, p.zzz};
  if constexpr (LQ::N != Q::N) {
    const int j = threadIdx.x & 15;
    int32_t to29 = 0;
#pragma unroll
    for (int q = 0; q < LQ::N; ++q)
      if (j == q) to29 = (int32_t)LQ::TO29[q];
    lp_step4(c, v[0], v[0], to29, v[1], v[1], to29, v[2], v[2], to29, v[3], v[3], to29);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    int64_t l[LQ::N];
    lp_canon<Cv>(v[k], l);  // canonical limbs, uniform over the wave
    if ((threadIdx.x & 63) == 0) {
#pragma unroll
      for (int i = 0; i < Q::N; ++i) rec[k * Q::N + i] = (k == 2 && p.inf) ? 0u : (uint32_t)l[i];
    }
  }
}

// the crowded buckets listed by k_fixup: one wave per bucket, its pieces added in lane-parallel
// arithmetic; any grid (waves stride over the list)
template <class Cv>
__global__ void __launch_bounds__(256) k_fixup_crowded(const uint32_t* __restrict__ crowd, uint32_t* __restrict__ acc29,
                                                       uint32_t nb, uint32_t nthreads) {
  KZ_TAIL_PRIO();
  constexpr int W29 = kW29<Fp29Of<Cv>>;
  const uint32_t n = (uint32_t)__builtin_amdgcn_readfirstlane((int)crowd[0]);
  const uint32_t nwaves = gridDim.x * (blockDim.x / 64);
  const LpCtx<Cv> c = lp_ctx<Cv>();
  for (uint32_t i = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64; i < n; i += nwaves) {
    const uint32_t key = (uint32_t)__builtin_amdgcn_readfirstlane((int)crowd[1 + 3 * i]);
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)crowd[2 + 3 * i]);
    const uint32_t c1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)crowd[3 + 3 * i]);
    LpXyzz<Cv> acc = lp_load_x29(c, acc29 + ((size_t)nb + nthreads + c0) * W29);
    for (uint32_t cc = c0 + 1; cc <= c1; ++cc) acc = lp_xyzz_add(c, acc, lp_load_x29(c, acc29 + ((size_t)nb + cc) * W29));
    lp_store_x29(c, acc29 + (size_t)key * W29, acc);
  }
}

// Bucket stores of two accumulations over the same sets (the point ranges of a chunked
// host-buffer batch, api.hip enqueue_batch_chunked): A[b] += B[b] where B's bucket is non-empty,
// counts added (the reduction only tests them for zero); empty buckets' records are never read.
template <class Cv>
__global__ void __launch_bounds__(256) k_merge_buckets(uint32_t nb, uint32_t* __restrict__ acc29,
                                                       uint32_t* __restrict__ cnt,
                                                       const uint32_t* __restrict__ acc29b,
                                                       const uint32_t* __restrict__ cntb) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint32_t kb = cntb[b];
  if (!kb) return;
  using Q = Fp29Of<Cv>;
  const uint32_t ka = cnt[b];
  const X29<Q> y = load_x29<Q>(acc29b, b);
  store_x29<Q>(acc29, b, ka ? x29_add<Cv, Q>(load_x29<Q>(acc29, b), y) : y);
  cnt[b] = ka + kb;
}

// ------------------------------------------------------------------------------ reduction
// Segment g covers buckets [g*SEG, (g+1)*SEG) of one set (SEG divides NBUCKETS).  Two threads
// per segment (adjacent lanes): half h runs the running sums over buckets [8h, 8h + 8) of the
// segment -- R_h = sum_{i<8} i S_{8h+i}, U_h = sum_{i<8} S_{8h+i} -- and after one exchange
//   R'_g = R_0 + R_1,  U_g = U_0 + U_1,  V_g = U_1  (records R, U and V = U + nseg)
// so that sum_i i S_{g*SEG+i} = R'_g + 8 V_g; the 8 V_g term is summed over all segments in
// k_reduce_bits and scaled once in k_reduce_bits_finish.  (Forming R_1 + 8 U_1 here put three
// doublings on the upper half's chain while the lower half idled: ~20 point operations per
// wave instead of ~16; the kernel is latency-bound at 1.5 waves per SIMD.)
// LOWP (the reduction and combination kernels): no raised issue priority -- the side stream of a
// split accumulation runs them beside the critical-path accumulation (api.hip run_msm_core)
template <class Cv, bool LOWP = false>
__global__ void __launch_bounds__(256, 2) k_reduce_segments(uint32_t nseg, const uint32_t* __restrict__ cnt,
                                                         const uint32_t* __restrict__ acc29,
                                                         Xyzz<Cv>* __restrict__ R, Xyzz<Cv>* __restrict__ U) {
  static_assert(SEG == 16, "two 8-bucket halves per segment");
  if constexpr (!LOWP) KZ_TAIL_PRIO();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = t >> 1, h = t & 1;
  using Q = Fp29Of<Cv>;  // radix 2^29 on the records; R, U written as records
  const X29<Q> O{F29<Q>::zero(), F29<Q>::zero(), F29<Q>::zero(), F29<Q>::zero(), true};
  X29<Q> run = O, acc = O;
  if (g < nseg) {
    const uint32_t base = g * SEG + 8 * h;
    for (int i = 7; i >= 1; --i) {
      if (cnt[base + i]) run = x29_add<Cv, Q>(run, load_x29<Q>(acc29, base + i));
      acc = x29_add<Cv, Q>(acc, run);
    }
    if (cnt[base]) run = x29_add<Cv, Q>(run, load_x29<Q>(acc29, base));
  }
  // h = 0 needs the partner's R_1, h = 1 the partner's U_0 (adjacent lanes, whole wave)
  const X29<Q> other = x29_swap_pair<Q>(h ? acc : run);
  if (g >= nseg) return;
  if (h == 0) {
    store_x29<Q>(reinterpret_cast<uint32_t*>(R), g, x29_add<Cv, Q>(acc, other));
  } else {
    store_x29<Q>(reinterpret_cast<uint32_t*>(U), g, x29_add<Cv, Q>(run, other));
    store_x29<Q>(reinterpret_cast<uint32_t*>(U), (size_t)nseg + g, run);  // V_g = U_1
  }
}

// The same records from 4 threads per segment (lanes 4g .. 4g + 3), for calls with few bucket
// sets -- the critical path of a split accumulation reduces only MSM#0's 8 sets (api.hip
// run_msm_core), ~0.5 waves per SIMD with 2 threads per segment, so the segment's serial chain
// sets the time.  Quarter h runs the running sums over buckets [4h, 4h + 4): r_h = sum_{i<4} i
// S_{4h+i}, u_h = sum_{i<4} S_{4h+i}; then, with V_3 = u_3, V_2 = u_2 + u_3, V_1 = u_1 + V_2,
//   sum_i i S_{g SEG + i} = sum_h (r_h + 4 h u_h) = R'_g + 4 V_g,   R'_g = sum_h r_h,
//   V_g = V_1 + V_2 + V_3,   U_g = u_0 + V_1
// in three exchange steps of one addition per lane: 7 + 3 serial additions per segment instead
// of 15 + 1.  The deferred scale of sum V_g is 4 (k_reduce_bits_finish<..., 4>).
// the value of lane `src` (every lane takes part), word by word so no second whole record is
// live (the reduction kernels sit at 256 VGPRs)
template <class Q>
KZ_DEV X29<Q> x29_from_lane(const X29<Q>& a, int src) {
  X29<Q> o;
#pragma unroll
  for (int k = 0; k < Q::N; ++k) {
    o.x.v[k] = (uint32_t)__shfl((int)a.x.v[k], src);
    o.y.v[k] = (uint32_t)__shfl((int)a.y.v[k], src);
    o.zz.v[k] = (uint32_t)__shfl((int)a.zz.v[k], src);
    o.zzz.v[k] = (uint32_t)__shfl((int)a.zzz.v[k], src);
  }
  o.inf = __shfl((int)a.inf, src) != 0;
  return o;
}
// lane `src`'s a1 where that lane has `c1`, else its a0 -- the select done word by word before the
// shuffle
template <class Q>
KZ_DEV X29<Q> x29_from_lane_sel(bool c1, const X29<Q>& a1, const X29<Q>& a0, int src) {
  X29<Q> o;
#pragma unroll
  for (int k = 0; k < Q::N; ++k) {
    o.x.v[k] = (uint32_t)__shfl((int)(c1 ? a1.x.v[k] : a0.x.v[k]), src);
    o.y.v[k] = (uint32_t)__shfl((int)(c1 ? a1.y.v[k] : a0.y.v[k]), src);
    o.zz.v[k] = (uint32_t)__shfl((int)(c1 ? a1.zz.v[k] : a0.zz.v[k]), src);
    o.zzz.v[k] = (uint32_t)__shfl((int)(c1 ? a1.zzz.v[k] : a0.zzz.v[k]), src);
  }
  o.inf = __shfl((int)(c1 ? a1.inf : a0.inf), src) != 0;
  return o;
}
template <class Q>
KZ_DEV void x29_swap_if(bool c, X29<Q>& a, X29<Q>& b) {
#pragma unroll
  for (int k = 0; k < Q::N; ++k) {
    uint32_t t = a.x.v[k]; a.x.v[k] = c ? b.x.v[k] : t; b.x.v[k] = c ? t : b.x.v[k];
    t = a.y.v[k]; a.y.v[k] = c ? b.y.v[k] : t; b.y.v[k] = c ? t : b.y.v[k];
    t = a.zz.v[k]; a.zz.v[k] = c ? b.zz.v[k] : t; b.zz.v[k] = c ? t : b.zz.v[k];
    t = a.zzz.v[k]; a.zzz.v[k] = c ? b.zzz.v[k] : t; b.zzz.v[k] = c ? t : b.zzz.v[k];
  }
  const bool t = a.inf;
  a.inf = c ? b.inf : t;
  b.inf = c ? t : b.inf;
}
// each step: one shuffle into b, lanes that add nothing get b = O, then acc += b on every lane
// (swaps put each lane's addend into acc first)
template <class Cv, bool LOWP = false>
__global__ void __launch_bounds__(256, 2) k_reduce_segments4(uint32_t nseg, const uint32_t* __restrict__ cnt,
                                                          const uint32_t* __restrict__ acc29,
                                                          Xyzz<Cv>* __restrict__ R, Xyzz<Cv>* __restrict__ U) {
  static_assert(SEG == 16, "four 4-bucket quarters per segment");
  if constexpr (!LOWP) KZ_TAIL_PRIO();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = t >> 2, h = t & 3;
  const int lane = (int)(threadIdx.x & 63u), q0 = lane & ~3;  // the segment's first lane in the wave
  using Q = Fp29Of<Cv>;
  const X29<Q> O{F29<Q>::zero(), F29<Q>::zero(), F29<Q>::zero(), F29<Q>::zero(), true};
  X29<Q> run = O, acc = O;  // u_h, r_h
  if (g < nseg) {
    const uint32_t base = g * SEG + 4 * h;
    for (int i = 3; i >= 1; --i) {
      if (cnt[base + i]) run = x29_add<Cv, Q>(run, load_x29<Q>(acc29, base + i));
      acc = x29_add<Cv, Q>(acc, run);
    }
    if (cnt[base]) run = x29_add<Cv, Q>(run, load_x29<Q>(acc29, base));
  }
  // step 1 -- lane 0: r0 + r1; lane 2: V2 = u2 + u3; lane 3: r3 + r2 (lane 2 holds u2 in acc)
  x29_swap_if<Q>(h == 2, acc, run);
  {
    const int src = q0 + (h == 0 ? 1 : h == 2 ? 3 : h == 3 ? 2 : 1);
    X29<Q> b = x29_from_lane_sel<Q>(h >= 2, run, acc, src);  // lanes 2, 3 export run (r2, u3)
    b.inf = b.inf || h == 1;
    acc = x29_add<Cv, Q>(acc, b);
  }
  // step 2 -- lane 0: R' = (r0 + r1) + (r2 + r3); lane 1: V1 = u1 + V2; lane 3: V2 + V3 = u3 + V2
  {
    const int src = q0 + (h == 0 ? 3 : 2);
    X29<Q> b = x29_from_lane<Q>(acc, src);
    b.inf = b.inf || h == 2;
    x29_swap_if<Q>((h & 1) != 0, acc, run);  // lanes 1, 3 add into u1, u3
    acc = x29_add<Cv, Q>(acc, b);
  }
  // step 3 -- lane 0: U = u0 + V1; lane 1: V = V1 + (V2 + V3)
  {
    const int src = q0 + (h == 0 ? 1 : 3);
    X29<Q> b = x29_from_lane<Q>(acc, src);
    b.inf = b.inf || h >= 2;
    x29_swap_if<Q>(h == 0, acc, run);  // lane 0: acc = u0, run = R'
    acc = x29_add<Cv, Q>(acc, b);
  }
  if (g >= nseg) return;
  if (h == 0) {
    store_x29<Q>(reinterpret_cast<uint32_t*>(R), g, run);
    store_x29<Q>(reinterpret_cast<uint32_t*>(U), g, acc);
  } else if (h == 1) {
    store_x29<Q>(reinterpret_cast<uint32_t*>(U), (size_t)nseg + g, acc);  // V_g
  }
}

// Window sums with a short dependency chain (~40 point operations per set; the earlier one
// workgroup per set with three serial 16-term segment levels needed ~130, 3.8 vs 1.2 ms):
//   W = sum_g (R'_g + U_g) + 8 sum_g V_g + SEG * sum_g g U_g,   sum_g g U_g = sum_j 2^j B_j,
//   B_j = sum of the NSEG / 2 U_g whose index g has bit j set (j < SEG_BITS: 11 for c = 16).
// k_reduce_bits: RB_PARTS workgroups per set -- SEG_BITS compute B_j, 4 compute quarter sums of
// R'_g + U_g, 2 compute half sums of V_g -- each a few points per thread (c = 16: 4), two levels
// of a thread-serial LDS tree, then 6 levels in lane-parallel arithmetic (single-batch reduce
// phase 0.853 -> 0.759 ms at 2^20, 0.55 -> 0.42 ms at 2^17: profiles/r05/ab_reduce_bits_lp.txt).  k_reduce_bits_finish: one wave per set, Horner over the bit sums, then
// 2 H + sum V, 3 doublings: 16 H + 8 sum V.
constexpr int RB_PARTS = Win<WBITS>::RB_PARTS;  // c = 16 (the most parts per set)

template <class Cv, int WB = WBITS, bool LOWP = false>
__global__ void __launch_bounds__(256) k_reduce_bits(const Xyzz<Cv>* __restrict__ R, const Xyzz<Cv>* __restrict__ U,
                                                     Xyzz<Cv>* __restrict__ parts) {
  if constexpr (!LOWP) KZ_TAIL_PRIO();
  using Wn = Win<WB>;
  constexpr uint32_t NSEG = Wn::NSEG, SB = Wn::SEG_BITS, RBP = Wn::RB_PARTS;
  const uint32_t set = blockIdx.x / RBP, j = blockIdx.x % RBP;
  const uint32_t t = threadIdx.x;
  // the segment index of the q-th g (q < NSEG / 2) whose bit j is set
  auto bit_g = [j](uint32_t q) { return ((q >> j) << (j + 1)) | (1u << j) | (q & ((1u << j) - 1)); };
  {  // radix 2^29 on the R/U/V records, inline additions
    using Q = Fp29Of<Cv>;
    constexpr int N = Q::N, W29 = kW29<Q>;
    __shared__ uint32_t lds29[W29 + 1][128];
    const uint32_t* R29 = reinterpret_cast<const uint32_t*>(R) + (size_t)set * NSEG * W29;
    const uint32_t* U29 = reinterpret_cast<const uint32_t*>(U) + (size_t)set * NSEG * W29;
    const uint32_t nsets = gridDim.x / RBP;  // V records follow the nsets * NSEG U records
    const uint32_t* V29 = reinterpret_cast<const uint32_t*>(U) + ((size_t)nsets + set) * NSEG * W29;
    X29<Q> v{F29<Q>::zero(), F29<Q>::zero(), F29<Q>::zero(), F29<Q>::zero(), true};
    if (j >= SB + 4) {  // half sums of V_g
#pragma unroll 1
      for (uint32_t q = t; q < NSEG / 2; q += 256) v = x29_add<Cv, Q>(v, load_x29<Q>(V29, (j - SB - 4) * (NSEG / 2) + q));
    } else if (j < SB) {
#pragma unroll 1
      for (uint32_t q = t; q < NSEG / 2; q += 256) v = x29_add<Cv, Q>(v, load_x29<Q>(U29, bit_g(q)));
    } else {
      const uint32_t base = (j - SB) * (NSEG / 4);
#pragma unroll 1
      for (uint32_t q = t; q < NSEG / 4; q += 256) {
        v = x29_add<Cv, Q>(v, load_x29<Q>(R29, base + q));
        v = x29_add<Cv, Q>(v, load_x29<Q>(U29, base + q));
      }
    }
    // two levels of the thread-serial LDS tree (256 -> 64 sums), one coordinate word per row
    for (int st = 128; st >= 64; st >>= 1) {
      if (t >= (uint32_t)st && t < 2u * st) {
#pragma unroll
        for (int k = 0; k < N; ++k) {
          lds29[k][t - st] = v.x.v[k];
          lds29[N + k][t - st] = v.y.v[k];
          lds29[2 * N + k][t - st] = v.zz.v[k];
          lds29[3 * N + k][t - st] = v.zzz.v[k];
        }
        lds29[W29][t - st] = v.inf ? 1u : 0u;
      }
      __syncthreads();
      if (t < (uint32_t)st) {
        X29<Q> o;
#pragma unroll
        for (int k = 0; k < N; ++k) {
          o.x.v[k] = lds29[k][t];
          o.y.v[k] = lds29[N + k][t];
          o.zz.v[k] = lds29[2 * N + k][t];
          o.zzz.v[k] = lds29[3 * N + k][t];
        }
        o.inf = lds29[W29][t] != 0;
        v = x29_add<Cv, Q>(v, o);
      }
      __syncthreads();
    }
    // the last 6 levels (64 -> 1) in lane-parallel arithmetic, one point addition per wave at a
    // time: a thread-serial level costs one serial addition (~25 us at this occupancy), a
    // lane-parallel addition ~1.5 us, and the upper levels have few additions to spread
    constexpr int LPW = 4 * 16 + 1;  // a point: x, y, zz, zzz (16 lanes each), the infinity flag
    uint32_t(*lpn)[LPW] = reinterpret_cast<uint32_t(*)[LPW]>(&lds29[0][0]);
    static_assert(sizeof(lds29) >= sizeof(uint32_t) * 64 * LPW, "LDS for 64 lane-parallel points");
    if (t < 64) {  // radix-29 limbs as they are (zero above N)
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        lpn[t][k] = k < N ? v.x.v[k < N ? k : 0] : 0u;
        lpn[t][16 + k] = k < N ? v.y.v[k < N ? k : 0] : 0u;
        lpn[t][32 + k] = k < N ? v.zz.v[k < N ? k : 0] : 0u;
        lpn[t][48 + k] = k < N ? v.zzz.v[k < N ? k : 0] : 0u;
      }
      lpn[t][64] = v.inf ? 1u : 0u;
    }
    __syncthreads();
    const LpCtx<Cv> c = lp_ctx<Cv>();
    const uint32_t wave = t >> 6, lane16 = t & 15;
    auto lp_get = [&](uint32_t k) {
      LpXyzz<Cv> P;
      P.x = (int32_t)lpn[k][lane16];
      P.y = (int32_t)lpn[k][16 + lane16];
      P.zz = (int32_t)lpn[k][32 + lane16];
      P.zzz = (int32_t)lpn[k][48 + lane16];
      P.inf = __builtin_amdgcn_readfirstlane((int)lpn[k][64]) != 0;
      return P;
    };
    auto lp_put = [&](uint32_t k, const LpXyzz<Cv>& P) {
      if ((t & 63) < 16) {
        lpn[k][lane16] = (uint32_t)P.x;
        lpn[k][16 + lane16] = (uint32_t)P.y;
        lpn[k][32 + lane16] = (uint32_t)P.zz;
        lpn[k][48 + lane16] = (uint32_t)P.zzz;
      }
      if ((t & 63) == 0) lpn[k][64] = P.inf ? 1u : 0u;
    };
    if constexpr (LpQ<Cv>::N != N) {  // BN254: x R29 (R29 = 2^261) -> x R (2^290), one product step per point
      int32_t from29 = 0;
#pragma unroll
      for (int q = 0; q < LpQ<Cv>::N; ++q)
        if (lane16 == (uint32_t)q) from29 = (int32_t)LpQ<Cv>::FROM29[q];
#pragma unroll 1
      for (uint32_t k = wave; k < 64; k += 4) {
        LpXyzz<Cv> P = lp_get(k);
        lp_step4(c, P.x, P.x, from29, P.y, P.y, from29, P.zz, P.zz, from29, P.zzz, P.zzz, from29);
        lp_put(k, P);
      }
      __syncthreads();
    } else {
      static_assert(LpQ<Cv>::N == N, "BLS12-381: radix-29 record limbs are the lane-parallel limbs (R29 = R)");
    }
#pragma unroll 1
    for (uint32_t half = 32; half >= 1; half >>= 1) {
      // each sum q < half read and written by one wave; the sums >= half only read
#pragma unroll 1
      for (uint32_t q = wave; q < half; q += 4) lp_put(q, lp_xyzz_add(c, lp_get(q), lp_get(q + half)));
      __syncthreads();
    }
    if (wave == 0) lp_store_xyzz(c, &parts[(size_t)set * RBP + j], lp_get(0));
  }
}

// One wave per set, lane-parallel arithmetic (lpfield.hpp): Horner over the bit sums (c = 16:
// 10 XYZZ doublings + 10 additions), the 4 quarter sums, 4 doublings -- ~80 row-parallel
// product steps instead of ~330 serial products on one lane (0.71 ms before).
// SEGT: threads per segment of the records (k_reduce_segments: 2, sum V scaled by 8;
// k_reduce_segments4: 4, scaled by 4)
template <class Cv, int WB = WBITS, bool LOWP = false, int SEGT = 2>
__global__ void __launch_bounds__(64) k_reduce_bits_finish(const Xyzz<Cv>* __restrict__ parts,
                                                           Xyzz<Cv>* __restrict__ winsum) {
  static_assert(SEGT == 2 || SEGT == 4, "segment threads");
  if constexpr (!LOWP) KZ_TAIL_PRIO();
  using Wn = Win<WB>;
  constexpr int SB = Wn::SEG_BITS;
  const uint32_t set = blockIdx.x;
  const LpCtx<Cv> c = lp_ctx<Cv>();
  const Xyzz<Cv>* P = parts + (size_t)set * Wn::RB_PARTS;
  LpXyzz<Cv> V = lp_load_xyzz(c, &P[SB - 1]);
#pragma unroll 1
  for (int j = SB - 2; j >= 0; --j) V = lp_xyzz_add(c, lp_xyzz_dbl(c, V), lp_load_xyzz(c, &P[j]));
  LpXyzz<Cv> W = lp_xyzz_add(c, lp_xyzz_add(c, lp_load_xyzz(c, &P[SB]), lp_load_xyzz(c, &P[SB + 1])),
                             lp_xyzz_add(c, lp_load_xyzz(c, &P[SB + 2]), lp_load_xyzz(c, &P[SB + 3])));
  // 2 threads per segment: 16 H + 8 sum V = 8 (2 H + sum V); 4: 16 H + 4 sum V = 4 (4 H + sum V)
  if constexpr (SEGT == 4) V = lp_xyzz_dbl(c, V);
  V = lp_xyzz_add(c, lp_xyzz_dbl(c, V), lp_xyzz_add(c, lp_load_xyzz(c, &P[SB + 4]), lp_load_xyzz(c, &P[SB + 5])));
#pragma unroll 1
  for (int i = 0; i < (SEGT == 4 ? 2 : 3); ++i) V = lp_xyzz_dbl(c, V);
  lp_store_xyzz(c, &winsum[set], lp_xyzz_add(c, W, V));
}

// Horner over windows for each MSM: res[m] = sum_w 2^(c w) winsum[set_base_m + w]
struct MsmWindows {
  uint32_t nmsm;
  uint32_t set_base[2];
  uint32_t nwin[2];
};
// One wave per MSM, lane-parallel arithmetic (lpfield.hpp): the running sum stays in XYZZ through
// the c doublings of a step (dbl-2008-s-1: 3 row-parallel product steps, as many as the a = 0
// Jacobian doubling) and takes the window sum with no coordinate change: 52 product steps per
// 16-bit window against 57 with a Jacobian running sum (+ 2 steps to XYZZ and 3 back around each
// addition).  ~52 steps per window instead of ~134 serial products (3.9 ms for 16 windows before).
template <class Cv, int WB = WBITS, bool LOWP = false>
__global__ void __launch_bounds__(64) k_window_combine(MsmWindows mw, const Xyzz<Cv>* __restrict__ winsum,
                                                       Xyzz<Cv>* __restrict__ res) {
  if constexpr (!LOWP) KZ_TAIL_PRIO();
  const uint32_t m = blockIdx.x;
  const LpCtx<Cv> c = lp_ctx<Cv>();
  const Xyzz<Cv>* W = winsum + mw.set_base[m];
  LpXyzz<Cv> acc = lp_load_xyzz(c, &W[mw.nwin[m] - 1]);
#pragma unroll 1
  for (int w = (int)mw.nwin[m] - 2; w >= 0; --w) {
    const LpXyzz<Cv> ws = lp_load_xyzz(c, &W[w]);
#pragma unroll 1
    for (int i = 0; i < WB; ++i) acc = lp_xyzz_dbl(c, acc);
    acc = lp_xyzz_add(c, acc, ws);
  }
  lp_store_xyzz(c, &res[m], acc);
}

}  // namespace kzgmi
