// Small MSMs (a few hundred terms, e.g. configs[0]'s 256-tuple batch): one wave per term computes
// [k]P in lane-parallel arithmetic (lpfield.hpp) and the waves sum their results up a binary tree
// with arrival counters -- no sort, no buckets, no bucket-sum reduction.
//
// Why: the bucket method's fixed costs do not shrink with n.  A 256-tuple batch (769 terms) still
// reduced 24 sets x 2^15 buckets (0.86 ms, latency-bound chains) and combined 16 windows (0.37 ms)
// for 8 K entries.  Here the latency is one scalar multiplication (a 255-bit signed radix-16
// double-and-add: ~256 XYZZ doublings of 3 row-parallel product steps and ~64 additions of 4) plus
// log2(terms) tree additions; the terms' waves run side by side on the chip's 1024 SIMDs.
//
// Tree: MSM m's terms are leaves 0 .. c_m - 1; at level L node v covers leaves [v 2^L, (v+1) 2^L).
// A wave holding node v's sum stores it, releases, and bumps its parent's counter; the second of
// two siblings to arrive adds the first's stored sum and climbs on; a node without a sibling
// climbs alone.  No wave ever waits for another (no spinning): the grid drains in any schedule.
// The root's wave writes res[m] (XYZZ, field.hpp form).  Points: the slot's radix-2^29 slots
// (BLS12-381: 14 limbs of x then y, the lane-parallel limb layout with the same R = 2^406;
// BN254: x 2^261, y 2^261 packed in 32-bit words, one product each into the 2^290 form).
// Reference: none (LICENSE only); the same sums as the bucket path (bit-exact A, B and MSM results
// in every small-n parity test).
#pragma once
#include "lpfield.hpp"
#include "msm.hpp"

namespace kzgmi {

// term classes of a small call: class k's terms are blocks [term_base[k], term_base[k] + count)
// and leaves [leaf_base[k], ...) of MSM msm[k]
struct SmallPlan {
  uint32_t nclass, nmsm;
  uint32_t term_base[MAX_CLASSES];
  uint32_t leaf_base[MAX_CLASSES];
  uint32_t msm[MAX_CLASSES];
  uint32_t count[2];       // leaves per MSM
  uint32_t node_base[2];   // first stored node of each MSM (levels back to back)
  uint32_t flag_base[2];   // first arrival counter of each MSM
};

// a stored tree node: row 0's 16 lanes of x, y, zz, zzz, then the infinity flag
constexpr int SMALL_NODE_WORDS = 4 * 16 + 4;

template <class Cv>
KZ_DEV void small_store(uint32_t* node, const LpXyzz<Cv>& p) {
  const int t = threadIdx.x;
  if (t < 16) {
    node[t] = (uint32_t)p.x;
    node[16 + t] = (uint32_t)p.y;
    node[32 + t] = (uint32_t)p.zz;
    node[48 + t] = (uint32_t)p.zzz;
  }
  if (t == 0) node[64] = p.inf ? 1u : 0u;
}
template <class Cv>
KZ_DEV LpXyzz<Cv> small_load(const uint32_t* node) {
  const int j = threadIdx.x & 15;  // every row takes the same value (lane-parallel convention)
  LpXyzz<Cv> p;
  p.x = (int32_t)node[j];
  p.y = (int32_t)node[16 + j];
  p.zz = (int32_t)node[32 + j];
  p.zzz = (int32_t)node[48 + j];
  p.inf = __builtin_amdgcn_readfirstlane((int)node[64]) != 0;
  return p;
}

// 5 bits of the scalar ending at bit pos + 3 (pos may be -1 .. 4W - 1): b_{pos+3} .. b_{pos-1}
template <int NW>
KZ_DEV uint32_t small_bits(const uint32_t (&k)[NW], int lo) {  // bits lo .. lo + 4 (lo >= -1)
  uint64_t v = 0;
  const int w = lo < 0 ? 0 : lo >> 5, s = lo < 0 ? 0 : lo & 31;
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    if (i == w) v |= (uint64_t)k[i];
    if (i == w + 1) v |= (uint64_t)k[i] << 32;
  }
  const uint32_t b = (uint32_t)(v >> s);
  return lo < 0 ? (b << 1) & 0x1fu : b & 0x1fu;
}

// [k]P, k < 2^(32 NW), signed radix-16 (Booth) digits d_w = -8 b_{4w+3} + 4 b_{4w+2} + 2 b_{4w+1}
// + b_{4w} + b_{4w-1} in [-8, 8], top down; table 1P .. 8P
template <class Cv, int NW>
KZ_DEV LpXyzz<Cv> small_mul(const LpCtx<Cv>& c, const LpXyzz<Cv>& P, const uint32_t (&k)[NW]) {
  LpXyzz<Cv> T[8];
  T[0] = P;
  T[1] = lp_xyzz_dbl(c, P);
#pragma unroll 1
  for (int j = 2; j < 8; ++j) T[j] = lp_xyzz_add(c, T[j - 1], P);
  constexpr int W = 8 * NW + 1;  // windows (the last takes b_{32 NW - 1} alone)
  LpXyzz<Cv> acc = P;
  acc.inf = true;
  bool started = false;
#pragma unroll 1
  for (int w = W - 1; w >= 0; --w) {
    const uint32_t b = small_bits<NW>(k, 4 * w - 1);  // b_{4w-1} .. b_{4w+3}
    const int d = (int)((b >> 1) & 7u) + (int)(b & 1u) - 8 * (int)((b >> 4) & 1u);
    if (started) {
#pragma unroll 1
      for (int i = 0; i < 4; ++i) acc = lp_xyzz_dbl(c, acc);
    }
    if (d != 0) {
      const int a = (d < 0 ? -d : d) - 1;
      LpXyzz<Cv> q = T[0];
#pragma unroll
      for (int j = 1; j < 8; ++j)
        if (a == j) q = T[j];
      if (d < 0) q.y = lp_sub(c, 0, q.y);
      acc = started ? lp_xyzz_add(c, acc, q) : q;
      started = true;
    }
  }
  return acc;
}

template <class Cv>
__global__ void __launch_bounds__(64) k_small_msm(TermList tl, SmallPlan sp, const Affine<Cv>* __restrict__ pts,
                                                  const uint8_t* __restrict__ inf, uint32_t* __restrict__ nodes,
                                                  uint32_t* __restrict__ flags, Xyzz<Cv>* __restrict__ res) {
  using Q = Fp29Of<Cv>;
  using LQ = LpQ<Cv>;
  KZ_TAIL_PRIO();
  const LpCtx<Cv> c = lp_ctx<Cv>();
  const uint32_t t = blockIdx.x, j = threadIdx.x & 15;
  uint32_t k = 0;
#pragma unroll 1
  for (uint32_t q = 1; q < sp.nclass; ++q)
    if (t >= sp.term_base[q]) k = q;
  const TermClass& C = tl.c[k];
  const uint32_t i = t - sp.term_base[k];
  const uint32_t m = sp.msm[k];
  uint32_t v = sp.leaf_base[k] + i;  // leaf of MSM m
  // the term's point in the accumulation's slot format (msm.hpp load_pt29) and scalar (uniform words)
  const uint32_t pi = C.pt_base + i;
  const uint32_t* slot = reinterpret_cast<const uint32_t*>(pts + pi);
  int32_t one = 0, from29 = 0;  // per-lane limbs of R mod p and R^2 / R29 mod p
#pragma unroll
  for (int q = 0; q < LQ::N; ++q)
    if (j == (uint32_t)q) {
      one = (int32_t)LQ::ONE[q];
      from29 = (int32_t)LQ::FROM29[q];
    }
  LpXyzz<Cv> P;
  if constexpr (kPackPts<Cv>) {  // BN254: x R29, y R29 as 32-bit words; R29 = 2^261, R = 2^290
    lp_step2(c, P.x, lp_raw_from_words<Cv>(slot), from29, P.y, lp_raw_from_words<Cv>(slot + Cv::FpP::N), from29);
  } else {  // BLS12-381: 14 radix-29 limbs of x, then of y; R29 = R = 2^406, the limbs as they are
    static_assert(Q::N == LQ::N, "radix-29 slot limbs are the lane-parallel limbs");
    P.x = j < (uint32_t)Q::N ? (int32_t)slot[j] : 0;
    P.y = j < (uint32_t)Q::N ? (int32_t)slot[Q::N + j] : 0;
  }
  P.zz = P.zzz = one;
  P.inf = inf[pi] != 0;
  const uint32_t* sw = C.scal + (size_t)C.scal_stride * i;
  LpXyzz<Cv> acc;
  if (C.scal_words == 8) {
    uint32_t kk[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) kk[q] = (uint32_t)__builtin_amdgcn_readfirstlane((int)sw[q]);
    acc = small_mul<Cv, 8>(c, P, kk);
  } else {
    // 4-word scalars are sign-magnitude: bit 127 is the sign (GLV half scalars; msm.hpp term_digits)
    uint32_t kk[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) kk[q] = (uint32_t)__builtin_amdgcn_readfirstlane((int)sw[q]);
    const bool neg = (kk[3] >> 31) != 0;
    kk[3] &= 0x7fffffffu;
    acc = small_mul<Cv, 4>(c, P, kk);
    if (neg) acc.y = lp_sub(c, 0, acc.y);
  }
  if (P.inf) acc.inf = true;
  // climb the tree
  uint32_t cnt = sp.count[m], node = sp.node_base[m], flag = sp.flag_base[m];
#pragma unroll 1
  while (cnt > 1) {
    const uint32_t partner = v ^ 1u;
    if (partner < cnt) {
      small_store<Cv>(nodes + (size_t)(node + v) * SMALL_NODE_WORDS, acc);
      __threadfence();
      uint32_t old = 0;
      if (threadIdx.x == 0)
        old = __hip_atomic_fetch_add(flags + flag + (v >> 1), 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      old = (uint32_t)__builtin_amdgcn_readfirstlane((int)old);
      if (old == 0) return;  // the sibling's wave carries on
      __threadfence();
      acc = lp_xyzz_add(c, acc, small_load<Cv>(nodes + (size_t)(node + partner) * SMALL_NODE_WORDS));
    }
    node += cnt;
    flag += (cnt + 1) >> 1;
    v >>= 1;
    cnt = (cnt + 1) >> 1;
  }
  lp_store_xyzz(c, &res[m], acc);
}

}  // namespace kzgmi
