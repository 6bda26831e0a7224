// ARCHIVED EXPERIMENT (not built): radix-2^28 accumulation, measured slower in situ -- see
// profiles/r01/probes/radix28.txt.  Needed the Fp28 constants tools/gen_params.py emitted then.
// Bucket accumulation in carry-free radix-2^28 arithmetic (field28.hpp): the same
// load-balanced chunking as k_accumulate (msm.hpp) -- each thread owns ACC_CHUNK consecutive
// sorted entries, bucket pieces cut by chunk boundaries go to part_first/part_last -- but
// the running bucket sums are lazily reduced radix-2^28 XYZZ points.  Inputs: the points in
// R28-Montgomery form (k_points_to28, canonical < p).  Outputs: canonical 32-bit-limb
// R32-Montgomery XYZZ records, so k_fixup and the bucket reduction are unchanged.
//
// Bounds (multiples of p; every mul28 input pair below has product < 100 p^2 << 2047 p^2):
//   bucket:  X < 8p, Y < 4p, ZZ < 2p, ZZZ < 2p        point (x2, y2): canonical < p
//   U2 = x2 ZZ, S2 = y2 ZZZ             < 2p
//   P = U2 + 8p - X  in (0, 10p)        R = S2 + 4p - Y  in (0, 6p)
//   PP = P^2, PPP = P PP, Q = X PP, RR = R^2            < 2p each
//   X3 = RR + 6p - PPP - 2Q in (0, 8p)   (RR + 6p - PPP > 4p > 2Q)
//   Y3 = R (Q + 8p - X3) + 2p - Y PPP in (0, 4p)
//   ZZ3 = ZZ PP, ZZZ3 = ZZZ PPP < 2p
// P == 0 mod p (the running sum equals +-Q) is tested on PP (< 2p: PP in {0, p}); such a
// chunk is handed to k_accumulate_redo (32-bit formulas with the doubling / infinity cases).
// A finite bucket never has ZZ = 0 or p, so zz == 0 exactly marks an empty running sum.
#pragma once
#include "field28.hpp"
#include "msm.hpp"

namespace kzgmi {

// y -> p - y for canonical y: in (0, p], which is all the bounds below need
template <class Q>
KZ_DEV F28<Q> neg28(const F28<Q>& y) {
  F28<Q> zero;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) zero.v[i] = 0;
  return sub28(zero, y, Q::MOD);
}

template <class Cv>
struct Acc28 {
  using F = F28<typename Cv::Fp28P>;
  F x, y, zz, zzz;
};
template <class Cv>
struct Aff28 {
  using F = F28<typename Cv::Fp28P>;
  F x, y;
};

// P + Q (Q affine).  Ordered so that each input coordinate dies as soon as it has been
// used (register pressure).  Returns false for the rare P == +-Q case (caller handles it).
template <class Cv>
KZ_DEV bool add28_affine(Acc28<Cv>& p, const Aff28<Cv>& q) {
  using Q = typename Cv::Fp28P;
  const auto P = sub28(mul28(q.x, p.zz), p.x, Q::P8);   // U2 + 8p - X
  const auto R = sub28(mul28(q.y, p.zzz), p.y, Q::P4);  // S2 + 4p - Y
  const auto PP = mul28(P, P);
  if (is_zero_lt2p(PP)) return false;
  const auto PPP = mul28(P, PP);
  p.zz = mul28(p.zz, PP);
  const auto Qv = mul28(p.x, PP);
  p.zzz = mul28(p.zzz, PPP);
  const auto YP = mul28(p.y, PPP);
  p.x = sub2_28(mul28(R, R), PPP, Qv, Q::P6);           // RR + 6p - PPP - 2Q
  p.y = sub28(mul28(R, sub28(Qv, p.x, Q::P8)), YP, Q::P2);
  return true;
}

// lazily reduced radix-2^28 coordinate (< 8p) -> canonical R32-Montgomery Fp
template <class Cv>
KZ_DEV Fp<typename Cv::FpP> to_r32(const F28<typename Cv::Fp28P>& a) {
  using Q = typename Cv::Fp28P;
  const auto c = canon_lt2p(mul28(a, F28<Q>::from_const(Q::TO32)));  // a R32 / R28 ... < 2p -> < p
  Fp<typename Cv::FpP> r;
  pack32<Q>(c, r.v);
  return r;
}

// store one bucket piece: each coordinate converted and written on its own (keeps the
// flush's register peak at the running sum plus one conversion)
template <class Cv>
KZ_DEV void acc28_flush(const Acc28<Cv>& acc, uint32_t key, uint32_t chunk, uint32_t start,
                        const uint32_t* __restrict__ off, const uint32_t* __restrict__ cnt,
                        Xyzz<Cv>* __restrict__ buckets, Xyzz<Cv>* __restrict__ part_first,
                        Xyzz<Cv>* __restrict__ part_last) {
  constexpr int N = Cv::FpP::N;
  const uint32_t o = off[key];
  const bool started_before = o < start;
  const bool ends_after = o + cnt[key] > start + ACC_CHUNK;
  Xyzz<Cv>* dst = started_before ? &part_first[chunk] : ends_after ? &part_last[chunk] : &buckets[key];
  uint4* d = reinterpret_cast<uint4*>(dst);
  auto put = [&](int c, const F28<typename Cv::Fp28P>& a) {
    const Fp<typename Cv::FpP> f = to_r32<Cv>(a);
    _Pragma("unroll") for (int k = 0; k < N / 4; ++k)
      d[c * (N / 4) + k] = make_uint4(f.v[4 * k], f.v[4 * k + 1], f.v[4 * k + 2], f.v[4 * k + 3]);
  };
  put(0, acc.x);
  put(1, acc.y);
  put(2, acc.zz);
  put(3, acc.zzz);
}

template <class Cv>
KZ_DEV Aff28<Cv> load_aff28(const uint32_t* __restrict__ pts28, uint32_t i) {
  constexpr int N = Cv::Fp28P::N;
  constexpr int W = 2 * N;  // words per point (28 BLS, 20 BN: multiples of 4)
  static_assert(W % 4 == 0, "16-byte granules");
  const uint4* src = reinterpret_cast<const uint4*>(pts28 + (size_t)i * W);
  uint32_t w[W];
  _Pragma("unroll") for (int k = 0; k < W / 4; ++k) {
    const uint4 q = src[k];
    w[4 * k] = q.x; w[4 * k + 1] = q.y; w[4 * k + 2] = q.z; w[4 * k + 3] = q.w;
  }
  Aff28<Cv> a;
  _Pragma("unroll") for (int k = 0; k < N; ++k) { a.x.v[k] = w[k]; a.y.v[k] = w[N + k]; }
  return a;
}

// entry value v = (point index << 1) | sign -> the (possibly negated) point
template <class Cv>
KZ_DEV Aff28<Cv> load_point28(const uint32_t* __restrict__ pts28, uint32_t v) {
  Aff28<Cv> q = load_aff28<Cv>(pts28, v >> 1);
  if (v & 1) q.y = neg28(q.y);
  return q;
}

// canonical R32-Montgomery affine points -> canonical R28-Montgomery (one mul28 per coordinate)
template <class Cv>
__global__ void __launch_bounds__(256) k_points_to28(const Affine<Cv>* __restrict__ pts, uint32_t n,
                                                     uint32_t* __restrict__ pts28) {
  using Q = typename Cv::Fp28P;
  constexpr int N = Q::N;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Affine<Cv> a = load_affine(pts, i);
  const auto k = F28<Q>::from_const(Q::TO28);
  const auto x = canon_lt2p(mul28(unpack28<Q>(a.x.v), k));
  const auto y = canon_lt2p(mul28(unpack28<Q>(a.y.v), k));
  uint32_t w[2 * N];
  _Pragma("unroll") for (int j = 0; j < N; ++j) { w[j] = x.v[j]; w[N + j] = y.v[j]; }
  uint4* d = reinterpret_cast<uint4*>(pts28 + (size_t)i * 2 * N);
  _Pragma("unroll") for (int j = 0; j < N / 2; ++j) d[j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
}

template <class Cv>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) k_accumulate28(const uint32_t* __restrict__ total_p,
                                                      const uint32_t* __restrict__ sorted_val,
                                                      const uint32_t* __restrict__ sorted_key,
                                                      const uint32_t* __restrict__ off,
                                                      const uint32_t* __restrict__ cnt,
                                                      const uint32_t* __restrict__ pts28,
                                                      Xyzz<Cv>* __restrict__ buckets,
                                                      Xyzz<Cv>* __restrict__ part_first,
                                                      Xyzz<Cv>* __restrict__ part_last,
                                                      uint32_t* __restrict__ redo) {
  using Q = typename Cv::Fp28P;
  const uint32_t total = *total_p;
  const uint32_t chunk = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t start = chunk * ACC_CHUNK;
  if (start >= total) return;
  const uint32_t end = min(start + ACC_CHUNK, total);
  Acc28<Cv> acc;
  _Pragma("unroll") for (int i = 0; i < Q::N; ++i) acc.x.v[i] = acc.y.v[i] = acc.zz.v[i] = acc.zzz.v[i] = 0;
  uint32_t cur = sorted_key[start];
  for (uint32_t e = start; e < end; ++e) {
    const uint32_t key = sorted_key[e];
    if (key != cur) {
      acc28_flush(acc, cur, chunk, start, off, cnt, buckets, part_first, part_last);
      _Pragma("unroll") for (int i = 0; i < Q::N; ++i) acc.zz.v[i] = 0;
      cur = key;
    }
    const uint32_t v = sorted_val[e];
    const Aff28<Cv> q = load_point28<Cv>(pts28, v);
    if (all_zero28(acc.zz)) {  // first point of a bucket piece
      acc.x = q.x;
      acc.y = q.y;
      acc.zz = acc.zzz = F28<Q>::from_const(Q::ONE);
    } else if (!add28_affine(acc, q)) {
      // P == +-Q (rare; every addition of a repeated point): hand the whole chunk to
      // k_accumulate_redo, which rewrites everything this chunk stores
      redo[1 + atomicAdd(redo, 1u)] = chunk;
      return;
    }
  }
  acc28_flush(acc, cur, chunk, start, off, cnt, buckets, part_first, part_last);
}

}  // namespace kzgmi
