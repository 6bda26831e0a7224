// kzgmi host orchestration + C-ABI (layers L3/L4 of SURVEY.md section 1).
//
// One translation unit: instantiates every kernel for BLS12-381 and BN254 and implements
// include/kzgmi.h.  Device memory lives in per-slot workspaces owned by the context and is
// grown on demand (never inside a timed steady state).  Every compute path is HIP-only:
// without a device the calls fail with KZGMI_ERR_DEVICE (no CPU fallback).
// Reference: none (LICENSE only); boundary contract = SURVEY.md 8b, BASELINE.json:5.
#include "launch.hpp"
#include "kzgmi.h"

#include <rocprofiler-sdk-roctx/roctx.h>

#include <sys/random.h>
#include <cstdio>
#define KZ_STR2(x) #x
#define KZ_STR(x) KZ_STR2(x)
#include <cstdlib>
#include <cstring>
#include <string>
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

using namespace kzgmi;

namespace {

thread_local std::string g_err = "";

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIPCHK(x)                                                                              \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) return fail(KZGMI_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define CHK(x)                  \
  do {                          \
    int r_ = (x);               \
    if (r_ != 0) return r_;     \
  } while (0)

// process-wide count of workspace (re)allocations: kzgmi_alloc_count(), so a caller (bench.py,
// tests) can check that kzgmi_ctx_reserve left nothing to allocate inside a timed region
std::atomic<uint64_t> g_allocs{0};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes == 0) bytes = 16;
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, bytes) != hipSuccess) return fail(KZGMI_ERR_OOM, "hipMalloc failed (" + std::to_string(bytes) + " bytes)");
    cap = bytes;
    g_allocs.fetch_add(1, std::memory_order_relaxed);
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T> T* as() const { return reinterpret_cast<T*>(p); }
};

// roctx range over a host-side scope (SURVEY.md 5 tracing): the enqueue of each batch phase and
// every blocking wait, visible in `rocprofv3 --marker-trace` beside the kernels they issue
struct Roctx {
  explicit Roctx(const char* m) { roctxRangePushA(m); }
  ~Roctx() { roctxRangePop(); }
  Roctx(const Roctx&) = delete;
  Roctx& operator=(const Roctx&) = delete;
};

// the batch phases in stream order, then "h2d": the host-to-HBM copy of a host-buffer call
// (kzgmi_batch_verify_ex_async), timed by its own pair of events
const char* const kPhaseNames = "convert,scalars,sort,accumulate,reduce,combine,pairing,h2d";
constexpr int kNumPhases = 8;
constexpr int kNumBatchPhases = 7;
enum Phase { PH_CONVERT = 0, PH_SCALARS, PH_SORT, PH_ACCUM, PH_REDUCE, PH_COMBINE, PH_PAIRING, PH_H2D };
constexpr int EV_H2D0 = kNumBatchPhases + 1, EV_H2D1 = kNumBatchPhases + 2;  // Slot::ev indices
constexpr size_t kRingBytes = size_t(16) << 20;  // pinned staging ring of pageable host inputs (x 2 per slot)

struct Slot {
  hipStream_t stream = nullptr;       // the slot's stream: every job on the slot is issued here
  hipEvent_t done_ev = nullptr;       // the slot's last job issued so far has completed
  bool done_rec = false;
  std::vector<hipEvent_t> dep_pool;   // entry dependencies of the slot's next job (kzgmi_stream_wait, the
  int ndep = 0;                        // H2D copy of host inputs): dep_pool[0, ndep)
  DevBuf pts, inf, scal_r, scal_s, scal_t, tpart, cnt, off, coarse, ent, total, sval, skey;
  DevBuf R, U, scratch, winsum, res, flags, stage, outb;
  DevBuf acc29;                                  // radix-29 bucket records (msm.hpp)
  DevBuf accq;                                   // k_accumulate's work-queue counter (large calls)
  DevBuf crowd;                                  // k_fixup's list of crowded buckets (msm.hpp k_fixup_crowded)
  DevBuf fs_leaves, fs_tmp, fs_top, pow, chal;  // Fiat-Shamir / powers-of-r randomisers
  DevBuf glv_r, glv_s, glv_t;                    // GLV half scalars (glv.hpp): [h0 x n | h1 x n]
  DevBuf digits;                                 // signed window digit codes of every term (msm.hpp)
  DevBuf small_nodes, small_flags;               // small calls' summation tree (msm_small.hpp)
  DevBuf acc29b, cntb, offb;                     // second bucket store of chunked batches (run_msm_core part)
  // split accumulation (run_msm_core): the second MSM's reduction and window combination run on
  // the context's side stream beside the first MSM's accumulation; side_ev[0] = its sets
  // accumulated, [1] = combined
  hipEvent_t side_ev[2] = {};
  int* host_flags = nullptr;  // pinned: [ok, err]
  uint8_t* host_out = nullptr;  // pinned: encoded MSM result of an async MSM job
  uint8_t* ring[2] = {};        // pinned staging of pageable host inputs (kRingBytes each, lazily)
  hipEvent_t ring_ev[2] = {};   // the DMA that last read ring[b]
  int ring_next = 0;
  hipEvent_t ev[kNumBatchPhases + 3] = {};  // phase marks 0..7, then the H2D pair
  hipEvent_t signal_ev = nullptr;  // kzgmi_slot_signal: this slot's stream -> the caller's stream
  bool ev_used[kNumBatchPhases + 3] = {};
  bool pending = false;
  bool partial_job = false;  // pending job produces a partial record, not a verdict
  int partial_of = 0;        // ... of a batch (1) or an MSM (2): a combine of that kind may chain behind it
  bool msm_job = false;      // pending job is an MSM whose encoded result lands in host_out
  int curve = 0;
  // every device buffer of the slot (kzgmi_ctx_destroy releases them all: a buffer added above
  // must be listed here)
  template <class F>
  void for_each_buf(F&& f) {
    DevBuf* bufs[] = {&pts, &inf, &scal_r, &scal_s, &scal_t, &tpart, &cnt, &off, &coarse, &ent, &total, &sval, &skey,
                      &R, &U, &scratch, &winsum, &res, &flags, &stage, &outb, &acc29, &accq, &crowd, &fs_leaves,
                      &fs_tmp, &fs_top, &pow, &chal, &glv_r, &glv_s, &glv_t, &digits, &small_nodes, &small_flags,
                      &acc29b, &cntb, &offb};
    for (DevBuf* b : bufs) f(*b);
  }
};

}  // namespace

struct kzgmi_ctx {
  int device = 0;
  std::vector<Slot> slots;
  int user_slots = 0;                   // slots in the caller's numbering (multi-device: over all devices)
  int prio_levels = 1;                  // stream priorities the slot streams cycle through
  bool profiling = false;
  // GLV split of full Fr scalars.  phi(P) = [lambda] P holds only on
  // G1, so BLS12-381 (cofactor > 1) uses it only for points known to be in G1: batch calls
  // with KZGMI_FLAG_SUBGROUP_CHECK or KZGMI_FLAG_TRUSTED_G1, MSMs after kzgmi_set_trusted_g1.
  // BN254 G1 is the whole curve (cofactor 1): always.
  bool glv_msm = true;      // enable knobs (kzgmi_set_glv; A/B measurements)
  bool glv_batch = true;
  bool msm_trusted_g1 = false;
  // accumulation grid cap: one resident round (CUs x 4 SIMDs x kAccWaves<Cv> waves x 64 lanes)
  // of equal chunks instead of 64-entry chunks in 2-3 partial rounds: 113 -> 116
  // batch-verifies/s pipelined when introduced (tools/ab.py).
  int ncu = 0;                // compute units: the accumulation grid cap (kAccWaves, msm.hpp)
  size_t acc_threads_env = 0;  // KZGMI_ACC_THREADS override of that cap (0 = none)
  int acc_queue = ACC_QUEUE_FACTOR;  // KZGMI_ACC_QUEUE: chunks per capped thread (<= 1: static grid)
  size_t acc_queue_min = ACC_QUEUE_MIN_LEN;  // KZGMI_ACC_QUEUE_MIN: shortest queue chunk (entries)
  size_t acc_queue_from = ACC_QUEUE_FROM;    // KZGMI_ACC_QUEUE_FROM: calls with fewer entries keep the static grid
  bool sort_split = false;     // KZGMI_SORT_SPLIT: split coarse-pass entries at every size (tests)
  bool sort_full_bins = false;  // KZGMI_SORT_FULL_BINS: the set-table-overflow fallback at every size (tests)
  int wbits_env = 0;           // KZGMI_WBITS: 13 or 16 forces the window width (tests, A/B)
  uint32_t small_terms = 4096;  // calls of at most this many terms: msm_small.hpp (KZGMI_SMALL_TERMS; 0: never)
  int host_chunks_env = 0;       // KZGMI_HOST_CHUNKS: ranges of a synchronous host-buffer batch (batch_host_chunked)
  int host_chunk_mode = 0;       // KZGMI_HOST_CHUNK_MODE=1: shard partials even where one bucket store applies
  // Split accumulation of two-MSM calls (run_msm_core): -1 synchronous device calls of at least
  // SPLIT_FROM entries with no other slot in flight (latency-bound), 0 never, 1 always
  // (KZGMI_SPLIT_ACC).  Single 2^20 BLS12-381 batches 8.02 -> 7.95 ms; 2^17 ones lose (2.95 ->
  // 3.01 ms: the side work outlasts the short second launch), so smaller calls keep one launch
  // (profiles/r06/split_accumulation.txt, ab_split_rev.txt)
  static constexpr size_t SPLIT_FROM = size_t(1) << 25;
  int split_acc = -1;
  bool split_low_prio = true;    // KZGMI_SPLIT_LOWPRIO: the side stream's kernels without the tail's raised issue priority
  bool split_side_fix = true;    // KZGMI_SPLIT_SIDEFIX: the first launch's piece joins on the side stream
  bool split_side_prio = true;   // KZGMI_SPLIT_SIDEPRIO: the side stream at the device's greatest priority
  // KZGMI_SPLIT_REV: MSM#0's sets (8 windows) in the first launch, its short tail on the side
  // stream, hidden behind MSM#1's 3x longer launch; MSM#1's tail after it on an idle chip.  0:
  // MSM#1's first, whose side tail outlasts the short second launch.  2^20: 7.95 vs 7.98 ms
  // (one launch 8.02; profiles/r06/ab_split_rev.txt)
  bool split_rev = true;
  // set by the synchronous device-buffer call while it enqueues: only such calls split (the first
  // batch of a pipeline is alone when it is enqueued too, and split it cost the 20-step bench
  // ~1 ms: its two launches, then a gap while the next batch's front end ran)
  bool sync_call = false;
  // reduction segments on 4 threads instead of 2 while that grid stays within seg4_waves waves per
  // SIMD (Launch::reduce; KZGMI_SEG4_WAVES, 0: always 2)
  int seg4_waves = 1;
  // accumulation order: a slot's k_accumulate waits for the accumulation D launches before it
  // (any slot), so at most D run at once and they start in submission order.  Without it 16
  // slots in flight ran their accumulations in bursts and their tails (pairing: one CU) together,
  // with no accumulation beside them, and the oldest batch -- the one the caller waits on to
  // reuse its slot -- finished last (tools/trace_gaps.py).  D = acc_order for calls of at least
  // ACC_ORDER_WIDE entries, acc_order_small below (a 2^17 batch's accumulation does not fill
  // the chip): pipelined 2^20 batches 184.7 vs 183.5/s (BN254 361 vs 347), 2^17 batches 1074 vs
  // 1028/s with D = 4 (925 with 2) -- profiles/r05/ab_acc_order*.txt.  Only where every slot has
  // a hardware queue of its own: a stream waiting for the event holds up the other slots of its
  // queue (at the default 4 queues 2^20 batches ran 160 vs 173/s with the order).
  // KZGMI_ACC_ORDER, KZGMI_ACC_ORDER_SMALL (0: off; set: also on shared queues)
  static constexpr int kAccOrderMax = 8;
  static constexpr size_t ACC_ORDER_WIDE = size_t(1) << 23;
  int acc_order = 2, acc_order_small = 4;
  hipEvent_t acc_ring[kAccOrderMax] = {};  // launch i's event at i % kAccOrderMax
  uint64_t acc_launches = 0;
  double phase_ms[kNumPhases] = {};  // running sums since profiling was (re)enabled
  // host-buffer inputs of every slot are copied on ONE stream, in submission order: each
  // batch's copy then gets the whole link and completes first-in first-out (16 concurrent
  // 256-MiB copies on the slots' own streams shared the link and all finished late)
  hipStream_t h2d_stream = nullptr;  // created with the context
  // The split accumulation's side stream: ONE per context, created at the first split.  Splits run
  // only on calls with no other slot in flight, so one suffices -- and every extra stream takes a
  // hardware queue: a side stream per slot (17 + 16 queues) oversubscribed the device's queue
  // slots and the whole 16-slot pipeline ran 180 -> 120 batch-verifies/s (gpurun call r6f)
  hipStream_t side_stream = nullptr;
  int phase_calls = 0;
  DevBuf table[2], table_base[2];
  bool table_ready[2] = {false, false};
  DevBuf lines_tmp, tmp;
  DevBuf gath;                       // multi-device: partial records gathered from every device
  DevBuf mdig, mdig_all;             // multi-device Fiat-Shamir: this device's / every device's subtree roots
  std::vector<kzgmi_ctx*> peers;     // multi-device: contexts of device_ids[1..] (kzgmi_ctx_create, n_devices > 1)
  std::vector<kzgmi_srs*> srs_list;  // live SRS objects: detached (device memory freed) on destroy
  std::vector<kzgmi_ck*> ck_list;    // live commit keys: same
};

// prover commit key: rows w = 0..15 of 2^(16 w)-shifted SRS points, [row][point] Montgomery affine
struct kzgmi_ck {
  int curve = 0;
  size_t n = 0;
  kzgmi_ctx* ctx = nullptr;
  DevBuf pts, inf;
};
constexpr int CK_ROWS = 16;  // 16-bit windows of a 255-bit Fr scalar

struct kzgmi_srs {
  int curve = 0;
  kzgmi_ctx* ctx = nullptr;
  DevBuf lines, q, q_inf;
  DevBuf g1;                        // the SRS's [1]_1: Montgomery affine point + its infinity byte after it,
  size_t g1_29_off = 0;             // then the same point in the accumulation's radix-29 format
  void* g1_29() const { return static_cast<uint8_t*>(g1.p) + g1_29_off; }
  std::vector<kzgmi_srs*> peers;    // multi-device context: the same SRS on each peer device
};

namespace {

int set_dev(kzgmi_ctx* c) {
  HIPCHK(hipSetDevice(c->device));
  return 0;
}

inline unsigned grid(size_t n, unsigned b) { return (unsigned)((n + b - 1) / b); }

// Start a job on slot s: its work goes on s.stream after the entry dependencies recorded since
// the slot's previous job (kzgmi_stream_wait, the H2D copy of host inputs).  Every entry point
// that issues work on a slot calls this first.
int begin_job(Slot& s) {
  for (int k = 0; k < s.ndep; ++k) HIPCHK(hipStreamWaitEvent(s.stream, s.dep_pool[k], 0));
  s.ndep = 0;
  return 0;
}

// The job's last operation is issued: done_ev marks its completion (kzgmi_slot_wait, the next
// job's begin_job, kzgmi_slot_signal)
int end_job(Slot& s) {
  HIPCHK(hipEventRecord(s.done_ev, s.stream));
  s.done_rec = true;
  return 0;
}

// Host wait for the slot's last job (an event, not a stream sync: an entry dependency recorded
// for the slot's next job must not be waited for here)
int sync_slot(Slot& s) {
  if (s.done_rec) HIPCHK(hipEventSynchronize(s.done_ev));
  return 0;
}
int sync_job(Slot& s) {
  CHK(end_job(s));
  return sync_slot(s);
}

// A new entry dependency of the slot's next job: work enqueued so far on `stream`
int add_dep(Slot& s, hipStream_t stream) {
  if (s.ndep == (int)s.dep_pool.size()) {
    hipEvent_t e = nullptr;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    s.dep_pool.push_back(e);
  }
  HIPCHK(hipEventRecord(s.dep_pool[s.ndep], stream));
  s.ndep += 1;
  return 0;
}

void mark(kzgmi_ctx* c, Slot& s, int idx) {
  if (!c->profiling) return;
  if (!s.ev[idx]) (void)hipEventCreate(&s.ev[idx]);
  (void)hipEventRecord(s.ev[idx], s.stream);
  s.ev_used[idx] = true;
}

void collect_phases(kzgmi_ctx* c, Slot& s) {
  if (!c->profiling) return;
  // phase k spans from the latest earlier recorded mark to mark k+1
  for (int k = 0; k < kNumBatchPhases; ++k) {
    if (!s.ev_used[k + 1]) continue;
    int j = k;
    while (j >= 0 && !s.ev_used[j]) --j;
    if (j < 0) continue;
    float ms = 0;
    if (hipEventElapsedTime(&ms, s.ev[j], s.ev[k + 1]) == hipSuccess) c->phase_ms[k] += ms;
  }
  if (s.ev_used[EV_H2D0] && s.ev_used[EV_H2D1]) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, s.ev[EV_H2D0], s.ev[EV_H2D1]) == hipSuccess) c->phase_ms[PH_H2D] += ms;
  }
  c->phase_calls += 1;
  for (bool& u : s.ev_used) u = false;
}

Seed make_seed(const uint8_t* seed32, uint8_t (&buf)[32]) {
  if (seed32) {
    memcpy(buf, seed32, 32);
  } else {
    size_t got = 0;
    while (got < 32) {
      ssize_t r = getrandom(buf + got, 32 - got, 0);
      if (r > 0) got += (size_t)r;
    }
  }
  Seed s;
  for (int k = 0; k < 8; ++k)
    s.w[k] = (uint32_t)buf[4 * k] << 24 | (uint32_t)buf[4 * k + 1] << 16 | (uint32_t)buf[4 * k + 2] << 8 | buf[4 * k + 3];
  return s;
}

int map_device_err(uint32_t e) {
  switch (e) {
    case DERR_NONE: return 0;
    case DERR_ENCODING: return fail(KZGMI_ERR_ENCODING, "invalid point encoding");
    case DERR_NOT_ON_CURVE: return fail(KZGMI_ERR_NOT_ON_CURVE, "point not on curve");
    case DERR_SCALAR: return fail(KZGMI_ERR_SCALAR, "non-canonical scalar (>= r)");
    case DERR_NOT_IN_SUBGROUP: return fail(KZGMI_ERR_NOT_IN_SUBGROUP, "point not in the order-r subgroup");
    case DERR_SHARD: return fail(KZGMI_ERR_SHARD, "a gathered partial record is marked failed (its shard was rejected)");
    default: return fail(KZGMI_ERR_DEVICE, "unknown device error");
  }
}

// ------------------------------------------------------------------------------ small MSMs
// The terms of tl (classes in order) as one wave each, MSM m's leaves in class order; the tree's
// stored nodes and arrival counters per MSM, level after level (msm_small.hpp).
template <class Cv>
int run_small_msm(kzgmi_ctx* c, Slot& s, const TermList& tl, const MsmWindows& mw, const Affine<Cv>* pts,
                  const uint8_t* inf, bool own_pts, bool dry) {
  SmallPlan sp{};
  sp.nclass = tl.nclass;
  sp.nmsm = mw.nmsm;
  uint32_t terms = 0, leaves[2] = {0, 0};
  for (uint32_t k = 0; k < tl.nclass; ++k) {
    const uint32_t m = mw.nmsm > 1 && tl.c[k].set_base >= mw.set_base[1] ? 1 : 0;
    sp.term_base[k] = terms;
    sp.msm[k] = m;
    sp.leaf_base[k] = leaves[m];
    terms += tl.c[k].count;
    leaves[m] += tl.c[k].count;
  }
  uint32_t nodes = 0, flags = 0;
  for (uint32_t m = 0; m < 2; ++m) {
    sp.count[m] = leaves[m];
    sp.node_base[m] = nodes;
    sp.flag_base[m] = flags;
    for (uint32_t cnt = leaves[m]; cnt > 1; cnt = (cnt + 1) >> 1) {
      nodes += cnt;
      flags += (cnt + 1) >> 1;
    }
  }
  CHK(s.small_nodes.ensure((size_t)(nodes + 1) * SMALL_NODE_WORDS * 4));
  CHK(s.small_flags.ensure((size_t)(flags + 1) * 4));
  CHK(s.res.ensure(2 * sizeof(Xyzz<Cv>)));
  if (dry) return 0;
  Roctx rx("kzgmi.msm.small");
  hipStream_t st = s.stream;
  using L = Launch<Cv>;
  if (!pts) pts = s.pts.template as<Affine<Cv>>();
  if (!inf) inf = s.inf.template as<uint8_t>();
  if (own_pts) {  // the slot's points into the radix-29 slots the kernel reads
    uint32_t npts = 0;
    for (uint32_t k = 0; k < tl.nclass; ++k)
      if (tl.c[k].count) npts = std::max(npts, tl.c[k].pt_base + tl.c[k].count);
    L::pts_to29(st, s.pts.template as<Affine<Cv>>(), npts);
  }
  mark(c, s, PH_SORT + 1);
  L::small_msm(st, tl, sp, terms, pts, inf, s.small_nodes.template as<uint32_t>(), s.small_flags.template as<uint32_t>(),
               flags + 1, s.res.template as<Xyzz<Cv>>());
  mark(c, s, PH_ACCUM + 1);
  mark(c, s, PH_REDUCE + 1);
  mark(c, s, PH_COMBINE + 1);
  HIPCHK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------ MSM core
// part (chunked host-buffer batches, enqueue_batch_chunked): 0 the whole call; 1 the first point
// range -- sort + accumulate into the slot's bucket store, no reduction; 2 a middle range -- into
// the second store (acc29b, cntb, offb), merged into the first; 3 the last range -- as 2, then the
// reduction and window combination of the merged store
template <class Cv>
int run_msm_core(kzgmi_ctx* c, Slot& s, const TermList& tl_in, uint32_t nsets, size_t emax, const MsmWindows& mw,
                 const Affine<Cv>* pts = nullptr, const uint8_t* inf = nullptr, bool pts29 = false,
                 bool dry = false, int wbits = WBITS, int part = 0) {
  const uint32_t nbuckets = wbits == 13 ? Win<13>::NBUCKETS : Win<WBITS>::NBUCKETS;
  const uint32_t bins = wbits == 13 ? Win<13>::BINS : Win<WBITS>::BINS;
  const uint32_t rb_parts = wbits == 13 ? Win<13>::RB_PARTS : Win<WBITS>::RB_PARTS;
  // pts == nullptr: the slot's freshly converted points, put into the accumulation's format
  // here unless convert_points stored them in it already (pts29); explicit pts (commit-key
  // rows) are stored in that format already (kzgmi_ck_load)
  const bool own_pts = pts == nullptr && !pts29;
  // small calls: one wave per term and a summation tree (msm_small.hpp) instead of buckets
  {
    bool small = part == 0 && c->small_terms && tl_in.total <= c->small_terms && mw.nmsm <= 2;
    for (uint32_t k = 0; k < tl_in.nclass; ++k) small = small && tl_in.c[k].win_off == 0;
    if (small) return run_small_msm<Cv>(c, s, tl_in, mw, pts, inf, own_pts, dry);
  }
  TermList tl = tl_in;  // + each class's offset in the digit array
  size_t ndig = 0;
  for (uint32_t k = 0; k < tl.nclass; ++k) {
    tl.c[k].dig_base = (uint32_t)ndig;
    ndig += (size_t)tl.c[k].count * tl.c[k].nwin;
  }
  if (ndig >= (1ull << 32)) return fail(KZGMI_ERR_ARG, "too many window digits for one call");
  CHK(s.digits.ensure(ndig * 4));
  using XY = Xyzz<Cv>;
  if (!pts) pts = s.pts.template as<Affine<Cv>>();  // default: the slot's converted points
  if (!inf) inf = s.inf.template as<uint8_t>();
  const uint32_t NB = nsets * nbuckets;
  // accumulation threads: 64-entry chunks (16 for small calls, msm.hpp ACC_CHUNK_SMALL), at most
  // one resident round of them (then equal longer chunks)
  const size_t chunk = emax <= ACC_SMALL_ENTRIES ? ACC_CHUNK_SMALL : ACC_CHUNK;
  size_t nchunks = (emax + chunk - 1) / chunk + 1;
  const size_t cap = c->acc_threads_env ? c->acc_threads_env : (size_t)c->ncu * 4 * kAccWaves<Cv> * 64;
  if (cap && nchunks > cap) nchunks = cap;
  // A call with no other slot of the context in flight is latency-bound: below the cap, give
  // every SIMD the same whole number of waves (shorter equal chunks).  A 2^17 batch at 13 bits
  // is 1.25 waves per SIMD, and its SIMDs with two waves ran 1.5x longer than those with one:
  // 4.36 -> 3.99 ms per batch.  Pipelined calls keep the longer chunks (fewer pieces to join:
  // 2^17 batches 1014 vs 966/s with the rounding; profiles/r03/misc_ab_r03.txt).
  // (kzgmi_ctx_reserve sizes the piece arrays for the rounded count)
  bool alone = true;
  for (const Slot& o : c->slots) alone &= &o == &s || !o.pending;
  alone |= dry;
  const size_t simd_lanes = (size_t)c->ncu * 4 * 64;
  if (alone && !c->acc_threads_env && emax > ACC_SMALL_ENTRIES && simd_lanes && nchunks < cap)
    nchunks = std::min(cap, (nchunks + simd_lanes - 1) / simd_lanes * simd_lanes);
  // Large radix-29 calls (the grid at its cap): c->acc_queue x cap shorter chunks taken from a
  // work queue by the cap's threads (msm.hpp k_accumulate), so an accumulation that starts behind
  // another slot's still ends on every CU at about the same time.  The part arrays and k_fixup
  // are sized for the chunk count.
  size_t acc_threads = 0;
  if (c->acc_queue > 1 && cap && nchunks == cap && cap % 256 == 0 && emax >= c->acc_queue_from) {
    acc_threads = cap;
    nchunks = std::min(cap * (size_t)c->acc_queue, std::max(cap, emax / c->acc_queue_min));
    if (nchunks <= cap) acc_threads = 0;
  }
  nchunks = (nchunks + 255) / 256 * 256;  // = the launched thread count (part arrays indexed by thread)
  // Split accumulation (latency): the two MSMs' sets (MSM#1's a suffix of the sets) accumulate
  // in two launches; the first launch's MSM reduces and combines on the slot's side stream beside
  // the second launch (split_rev: which MSM goes first).
  const uint32_t split_set = mw.nmsm == 2 ? mw.set_base[1] : 0;
  const bool can_split = part == 0 && mw.set_base[0] == 0 && split_set > 0 && split_set + mw.nwin[1] == nsets &&
                         mw.nwin[0] == split_set && c->split_acc != 0;
  // auto: only where the second MSM's tail is the longer one (BLS12-381 without GLV: 16 windows
  // against 8).  GLV batches (BN254, trusted BLS12-381 points) have 8 windows in both MSMs: the
  // split only adds its side-stream contention (BN254 2^22: 14.70 -> 15.18 ms)
  const bool split = can_split && (c->split_acc > 0 || (alone && c->sync_call && emax >= kzgmi_ctx::SPLIT_FROM &&
                                                        mw.nwin[1] > mw.nwin[0]));
  const size_t nchunks_b = nchunks, acc_threads_b = acc_threads;  // the second launch's grid
  // pieces: [A's first | A's last | B's first | B's last] when A's joins run on the side stream
  const size_t pieces = can_split && c->split_side_fix ? nchunks + nchunks_b : std::max(nchunks, nchunks_b);
  const size_t crowd_words = 1 + 3 * (pieces / FIX_LP_FROM + 2);  // at most one per FIX_LP_FROM + 1 chunks
  CHK(s.cnt.ensure((size_t)NB * 4));
  CHK(s.off.ensure((size_t)NB * 4));
  const bool second = part >= 2;  // this range accumulates into the second store, then merges
  if (second) {
    CHK(s.cntb.ensure((size_t)NB * 4));
    CHK(s.offb.ensure((size_t)NB * 4));
  }
  DevBuf& CNT = second ? s.cntb : s.cnt;
  DevBuf& OFF = second ? s.offb : s.off;
  DevBuf& ACC = second ? s.acc29b : s.acc29;
  CHK(s.coarse.ensure((size_t)3 * nsets * bins * 4));
  CHK(s.ent.ensure(emax * 8));
  CHK(s.total.ensure(16));
  if (acc_threads || acc_threads_b) CHK(s.accq.ensure(16));
  CHK(s.crowd.ensure(4 * crowd_words * (can_split ? 2 : 1)));  // a split's second list after the first
  CHK(s.sval.ensure(emax * 4 + 16));  // + 16: k_accumulate reads values 4 at a time, up to 3 past the end
  CHK(s.skey.ensure(emax * 4));
  constexpr int W29 = kW29<Fp29Of<Cv>>;
  // buckets and bucket pieces are radix-29 records in acc29 (msm.hpp)
  CHK(s.acc29.ensure(((size_t)NB + 2 * pieces) * W29 * 4));
  if (second) CHK(s.acc29b.ensure(((size_t)NB + 2 * nchunks) * W29 * 4));
  const size_t seg_rec = (size_t)W29 * 4;  // a radix-29 record
  CHK(s.R.ensure((size_t)NB / SEG * seg_rec));
  CHK(s.U.ensure((size_t)NB / SEG * seg_rec * 2));  // U records, then the V records
  CHK(s.scratch.ensure((size_t)nsets * rb_parts * sizeof(XY)));  // k_reduce_bits partial sums
  CHK(s.winsum.ensure((size_t)nsets * sizeof(XY)));
  CHK(s.res.ensure(2 * sizeof(XY)));
  if (dry) return 0;  // kzgmi_ctx_reserve: workspace sized, nothing enqueued
  if (split && !c->side_stream) {  // at the slot stream's priority, or the device's greatest
    int prio = 0, least = 0, greatest = 0;
    HIPCHK(hipStreamGetPriority(s.stream, &prio));
    if (c->split_side_prio && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess) prio = greatest;
    HIPCHK(hipStreamCreateWithPriority(&c->side_stream, hipStreamNonBlocking, prio));
  }
  if (split && !s.side_ev[0])
    for (auto& e : s.side_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  Roctx rx("kzgmi.msm.sort+accumulate+reduce+combine");
  hipStream_t st = s.stream;
  using L = Launch<Cv>;
  if (own_pts) {
    uint32_t npts = 0;
    for (uint32_t k = 0; k < tl.nclass; ++k)
      if (tl.c[k].count) npts = std::max(npts, tl.c[k].pt_base + tl.c[k].count);
    L::pts_to29(st, s.pts.template as<Affine<Cv>>(), npts);
  }
  L::sort(st, tl, nsets, inf, s.digits.template as<uint32_t>(), s.coarse.template as<uint32_t>(), s.ent.template as<uint64_t>(), emax,
          (c->sort_split ? L::SORT_SPLIT : 0) | (c->sort_full_bins ? L::SORT_FULL_BINS : 0),
          OFF.template as<uint32_t>(), CNT.template as<uint32_t>(), s.total.template as<uint32_t>(),
          s.sval.template as<uint32_t>(), s.skey.template as<uint32_t>(), wbits);
  mark(c, s, PH_SORT + 1);
  hipEvent_t* order_ev = nullptr;  // accumulation order (kzgmi_ctx::acc_order)
  const int order = emax >= kzgmi_ctx::ACC_ORDER_WIDE ? c->acc_order : c->acc_order_small;
  if (order > 0 && c->slots.size() > 1) {
    constexpr uint64_t M = kzgmi_ctx::kAccOrderMax;
    const uint64_t i = c->acc_launches++;
    if (i >= (uint64_t)order && c->acc_ring[(i - order) % M])  // the accumulation `order` launches back
      HIPCHK(hipStreamWaitEvent(st, c->acc_ring[(i - order) % M], 0));
    order_ev = &c->acc_ring[i % M];  // (launch i - M's event: no later launch waits for it)
    if (!*order_ev) HIPCHK(hipEventCreateWithFlags(order_ev, hipEventDisableTiming));
  }
  if (split) {
    // sets [split_set, nsets) are the sorted entries [coff[split_set * bins], total)
    const uint32_t* mid = s.coarse.template as<uint32_t>() + (size_t)nsets * bins + (size_t)split_set * bins;
    const uint32_t h = split_set, hn = nsets - split_set;
    uint32_t* acc = s.acc29.template as<uint32_t>();
    uint32_t* crowd_a = s.crowd.template as<uint32_t>();
    uint32_t* crowd_b = crowd_a + crowd_words;
    // launch A's pieces follow the buckets, launch B's follow A's: A's joins may run on the side
    // stream while B accumulates.  Order: MSM#1's sets [mid, total) first (split_rev 0), or
    // MSM#0's [0, mid) first (1); the first launch's MSM finishes on the side stream.
    const bool rev = c->split_rev;
    const uint32_t* total_a = rev ? mid : s.total.template as<uint32_t>();
    const uint32_t* lo_a = rev ? nullptr : mid;
    const uint32_t* total_b = rev ? s.total.template as<uint32_t>() : mid;
    const uint32_t* lo_b = rev ? mid : nullptr;
    const uint32_t nb_b = c->split_side_fix ? (uint32_t)(NB + 2 * nchunks) : NB;
    L::accumulate(st, nchunks, total_a, s.sval.template as<uint32_t>(), s.skey.template as<uint32_t>(),
                  s.off.template as<uint32_t>(), s.cnt.template as<uint32_t>(), pts, acc, NB, acc_threads,
                  acc_threads ? s.accq.template as<uint32_t>() : nullptr, crowd_a, lo_a,
                  c->split_side_fix ? nullptr : st);
    hipStream_t sd = c->side_stream;
    HIPCHK(hipEventRecord(s.side_ev[0], st));
    HIPCHK(hipStreamWaitEvent(sd, s.side_ev[0], 0));
    L::accumulate(st, nchunks_b, total_b, s.sval.template as<uint32_t>(), s.skey.template as<uint32_t>(),
                  s.off.template as<uint32_t>(), s.cnt.template as<uint32_t>(), pts, acc, nb_b, acc_threads_b,
                  acc_threads_b ? s.accq.template as<uint32_t>() : nullptr, crowd_b, lo_b, st);
    if (order_ev) HIPCHK(hipEventRecord(*order_ev, st));
    // MSM m's reduction and window combination on stream q: bucket records, R / U+V records, bit
    // sums and window sums at the offsets of its sets
    const size_t nseg = nbuckets / SEG;
    uint32_t* R29 = s.R.template as<uint32_t>();
    uint32_t* U29 = s.U.template as<uint32_t>();
    auto tail = [&](hipStream_t q, int m, bool lowp) {
      const uint32_t s0 = m ? h : 0, ns = m ? hn : h;
      L::reduce(q, ns, s.cnt.template as<uint32_t>() + (size_t)s0 * nbuckets, acc + (size_t)s0 * nbuckets * W29,
                reinterpret_cast<XY*>(R29 + s0 * nseg * W29), reinterpret_cast<XY*>(U29 + 2 * s0 * nseg * W29),
                s.scratch.template as<XY>() + (size_t)s0 * rb_parts, s.winsum.template as<XY>() + s0, wbits, lowp,
                c->seg4_waves, 4 * c->ncu);
      if (q == st) mark(c, s, PH_REDUCE + 1);
      L::window_combine(q, MsmWindows{1, {s0, 0}, {mw.nwin[m], 0}}, s.winsum.template as<XY>(),
                        s.res.template as<XY>() + m, wbits, lowp);
    };
    // side: (A's piece joins,) the first launch's MSM
    if (c->split_side_fix)
      L::fixup(sd, nchunks, total_a, s.skey.template as<uint32_t>(), s.off.template as<uint32_t>(),
               s.cnt.template as<uint32_t>(), acc, NB, crowd_a, lo_a);
    tail(sd, rev ? 0 : 1, c->split_low_prio);
    HIPCHK(hipEventRecord(s.side_ev[1], sd));
    mark(c, s, PH_ACCUM + 1);
    tail(st, rev ? 1 : 0, false);
    HIPCHK(hipStreamWaitEvent(st, s.side_ev[1], 0));
    mark(c, s, PH_COMBINE + 1);
    HIPCHK(hipGetLastError());
    return 0;
  }
  L::accumulate(st, nchunks, s.total.template as<uint32_t>(), s.sval.template as<uint32_t>(), s.skey.template as<uint32_t>(),
                OFF.template as<uint32_t>(), CNT.template as<uint32_t>(), pts, ACC.template as<uint32_t>(), NB,
                acc_threads, acc_threads ? s.accq.template as<uint32_t>() : nullptr, s.crowd.template as<uint32_t>(),
                nullptr, st);
  if (order_ev) HIPCHK(hipEventRecord(*order_ev, st));
  if (second)
    L::merge_buckets(st, NB, s.acc29.template as<uint32_t>(), s.cnt.template as<uint32_t>(),
                     s.acc29b.template as<uint32_t>(), s.cntb.template as<uint32_t>());
  mark(c, s, PH_ACCUM + 1);
  if (part == 1 || part == 2) {
    HIPCHK(hipGetLastError());
    return 0;  // more ranges follow
  }
  L::reduce(st, nsets, s.cnt.template as<uint32_t>(), s.acc29.template as<uint32_t>(), s.R.template as<XY>(),
            s.U.template as<XY>(), s.scratch.template as<XY>(), s.winsum.template as<XY>(), wbits, false, c->seg4_waves,
            4 * c->ncu);
  mark(c, s, PH_REDUCE + 1);
  L::window_combine(st, mw, s.winsum.template as<XY>(), s.res.template as<XY>(), wbits);
  mark(c, s, PH_COMBINE + 1);
  HIPCHK(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------ Fiat-Shamir
constexpr uint32_t kAllFlags = KZGMI_FLAG_COMPRESSED | KZGMI_FLAG_SUBGROUP_CHECK | KZGMI_FLAG_POWERS |
                               KZGMI_FLAG_FIAT_SHAMIR | KZGMI_FLAG_TRUSTED_G1;

uint32_t next_pow2(uint32_t x) {
  uint32_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

// 4096-leaf subtree roots of tuples [0, n) (global indices offset + i) -> returned device pointer
template <class Cv>
int enqueue_fs_digests(Slot& s, const void* dC, const void* dpi, const void* dz, const void* dy, size_t n,
                       uint64_t offset, bool compressed, const uint32_t** digests_out) {
  using L = Launch<Cv>;
  const uint32_t nch = (uint32_t)((n + FS_CHUNK - 1) / FS_CHUNK);
  const size_t slots = (size_t)nch * FS_CHUNK;
  CHK(s.fs_leaves.ensure(slots * 32));
  CHK(s.fs_tmp.ensure(slots * 24 + 64));
  HIPCHK(hipMemsetAsync(s.fs_leaves.p, 0, slots * 32, s.stream));
  L::fs_leaves(s.stream, (const uint8_t*)dC, (const uint8_t*)dpi, (const uint8_t*)dz, (const uint8_t*)dy, (uint32_t)n,
               offset, compressed, s.fs_leaves.template as<uint32_t>());
  *digests_out = L::fs_reduce(s.stream, s.fs_leaves.template as<uint32_t>(), (uint32_t)slots, nch,
                              s.fs_tmp.template as<uint32_t>());
  return 0;
}

// chunk digests (device) -> root -> r and its power table in s.pow, r (BE words) in s.chal
template <class Cv>
int enqueue_fs_challenge(Slot& s, const uint32_t* digests, uint32_t nch, uint64_t n_total) {
  using L = Launch<Cv>;
  const uint32_t p2 = next_pow2(nch);
  CHK(s.fs_top.ensure((size_t)p2 * 32 * 2 + 64));
  CHK(s.pow.ensure(FS_POW_BITS * sizeof(Fp<typename Cv::FrP>)));
  CHK(s.chal.ensure(32));
  uint32_t* top = s.fs_top.template as<uint32_t>();
  HIPCHK(hipMemcpyAsync(top, digests, (size_t)nch * 32, hipMemcpyDeviceToDevice, s.stream));
  L::fs_pad(s.stream, top, nch, p2);
  const uint32_t* root = L::fs_reduce(s.stream, top, p2, 1, top + 8 * (size_t)p2);
  L::fs_challenge(s.stream, root, n_total, s.pow.p, s.chal.template as<uint32_t>());
  return 0;
}

// the workspaces enqueue_fs_digests + enqueue_fs_challenge grow for a batch of n tuples
template <class Cv>
int reserve_fs(Slot& s, size_t n) {
  const uint32_t nch = (uint32_t)((n + FS_CHUNK - 1) / FS_CHUNK);
  const size_t slots = (size_t)nch * FS_CHUNK;
  CHK(s.fs_leaves.ensure(slots * 32));
  CHK(s.fs_tmp.ensure(slots * 24 + 64));
  CHK(s.fs_top.ensure((size_t)next_pow2(nch) * 32 * 2 + 64));
  CHK(s.pow.ensure(FS_POW_BITS * sizeof(Fp<typename Cv::FrP>)));
  CHK(s.chal.ensure(32));
  return 0;
}

// Window width of a call from its entry count at c = 16 (msm.hpp Win): c = 13 for mid-size calls,
// 2^20 < entries <= max13 (batches: 2^15 < n <= 2^17, max13 = 2^22; MSMs: 2^16 < n <= 2^17,
// max13 = 2^21) -- 8x fewer buckets for 5/4 the terms, where the bucket-sum reduction is a large
// share of the pipelined work (2^17-tuple batches 875 -> 1024/s, 2^17-point MSMs 193 -> 224 M
// pts/s; profiles/r03/misc_ab_r03.txt).  Not for larger calls (a 2^18-point MSM: 270 -> 242)
// nor tiny ones, whose latency it raises: the top window of a 10 x 13-bit split of a 128-bit
// magnitude holds 11 bits (of a 20 x 13 split of 256 bits, 9), so its terms crowd into a few
// hundred buckets whose pieces k_fixup joins serially (n = 256: 3.0 -> 3.3 ms).  At 14 bits the
// top windows keep 2 and 4 bits: a 2^17 batch took 19 ms.  KZGMI_WBITS=13/16 forces one.
int call_wbits(const kzgmi_ctx* c, size_t entries16, size_t max13) {
  if (c->wbits_env == 13 || c->wbits_env == WBITS) return c->wbits_env;
  return entries16 > (size_t(1) << 20) && entries16 <= max13 ? 13 : WBITS;
}
// windows of a 127-bit magnitude (randomisers, GLV halves) and of a full 255-bit scalar at width c
// (signed digits: the top window takes the last carry)
inline uint32_t windows_half(int wb) { return (uint32_t)((128 + wb - 1) / wb); }
inline uint32_t windows_full(int wb) { return (uint32_t)((256 + wb - 1) / wb); }

// ------------------------------------------------------------------------------ batch
template <class Cv>
int enqueue_batch(kzgmi_ctx* c, Slot& s, const kzgmi_srs* srs, const void* dC, const void* dz, const void* dy,
                  const void* dpi, size_t n, const Seed& seed, uint64_t offset, void* d_partial_out,
                  uint32_t flags, bool dry = false) {
  using XY = Xyzz<Cv>;
  using FrF = Fp<typename Cv::FrP>;
  const bool glv = c->glv_batch &&
                   (Cv::ID == 1 || (flags & (KZGMI_FLAG_SUBGROUP_CHECK | KZGMI_FLAG_TRUSTED_G1)) != 0);
  const size_t PH = 2 * n + 1;  // GLV: phi(pts[j]) at pts[PH + j]
  const size_t npts = glv ? 2 * PH : PH;
  using L = Launch<Cv>;
  CHK(s.pts.ensure(npts * sizeof(Affine<Cv>)));
  CHK(s.inf.ensure(npts));
  // powers: r_i = r^i (255-bit, caller-supplied r).  Fiat-Shamir: r from the transcript, then
  // the seeded 127-bit randomisers with seed = r (so 32n MSM entries, as with a host seed).
  const bool powers = (flags & KZGMI_FLAG_POWERS) != 0;
  if (glv) {
    CHK(s.glv_s.ensure(n * 32));
    CHK(s.glv_t.ensure(32));
    if (powers) CHK(s.glv_r.ensure(n * 32));
  }
  CHK(s.scal_r.ensure(n * (powers ? 32 : 16)));
  CHK(s.scal_s.ensure(n * 32));
  CHK(s.scal_t.ensure(32));
  CHK(s.tpart.ensure(L::tpart_bytes((uint32_t)n)));
  CHK(s.flags.ensure(16));
  if (dry) {  // kzgmi_ctx_reserve: the randomiser workspaces of this mode, no launches
    if (flags & KZGMI_FLAG_FIAT_SHAMIR) CHK(reserve_fs<Cv>(s, n));
    else if (flags & KZGMI_FLAG_POWERS) CHK(s.pow.ensure(FS_POW_BITS * sizeof(FrF)));
  }
  hipStream_t st = s.stream;
  uint32_t* err = s.flags.template as<uint32_t>() + 1;
  Affine<Cv>* pts = s.pts.template as<Affine<Cv>>();
  uint8_t* inf = s.inf.template as<uint8_t>();
  // points that only feed the radix-29 accumulation are converted straight into its format
  // (with GLV their images too: k_endo_points29); decompression and the subgroup check work in
  // the 32-bit form, converted afterwards by run_msm_core's k_pts_to29
  const bool pts29 = !(flags & (KZGMI_FLAG_COMPRESSED | KZGMI_FLAG_SUBGROUP_CHECK));
  const uint32_t nn = (uint32_t)n;
  uint32_t* gs = s.glv_s.template as<uint32_t>();
  uint32_t* gt = s.glv_t.template as<uint32_t>();
  uint32_t* gr = s.glv_r.template as<uint32_t>();
  // decode + validate the points, derive the randomisers and the MSM scalars
  auto front = [&]() -> int {
    Roctx rx("kzgmi.batch.convert+scalars");
    CHK(begin_job(s));
    mark(c, s, 0);
    HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, st));
    if (flags & KZGMI_FLAG_COMPRESSED) {
      L::decompress_points(st, (const uint8_t*)dpi, (uint32_t)n, pts, inf, err);
      L::decompress_points(st, (const uint8_t*)dC, (uint32_t)n, pts + n, inf + n, err);
    } else if (glv && pts29) {  // with phi(P) stored by the same pass (no k_endo_points29 over 2n points)
      L::convert_points(st, (const uint8_t*)dpi, (uint32_t)n, pts, inf, err, true, pts + PH, inf + PH);
      L::convert_points(st, (const uint8_t*)dC, (uint32_t)n, pts + n, inf + n, err, true, pts + PH + n, inf + PH + n);
    } else {
      L::convert_points(st, (const uint8_t*)dpi, (uint32_t)n, pts, inf, err, pts29);
      L::convert_points(st, (const uint8_t*)dC, (uint32_t)n, pts + n, inf + n, err, pts29);
    }
    if (flags & KZGMI_FLAG_SUBGROUP_CHECK) L::subgroup_check(st, pts, inf, (uint32_t)(2 * n), err);
    // the SRS's [1]_1 as the last term of MSM#1: -t [1]_1
    HIPCHK(hipMemcpyAsync(pts + 2 * n, pts29 ? srs->g1_29() : srs->g1.p, sizeof(Affine<Cv>), hipMemcpyDeviceToDevice, st));
    HIPCHK(hipMemcpyAsync(inf + 2 * n, srs->g1.template as<uint8_t>() + sizeof(Affine<Cv>), 1, hipMemcpyDeviceToDevice, st));
    if (glv && pts29)  // the converts stored the 2n images: G1's alone
      L::endo_points(st, pts + 2 * n, inf + 2 * n, 1, pts + PH + 2 * n, inf + PH + 2 * n, true);
    else if (glv)
      L::endo_points(st, pts, inf, (uint32_t)PH, pts + PH, inf + PH, pts29);
    mark(c, s, PH_CONVERT + 1);
    if (flags & KZGMI_FLAG_FIAT_SHAMIR) {  // r from the transcript of this (whole) batch
      const uint32_t* digests = nullptr;
      CHK(enqueue_fs_digests<Cv>(s, dC, dpi, dz, dy, n, 0, (flags & KZGMI_FLAG_COMPRESSED) != 0, &digests));
      CHK(enqueue_fs_challenge<Cv>(s, digests, (uint32_t)((n + FS_CHUNK - 1) / FS_CHUNK), n));
    } else if (flags & KZGMI_FLAG_POWERS) {  // r supplied by the caller in place of the seed
      CHK(s.pow.ensure(FS_POW_BITS * sizeof(FrF)));
      L::pow_table(st, seed, s.pow.p, err);
    }
    if (powers)
      L::scalar_prep_pow(st, s.pow.p, offset, (const uint8_t*)dz, (const uint8_t*)dy, (uint32_t)n,
                         s.scal_r.template as<uint32_t>(), s.scal_s.template as<uint32_t>(), s.tpart.p,
                         s.scal_t.template as<uint32_t>(), err);
    else
      L::scalar_prep(st, seed, (flags & KZGMI_FLAG_FIAT_SHAMIR) ? s.chal.template as<uint32_t>() : nullptr, offset, (const uint8_t*)dz, (const uint8_t*)dy, (uint32_t)n,
                     s.scal_r.template as<uint32_t>(), s.scal_s.template as<uint32_t>(), s.tpart.p,
                     s.scal_t.template as<uint32_t>(), err, glv ? gs : nullptr, glv ? gs + 4 * (size_t)n : nullptr);
    if (glv) {  // (s_i split by k_scalar_prep itself unless the powers form produced it)
      if (powers) L::glv_split(st, s.scal_s.template as<uint32_t>(), 8, nn, gs, gs + 4 * (size_t)n);
      L::glv_split(st, s.scal_t.template as<uint32_t>(), 8, 1, gt, gt + 4);
      if (powers) L::glv_split(st, s.scal_r.template as<uint32_t>(), 8, nn, gr, gr + 4 * (size_t)n);
    }
    mark(c, s, PH_SCALARS + 1);
    return 0;
  };
  if (!dry) CHK(front());
  TermList tl{};
  const uint32_t ph = (uint32_t)PH;
  // c = 16: H = 8 windows for 127-bit magnitudes, F = 16 for full scalars; c = 13: 10 and 20
  const int wb = call_wbits(c, (size_t)(powers ? 48 : 32) * n, size_t(1) << 22);
  const uint32_t H = windows_half(wb), F = windows_full(wb);
  if (glv) {  // every MSM in H windows of half scalars: sets 0..H-1 (MSM#0), H..2H-1 (MSM#1)
    const uint32_t* rr = s.scal_r.template as<uint32_t>();
    uint32_t k = 0;
    if (!powers) {
      tl.c[k++] = {nn, 0, 4, H, 0, 4, rr};                     // MSM#0: r_i pi_i
      tl.c[k++] = {nn, nn, 4, H, H, 4, rr};                    // MSM#1: r_i C_i
    } else {
      tl.c[k++] = {nn, 0, 4, H, 0, 4, gr};                     // MSM#0: r_i pi_i = h0 pi + h1 phi(pi)
      tl.c[k++] = {nn, ph, 4, H, 0, 4, gr + 4 * (size_t)n};
      tl.c[k++] = {nn, nn, 4, H, H, 4, gr};                    // MSM#1: r_i C_i
      tl.c[k++] = {nn, ph + nn, 4, H, H, 4, gr + 4 * (size_t)n};
    }
    tl.c[k++] = {nn, 0, 4, H, H, 4, gs};                       //        s_i pi_i
    tl.c[k++] = {nn, ph, 4, H, H, 4, gs + 4 * (size_t)n};
    tl.c[k++] = {1, 2 * nn, 4, H, H, 0, gt};                   //        -t G1
    tl.c[k++] = {1, ph + 2 * nn, 4, H, H, 0, gt + 4};
    tl.nclass = k;
    tl.total = 0;
    for (uint32_t j = 0; j < k; ++j) tl.total += tl.c[j].count;
    const MsmWindows mw{2, {0, H}, {H, H}};
    CHK(run_msm_core<Cv>(c, s, tl, 2 * H, (size_t)(powers ? 6 : 4) * H * n + 2 * H + 16, mw, nullptr, nullptr,
                         pts29, dry, wb));
  } else if (!powers) {  // 127-bit r_i: MSM#0 in H windows (sets 0..H-1), MSM#1 in F (sets H..H+F-1)
    tl.c[0] = {nn, 0, 4, H, 0, 4, s.scal_r.template as<uint32_t>()};          // MSM#0: r_i pi_i
    tl.c[1] = {nn, nn, 4, H, H, 4, s.scal_r.template as<uint32_t>()};         // MSM#1: r_i C_i
    tl.c[2] = {nn, 0, 8, F, H, 8, s.scal_s.template as<uint32_t>()};          //        s_i pi_i
    tl.c[3] = {1, 2 * nn, 8, F, H, 0, s.scal_t.template as<uint32_t>()};      //        -t G1
  }
  if (!glv && powers) {  // r_i = r^i, full Fr: both MSMs in F windows (sets 0..F-1, F..2F-1)
    tl.c[0] = {nn, 0, 8, F, 0, 8, s.scal_r.template as<uint32_t>()};
    tl.c[1] = {nn, nn, 8, F, F, 8, s.scal_r.template as<uint32_t>()};
    tl.c[2] = {nn, 0, 8, F, F, 8, s.scal_s.template as<uint32_t>()};
    tl.c[3] = {1, 2 * nn, 8, F, F, 0, s.scal_t.template as<uint32_t>()};
  }
  if (!glv) {
    tl.nclass = 4;
    tl.total = 3 * nn + 1;
    const MsmWindows mw = powers ? MsmWindows{2, {0, F}, {F, F}} : MsmWindows{2, {0, H}, {H, F}};
    CHK(run_msm_core<Cv>(c, s, tl, powers ? 2 * F : H + F, (size_t)(powers ? 3 * F : 2 * H + F) * n + F + 16, mw,
                         nullptr, nullptr, pts29, dry, wb));
  }
  if (dry) return 0;
  Roctx rx("kzgmi.batch.pairing");
  if (d_partial_out) {
    L::partial_out(st, s.res.template as<XY>(), 2, err, (XY*)d_partial_out);  // marked if this shard failed
  } else {
    L::pairing_check(st, s.res.template as<XY>(), srs->lines.template as<Line<Cv>>(), srs->q_inf.template as<uint8_t>(),
                     s.flags.template as<int>());
    mark(c, s, PH_PAIRING + 1);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, st));
  CHK(end_job(s));
  s.pending = true;
  s.partial_job = d_partial_out != nullptr;
  s.partial_of = s.partial_job ? 1 : 0;
  s.msm_job = false;
  s.curve = Cv::ID;
  return 0;
}

int finish_slot(kzgmi_ctx* c, Slot& s, int* ok_out) {
  {
    Roctx rx("kzgmi.slot_wait");
    CHK(sync_slot(s));
  }
  s.pending = false;
  collect_phases(c, s);
  int e = map_device_err((uint32_t)s.host_flags[1]);
  if (e) return e;
  if (ok_out) *ok_out = (s.partial_job || s.msm_job) ? 1 : s.host_flags[0];
  return 0;
}

template <class F>
int dispatch(int curve, F&& f) {
  if (curve == 0) return f(Bls12_381{});
  if (curve == 1) return f(Bn254{});
  return fail(KZGMI_ERR_ARG, "unknown curve");
}

size_t g1_bytes(int curve) { return curve == 0 ? 96 : 64; }
size_t g2_bytes(int curve) { return curve == 0 ? 192 : 128; }

int check_ctx(kzgmi_ctx* c, int slot = 0) {
  if (!c) return fail(KZGMI_ERR_ARG, "null context");
  if (slot < 0 || slot >= (int)c->slots.size()) return fail(KZGMI_ERR_ARG, "bad slot");
  return set_dev(c);
}

kzgmi_ctx* dev_ctx(kzgmi_ctx* c, int d) { return d == 0 ? c : c->peers[d - 1]; }

// Multi-device context (kzgmi_ctx_create with D > 1 devices): the caller's slot s runs on device
// s % D as that device's local slot s / D -- whole batches / MSMs per device, each device with
// its own lane pipeline; caller slot d < D is device d's local slot 0, which is also the
// device's shard slot of the synchronous strong split.  Only the outermost C-ABI call of a
// host thread translates (entry points calling each other pass local slots): t_route_depth.
thread_local int t_route_depth = 0;
struct RouteGuard {
  RouteGuard() { ++t_route_depth; }
  ~RouteGuard() { --t_route_depth; }
  RouteGuard(const RouteGuard&) = delete;
  RouteGuard& operator=(const RouteGuard&) = delete;
};
int route_slot(kzgmi_ctx*& c, const kzgmi_srs** srs, int& slot) {
  if (t_route_depth != 1 || !c || c->peers.empty()) return 0;
  const int D = 1 + (int)c->peers.size();
  if (slot < 0 || slot >= c->user_slots) return fail(KZGMI_ERR_ARG, "bad slot");
  const int d = slot % D;
  if (srs && *srs) {
    if ((*srs)->ctx != c || (*srs)->peers.size() != c->peers.size())
      return fail(KZGMI_ERR_ARG, "srs does not belong to this context");
    if (d > 0) *srs = (*srs)->peers[d - 1];
  }
  c = dev_ctx(c, d);
  slot /= D;
  return 0;
}
#define KZ_ROUTE(c, srsp, slot) \
  RouteGuard route_guard_;       \
  CHK(route_slot(c, srsp, slot))

int batch_multi_host(kzgmi_ctx* c, const kzgmi_srs* srs, const uint8_t* commitments, const uint8_t* zs,
                     const uint8_t* ys, const uint8_t* proofs, size_t n, const uint8_t* seed32, uint32_t flags,
                     int* ok_out);
int msm_multi_host(kzgmi_ctx* c, kzgmi_curve curve, const uint8_t* points, const uint8_t* scalars, size_t n,
                   uint8_t* out);

// synchronous entry points that run on slot 0 must not overwrite a pending async job's
// flags / result buffers (its later kzgmi_slot_wait would report theirs)
int slot0_idle(kzgmi_ctx* c) {
  if (c->slots[0].pending)
    return fail(KZGMI_ERR_ARG, "slot 0 busy: complete its pending job (kzgmi_slot_wait / kzgmi_msm_wait) first");
  for (size_t d = 0; d < c->peers.size(); ++d)  // multi-device: the shard slots (caller slots 1..D-1)
    if (c->peers[d]->slots[0].pending)
      return fail(KZGMI_ERR_ARG, "slot " + std::to_string(d + 1) + " busy: a synchronous multi-device call uses "
                                 "every device's first slot");
  return 0;
}

template <class Cv>
int ensure_table(kzgmi_ctx* c, hipStream_t st) {
  if (c->table_ready[Cv::ID]) return 0;
  CHK(c->table_base[Cv::ID].ensure(32 * sizeof(Xyzz<Cv>)));
  CHK(c->table[Cv::ID].ensure(32 * 256 * sizeof(Affine<Cv>)));
  Launch<Cv>::gen_table(st, c->table_base[Cv::ID].template as<Xyzz<Cv>>(), c->table[Cv::ID].template as<Affine<Cv>>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(st));
  c->table_ready[Cv::ID] = true;
  return 0;
}

// ---------------------------------------------------------------- host buffers (PCIe path)
// Pinned host ranges the library may DMA from directly: kzgmi_host_alloc blocks and
// kzgmi_host_register'ed ranges, keyed by start address.
struct HostRange {
  uintptr_t hi;
  bool owned;  // kzgmi_host_alloc (hipHostFree) vs kzgmi_host_register (hipHostUnregister)
};
std::mutex g_host_mu;
std::map<uintptr_t, HostRange> g_host;

bool host_pinned(const void* p, size_t bytes) {
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> lk(g_host_mu);
  auto it = g_host.upper_bound(a);
  if (it == g_host.begin()) return false;
  --it;
  return a >= it->first && a + bytes <= it->second.hi;
}

// Parallel memcpy for pageable -> pinned staging: one memcpy thread reaches ~10-20 GB/s, below
// PCIe Gen5's ~50 GB/s, so the copy is split over KZGMI_COPY_THREADS workers (default 8) plus
// the caller.  One job at a time (contexts on several host threads take turns).
class CopyPool {
 public:
  CopyPool() {
    const char* e = getenv("KZGMI_COPY_THREADS");
    nthreads_ = e ? std::max(1, atoi(e)) : 8;
  }
  void copy(void* dst, const void* src, size_t len) {
    if (len < (size_t(2) << 20) || nthreads_ <= 1) {
      memcpy(dst, src, len);
      return;
    }
    std::lock_guard<std::mutex> job(job_mu_);
    start();
    const int parts = (int)workers_.size() + 1;
    {
      std::lock_guard<std::mutex> lk(mu_);
      dst_ = (uint8_t*)dst;
      src_ = (const uint8_t*)src;
      len_ = len;
      parts_ = parts;
      left_ = parts - 1;
      ++gen_;
    }
    cv_.notify_all();
    part(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return left_ == 0; });
  }

 private:
  void start() {
    if (!workers_.empty()) return;
    for (int i = 1; i < nthreads_; ++i) {
      workers_.emplace_back([this, i] { loop(i); });
      workers_.back().detach();  // the pool lives as long as the process (never destroyed)
    }
  }
  void part(int i) {
    const size_t per = (len_ / parts_ + 63) & ~size_t(63);
    const size_t lo = std::min(len_, per * i), hi = std::min(len_, per * (i + 1));
    if (hi > lo) memcpy(dst_ + lo, src_ + lo, hi - lo);
  }
  void loop(int i) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
      }
      part(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--left_ == 0) done_.notify_one();
    }
  }
  int nthreads_ = 8;  // fixed by the constructor (the pool is a function-local static: thread-safe)
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> workers_;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
  size_t len_ = 0;
  int parts_ = 1, left_ = 0;
  uint64_t gen_ = 0;
};
CopyPool* copy_pool() {
  static CopyPool* p = new CopyPool();  // never destroyed: its workers are detached
  return p;
}

// enqueue host -> device on the copy stream cs: pinned ranges by DMA directly (asynchronous);
// pageable ones through the slot's two pinned ring buffers, the host copy of chunk k+1
// overlapping the DMA of chunk k (the call returns when the last chunk is staged)
int h2d(Slot& s, hipStream_t cs, void* dst, const void* src, size_t bytes) {
  if (!bytes) return 0;
  if (host_pinned(src, bytes)) {
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, cs));
    return 0;
  }
  for (int b = 0; b < 2; ++b) {
    if (!s.ring[b]) {
      if (hipHostMalloc((void**)&s.ring[b], kRingBytes, hipHostMallocDefault) != hipSuccess) {
        s.ring[b] = nullptr;
        return fail(KZGMI_ERR_OOM, "pinned staging allocation failed");
      }
      g_allocs.fetch_add(1, std::memory_order_relaxed);
    }
    if (!s.ring_ev[b]) {
      HIPCHK(hipEventCreateWithFlags(&s.ring_ev[b], hipEventDisableTiming));
      HIPCHK(hipEventRecord(s.ring_ev[b], cs));  // so the first wait on it has a record
    }
  }
  for (size_t off = 0; off < bytes; off += kRingBytes) {
    const size_t len = std::min(kRingBytes, bytes - off);
    const int b = s.ring_next;
    s.ring_next ^= 1;
    HIPCHK(hipEventSynchronize(s.ring_ev[b]));  // its previous DMA has read it
    copy_pool()->copy(s.ring[b], (const uint8_t*)src + off, len);
    HIPCHK(hipMemcpyAsync((uint8_t*)dst + off, s.ring[b], len, hipMemcpyHostToDevice, cs));
    HIPCHK(hipEventRecord(s.ring_ev[b], cs));
  }
  return 0;
}

std::vector<size_t> split_units(size_t n, int D);  // below: balanced ranges in units of 4096 tuples

// A synchronous host-buffer batch (plain flags, or TRUSTED_G1; BN254 and declared-G1 points take
// the GLV form) as k point ranges on one slot: range j's copy (the context's copy stream) overlaps
// the previous ranges' front end and accumulation on the slot's stream, every range accumulates
// into the same bucket sets (a second store merged into the first, run_msm_core parts 1..3), the
// G1 term joins the last range (its scalar needs every range's r_i y_i), and one reduction,
// combination and pairing decide.  Same r_i (global index), same sums as enqueue_batch; the
// inputs land in the slot's stage buffer.
template <class Cv>
int enqueue_batch_chunked(kzgmi_ctx* c, Slot& s, const kzgmi_srs* srs, const uint8_t* hC, const uint8_t* hz,
                          const uint8_t* hy, const uint8_t* hpi, size_t n, const Seed& seed, uint32_t flags, int k) {
  using XY = Xyzz<Cv>;
  using L = Launch<Cv>;
  using FrF = Fp<typename Cv::FrP>;
  const bool glv = c->glv_batch && (Cv::ID == 1 || (flags & KZGMI_FLAG_TRUSTED_G1) != 0);
  const size_t gb = g1_bytes(Cv::ID);
  const size_t PH = 2 * n + 1;  // GLV: phi(pts[j]) at pts[PH + j]
  CHK(s.pts.ensure((glv ? 2 * PH : PH) * sizeof(Affine<Cv>)));
  CHK(s.inf.ensure(glv ? 2 * PH : PH));
  CHK(s.scal_r.ensure(n * 16));
  CHK(s.scal_s.ensure(n * 32));
  CHK(s.scal_t.ensure(32));
  if (glv) {
    CHK(s.glv_s.ensure(n * 32));
    CHK(s.glv_t.ensure(32));
  }
  CHK(s.tpart.ensure(L::tpart_bytes((uint32_t)n)));
  CHK(s.flags.ensure(16));
  CHK(s.stage.ensure(n * (2 * gb + 64)));
  uint8_t* dC = s.stage.template as<uint8_t>();
  uint8_t* dpi = dC + n * gb;
  uint8_t* dz = dC + 2 * n * gb;
  uint8_t* dy = dz + 32 * n;
  Affine<Cv>* pts = s.pts.template as<Affine<Cv>>();
  uint8_t* inf = s.inf.template as<uint8_t>();
  uint32_t* sr = s.scal_r.template as<uint32_t>();
  uint32_t* ss = s.scal_s.template as<uint32_t>();
  uint32_t* stt = s.scal_t.template as<uint32_t>();
  uint32_t* gs = s.glv_s.template as<uint32_t>();  // [h0 x n | h1 x n]
  uint32_t* gt = s.glv_t.template as<uint32_t>();
  FrF* tpart = reinterpret_cast<FrF*>(s.tpart.p);
  uint32_t* err = s.flags.template as<uint32_t>() + 1;
  const int wb = call_wbits(c, (size_t)32 * n, size_t(1) << 22);
  const uint32_t H = windows_half(wb), F = windows_full(wb);
  const MsmWindows mw = glv ? MsmWindows{2, {0, H}, {H, H}} : MsmWindows{2, {0, H}, {H, F}};
  const uint32_t nsets = glv ? 2 * H : H + F;
  const uint32_t nn = (uint32_t)n, ph = (uint32_t)PH;
  // the first range short (its copy is the only one nothing overlaps), the others equal
  std::vector<size_t> nk(k);
  {
    const size_t units = (n + FS_CHUNK - 1) / FS_CHUNK;
    const size_t u0 = k > 1 ? std::max<size_t>(1, units / (2 * (size_t)k)) : units;
    nk[0] = std::min(n, u0 * FS_CHUNK);
    const std::vector<size_t> rest = split_units(n - nk[0], k - 1 > 0 ? k - 1 : 1);
    for (int j = 1; j < k; ++j) nk[j] = rest[j - 1];
  }
  auto terms = [&](size_t lo, size_t nj, bool last) {
    TermList tl{};
    const uint32_t l = (uint32_t)lo, m = (uint32_t)nj;
    uint32_t q = 0;
    tl.c[q++] = {m, l, 4, H, 0, 4, sr + 4 * lo};           // MSM#0: r_i pi_i
    tl.c[q++] = {m, nn + l, 4, H, H, 4, sr + 4 * lo};      // MSM#1: r_i C_i
    if (glv) {
      tl.c[q++] = {m, l, 4, H, H, 4, gs + 4 * lo};         //        s_i pi_i = h0 pi + h1 phi(pi)
      tl.c[q++] = {m, ph + l, 4, H, H, 4, gs + 4 * (n + lo)};
      if (last) {
        tl.c[q++] = {1, 2 * nn, 4, H, H, 0, gt};           //        -t G1
        tl.c[q++] = {1, ph + 2 * nn, 4, H, H, 0, gt + 4};
      }
    } else {
      tl.c[q++] = {m, l, 8, F, H, 8, ss + 8 * lo};         //        s_i pi_i
      if (last) tl.c[q++] = {1, 2 * nn, 8, F, H, 0, stt};  //        -t G1
    }
    tl.nclass = q;
    tl.total = 0;
    for (uint32_t j = 0; j < q; ++j) tl.total += tl.c[j].count;
    return tl;
  };
  auto emax_of = [&](size_t nj) {
    return glv ? (size_t)4 * H * nj + 2 * H + 16 : (size_t)(2 * H + F) * nj + F + 16;
  };
  size_t nmax = 0;
  for (size_t v : nk) nmax = std::max(nmax, v);
  // every workspace at its final size before the first launch (a later growth would free a buffer
  // an earlier range's kernels are still using)
  CHK(run_msm_core<Cv>(c, s, terms(0, nmax, true), nsets, emax_of(nmax), mw, nullptr, nullptr, true, true, wb, 3));
  hipStream_t st = s.stream, cs = c->h2d_stream;
  if (s.done_rec) HIPCHK(hipStreamWaitEvent(cs, s.done_ev, 0));  // the stage buffer is free
  size_t lo = 0;
  for (int j = 0; j < k; ++j) {
    const size_t nj = nk[j];
    const bool last = j == k - 1;
    CHK(h2d(s, cs, dC + lo * gb, hC + lo * gb, nj * gb));
    CHK(h2d(s, cs, dpi + lo * gb, hpi + lo * gb, nj * gb));
    CHK(h2d(s, cs, dz + 32 * lo, hz + 32 * lo, nj * 32));
    CHK(h2d(s, cs, dy + 32 * lo, hy + 32 * lo, nj * 32));
    CHK(add_dep(s, cs));
    CHK(begin_job(s));  // this range's kernels wait for its copy only
    if (j == 0) {
      mark(c, s, 0);
      HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, st));
      HIPCHK(hipMemcpyAsync(pts + 2 * n, srs->g1_29(), sizeof(Affine<Cv>), hipMemcpyDeviceToDevice, st));
      HIPCHK(hipMemcpyAsync(inf + 2 * n, srs->g1.template as<uint8_t>() + sizeof(Affine<Cv>), 1,
                            hipMemcpyDeviceToDevice, st));
      if (glv) L::endo_points(st, pts + 2 * n, inf + 2 * n, 1, pts + PH + 2 * n, inf + PH + 2 * n, true);
    }
    if (glv) {  // phi(P) stored by the same pass
      L::convert_points(st, dpi + lo * gb, (uint32_t)nj, pts + lo, inf + lo, err, true, pts + PH + lo, inf + PH + lo);
      L::convert_points(st, dC + lo * gb, (uint32_t)nj, pts + n + lo, inf + n + lo, err, true, pts + PH + n + lo,
                        inf + PH + n + lo);
    } else {
      L::convert_points(st, dpi + lo * gb, (uint32_t)nj, pts + lo, inf + lo, err, true);
      L::convert_points(st, dC + lo * gb, (uint32_t)nj, pts + n + lo, inf + n + lo, err, true);
    }
    // range j's per-block r_i y_i sums land at its blocks of tpart (lo is a multiple of PREP_BLOCK)
    L::scalar_prep(st, seed, nullptr, lo, dz + 32 * lo, dy + 32 * lo, (uint32_t)nj, sr + 4 * lo, ss + 8 * lo,
                   tpart + lo / PREP_BLOCK, stt, err, glv ? gs + 4 * lo : nullptr, glv ? gs + 4 * (n + lo) : nullptr);
    if (last) {  // -t over every range (then its GLV halves)
      L::tsum(st, tpart, (uint32_t)((n + PREP_BLOCK - 1) / PREP_BLOCK), stt);
      if (glv) L::glv_split(st, stt, 8, 1, gt, gt + 4);
    }
    const int part = k == 1 ? 0 : j == 0 ? 1 : last ? 3 : 2;
    CHK(run_msm_core<Cv>(c, s, terms(lo, nj, last), nsets, emax_of(nj), mw, nullptr, nullptr, true, false, wb, part));
    lo += nj;
  }
  L::pairing_check(st, s.res.template as<XY>(), srs->lines.template as<Line<Cv>>(), srs->q_inf.template as<uint8_t>(),
                   s.flags.template as<int>());
  mark(c, s, PH_PAIRING + 1);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, st));
  CHK(end_job(s));
  s.pending = true;
  s.partial_job = false;
  s.partial_of = 0;
  s.msm_job = false;
  s.curve = Cv::ID;
  return 0;
}

}  // namespace

// ================================================================================ C ABI
extern "C" {

const char* kzgmi_version(void) { return "kzgmi 0.5 (abi " KZ_STR(KZGMI_ABI_VERSION) ", gfx950, HIP)"; }
int kzgmi_abi_version(void) { return KZGMI_ABI_VERSION; }
uint64_t kzgmi_alloc_count(void) { return g_allocs.load(std::memory_order_relaxed); }
const char* kzgmi_last_error(void) { return g_err.c_str(); }
const char* kzgmi_phase_names(void) { return kPhaseNames; }

int kzgmi_ctx_create_device(kzgmi_ctx** out, int device_id, int pipeline_slots) {
  if (!out || device_id < 0 || pipeline_slots < 1 || pipeline_slots > 64) return fail(KZGMI_ERR_ARG, "bad ctx args");
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device_id)
    return fail(KZGMI_ERR_DEVICE, "no HIP device " + std::to_string(device_id) + " (found " + std::to_string(ndev) + ")");
  HIPCHK(hipSetDevice(device_id));
  kzgmi_ctx* c = new kzgmi_ctx();
  c->device = device_id;
  int ncu = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device_id) == hipSuccess && ncu > 0)
    c->ncu = ncu;
  if (const char* e = getenv("KZGMI_ACC_THREADS")) c->acc_threads_env = (size_t)strtoull(e, nullptr, 10);
  if (const char* e = getenv("KZGMI_ACC_QUEUE")) c->acc_queue = atoi(e);
  if (const char* e = getenv("KZGMI_ACC_QUEUE_MIN")) c->acc_queue_min = std::max<size_t>(4, strtoull(e, nullptr, 10));
  if (const char* e = getenv("KZGMI_ACC_QUEUE_FROM")) c->acc_queue_from = strtoull(e, nullptr, 10);
  if (const char* e = getenv("KZGMI_SORT_SPLIT")) c->sort_split = atoi(e) != 0;
  if (const char* e = getenv("KZGMI_SORT_FULL_BINS")) c->sort_full_bins = atoi(e) != 0;
  if (const char* e = getenv("KZGMI_WBITS")) c->wbits_env = atoi(e);
  if (const char* e = getenv("KZGMI_SMALL_TERMS")) c->small_terms = (uint32_t)strtoul(e, nullptr, 10);
  if (const char* e = getenv("KZGMI_HOST_CHUNKS")) c->host_chunks_env = std::max(1, atoi(e));
  if (const char* e = getenv("KZGMI_HOST_CHUNK_MODE")) c->host_chunk_mode = atoi(e);
  if (const char* e = getenv("KZGMI_SPLIT_ACC")) c->split_acc = atoi(e) < 0 ? -1 : std::min(1, atoi(e));
  if (const char* e = getenv("KZGMI_SPLIT_LOWPRIO")) c->split_low_prio = atoi(e) != 0;
  if (const char* e = getenv("KZGMI_SEG4_WAVES")) c->seg4_waves = std::max(0, atoi(e));
  if (const char* e = getenv("KZGMI_SPLIT_SIDEFIX")) c->split_side_fix = atoi(e) != 0;
  if (const char* e = getenv("KZGMI_SPLIT_SIDEPRIO")) c->split_side_prio = atoi(e) != 0;
  if (const char* e = getenv("KZGMI_SPLIT_REV")) c->split_rev = atoi(e) != 0;
  // HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 unless set before the runtime
  // starts) and serialises the streams of one queue, so every slot in flight needs a queue of its
  // own (16 slots on 24 queues pipeline; 24 on 24 ran 3.6x slower).  The runtime keeps that many
  // queues PER STREAM PRIORITY: when the slots (+ the copy stream) outnumber the queues, the slot
  // streams cycle through the device's priority levels, which multiplies the queues they get --
  // at the default 4 queues, 2^20 batches run 173 vs 161/s (0.96 of the 179.5/s on 24 queues)
  // and 2^17 batches 814 vs 577/s (profiles/r05/ab_stream_prio*.txt).  KZGMI_STREAM_PRIO=0/1
  // forces it off / on.
  const char* qenv = getenv("GPU_MAX_HW_QUEUES");
  const int queues = qenv ? std::max(1, atoi(qenv)) : 4;
  int prio_least = 0, prio_greatest = 0;
  bool spread = pipeline_slots + 1 > queues;
  if (const char* e = getenv("KZGMI_STREAM_PRIO")) spread = atoi(e) != 0;
  spread = spread && hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) == hipSuccess &&
           prio_least != prio_greatest;
  c->prio_levels = spread ? std::abs(prio_least - prio_greatest) + 1 : 1;
  {
    static std::atomic<bool> warned{false};
    if (pipeline_slots > 1 && pipeline_slots + 1 > queues * c->prio_levels && !getenv("KZGMI_QUIET") &&
        !warned.exchange(true))
      fprintf(stderr, "kzgmi: %d pipeline slots on %d hardware queues (GPU_MAX_HW_QUEUES x %d stream priorities): "
                      "slots sharing a queue run one after another\n",
              pipeline_slots, queues * c->prio_levels, c->prio_levels);
  }
  if (pipeline_slots + 1 > queues * c->prio_levels) c->acc_order = c->acc_order_small = 0;  // shared queues
  if (const char* e = getenv("KZGMI_ACC_ORDER")) c->acc_order = std::min(std::max(0, atoi(e)), kzgmi_ctx::kAccOrderMax);
  if (const char* e = getenv("KZGMI_ACC_ORDER_SMALL"))
    c->acc_order_small = std::min(std::max(0, atoi(e)), kzgmi_ctx::kAccOrderMax);
  bool okc = hipStreamCreateWithFlags(&c->h2d_stream, hipStreamNonBlocking) == hipSuccess;
  c->slots.resize(pipeline_slots);
  c->user_slots = pipeline_slots;
  for (size_t k = 0; k < c->slots.size() && okc; ++k) {
    Slot& s = c->slots[k];
    const int step = prio_least > prio_greatest ? 1 : -1;  // from the greatest priority towards the least
    okc = (spread ? hipStreamCreateWithPriority(&s.stream, hipStreamNonBlocking,
                                                prio_greatest + step * (int)(k % c->prio_levels))
                  : hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking)) == hipSuccess;
    okc = okc && hipEventCreateWithFlags(&s.done_ev, hipEventDisableTiming) == hipSuccess &&
          hipEventCreateWithFlags(&s.signal_ev, hipEventDisableTiming) == hipSuccess &&
          hipHostMalloc((void**)&s.host_flags, 16, hipHostMallocDefault) == hipSuccess &&
          hipHostMalloc((void**)&s.host_out, 128, hipHostMallocDefault) == hipSuccess;
  }
  if (!okc) {
    kzgmi_ctx_destroy(c);
    return fail(KZGMI_ERR_DEVICE, "stream/event/pinned allocation failed");
  }
  *out = c;
  return 0;
}

void kzgmi_ctx_destroy(kzgmi_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->side_stream) {  // its kernels read slot buffers: drained before any is released
    (void)hipStreamSynchronize(c->side_stream);
    (void)hipStreamDestroy(c->side_stream);
  }
  for (auto& s : c->slots) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    s.for_each_buf([](DevBuf& b) { b.release(); });
    for (auto& e : s.ev)
      if (e) (void)hipEventDestroy(e);
    if (s.signal_ev) (void)hipEventDestroy(s.signal_ev);
    if (s.done_ev) (void)hipEventDestroy(s.done_ev);
    for (auto& e : s.dep_pool) (void)hipEventDestroy(e);
    for (int b = 0; b < 2; ++b) {
      if (s.ring_ev[b]) (void)hipEventDestroy(s.ring_ev[b]);
      if (s.ring[b]) (void)hipHostFree(s.ring[b]);
    }
    for (auto& e : s.side_ev)
      if (e) (void)hipEventDestroy(e);
    if (s.host_flags) (void)hipHostFree(s.host_flags);
    if (s.host_out) (void)hipHostFree(s.host_out);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  for (hipEvent_t e : c->acc_ring)
    if (e) (void)hipEventDestroy(e);
  for (int k = 0; k < 2; ++k) { c->table[k].release(); c->table_base[k].release(); }
  if (c->h2d_stream) {
    (void)hipStreamSynchronize(c->h2d_stream);
    (void)hipStreamDestroy(c->h2d_stream);
  }

  c->lines_tmp.release();
  c->tmp.release();
  for (kzgmi_ck* ck : c->ck_list) {  // detach: later kzgmi_ck_free() only deletes the struct
    ck->pts.release();
    ck->inf.release();
    ck->ctx = nullptr;
  }
  for (kzgmi_srs* srs : c->srs_list) {  // detach: later kzgmi_srs_free() only deletes the struct
    srs->lines.release();
    srs->q.release();
    srs->q_inf.release();
    srs->g1.release();
    srs->ctx = nullptr;
  }
  c->gath.release();
  c->mdig.release();
  c->mdig_all.release();
  std::vector<kzgmi_ctx*> peers;
  peers.swap(c->peers);
  delete c;
  for (kzgmi_ctx* p : peers) kzgmi_ctx_destroy(p);
}

int kzgmi_ctx_reserve(kzgmi_ctx* c, kzgmi_curve curve, size_t n, uint32_t flags) {
  CHK(check_ctx(c));
  if (flags & ~kAllFlags) return fail(KZGMI_ERR_ARG, "unknown flags");
  if ((flags & KZGMI_FLAG_POWERS) && (flags & KZGMI_FLAG_FIAT_SHAMIR))
    return fail(KZGMI_ERR_ARG, "KZGMI_FLAG_POWERS and KZGMI_FLAG_FIAT_SHAMIR are exclusive");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "batch too large (max 2^26 tuples per call)");
  for (auto& s : c->slots)
    if (s.pending) return fail(KZGMI_ERR_ARG, "kzgmi_ctx_reserve with jobs in flight");
  const Seed none{};
  for (auto& s : c->slots) {
    if (n)
      CHK(dispatch(curve, [&](auto cv) -> int {
        return enqueue_batch<decltype(cv)>(c, s, nullptr, nullptr, nullptr, nullptr, nullptr, n, none, 0, nullptr, flags,
                                           /*dry=*/true);
      }));
    for (auto& e : s.ev)  // the phase events kzgmi_set_profiling records
      if (!e) HIPCHK(hipEventCreate(&e));
  }
  // multi-device context: every device's slots take whole batches of up to n (the async entry
  // points pipeline them per device; the synchronous split runs smaller shards on the same slots)
  for (kzgmi_ctx* p : c->peers) CHK(kzgmi_ctx_reserve(p, curve, n, flags));
  return set_dev(c);
}

int kzgmi_srs_load(kzgmi_ctx* c, kzgmi_curve curve, const uint8_t* g1, const uint8_t* g2, const uint8_t* tau_g2,
                   kzgmi_srs** out) {
  CHK(check_ctx(c));
  if (!g2 || !tau_g2 || !out) return fail(KZGMI_ERR_ARG, "null srs argument");
  *out = nullptr;
  CHK(slot0_idle(c));
  int rc = dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    Slot& s = c->slots[0];
    const size_t gb = g2_bytes(Cv::ID), g1b = g1_bytes(Cv::ID);
    kzgmi_srs* srs = new kzgmi_srs();
    srs->curve = Cv::ID;
    srs->ctx = c;
    int r = 0;
    if ((r = s.stage.ensure(2 * gb + g1b)) || (r = s.flags.ensure(16)) || (r = srs->q.ensure(2 * sizeof(G2Aff<Cv>))) ||
        (r = srs->q_inf.ensure(16)) || (r = srs->lines.ensure(2 * Launch<Cv>::num_lines() * sizeof(Line<Cv>))) ||
        (r = srs->g1.ensure(2 * sizeof(Affine<Cv>) + 16))) {
      delete srs;
      return r;
    }
    // slot 0 = [tau]_2, slot 1 = [1]_2, then [1]_1
    std::vector<uint8_t> h(2 * gb + g1b);
    memcpy(h.data(), tau_g2, gb);
    memcpy(h.data() + gb, g2, gb);
    if (g1) memcpy(h.data() + 2 * gb, g1, g1b);
    if (int rb = begin_job(s)) {
      kzgmi_srs_free(srs);
      return rb;
    }
    hipStream_t st = s.stream;
    Affine<Cv>* g1p = srs->g1.template as<Affine<Cv>>();
    uint8_t* g1inf = srs->g1.template as<uint8_t>() + sizeof(Affine<Cv>);
    uint8_t g1inf_h = 0;
    bool okk = hipMemcpyAsync(s.stage.p, h.data(), h.size(), hipMemcpyHostToDevice, st) == hipSuccess &&
               hipMemsetAsync(s.flags.p, 0, 16, st) == hipSuccess;
    if (okk) {
      uint32_t* err = s.flags.template as<uint32_t>() + 1;
      Launch<Cv>::convert_g2(st, s.stage.template as<uint8_t>(), 2, srs->q.template as<G2Aff<Cv>>(), srs->q_inf.template as<uint8_t>(),
                                         err);
      Launch<Cv>::precompute_lines(st, srs->q.template as<G2Aff<Cv>>(), srs->lines.template as<Line<Cv>>());
      if (g1) {  // validated like any input point, and it must be in G1 (GLV and the check rely on it)
        Launch<Cv>::convert_points(st, s.stage.template as<uint8_t>() + 2 * gb, 1, g1p, g1inf, err);
        Launch<Cv>::subgroup_check(st, g1p, g1inf, 1, err);
      } else {   // NULL: the standard generator
        Launch<Cv>::set_generator(st, g1p, g1inf);
      }
      srs->g1_29_off = sizeof(Affine<Cv>) + 16;
      Affine<Cv>* g1p29 = static_cast<Affine<Cv>*>(srs->g1_29());
      okk = hipMemcpyAsync(g1p29, g1p, sizeof(Affine<Cv>), hipMemcpyDeviceToDevice, st) == hipSuccess;
      Launch<Cv>::pts_to29(st, g1p29, 1);
      okk = okk && hipGetLastError() == hipSuccess &&
            hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, st) == hipSuccess &&
            hipMemcpyAsync(&g1inf_h, g1inf, 1, hipMemcpyDeviceToHost, st) == hipSuccess && sync_job(s) == 0;
    }
    if (!okk) {
      kzgmi_srs_free(srs);
      return fail(KZGMI_ERR_DEVICE, "srs upload/precompute failed");
    }
    int e = map_device_err((uint32_t)s.host_flags[1]);
    if (!e && g1inf_h) e = fail(KZGMI_ERR_ARG, "SRS G1 element is the point at infinity");
    if (e) {
      kzgmi_srs_free(srs);
      return e;
    }
    c->srs_list.push_back(srs);
    *out = srs;
    return 0;
  });
  if (rc) return rc;
  for (kzgmi_ctx* p : c->peers) {  // multi-device context: the same SRS on every device
    kzgmi_srs* ps = nullptr;
    if (int r = kzgmi_srs_load(p, curve, g1, g2, tau_g2, &ps)) {
      kzgmi_srs_free(*out);
      *out = nullptr;
      return r;
    }
    (*out)->peers.push_back(ps);
  }
  return set_dev(c);
}

void kzgmi_srs_free(kzgmi_srs* srs) {
  if (!srs) return;
  for (kzgmi_srs* p : srs->peers) kzgmi_srs_free(p);
  srs->peers.clear();
  if (kzgmi_ctx* c = srs->ctx) {  // still attached: free its device memory on its device
    (void)hipSetDevice(c->device);
    auto& v = c->srs_list;
    v.erase(std::remove(v.begin(), v.end(), srs), v.end());
    srs->lines.release();
    srs->q.release();
    srs->q_inf.release();
    srs->g1.release();
  }
  delete srs;  // a detached SRS (its context already destroyed) owns no device memory
}

int kzgmi_batch_verify_device_async(kzgmi_ctx* c, const kzgmi_srs* srs, int slot, const void* dC, const void* dz,
                                    const void* dy, const void* dpi, size_t n, const uint8_t* seed32) {
  return kzgmi_batch_verify_device_ex_async(c, srs, slot, dC, dz, dy, dpi, n, seed32, 0);
}

int kzgmi_batch_verify_device_ex_async(kzgmi_ctx* c, const kzgmi_srs* srs, int slot, const void* dC, const void* dz,
                                       const void* dy, const void* dpi, size_t n, const uint8_t* seed32,
                                       uint32_t flags) {
  KZ_ROUTE(c, &srs, slot);
  if (flags & ~kAllFlags) return fail(KZGMI_ERR_ARG, "unknown flags");
  if ((flags & KZGMI_FLAG_POWERS) && (flags & KZGMI_FLAG_FIAT_SHAMIR))
    return fail(KZGMI_ERR_ARG, "KZGMI_FLAG_POWERS and KZGMI_FLAG_FIAT_SHAMIR are exclusive");
  if ((flags & KZGMI_FLAG_POWERS) && !seed32) return fail(KZGMI_ERR_ARG, "KZGMI_FLAG_POWERS needs r in seed32");
  CHK(check_ctx(c, slot));
  if (!srs || srs->ctx != c) return fail(KZGMI_ERR_ARG, "srs does not belong to this context");
  if (n && (!dC || !dz || !dy || !dpi)) return fail(KZGMI_ERR_ARG, "null input");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "batch too large (max 2^26 tuples per call)");
  Slot& s = c->slots[slot];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot busy: call kzgmi_slot_wait first");
  uint8_t sb[32];
  Seed seed = make_seed(seed32, sb);
  if (n == 0) {
    CHK(set_dev(c));
    CHK(sync_slot(s));  // host_flags may still be the target of a copy
    s.host_flags[0] = 1;
    s.host_flags[1] = 0;
    s.pending = true;
    s.partial_job = false;
    s.partial_of = 0;
    s.msm_job = false;
    return 0;
  }
  Roctx rx("kzgmi_batch_verify_device_ex_async");
  return dispatch(srs->curve, [&](auto cv) -> int {
    return enqueue_batch<decltype(cv)>(c, s, srs, dC, dz, dy, dpi, n, seed, 0, nullptr, flags);
  });
}

int kzgmi_slot_wait(kzgmi_ctx* c, int slot, int* ok_out) {
  KZ_ROUTE(c, nullptr, slot);
  CHK(check_ctx(c, slot));
  Slot& s = c->slots[slot];
  if (!s.pending) return fail(KZGMI_ERR_ARG, "slot has no pending batch");
  return finish_slot(c, s, ok_out);
}

int kzgmi_batch_verify_device(kzgmi_ctx* c, const kzgmi_srs* srs, const void* dC, const void* dz, const void* dy,
                              const void* dpi, size_t n, const uint8_t* seed32, int* ok_out) {
  if (!ok_out) return fail(KZGMI_ERR_ARG, "null ok_out");
  c->sync_call = true;
  const int rc = kzgmi_batch_verify_device_async(c, srs, 0, dC, dz, dy, dpi, n, seed32);
  c->sync_call = false;
  CHK(rc);
  return kzgmi_slot_wait(c, 0, ok_out);
}

}  // extern "C"
namespace {
// The host arrays of one batch into the slot's stage buffer on the context's FIFO copy stream
// (pinned ranges DMA'd directly, pageable ones staged by the copy pool before this returns); the
// slot's next job waits for the copy.
int stage_host_batch(kzgmi_ctx* c, Slot& s, const kzgmi_srs* srs, uint32_t flags, const uint8_t* commitments,
                     const uint8_t* zs, const uint8_t* ys, const uint8_t* proofs, size_t n, const uint8_t** dC_out,
                     const uint8_t** dz_out, const uint8_t** dy_out, const uint8_t** dpi_out) {
  const size_t gb = (flags & KZGMI_FLAG_COMPRESSED) ? g1_bytes(srs->curve) / 2 : g1_bytes(srs->curve);
  CHK(s.stage.ensure(n * (2 * gb + 64)));
  uint8_t* dC = s.stage.template as<uint8_t>();
  uint8_t* dpi = dC + n * gb;
  uint8_t* dz = dC + 2 * n * gb;
  uint8_t* dy = dz + 32 * n;
  hipStream_t cs = c->h2d_stream;
  // the copy overwrites s.stage: after the slot's previous job
  if (s.done_rec) HIPCHK(hipStreamWaitEvent(cs, s.done_ev, 0));
  if (c->profiling) {
    if (!s.ev[EV_H2D0]) HIPCHK(hipEventCreate(&s.ev[EV_H2D0]));
    if (!s.ev[EV_H2D1]) HIPCHK(hipEventCreate(&s.ev[EV_H2D1]));
    HIPCHK(hipEventRecord(s.ev[EV_H2D0], cs));
  }
  CHK(h2d(s, cs, dC, commitments, n * gb));
  CHK(h2d(s, cs, dpi, proofs, n * gb));
  CHK(h2d(s, cs, dz, zs, n * 32));
  CHK(h2d(s, cs, dy, ys, n * 32));
  if (c->profiling) HIPCHK(hipEventRecord(s.ev[EV_H2D1], cs));
  CHK(add_dep(s, cs));  // the batch's kernels wait for its copy only
  *dC_out = dC;
  *dz_out = dz;
  *dy_out = dy;
  *dpi_out = dpi;
  return 0;
}

std::vector<size_t> split_units(size_t n, int D);  // below: balanced ranges in units of 4096 tuples

// Synchronous host-buffer batches on one device: the PCIe copy (~5 ms per 2^20 batch) would sit
// in front of the whole computation.  Split into k point ranges (units of 4096 tuples) on slots
// 0..k-1: range j's shard partial starts as soon as its own copy has landed, while the next
// range copies, and one combine + pairing on slot 0 decides (the same sums: r_i use the global
// index; a failed range marks its partial records, so the combine reports its error).  Batches
// without flags (or with TRUSTED_G1) instead accumulate every range into one bucket store
// (enqueue_batch_chunked): no per-range reduction.  From 2^17 tuples: 4 ranges with one store (2^20 pinned: 13.7 -> 11.0
// ms, pageable 14.1 -> 11.3), 2 with partials (12.1 / 12.5 ms; profiles/r05/host_latency_*.txt).
// KZGMI_HOST_CHUNKS overrides (1: never); not with Fiat-Shamir (the challenge needs every range
// first) or when slots 0..k-1 are not all idle.
bool one_store_flags(uint32_t flags) { return (flags & ~KZGMI_FLAG_TRUSTED_G1) == 0; }
int host_chunks(const kzgmi_ctx* c, size_t n, uint32_t flags, int curve) {
  (void)curve;
  if (flags & KZGMI_FLAG_FIAT_SHAMIR) return 1;
  const bool one_store = one_store_flags(flags) && c->host_chunk_mode != 1;
  int k = n >= (size_t(1) << 17) ? (one_store ? 4 : 2) : 1;
  if (c->host_chunks_env) k = c->host_chunks_env;
  k = std::min<int>(k, (int)((n + FS_CHUNK - 1) / FS_CHUNK));
  // the one-store form runs every range on slot 0 (slot0_idle checked it); the shard-partial
  // form takes slots 0..k-1, which must exist and be idle
  if (one_store) return std::max(k, 1);
  k = std::min<int>(k, (int)c->slots.size());
  for (int j = 0; j < k; ++j)
    if (c->slots[j].pending) return 1;
  return std::max(k, 1);
}

int batch_host_chunked(kzgmi_ctx* c, const kzgmi_srs* srs, const uint8_t* commitments, const uint8_t* zs,
                       const uint8_t* ys, const uint8_t* proofs, size_t n, const uint8_t* seed32, uint32_t flags,
                       int k, int* ok_out) {
  Roctx rx("kzgmi_batch_verify_ex.chunked");
  uint8_t sb[32];
  if (!seed32) {  // one verifier-private seed for every range
    make_seed(nullptr, sb);
    seed32 = sb;
  }
  if (one_store_flags(flags) && c->host_chunk_mode != 1) {
    // one bucket store for every range (no per-range reduction)
    Slot& s = c->slots[0];
    uint8_t sb2[32];
    const Seed seed = make_seed(seed32, sb2);
    const int r = dispatch(srs->curve, [&](auto cv) -> int {
      return enqueue_batch_chunked<decltype(cv)>(c, s, srs, commitments, zs, ys, proofs, n, seed, flags, k);
    });
    if (r) {
      // whatever was enqueued drains before the error returns: the slot's kernels of this call
      // (end_job never ran, so done_ev still marks the previous job) and the copies that may
      // still read the caller's buffers
      const std::string msg = g_err;
      (void)hipStreamSynchronize(s.stream);
      (void)hipStreamSynchronize(c->h2d_stream);
      s.ndep = 0;
      s.pending = false;
      return fail(r, msg);
    }
    return kzgmi_slot_wait(c, 0, ok_out);
  }
  const size_t gb = (flags & KZGMI_FLAG_COMPRESSED) ? g1_bytes(srs->curve) / 2 : g1_bytes(srs->curve);
  const size_t rec = 2 * kzgmi_partial_bytes((kzgmi_curve)srs->curve);
  CHK(c->gath.ensure((size_t)k * rec));
  const std::vector<size_t> nk = split_units(n, k);
  size_t lo = 0;
  int started = 0, r = 0;
  for (int j = 0; j < k && !r; ++j) {
    const uint8_t *dC, *dz, *dy, *dpi;
    r = stage_host_batch(c, c->slots[j], srs, flags, commitments + lo * gb, zs + lo * 32, ys + lo * 32,
                         proofs + lo * gb, nk[j], &dC, &dz, &dy, &dpi);
    if (!r)
      r = kzgmi_batch_partial_device_async(c, srs, j, dC, dz, dy, dpi, nk[j], lo, seed32, flags,
                                           (uint8_t*)c->gath.p + (size_t)j * rec);
    if (!r) ++started;
    lo += nk[j];
  }
  // every started range completes before the combine reads the records (a range's own error is
  // carried by its marked records)
  const std::string msg = r ? g_err : std::string();
  for (int j = 0; j < started; ++j) (void)kzgmi_slot_wait(c, j, nullptr);
  if (r) return fail(r, msg);
  return kzgmi_batch_combine_device(c, srs, c->gath.p, k, ok_out);
}
}  // namespace
extern "C" {

int kzgmi_batch_verify(kzgmi_ctx* c, const kzgmi_srs* srs, const uint8_t* commitments, const uint8_t* zs,
                       const uint8_t* ys, const uint8_t* proofs, size_t n, const uint8_t* seed32, int* ok_out) {
  return kzgmi_batch_verify_ex(c, srs, commitments, zs, ys, proofs, n, seed32, 0, ok_out);
}

int kzgmi_batch_verify_ex(kzgmi_ctx* c, const kzgmi_srs* srs, const uint8_t* commitments, const uint8_t* zs,
                          const uint8_t* ys, const uint8_t* proofs, size_t n, const uint8_t* seed32, uint32_t flags,
                          int* ok_out) {
  CHK(check_ctx(c));
  if (!srs || !ok_out) return fail(KZGMI_ERR_ARG, "null argument");
  if (srs->ctx != c) return fail(KZGMI_ERR_ARG, "srs does not belong to this context");
  if (n && (!commitments || !zs || !ys || !proofs)) return fail(KZGMI_ERR_ARG, "null input");
  CHK(slot0_idle(c));
  if (!c->peers.empty()) return batch_multi_host(c, srs, commitments, zs, ys, proofs, n, seed32, flags, ok_out);
  const int k = host_chunks(c, n, flags, srs->curve);
  if (k > 1) return batch_host_chunked(c, srs, commitments, zs, ys, proofs, n, seed32, flags, k, ok_out);
  CHK(kzgmi_batch_verify_ex_async(c, srs, 0, commitments, zs, ys, proofs, n, seed32, flags));
  return kzgmi_slot_wait(c, 0, ok_out);
}

int kzgmi_batch_verify_ex_async(kzgmi_ctx* c, const kzgmi_srs* srs, int slot, const uint8_t* commitments,
                                const uint8_t* zs, const uint8_t* ys, const uint8_t* proofs, size_t n,
                                const uint8_t* seed32, uint32_t flags) {
  if (!srs) return fail(KZGMI_ERR_ARG, "null argument");
  KZ_ROUTE(c, &srs, slot);
  CHK(check_ctx(c, slot));
  if (srs->ctx != c) return fail(KZGMI_ERR_ARG, "srs does not belong to this context");
  if (n && (!commitments || !zs || !ys || !proofs)) return fail(KZGMI_ERR_ARG, "null input");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "batch too large (max 2^26 tuples per call)");
  if (flags & ~kAllFlags) return fail(KZGMI_ERR_ARG, "unknown flags");
  Slot& s = c->slots[slot];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot busy: call kzgmi_slot_wait first");
  if (n == 0) return kzgmi_batch_verify_device_ex_async(c, srs, slot, nullptr, nullptr, nullptr, nullptr, 0, seed32, flags);
  Roctx rx("kzgmi_batch_verify_ex_async");
  const uint8_t *dC, *dz, *dy, *dpi;
  CHK(stage_host_batch(c, s, srs, flags, commitments, zs, ys, proofs, n, &dC, &dz, &dy, &dpi));
  const int r = kzgmi_batch_verify_device_ex_async(c, srs, slot, dC, dz, dy, dpi, n, seed32, flags);
  if (c->profiling) s.ev_used[EV_H2D0] = s.ev_used[EV_H2D1] = (r == 0);
  return r;
}

// ------------------------------------------------------------------------------ pinned host memory
int kzgmi_host_alloc(size_t bytes, void** out) {
  if (!out || bytes == 0) return fail(KZGMI_ERR_ARG, "bad argument");
  *out = nullptr;
  void* p = nullptr;
  HIPCHK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
  std::lock_guard<std::mutex> lk(g_host_mu);
  g_host[(uintptr_t)p] = HostRange{(uintptr_t)p + bytes, true};
  *out = p;
  return 0;
}

void kzgmi_host_free(void* p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host.find((uintptr_t)p);
    if (it == g_host.end() || !it->second.owned) return;  // not ours: leave it alone
    g_host.erase(it);
  }
  (void)hipHostFree(p);
}

int kzgmi_host_register(void* p, size_t bytes) {
  if (!p || bytes == 0) return fail(KZGMI_ERR_ARG, "bad argument");
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    if (g_host.count((uintptr_t)p)) return fail(KZGMI_ERR_ARG, "range already registered");
  }
  HIPCHK(hipHostRegister(p, bytes, hipHostRegisterDefault));
  std::lock_guard<std::mutex> lk(g_host_mu);
  g_host[(uintptr_t)p] = HostRange{(uintptr_t)p + bytes, false};
  return 0;
}

int kzgmi_host_unregister(void* p) {
  {
    std::lock_guard<std::mutex> lk(g_host_mu);
    auto it = g_host.find((uintptr_t)p);
    if (it == g_host.end() || it->second.owned) return fail(KZGMI_ERR_ARG, "range was not registered");
    g_host.erase(it);
  }
  HIPCHK(hipHostUnregister(p));
  return 0;
}

int kzgmi_last_combination(kzgmi_ctx* c, uint8_t* a_out, uint8_t* b_out) {
  CHK(check_ctx(c));
  if (!a_out || !b_out) return fail(KZGMI_ERR_ARG, "null output");
  CHK(slot0_idle(c));
  Slot& s = c->slots[0];
  if (!s.res.p) return fail(KZGMI_ERR_ARG, "no batch has run on slot 0");
  return dispatch(s.curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    const size_t gb = g1_bytes(Cv::ID);
    CHK(s.outb.ensure(2 * gb));
    CHK(begin_job(s));
    Launch<Cv>::encode_points(s.stream, s.res.template as<Xyzz<Cv>>(), 2, s.outb.template as<uint8_t>());
    HIPCHK(hipGetLastError());
    std::vector<uint8_t> h(2 * gb);
    HIPCHK(hipMemcpyAsync(h.data(), s.outb.p, 2 * gb, hipMemcpyDeviceToHost, s.stream));
    CHK(sync_job(s));
    memcpy(a_out, h.data(), gb);
    memcpy(b_out, h.data() + gb, gb);
    return 0;
  });
}

// ------------------------------------------------------------------------------ MSM
}  // extern "C"
namespace {
template <class Cv>
int enqueue_msm(kzgmi_ctx* c, Slot& s, const void* dpts, const void* dsc, size_t n, bool allow_glv = true) {
  const bool glv = allow_glv && c->glv_msm && (Cv::ID == 1 || c->msm_trusted_g1);
  CHK(s.pts.ensure((glv ? 2 : 1) * n * sizeof(Affine<Cv>)));
  CHK(s.inf.ensure((glv ? 2 : 1) * n));
  CHK(s.scal_s.ensure(n * 32));
  if (glv) CHK(s.glv_s.ensure(n * 32));
  CHK(s.flags.ensure(16));
  CHK(begin_job(s));
  hipStream_t st = s.stream;
  mark(c, s, 0);
  HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, st));
  uint32_t* err = s.flags.template as<uint32_t>() + 1;
  Affine<Cv>* pts = s.pts.template as<Affine<Cv>>();
  uint8_t* inf = s.inf.template as<uint8_t>();
  const bool pts29 = true;
  if (glv && pts29)  // phi(P) stored by the converting pass
    Launch<Cv>::convert_points(st, (const uint8_t*)dpts, (uint32_t)n, pts, inf, err, true, pts + n, inf + n);
  else
    Launch<Cv>::convert_points(st, (const uint8_t*)dpts, (uint32_t)n, pts, inf, err, pts29);
  if (glv && !pts29) Launch<Cv>::endo_points(st, pts, inf, (uint32_t)n, pts + n, inf + n, pts29);
  mark(c, s, PH_CONVERT + 1);
  uint32_t* sc = s.scal_s.template as<uint32_t>();
  Launch<Cv>::convert_scalars(st, (const uint8_t*)dsc, (uint32_t)n, sc, err);
  uint32_t* gs = s.glv_s.template as<uint32_t>();
  if (glv) Launch<Cv>::glv_split(st, sc, 8, (uint32_t)n, gs, gs + 4 * n);
  mark(c, s, PH_SCALARS + 1);
  TermList tl{};
  const uint32_t nn = (uint32_t)n;
  const int wb = call_wbits(c, (size_t)16 * n, size_t(1) << 21);
  const uint32_t H = windows_half(wb), F = windows_full(wb);
  if (glv) {  // sum k_i P_i = sum h0_i P_i + h1_i phi(P_i): H windows, H bucket sets
    tl.c[0] = {nn, 0, 4, H, 0, 4, gs};
    tl.c[1] = {nn, nn, 4, H, 0, 4, gs + 4 * n};
    tl.nclass = 2;
    tl.total = 2 * nn;
    const MsmWindows mw{1, {0, 0}, {H, 0}};
    CHK(run_msm_core<Cv>(c, s, tl, H, (size_t)2 * H * n + 16, mw, nullptr, nullptr, pts29, false, wb));
  } else {
    tl.c[0] = {nn, 0, 8, F, 0, 8, sc};
    tl.nclass = 1;
    tl.total = nn;
    const MsmWindows mw{1, {0, 0}, {F, 0}};
    CHK(run_msm_core<Cv>(c, s, tl, F, (size_t)F * n + 16, mw, nullptr, nullptr, pts29, false, wb));
  }
  s.curve = Cv::ID;
  return 0;
}

int read_flags_sync(kzgmi_ctx* c, Slot& s) {
  HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, s.stream));
  CHK(sync_job(s));
  collect_phases(c, s);
  return map_device_err((uint32_t)s.host_flags[1]);
}
}  // namespace
extern "C" {

// ------------------------------------------------------------------------------ prover commit key
int kzgmi_ck_load(kzgmi_ctx* c, kzgmi_curve curve, const uint8_t* g1_powers, size_t n, kzgmi_ck** out) {
  CHK(check_ctx(c));
  if (!g1_powers || !out || n == 0) return fail(KZGMI_ERR_ARG, "bad commit key argument");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "commit key too large (max 2^26 points)");
  Slot& s = c->slots[0];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot 0 busy: call kzgmi_slot_wait first");
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    using L = Launch<Cv>;
    const size_t gb = g1_bytes(Cv::ID);
    kzgmi_ck* ck = new kzgmi_ck();
    ck->curve = Cv::ID;
    ck->n = n;
    ck->ctx = c;
    int r = 0;
    if ((r = ck->pts.ensure((size_t)CK_ROWS * n * sizeof(Affine<Cv>))) || (r = ck->inf.ensure((size_t)CK_ROWS * n)) ||
        (r = s.stage.ensure(n * gb)) || (r = s.flags.ensure(16))) {
      delete ck;
      return r;
    }
    if (int rb = begin_job(s)) {
      delete ck;
      return rb;
    }
    hipStream_t st = s.stream;
    Affine<Cv>* pts = ck->pts.template as<Affine<Cv>>();
    uint8_t* inf = ck->inf.template as<uint8_t>();
    bool okk = hipMemcpyAsync(s.stage.p, g1_powers, n * gb, hipMemcpyHostToDevice, st) == hipSuccess &&
               hipMemsetAsync(s.flags.p, 0, 16, st) == hipSuccess;
    if (okk) {
      L::convert_points(st, s.stage.template as<uint8_t>(), (uint32_t)n, pts, inf, s.flags.template as<uint32_t>() + 1);
      for (int w = 1; w < CK_ROWS; ++w)
        L::shift_points(st, pts + (size_t)(w - 1) * n, inf + (size_t)(w - 1) * n, (uint32_t)n, pts + (size_t)w * n,
                        inf + (size_t)w * n);
      L::pts_to29(st, pts, (uint32_t)(CK_ROWS * n));  // resident in the accumulation's format
      okk = okk && hipGetLastError() == hipSuccess &&
            hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, st) == hipSuccess && sync_job(s) == 0;
    }
    if (!okk) {
      delete ck;
      return fail(KZGMI_ERR_DEVICE, "commit key upload/precompute failed");
    }
    if (int e = map_device_err((uint32_t)s.host_flags[1])) {
      delete ck;
      return e;
    }
    c->ck_list.push_back(ck);
    *out = ck;
    return 0;
  });
}

void kzgmi_ck_free(kzgmi_ck* ck) {
  if (!ck) return;
  if (kzgmi_ctx* c = ck->ctx) {
    (void)hipSetDevice(c->device);
    auto& v = c->ck_list;
    v.erase(std::remove(v.begin(), v.end(), ck), v.end());
    ck->pts.release();
    ck->inf.release();
  }
  delete ck;
}

int kzgmi_commit_device_async(kzgmi_ctx* c, const kzgmi_ck* ck, int slot, const void* d_coeffs, size_t m) {
  KZ_ROUTE(c, nullptr, slot);  // (commit keys live on the primary device: its slots only)
  CHK(check_ctx(c, slot));
  if (!ck || ck->ctx != c) return fail(KZGMI_ERR_ARG, "commit key does not belong to this context");
  if (m && !d_coeffs) return fail(KZGMI_ERR_ARG, "null argument");
  if (m > ck->n) return fail(KZGMI_ERR_ARG, "more coefficients than commit-key points");
  Slot& s = c->slots[slot];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot busy: call kzgmi_msm_wait first");
  return dispatch(ck->curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    using L = Launch<Cv>;
    const size_t gb = g1_bytes(Cv::ID);
    CHK(s.flags.ensure(16));
    CHK(s.outb.ensure(gb));
    CHK(s.res.ensure(2 * sizeof(Xyzz<Cv>)));
    CHK(begin_job(s));
    hipStream_t st = s.stream;
    HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, st));
    if (m == 0) {
      HIPCHK(hipMemsetAsync(s.res.p, 0, sizeof(Xyzz<Cv>), st));  // zz = 0: infinity
    } else {
      CHK(s.scal_s.ensure(m * 32));
      mark(c, s, 0);
      L::convert_scalars(st, (const uint8_t*)d_coeffs, (uint32_t)m, s.scal_s.template as<uint32_t>(),
                         s.flags.template as<uint32_t>() + 1);
      mark(c, s, PH_SCALARS + 1);
      // one class per 16-bit window w: the points of row w (2^(16 w) P_i) take digit w of the
      // coefficient; every class feeds the same bucket set, so no per-window reduction and no
      // window combination
      TermList tl{};
      for (int w = 0; w < CK_ROWS; ++w)
        tl.c[w] = {(uint32_t)m, (uint32_t)(w * ck->n), 8, 1, 0, 8, s.scal_s.template as<uint32_t>(), (uint32_t)w};
      tl.nclass = CK_ROWS;
      tl.total = (uint32_t)(CK_ROWS * m);
      MsmWindows mw{1, {0, 0}, {1, 0}};
      CHK(run_msm_core<Cv>(c, s, tl, 1, (size_t)CK_ROWS * m + 16, mw, ck->pts.template as<Affine<Cv>>(),
                           ck->inf.template as<uint8_t>()));
    }
    Launch<Cv>::encode_points(st, s.res.template as<Xyzz<Cv>>(), 1, s.outb.template as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s.host_out, s.outb.p, gb, hipMemcpyDeviceToHost, st));
    HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, st));
    CHK(end_job(s));
    s.pending = true;
    s.partial_job = false;
    s.partial_of = 0;
    s.msm_job = true;
    s.curve = Cv::ID;
    return 0;
  });
}

int kzgmi_commit_device(kzgmi_ctx* c, const kzgmi_ck* ck, const void* d_coeffs, size_t m, uint8_t* out) {
  if (!out) return fail(KZGMI_ERR_ARG, "null argument");
  CHK(kzgmi_commit_device_async(c, ck, 0, d_coeffs, m));
  return kzgmi_msm_wait(c, 0, out);
}

int kzgmi_commit(kzgmi_ctx* c, const kzgmi_ck* ck, const uint8_t* coeffs, size_t m, uint8_t* out) {
  CHK(check_ctx(c));
  if (!ck || (m && !coeffs)) return fail(KZGMI_ERR_ARG, "null argument");
  if (m == 0) return kzgmi_commit_device(c, ck, nullptr, 0, out);
  CHK(slot0_idle(c));
  Slot& s = c->slots[0];
  CHK(s.stage.ensure(m * 32));
  CHK(begin_job(s));  // the commit's job starts in the same lane, behind this copy
  HIPCHK(hipMemcpyAsync(s.stage.p, coeffs, m * 32, hipMemcpyHostToDevice, s.stream));
  return kzgmi_commit_device(c, ck, s.stage.p, m, out);
}

int kzgmi_msm_g1_device(kzgmi_ctx* c, kzgmi_curve curve, const void* dpts, const void* dsc, size_t n, uint8_t* out) {
  CHK(check_ctx(c));
  if (!out || (n && (!dpts || !dsc))) return fail(KZGMI_ERR_ARG, "null argument");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "MSM too large (max 2^26 points per call)");
  CHK(slot0_idle(c));
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    Slot& s = c->slots[0];
    const size_t gb = g1_bytes(Cv::ID);
    if (n == 0) {
      memset(out, 0, gb);
      if (Cv::ID == 0) out[0] = 0x40;
      return 0;
    }
    CHK(enqueue_msm<Cv>(c, s, dpts, dsc, n));
    CHK(s.outb.ensure(gb));
    Launch<Cv>::encode_points(s.stream, s.res.template as<Xyzz<Cv>>(), 1, s.outb.template as<uint8_t>());
    HIPCHK(hipGetLastError());
    CHK(read_flags_sync(c, s));
    HIPCHK(hipMemcpy(out, s.outb.p, gb, hipMemcpyDeviceToHost));
    return 0;
  });
}

int kzgmi_msm_g1_device_async(kzgmi_ctx* c, kzgmi_curve curve, int slot, const void* dpts, const void* dsc,
                              size_t n) {
  KZ_ROUTE(c, nullptr, slot);
  CHK(check_ctx(c, slot));
  if (n && (!dpts || !dsc)) return fail(KZGMI_ERR_ARG, "null argument");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "MSM too large (max 2^26 points per call)");
  Slot& s = c->slots[slot];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot busy: call kzgmi_msm_wait first");
  Roctx rx("kzgmi_msm_g1_device_async");
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    const size_t gb = g1_bytes(Cv::ID);
    if (n == 0) {
      CHK(sync_slot(s));  // host_out/host_flags may still be copy targets
      memset(s.host_out, 0, gb);
      if (Cv::ID == 0) s.host_out[0] = 0x40;
      s.host_flags[0] = 1;
      s.host_flags[1] = 0;
    } else {
      CHK(enqueue_msm<Cv>(c, s, dpts, dsc, n));
      CHK(s.outb.ensure(gb));
      Launch<Cv>::encode_points(s.stream, s.res.template as<Xyzz<Cv>>(), 1, s.outb.template as<uint8_t>());
      HIPCHK(hipGetLastError());
      HIPCHK(hipMemcpyAsync(s.host_out, s.outb.p, gb, hipMemcpyDeviceToHost, s.stream));
      HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, s.stream));
      CHK(end_job(s));
    }
    s.pending = true;
    s.partial_job = false;
    s.partial_of = 0;
    s.msm_job = true;
    s.curve = Cv::ID;
    return 0;
  });
}

int kzgmi_msm_wait(kzgmi_ctx* c, int slot, uint8_t* out) {
  KZ_ROUTE(c, nullptr, slot);
  CHK(check_ctx(c, slot));
  Slot& s = c->slots[slot];
  if (!s.pending || !s.msm_job) return fail(KZGMI_ERR_ARG, "slot has no pending MSM");
  int ok = 0;
  CHK(finish_slot(c, s, &ok));
  if (out) memcpy(out, s.host_out, g1_bytes(s.curve));
  return 0;
}

int kzgmi_msm_g1(kzgmi_ctx* c, kzgmi_curve curve, const uint8_t* points, const uint8_t* scalars, size_t n,
                 uint8_t* out) {
  CHK(check_ctx(c));
  if (!out || (n && (!points || !scalars))) return fail(KZGMI_ERR_ARG, "null argument");
  if (curve != KZGMI_BLS12_381 && curve != KZGMI_BN254) return fail(KZGMI_ERR_ARG, "unknown curve");
  if (n == 0) return kzgmi_msm_g1_device(c, curve, nullptr, nullptr, 0, out);
  CHK(slot0_idle(c));
  if (!c->peers.empty()) return msm_multi_host(c, curve, points, scalars, n, out);
  Slot& s = c->slots[0];
  const size_t gb = g1_bytes(curve);
  CHK(s.stage.ensure(n * (gb + 32)));
  uint8_t* dp = s.stage.template as<uint8_t>();
  uint8_t* ds = dp + n * gb;
  CHK(begin_job(s));  // the MSM's job starts in the same lane, behind these copies
  HIPCHK(hipMemcpyAsync(dp, points, n * gb, hipMemcpyHostToDevice, s.stream));
  HIPCHK(hipMemcpyAsync(ds, scalars, n * 32, hipMemcpyHostToDevice, s.stream));
  return kzgmi_msm_g1_device(c, curve, dp, ds, n, out);
}

// ------------------------------------------------------------------------------ multi-GPU
size_t kzgmi_partial_bytes(kzgmi_curve curve) {
  return curve == KZGMI_BLS12_381 ? sizeof(Xyzz<Bls12_381>) : sizeof(Xyzz<Bn254>);
}

int kzgmi_batch_partial_device_async(kzgmi_ctx* c, const kzgmi_srs* srs, int slot, const void* dC, const void* dz,
                                     const void* dy, const void* dpi, size_t n, uint64_t index_offset,
                                     const uint8_t* seed32, uint32_t flags, void* d_partial_out) {
  KZ_ROUTE(c, &srs, slot);
  Roctx rx("kzgmi_batch_partial_device_async");
  if (flags & ~kAllFlags) return fail(KZGMI_ERR_ARG, "unknown flags");
  if (flags & KZGMI_FLAG_FIAT_SHAMIR)
    return fail(KZGMI_ERR_ARG, "shards take the Fiat-Shamir r as seed32 (see kzgmi_fs_challenge_from_digests_device)");
  // r^i is built from the FS_POW_BITS = 32 low bits of the global index (fs.hpp): indices at or
  // above 2^32 would wrap and repeat randomisers
  if ((flags & KZGMI_FLAG_POWERS) && (index_offset > (1ull << 32) || n > (1ull << 32) - index_offset))
    return fail(KZGMI_ERR_ARG, "KZGMI_FLAG_POWERS needs index_offset + n <= 2^32");
  CHK(check_ctx(c, slot));
  if (!srs || srs->ctx != c || !d_partial_out) return fail(KZGMI_ERR_ARG, "bad argument");
  if (!seed32) return fail(KZGMI_ERR_ARG, "sharded verification needs an explicit shared seed");
  if (n && (!dC || !dz || !dy || !dpi)) return fail(KZGMI_ERR_ARG, "null input");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "batch too large (max 2^26 tuples per call)");
  Slot& s = c->slots[slot];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot busy: call kzgmi_slot_wait first");
  uint8_t sb[32];
  Seed seed = make_seed(seed32, sb);
  return dispatch(srs->curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    if (n == 0) {  // empty shard: both partials are the point at infinity (zz = 0)
      CHK(s.flags.ensure(16));
      CHK(begin_job(s));
      HIPCHK(hipMemsetAsync(d_partial_out, 0, 2 * sizeof(Xyzz<Cv>), s.stream));
      HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, s.stream));  // a chained combine keeps the error word
      CHK(sync_job(s));
      s.host_flags[0] = 1;
      s.host_flags[1] = 0;
      s.pending = true;
      s.partial_job = true;
      s.partial_of = 1;
      s.msm_job = false;
      s.curve = Cv::ID;
      return 0;
    }
    return enqueue_batch<Cv>(c, s, srs, dC, dz, dy, dpi, n, seed, index_offset, d_partial_out, flags);
  });
}

int kzgmi_batch_partial_device(kzgmi_ctx* c, const kzgmi_srs* srs, const void* dC, const void* dz, const void* dy,
                               const void* dpi, size_t n, uint64_t index_offset, const uint8_t* seed32,
                               void* d_partial_out) {
  CHK(kzgmi_batch_partial_device_async(c, srs, 0, dC, dz, dy, dpi, n, index_offset, seed32, 0, d_partial_out));
  return kzgmi_slot_wait(c, 0, nullptr);
}

int kzgmi_batch_combine_device_async(kzgmi_ctx* c, const kzgmi_srs* srs, int slot, const void* d_partials,
                                     int n_parts) {
  KZ_ROUTE(c, &srs, slot);
  CHK(check_ctx(c, slot));
  if (!srs || srs->ctx != c || !d_partials || n_parts < 1) return fail(KZGMI_ERR_ARG, "bad argument");
  Slot& s = c->slots[slot];
  // chained: behind this slot's own pending batch partial (one kzgmi_slot_wait completes both;
  // the partial's error word is kept, the pairing writes the verdict word)
  const bool chain = s.pending && s.partial_of == 1;
  if (s.pending && !chain) return fail(KZGMI_ERR_ARG, "slot busy: call kzgmi_slot_wait first");
  if (chain && s.curve != srs->curve) return fail(KZGMI_ERR_ARG, "chained combine: curve differs from the partial's");
  return dispatch(srs->curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    using XY = Xyzz<Cv>;
    CHK(s.res.ensure(2 * sizeof(XY)));
    CHK(s.flags.ensure(16));
    CHK(begin_job(s));  // chained: the lane the partial ended in
    hipStream_t st = s.stream;
    if (!chain) {
      HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, st));
      mark(c, s, PH_COMBINE);
    }
    Launch<Cv>::sum_partials(st, (const XY*)d_partials, (uint32_t)n_parts, 2, 2, s.res.template as<XY>(),
                             s.flags.template as<uint32_t>() + 1);
    Launch<Cv>::pairing_check(st, s.res.template as<XY>(), srs->lines.template as<Line<Cv>>(),
                              srs->q_inf.template as<uint8_t>(), s.flags.template as<int>());
    mark(c, s, PH_PAIRING + 1);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, st));
    CHK(end_job(s));
    s.pending = true;
    s.partial_job = false;
    s.partial_of = 0;
    s.msm_job = false;
    s.curve = Cv::ID;
    return 0;
  });
}

int kzgmi_batch_combine_device(kzgmi_ctx* c, const kzgmi_srs* srs, const void* d_partials, int n_parts, int* ok_out) {
  if (!ok_out) return fail(KZGMI_ERR_ARG, "null ok_out");
  CHK(kzgmi_batch_combine_device_async(c, srs, 0, d_partials, n_parts));
  return kzgmi_slot_wait(c, 0, ok_out);
}

int kzgmi_g1_validate_device(kzgmi_ctx* c, kzgmi_curve curve, const void* d_points, size_t n, uint32_t flags) {
  CHK(check_ctx(c));
  if (flags & ~(KZGMI_FLAG_COMPRESSED | KZGMI_FLAG_SUBGROUP_CHECK)) return fail(KZGMI_ERR_ARG, "unknown flags");
  if (n && !d_points) return fail(KZGMI_ERR_ARG, "null input");
  if (n > (1u << 27)) return fail(KZGMI_ERR_ARG, "too many points (max 2^27 per call)");
  if (n == 0) return 0;
  Slot& s = c->slots[0];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot 0 busy: call kzgmi_slot_wait first");
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    using L = Launch<Cv>;
    CHK(s.pts.ensure(n * sizeof(Affine<Cv>)));
    CHK(s.inf.ensure(n));
    CHK(s.flags.ensure(16));
    CHK(begin_job(s));
    hipStream_t st = s.stream;
    HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, st));
    uint32_t* err = s.flags.template as<uint32_t>() + 1;
    if (flags & KZGMI_FLAG_COMPRESSED)
      L::decompress_points(st, (const uint8_t*)d_points, (uint32_t)n, s.pts.template as<Affine<Cv>>(),
                           s.inf.template as<uint8_t>(), err);
    else
      L::convert_points(st, (const uint8_t*)d_points, (uint32_t)n, s.pts.template as<Affine<Cv>>(),
                        s.inf.template as<uint8_t>(), err);
    if (flags & KZGMI_FLAG_SUBGROUP_CHECK)
      L::subgroup_check(st, s.pts.template as<Affine<Cv>>(), s.inf.template as<uint8_t>(), (uint32_t)n, err);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, st));
    CHK(end_job(s));
    s.pending = true;
    s.partial_job = true;
    s.msm_job = false;
    return finish_slot(c, s, nullptr);
  });
}

// the chunk digests of kzgmi_fs_chunk_digests_device, enqueued on slot 0's stream (no wait)
static int fs_chunk_digests_enqueue(kzgmi_ctx* c, kzgmi_curve curve, const void* dC, const void* dz, const void* dy,
                                    const void* dpi, size_t n, uint64_t index_offset, uint32_t flags, void* d_out) {
  CHK(check_ctx(c));
  if (!d_out || (n && (!dC || !dz || !dy || !dpi)) || n == 0) return fail(KZGMI_ERR_ARG, "bad argument");
  if (index_offset % FS_CHUNK) return fail(KZGMI_ERR_ARG, "index_offset must be a multiple of 4096");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "too many tuples (max 2^26 per call)");
  Slot& s = c->slots[0];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot 0 busy: call kzgmi_slot_wait first");
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    const uint32_t* dg = nullptr;
    CHK(begin_job(s));
    CHK(enqueue_fs_digests<Cv>(s, dC, dpi, dz, dy, n, index_offset, (flags & KZGMI_FLAG_COMPRESSED) != 0, &dg));
    const size_t nch = (n + FS_CHUNK - 1) / FS_CHUNK;
    HIPCHK(hipMemcpyAsync(d_out, dg, nch * 32, hipMemcpyDeviceToDevice, s.stream));
    HIPCHK(hipGetLastError());
    return end_job(s);
  });
}

int kzgmi_fs_chunk_digests_device(kzgmi_ctx* c, kzgmi_curve curve, const void* dC, const void* dz, const void* dy,
                                  const void* dpi, size_t n, uint64_t index_offset, uint32_t flags, void* d_out) {
  CHK(fs_chunk_digests_enqueue(c, curve, dC, dz, dy, dpi, n, index_offset, flags, d_out));
  return sync_slot(c->slots[0]);
}

int kzgmi_fs_challenge_from_digests_device(kzgmi_ctx* c, kzgmi_curve curve, const void* d_digests, size_t nchunks,
                                           uint64_t n_total, uint8_t* r_out) {
  CHK(check_ctx(c));
  if (!d_digests || !r_out || nchunks == 0 || nchunks > (1u << 22)) return fail(KZGMI_ERR_ARG, "bad argument");
  if ((n_total + FS_CHUNK - 1) / FS_CHUNK != nchunks) return fail(KZGMI_ERR_ARG, "nchunks != ceil(n_total / 4096)");
  Slot& s = c->slots[0];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot 0 busy: call kzgmi_slot_wait first");
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    CHK(begin_job(s));
    CHK(enqueue_fs_challenge<Cv>(s, (const uint32_t*)d_digests, (uint32_t)nchunks, n_total));
    uint32_t w[8];
    HIPCHK(hipMemcpyAsync(w, s.chal.p, 32, hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipGetLastError());
    CHK(sync_job(s));
    for (int k = 0; k < 8; ++k)
      for (int b = 0; b < 4; ++b) r_out[4 * k + b] = (uint8_t)(w[k] >> (24 - 8 * b));
    return 0;
  });
}

int kzgmi_fs_challenge_device(kzgmi_ctx* c, kzgmi_curve curve, const void* dC, const void* dz, const void* dy,
                              const void* dpi, size_t n, uint32_t flags, uint8_t* r_out) {
  CHK(check_ctx(c));
  if (!r_out || n == 0 || !dC || !dz || !dy || !dpi) return fail(KZGMI_ERR_ARG, "bad argument");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "too many tuples (max 2^26 per call)");
  Slot& s = c->slots[0];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot 0 busy: call kzgmi_slot_wait first");
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    const uint32_t* dg = nullptr;
    CHK(begin_job(s));
    CHK(enqueue_fs_digests<Cv>(s, dC, dpi, dz, dy, n, 0, (flags & KZGMI_FLAG_COMPRESSED) != 0, &dg));
    CHK(enqueue_fs_challenge<Cv>(s, dg, (uint32_t)((n + FS_CHUNK - 1) / FS_CHUNK), n));
    uint32_t w[8];
    HIPCHK(hipMemcpyAsync(w, s.chal.p, 32, hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipGetLastError());
    CHK(sync_job(s));
    for (int k = 0; k < 8; ++k)
      for (int b = 0; b < 4; ++b) r_out[4 * k + b] = (uint8_t)(w[k] >> (24 - 8 * b));
    return 0;
  });
}

int kzgmi_g1_compress_device(kzgmi_ctx* c, kzgmi_curve curve, const void* d_points, size_t n, void* d_out) {
  CHK(check_ctx(c));
  if (n && (!d_points || !d_out)) return fail(KZGMI_ERR_ARG, "null argument");
  if (n > (1u << 27)) return fail(KZGMI_ERR_ARG, "too many points (max 2^27 per call)");
  CHK(slot0_idle(c));
  Slot& s = c->slots[0];
  return dispatch(curve, [&](auto cv) -> int {
    CHK(begin_job(s));
    Launch<decltype(cv)>::compress_points(s.stream, (const uint8_t*)d_points, (uint32_t)n, (uint8_t*)d_out);
    HIPCHK(hipGetLastError());
    CHK(sync_job(s));
    return 0;
  });
}

int kzgmi_msm_partial_device(kzgmi_ctx* c, kzgmi_curve curve, const void* dpts, const void* dsc, size_t n,
                             void* d_partial_out) {
  CHK(check_ctx(c));
  if (!d_partial_out || (n && (!dpts || !dsc))) return fail(KZGMI_ERR_ARG, "bad argument");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "MSM too large (max 2^26 points per call)");
  CHK(slot0_idle(c));
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    Slot& s = c->slots[0];
    if (n == 0) {
      Xyzz<Cv> h;
      memset(&h, 0, sizeof(h));
      HIPCHK(hipMemcpy(d_partial_out, &h, sizeof(h), hipMemcpyHostToDevice));
      return 0;
    }
    CHK(enqueue_msm<Cv>(c, s, dpts, dsc, n));
    Launch<Cv>::partial_out(s.stream, s.res.template as<Xyzz<Cv>>(), 1, s.flags.template as<uint32_t>() + 1,
                            (Xyzz<Cv>*)d_partial_out);
    return read_flags_sync(c, s);
  });
}

int kzgmi_msm_partial_device_async(kzgmi_ctx* c, kzgmi_curve curve, int slot, const void* dpts, const void* dsc,
                                   size_t n, void* d_partial_out) {
  KZ_ROUTE(c, nullptr, slot);
  CHK(check_ctx(c, slot));
  Roctx rx("kzgmi_msm_partial_device_async");
  if (!d_partial_out || (n && (!dpts || !dsc))) return fail(KZGMI_ERR_ARG, "bad argument");
  if (n > (1u << 26)) return fail(KZGMI_ERR_ARG, "MSM too large (max 2^26 points per call)");
  Slot& s = c->slots[slot];
  if (s.pending) return fail(KZGMI_ERR_ARG, "slot busy: call kzgmi_slot_wait first");
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    if (n == 0) {
      CHK(s.flags.ensure(16));
      CHK(sync_slot(s));  // host_flags may still be a copy target
      CHK(begin_job(s));
      HIPCHK(hipMemsetAsync(d_partial_out, 0, sizeof(Xyzz<Cv>), s.stream));  // ZZ = 0: infinity
      HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, s.stream));  // a chained combine keeps the error word
      CHK(end_job(s));
      s.host_flags[0] = 1;
      s.host_flags[1] = 0;
    } else {
      CHK(enqueue_msm<Cv>(c, s, dpts, dsc, n));
      Launch<Cv>::partial_out(s.stream, s.res.template as<Xyzz<Cv>>(), 1, s.flags.template as<uint32_t>() + 1,
                              (Xyzz<Cv>*)d_partial_out);
      HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, s.stream));
      CHK(end_job(s));
    }
    s.pending = true;
    s.partial_job = true;
    s.partial_of = 2;
    s.msm_job = false;
    s.curve = Cv::ID;
    return 0;
  });
}

int kzgmi_msm_combine_device_async(kzgmi_ctx* c, kzgmi_curve curve, int slot, const void* d_partials, int n_parts) {
  KZ_ROUTE(c, nullptr, slot);
  CHK(check_ctx(c, slot));
  if (!d_partials || n_parts < 1) return fail(KZGMI_ERR_ARG, "bad argument");
  Slot& s = c->slots[slot];
  const bool chain = s.pending && s.partial_of == 2;  // behind this slot's own MSM partial
  if (s.pending && !chain) return fail(KZGMI_ERR_ARG, "slot busy: call kzgmi_msm_wait first");
  if (chain && s.curve != (int)curve) return fail(KZGMI_ERR_ARG, "chained combine: curve differs from the partial's");
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    using XY = Xyzz<Cv>;
    const size_t gb = g1_bytes(Cv::ID);
    CHK(s.res.ensure(2 * sizeof(XY)));
    CHK(s.outb.ensure(gb));
    CHK(s.flags.ensure(16));
    CHK(begin_job(s));  // chained: the lane the partial ended in
    if (!chain) HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, s.stream));
    Launch<Cv>::sum_partials(s.stream, (const XY*)d_partials, (uint32_t)n_parts, 1, 1, s.res.template as<XY>(),
                             s.flags.template as<uint32_t>() + 1);
    Launch<Cv>::encode_points(s.stream, s.res.template as<XY>(), 1, s.outb.template as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s.host_out, s.outb.p, gb, hipMemcpyDeviceToHost, s.stream));
    HIPCHK(hipMemcpyAsync(s.host_flags, s.flags.p, 8, hipMemcpyDeviceToHost, s.stream));
    CHK(end_job(s));
    s.pending = true;
    s.partial_job = false;
    s.partial_of = 0;
    s.msm_job = true;
    s.curve = Cv::ID;
    return 0;
  });
}

int kzgmi_msm_combine_device(kzgmi_ctx* c, kzgmi_curve curve, const void* d_partials, int n_parts, uint8_t* out) {
  CHK(check_ctx(c));
  if (!d_partials || n_parts < 1 || !out) return fail(KZGMI_ERR_ARG, "bad argument");
  CHK(slot0_idle(c));
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    using XY = Xyzz<Cv>;
    Slot& s = c->slots[0];
    const size_t gb = g1_bytes(Cv::ID);
    CHK(s.res.ensure(2 * sizeof(XY)));
    CHK(s.outb.ensure(gb));
    CHK(s.flags.ensure(16));
    CHK(begin_job(s));
    HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, s.stream));
    Launch<Cv>::sum_partials(s.stream, (const XY*)d_partials, (uint32_t)n_parts, 1, 1, s.res.template as<XY>(),
                             s.flags.template as<uint32_t>() + 1);
    Launch<Cv>::encode_points(s.stream, s.res.template as<XY>(), 1, s.outb.template as<uint8_t>());
    HIPCHK(hipGetLastError());
    CHK(read_flags_sync(c, s));
    HIPCHK(hipMemcpy(out, s.outb.p, gb, hipMemcpyDeviceToHost));
    return 0;
  });
}

// ------------------------------------------------------------------------------ pairing
int kzgmi_pairing(kzgmi_ctx* c, kzgmi_curve curve, const uint8_t* g1, const uint8_t* g2, uint8_t* out) {
  CHK(check_ctx(c));
  if (!g1 || !g2 || !out) return fail(KZGMI_ERR_ARG, "null argument");
  CHK(slot0_idle(c));
  // BLS12-381: the pairing program's hard part is the x-chain of 3 (p^4 - p^2 + 1) / r, so it
  // yields e(P, Q)^3 (as the oracle and pyspec do); e(P, Q) = e([3^-1 mod r] P, Q)^3 for P in G1,
  // so P is first scaled by 3^-1 mod r with the library's MSM on one point, GLV forced off (the
  // GLV split is exact only on G1, and kzgmi_set_trusted_g1 must not change this diagnostic)
  uint8_t g1s[96];
  if (curve == KZGMI_BLS12_381) {
    static const uint8_t kInv3[32] = {0x4d, 0x49, 0x1a, 0x37, 0x71, 0x13, 0xa8, 0xda, 0xcc, 0xd1, 0x3a,
                                      0xb0, 0x06, 0x6b, 0xe5, 0x58, 0xe2, 0x7e, 0x6d, 0x57, 0x55, 0x54,
                                      0x3d, 0x54, 0xaa, 0xaa, 0xaa, 0xaa, 0x00, 0x00, 0x00, 0x01};
    using Cv = Bls12_381;
    Slot& s = c->slots[0];
    CHK(s.stage.ensure(96 + 32));
    CHK(s.outb.ensure(96));
    uint8_t* dp = s.stage.template as<uint8_t>();
    CHK(begin_job(s));  // the MSM's job starts in the same lane, behind these copies
    HIPCHK(hipMemcpyAsync(dp, g1, 96, hipMemcpyHostToDevice, s.stream));
    HIPCHK(hipMemcpyAsync(dp + 96, kInv3, 32, hipMemcpyHostToDevice, s.stream));
    CHK(enqueue_msm<Cv>(c, s, dp, dp + 96, 1, /*allow_glv=*/false));
    Launch<Cv>::encode_points(s.stream, s.res.template as<Xyzz<Cv>>(), 1, s.outb.template as<uint8_t>());
    HIPCHK(hipGetLastError());
    CHK(read_flags_sync(c, s));
    HIPCHK(hipMemcpy(g1s, s.outb.p, 96, hipMemcpyDeviceToHost));
    g1 = g1s;
  }
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    Slot& s = c->slots[0];
    const size_t gb1 = g1_bytes(Cv::ID), gb2 = g2_bytes(Cv::ID);
    const size_t fb = 12 * Cv::FP_BYTES;
    CHK(s.stage.ensure(gb1 + 2 * gb2 + 64));
    CHK(s.pts.ensure(sizeof(Affine<Cv>)));
    CHK(s.inf.ensure(16));
    CHK(s.flags.ensure(16));
    CHK(s.outb.ensure(fb));
    CHK(c->lines_tmp.ensure(2 * Launch<Cv>::num_lines() * sizeof(Line<Cv>) + 4 * sizeof(G2Aff<Cv>) + 64));
    std::vector<uint8_t> h(gb1 + 2 * gb2);
    memcpy(h.data(), g1, gb1);
    memcpy(h.data() + gb1, g2, gb2);
    memcpy(h.data() + gb1 + gb2, g2, gb2);
    CHK(begin_job(s));
    hipStream_t st = s.stream;
    uint8_t* d = s.stage.template as<uint8_t>();
    Line<Cv>* lines = c->lines_tmp.template as<Line<Cv>>();
    G2Aff<Cv>* q = reinterpret_cast<G2Aff<Cv>*>(lines + 2 * Launch<Cv>::num_lines());
    uint8_t* qinf = s.inf.template as<uint8_t>() + 8;
    HIPCHK(hipMemcpyAsync(d, h.data(), h.size(), hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, st));
    uint32_t* err = s.flags.template as<uint32_t>() + 1;
    Launch<Cv>::convert_points(st, d, 1, s.pts.template as<Affine<Cv>>(), s.inf.template as<uint8_t>(), err);
    Launch<Cv>::convert_g2(st, d + gb1, 2, q, qinf, err);
    Launch<Cv>::precompute_lines(st, q, lines);
    Launch<Cv>::pairing_one(st, s.pts.template as<Affine<Cv>>(), s.inf.template as<uint8_t>(), lines, qinf, s.outb.template as<uint8_t>());
    HIPCHK(hipGetLastError());
    CHK(read_flags_sync(c, s));
    HIPCHK(hipMemcpy(out, s.outb.p, fb, hipMemcpyDeviceToHost));
    return 0;
  });
}

// ------------------------------------------------------------------------------ generators
int kzgmi_gen_g1(kzgmi_ctx* c, kzgmi_curve curve, const void* d_scalars, size_t n, void* d_points_out) {
  CHK(check_ctx(c));
  if (n && (!d_scalars || !d_points_out)) return fail(KZGMI_ERR_ARG, "null argument");
  CHK(slot0_idle(c));
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    Slot& s = c->slots[0];
    CHK(begin_job(s));
    CHK(ensure_table<Cv>(c, s.stream));
    CHK(s.flags.ensure(16));
    HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, s.stream));
    if (n)
      Launch<Cv>::gen_g1(s.stream, (const uint8_t*)d_scalars, (uint32_t)n, c->table[Cv::ID].template as<Affine<Cv>>(),
                         (uint8_t*)d_points_out, s.flags.template as<uint32_t>() + 1);
    HIPCHK(hipGetLastError());
    return read_flags_sync(c, s);
  });
}

int kzgmi_gen_tuples(kzgmi_ctx* c, kzgmi_curve curve, const uint8_t* tau32, const uint8_t* seed32, size_t n,
                     void* dC, void* dz, void* dy, void* dpi) {
  CHK(check_ctx(c));
  if (!tau32 || !seed32 || (n && (!dC || !dz || !dy || !dpi))) return fail(KZGMI_ERR_ARG, "null argument");
  CHK(slot0_idle(c));
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    using FrF = Fp<typename Cv::FrP>;
    Slot& s = c->slots[0];
    CHK(begin_job(s));
    CHK(ensure_table<Cv>(c, s.stream));
    FrF tau;
    for (int k = 0; k < 8; ++k)
      tau.v[k] = (uint32_t)tau32[31 - 4 * k] | (uint32_t)tau32[30 - 4 * k] << 8 | (uint32_t)tau32[29 - 4 * k] << 16 |
                 (uint32_t)tau32[28 - 4 * k] << 24;
    // tau must be canonical
    for (int k = 7; k >= 0; --k) {
      if (tau.v[k] < Cv::FrP::MOD[k]) break;
      if (tau.v[k] > Cv::FrP::MOD[k] || k == 0) return fail(KZGMI_ERR_SCALAR, "tau >= r");
    }
    uint8_t sb[32];
    Seed seed = make_seed(seed32, sb);
    if (n)
      Launch<Cv>::gen_tuples(s.stream, seed, tau.v, (uint32_t)n, c->table[Cv::ID].template as<Affine<Cv>>(),
                                                           (uint8_t*)dC, (uint8_t*)dz, (uint8_t*)dy, (uint8_t*)dpi);
    HIPCHK(hipGetLastError());
    CHK(sync_job(s));
    return 0;
  });
}

int kzgmi_g2_mul(kzgmi_ctx* c, kzgmi_curve curve, const uint8_t* g2, const uint8_t* k32, uint8_t* out) {
  CHK(check_ctx(c));
  if (!g2 || !k32 || !out) return fail(KZGMI_ERR_ARG, "null argument");
  CHK(slot0_idle(c));
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    Slot& s = c->slots[0];
    const size_t gb = g2_bytes(Cv::ID);
    CHK(s.stage.ensure(2 * gb + 64));
    CHK(s.inf.ensure(16));
    CHK(s.flags.ensure(16));
    CHK(c->tmp.ensure(2 * sizeof(G2Aff<Cv>)));
    uint32_t k[8];
    for (int j = 0; j < 8; ++j)
      k[j] = (uint32_t)k32[31 - 4 * j] | (uint32_t)k32[30 - 4 * j] << 8 | (uint32_t)k32[29 - 4 * j] << 16 |
             (uint32_t)k32[28 - 4 * j] << 24;
    for (int j = 7; j >= 0; --j) {
      if (k[j] < Cv::FrP::MOD[j]) break;
      if (k[j] > Cv::FrP::MOD[j] || j == 0) return fail(KZGMI_ERR_SCALAR, "k >= r");
    }
    CHK(begin_job(s));
    hipStream_t st = s.stream;
    uint8_t* d = s.stage.template as<uint8_t>();
    HIPCHK(hipMemcpyAsync(d, g2, gb, hipMemcpyHostToDevice, st));
    HIPCHK(hipMemsetAsync(s.flags.p, 0, 16, st));
    Launch<Cv>::convert_g2(st, d, 1, c->tmp.template as<G2Aff<Cv>>(), s.inf.template as<uint8_t>(),
                           s.flags.template as<uint32_t>() + 1);
    Launch<Cv>::g2_mul(st, c->tmp.template as<G2Aff<Cv>>(), s.inf.template as<uint8_t>(), k, d + gb);
    HIPCHK(hipGetLastError());
    CHK(read_flags_sync(c, s));
    HIPCHK(hipMemcpy(out, d + gb, gb, hipMemcpyDeviceToHost));
    return 0;
  });
}

int kzgmi_probe_fpmul(kzgmi_ctx* c, kzgmi_curve curve, double* muls_per_s) {
  CHK(check_ctx(c));
  if (!muls_per_s) return fail(KZGMI_ERR_ARG, "null argument");
  CHK(slot0_idle(c));
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    Slot& s = c->slots[0];
    const uint32_t blocks = 256 * 16, iters = 2048;
    CHK(c->tmp.ensure((size_t)blocks * 256 * 4));
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    CHK(begin_job(s));
    Launch<Cv>::fpmul_probe(s.stream, blocks, 16, c->tmp.template as<uint32_t>());  // warm-up
    HIPCHK(hipEventRecord(e0, s.stream));
    Launch<Cv>::fpmul_probe(s.stream, blocks, iters, c->tmp.template as<uint32_t>());
    HIPCHK(hipEventRecord(e1, s.stream));
    CHK(sync_job(s));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    *muls_per_s = (double)blocks * 256.0 * iters * 8.0 / (ms * 1e-3);
    return 0;
  });
}

// ------------------------------------------------------------------------------ profiling
int kzgmi_set_glv(kzgmi_ctx* c, int msm, int batch) {
  CHK(check_ctx(c));
  for (auto& s : c->slots)
    if (s.pending) return fail(KZGMI_ERR_ARG, "kzgmi_set_glv with jobs in flight");
  c->glv_msm = msm != 0;
  c->glv_batch = batch != 0;
  for (kzgmi_ctx* p : c->peers) CHK(kzgmi_set_glv(p, msm, batch));
  return set_dev(c);
}

int kzgmi_set_split_acc(kzgmi_ctx* c, int mode) {
  CHK(check_ctx(c));
  if (mode < -1 || mode > 1) return fail(KZGMI_ERR_ARG, "split mode must be -1, 0 or 1");
  for (auto& s : c->slots)
    if (s.pending) return fail(KZGMI_ERR_ARG, "kzgmi_set_split_acc with jobs in flight");
  c->split_acc = mode;
  for (kzgmi_ctx* p : c->peers) CHK(kzgmi_set_split_acc(p, mode));
  return set_dev(c);
}

int kzgmi_set_trusted_g1(kzgmi_ctx* c, int on) {
  CHK(check_ctx(c));
  for (auto& s : c->slots)
    if (s.pending) return fail(KZGMI_ERR_ARG, "kzgmi_set_trusted_g1 with jobs in flight");
  c->msm_trusted_g1 = on != 0;
  for (kzgmi_ctx* p : c->peers) CHK(kzgmi_set_trusted_g1(p, on));
  return set_dev(c);
}

int kzgmi_set_profiling(kzgmi_ctx* c, int on) {
  if (!c) return fail(KZGMI_ERR_ARG, "null context");
  c->profiling = on != 0;
  for (int k = 0; k < kNumPhases; ++k) c->phase_ms[k] = 0;
  c->phase_calls = 0;
  // multi-device context: every device records its phases; kzgmi_get_phase_ms reports the
  // primary device's (the peers' shards run the same phases concurrently)
  for (kzgmi_ctx* p : c->peers) CHK(kzgmi_set_profiling(p, on));
  return 0;
}

int kzgmi_get_phase_ms(kzgmi_ctx* c, double* out, int max_n) {
  if (!c || !out) return fail(KZGMI_ERR_ARG, "null argument");
  int k = max_n < kNumPhases ? max_n : kNumPhases;
  for (int i = 0; i < k; ++i) out[i] = c->phase_calls ? c->phase_ms[i] / c->phase_calls : 0.0;
  return k;
}

// ------------------------------------------------------------------------------ stream order
int kzgmi_stream_wait(kzgmi_ctx* c, int slot, void* stream) {
  KZ_ROUTE(c, nullptr, slot);
  CHK(check_ctx(c, slot));
  // an entry dependency of the slot's next job (begin_job), whichever lane that job starts in
  return add_dep(c->slots[slot], (hipStream_t)stream);
}

int kzgmi_slot_signal(kzgmi_ctx* c, int slot, void* stream) {
  KZ_ROUTE(c, nullptr, slot);
  CHK(check_ctx(c, slot));
  Slot& s = c->slots[slot];
  if (!s.signal_ev) HIPCHK(hipEventCreateWithFlags(&s.signal_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(s.signal_ev, s.stream));
  HIPCHK(hipStreamWaitEvent((hipStream_t)stream, s.signal_ev, 0));
  return 0;
}

int kzgmi_partial_encode_device(kzgmi_ctx* c, kzgmi_curve curve, const void* d_records, size_t count, uint8_t* out) {
  CHK(check_ctx(c));
  if (!d_records || !out || count == 0 || count > 4096) return fail(KZGMI_ERR_ARG, "bad argument");
  CHK(slot0_idle(c));
  return dispatch(curve, [&](auto cv) -> int {
    using Cv = decltype(cv);
    Slot& s = c->slots[0];
    const size_t gb = g1_bytes(Cv::ID);
    CHK(s.outb.ensure(count * gb));
    CHK(begin_job(s));
    Launch<Cv>::encode_points(s.stream, (const Xyzz<Cv>*)d_records, (uint32_t)count, s.outb.template as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(out, s.outb.p, count * gb, hipMemcpyDeviceToHost, s.stream));
    CHK(sync_job(s));
    return 0;
  });
}

// ------------------------------------------------------------------------------ multi-device context
int kzgmi_ctx_create(kzgmi_ctx** out, const int* device_ids, int n_devices, int pipeline_slots) {
  if (!out || !device_ids || n_devices < 1 || n_devices > 64) return fail(KZGMI_ERR_ARG, "bad ctx args");
  *out = nullptr;
  if (pipeline_slots < 1 || pipeline_slots > 64) return fail(KZGMI_ERR_ARG, "bad ctx args");
  kzgmi_ctx* c = nullptr;
  // every device holds ceil(slots / n_devices) local slots (route_slot)
  const int local = (pipeline_slots + n_devices - 1) / n_devices;
  CHK(kzgmi_ctx_create_device(&c, device_ids[0], local));
  for (int k = 1; k < n_devices; ++k) {
    kzgmi_ctx* p = nullptr;
    if (int r = kzgmi_ctx_create_device(&p, device_ids[k], local)) {
      kzgmi_ctx_destroy(c);
      return r;
    }
    c->peers.push_back(p);
  }
  c->user_slots = pipeline_slots;
  CHK(set_dev(c));
  *out = c;
  return 0;
}

int kzgmi_ctx_num_devices(const kzgmi_ctx* c) { return c ? 1 + (int)c->peers.size() : 0; }

int kzgmi_slot_device(const kzgmi_ctx* c, int slot) {
  if (!c || slot < 0 || slot >= c->user_slots) return fail(KZGMI_ERR_ARG, "bad slot");
  const int D = 1 + (int)c->peers.size();
  return slot % D == 0 ? c->device : c->peers[slot % D - 1]->device;
}

}  // extern "C"

// Shards run concurrently (one async partial per device on its slot 0), the partial records are
// copied to the primary device (hipMemcpyPeer over xGMI: 2 XYZZ records per device), and the
// primary sums them and runs the pairing check -- the single-process form of the RCCL
// all-gather that kzgmi/distributed.py does across processes.
namespace {

// wait every device's slot 0 (first error wins; every slot is completed either way)
int wait_all(kzgmi_ctx* c, int started) {
  int first = 0;
  std::string msg;
  for (int d = 0; d < started; ++d) {
    int r = kzgmi_slot_wait(dev_ctx(c, d), 0, nullptr);
    if (r && !first) {
      first = r;
      msg = g_err;
    }
  }
  if (first) return fail(first, msg);
  return 0;
}

// children's records (in their `gath`, complete: wait_all synchronised every peer's slot 0) ->
// c->gath[d], copied on the primary's slot-0 stream, the stream kzgmi_batch_combine_device /
// kzgmi_msm_combine_device then read them on -- so the order is explicit, not left to how the
// runtime orders a null-stream peer copy against a non-blocking stream
int gather_records(kzgmi_ctx* c, size_t rec) {
  CHK(set_dev(c));
  CHK(begin_job(c->slots[0]));  // the combine's job starts in the same lane, behind these copies
  for (size_t d = 1; d <= c->peers.size(); ++d) {
    kzgmi_ctx* p = c->peers[d - 1];
    HIPCHK(hipMemcpyPeerAsync((uint8_t*)c->gath.p + d * rec, c->device, p->gath.p, p->device, rec, c->slots[0].stream));
  }
  return 0;
}

int batch_multi(kzgmi_ctx* c, const kzgmi_srs* srs, const void* const* dC, const void* const* dz,
                const void* const* dy, const void* const* dpi, const size_t* nd, const uint8_t* seed32,
                uint32_t flags, int* ok_out) {
  const int D = 1 + (int)c->peers.size();
  if (srs->peers.size() != c->peers.size()) return fail(KZGMI_ERR_ARG, "srs was not loaded on this context");
  const kzgmi_curve curve = (kzgmi_curve)srs->curve;
  const size_t rec = 2 * kzgmi_partial_bytes(curve);
  std::vector<uint64_t> off(D + 1, 0);
  for (int d = 0; d < D; ++d) {
    if (nd[d] && (!dC[d] || !dz[d] || !dy[d] || !dpi[d])) return fail(KZGMI_ERR_ARG, "null input");
    if (nd[d] > (1u << 26)) return fail(KZGMI_ERR_ARG, "shard too large (max 2^26 tuples per device)");
    off[d + 1] = off[d] + nd[d];
  }
  uint8_t sb[32];
  if (flags & KZGMI_FLAG_FIAT_SHAMIR) {  // one transcript over the whole batch: subtree roots gathered
    if (flags & KZGMI_FLAG_POWERS) return fail(KZGMI_ERR_ARG, "KZGMI_FLAG_POWERS and KZGMI_FLAG_FIAT_SHAMIR are exclusive");
    const uint64_t ntot = off[D];
    if (ntot == 0) {
      *ok_out = 1;
      return 0;
    }
    const size_t nch_tot = (ntot + FS_CHUNK - 1) / FS_CHUNK;
    CHK(c->mdig_all.ensure(nch_tot * 32));
    // every device hashes its subtrees concurrently (enqueued first), then each device's
    // digests are waited for and copied to the primary, ordered before the challenge derivation
    // on the primary's slot-0 stream
    for (int d = 0; d < D; ++d) {
      if (!nd[d]) continue;
      if (off[d] % FS_CHUNK) return fail(KZGMI_ERR_ARG, "Fiat-Shamir shards must start at multiples of 4096 tuples");
      kzgmi_ctx* p = dev_ctx(c, d);
      const size_t nch = (nd[d] + FS_CHUNK - 1) / FS_CHUNK;
      CHK(set_dev(p));
      CHK(p->mdig.ensure(nch * 32));
      CHK(fs_chunk_digests_enqueue(p, curve, dC[d], dz[d], dy[d], dpi[d], nd[d], off[d],
                                   flags & KZGMI_FLAG_COMPRESSED, p->mdig.p));
    }
    size_t at = 0;
    for (int d = 0; d < D; ++d) {
      if (!nd[d]) continue;
      kzgmi_ctx* p = dev_ctx(c, d);
      const size_t nch = (nd[d] + FS_CHUNK - 1) / FS_CHUNK;
      CHK(set_dev(p));
      CHK(sync_slot(p->slots[0]));
      CHK(set_dev(c));
      CHK(begin_job(c->slots[0]));  // the challenge's job follows in this lane
      HIPCHK(hipMemcpyPeerAsync((uint8_t*)c->mdig_all.p + at * 32, c->device, p->mdig.p, p->device, nch * 32,
                                c->slots[0].stream));
      at += nch;
    }
    CHK(kzgmi_fs_challenge_from_digests_device(c, curve, c->mdig_all.p, nch_tot, ntot, sb));
    seed32 = sb;
    flags &= ~KZGMI_FLAG_FIAT_SHAMIR;
  } else if (!seed32) {
    uint8_t tmp[32];
    make_seed(nullptr, tmp);  // one verifier-private seed shared by every shard
    memcpy(sb, tmp, 32);
    seed32 = sb;
  }
  CHK(set_dev(c));
  CHK(c->gath.ensure(D * rec));
  for (int d = 0; d < D; ++d) {
    kzgmi_ctx* p = dev_ctx(c, d);
    int r = 0;
    if (d > 0) {
      r = set_dev(p);
      if (!r) r = p->gath.ensure(rec);
    }
    if (!r)
      r = kzgmi_batch_partial_device_async(p, d == 0 ? srs : srs->peers[d - 1], 0, dC[d], dz[d], dy[d], dpi[d], nd[d],
                                           off[d], seed32, flags, d == 0 ? c->gath.p : p->gath.p);
    if (r) {
      std::string msg = g_err;
      (void)wait_all(c, d);
      return fail(r, msg);
    }
  }
  CHK(wait_all(c, D));
  CHK(gather_records(c, rec));
  return kzgmi_batch_combine_device(c, srs, c->gath.p, D, ok_out);
}

int msm_multi(kzgmi_ctx* c, kzgmi_curve curve, const void* const* dp, const void* const* ds, const size_t* nd,
              uint8_t* out) {
  const int D = 1 + (int)c->peers.size();
  if (curve != KZGMI_BLS12_381 && curve != KZGMI_BN254) return fail(KZGMI_ERR_ARG, "unknown curve");
  const size_t rec = kzgmi_partial_bytes(curve);
  CHK(set_dev(c));
  CHK(c->gath.ensure(D * rec));
  for (int d = 0; d < D; ++d) {
    kzgmi_ctx* p = dev_ctx(c, d);
    int r = 0;
    if (d > 0) {
      r = set_dev(p);
      if (!r) r = p->gath.ensure(rec);
    }
    if (!r) r = kzgmi_msm_partial_device_async(p, curve, 0, dp[d], ds[d], nd[d], d == 0 ? c->gath.p : p->gath.p);
    if (r) {
      std::string msg = g_err;
      (void)wait_all(c, d);
      return fail(r, msg);
    }
  }
  CHK(wait_all(c, D));
  CHK(gather_records(c, rec));
  return kzgmi_msm_combine_device(c, curve, c->gath.p, D, out);
}

// balanced split of n tuples/points over the devices in units of 4096 (Fiat-Shamir subtrees)
std::vector<size_t> split_units(size_t n, int D) {
  const size_t units = (n + FS_CHUNK - 1) / FS_CHUNK;
  std::vector<size_t> nd(D);
  size_t lo = 0;
  for (int d = 0; d < D; ++d) {
    size_t u1 = units * (d + 1) / D;
    size_t hi = std::min(n, u1 * FS_CHUNK);
    nd[d] = hi - lo;
    lo = hi;
  }
  return nd;
}

int batch_multi_host(kzgmi_ctx* c, const kzgmi_srs* srs, const uint8_t* commitments, const uint8_t* zs,
                     const uint8_t* ys, const uint8_t* proofs, size_t n, const uint8_t* seed32, uint32_t flags,
                     int* ok_out) {
  const int D = 1 + (int)c->peers.size();
  const size_t gb = (flags & KZGMI_FLAG_COMPRESSED) ? g1_bytes(srs->curve) / 2 : g1_bytes(srs->curve);
  std::vector<size_t> nd = split_units(n, D);
  std::vector<const void*> pC(D), pz(D), py(D), ppi(D);
  size_t lo = 0;
  for (int d = 0; d < D; ++d) {
    kzgmi_ctx* p = dev_ctx(c, d);
    Slot& s = p->slots[0];
    CHK(set_dev(p));
    CHK(s.stage.ensure(nd[d] * (2 * gb + 64)));
    uint8_t* base = s.stage.template as<uint8_t>();
    pC[d] = base;
    ppi[d] = base + nd[d] * gb;
    pz[d] = base + 2 * nd[d] * gb;
    py[d] = base + 2 * nd[d] * gb + 32 * nd[d];
    CHK(begin_job(s));  // the shard's job starts in the same lane, behind these copies
    if (nd[d]) {
      HIPCHK(hipMemcpyAsync((void*)pC[d], commitments + lo * gb, nd[d] * gb, hipMemcpyHostToDevice, s.stream));
      HIPCHK(hipMemcpyAsync((void*)ppi[d], proofs + lo * gb, nd[d] * gb, hipMemcpyHostToDevice, s.stream));
      HIPCHK(hipMemcpyAsync((void*)pz[d], zs + lo * 32, nd[d] * 32, hipMemcpyHostToDevice, s.stream));
      HIPCHK(hipMemcpyAsync((void*)py[d], ys + lo * 32, nd[d] * 32, hipMemcpyHostToDevice, s.stream));
    }
    lo += nd[d];
  }
  return batch_multi(c, srs, pC.data(), pz.data(), py.data(), ppi.data(), nd.data(), seed32, flags, ok_out);
}

int msm_multi_host(kzgmi_ctx* c, kzgmi_curve curve, const uint8_t* points, const uint8_t* scalars, size_t n,
                   uint8_t* out) {
  const int D = 1 + (int)c->peers.size();
  const size_t gb = g1_bytes(curve);
  std::vector<size_t> nd = split_units(n, D);
  std::vector<const void*> pp(D), ps(D);
  size_t lo = 0;
  for (int d = 0; d < D; ++d) {
    kzgmi_ctx* p = dev_ctx(c, d);
    Slot& s = p->slots[0];
    CHK(set_dev(p));
    CHK(s.stage.ensure(nd[d] * (gb + 32)));
    pp[d] = s.stage.p;
    ps[d] = s.stage.template as<uint8_t>() + nd[d] * gb;
    CHK(begin_job(s));
    if (nd[d]) {
      HIPCHK(hipMemcpyAsync((void*)pp[d], points + lo * gb, nd[d] * gb, hipMemcpyHostToDevice, s.stream));
      HIPCHK(hipMemcpyAsync((void*)ps[d], scalars + lo * 32, nd[d] * 32, hipMemcpyHostToDevice, s.stream));
    }
    lo += nd[d];
  }
  return msm_multi(c, curve, pp.data(), ps.data(), nd.data(), out);
}

}  // namespace

extern "C" {

int kzgmi_batch_verify_multi_device(kzgmi_ctx* c, const kzgmi_srs* srs, const void* const* d_commitments,
                                    const void* const* d_zs, const void* const* d_ys, const void* const* d_proofs,
                                    const size_t* n_per_device, const uint8_t* seed32, uint32_t flags, int* ok_out) {
  CHK(check_ctx(c));
  if (!srs || srs->ctx != c || !ok_out || !d_commitments || !d_zs || !d_ys || !d_proofs || !n_per_device)
    return fail(KZGMI_ERR_ARG, "bad argument");
  if (flags & ~kAllFlags) return fail(KZGMI_ERR_ARG, "unknown flags");
  if ((flags & KZGMI_FLAG_POWERS) && !seed32) return fail(KZGMI_ERR_ARG, "KZGMI_FLAG_POWERS needs r in seed32");
  CHK(slot0_idle(c));
  return batch_multi(c, srs, d_commitments, d_zs, d_ys, d_proofs, n_per_device, seed32, flags, ok_out);
}

int kzgmi_msm_g1_multi_device(kzgmi_ctx* c, kzgmi_curve curve, const void* const* d_points,
                              const void* const* d_scalars, const size_t* n_per_device, uint8_t* out) {
  CHK(check_ctx(c));
  if (!d_points || !d_scalars || !n_per_device || !out) return fail(KZGMI_ERR_ARG, "bad argument");
  CHK(slot0_idle(c));
  return msm_multi(c, curve, d_points, d_scalars, n_per_device, out);
}

}  // extern "C"
