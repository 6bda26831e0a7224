/* kzgmi -- MI355X-native KZG batch verifier: the drop-in C-ABI boundary.
 *
 * Reference interface replaced: the reference snapshot contains no code
 * (/root/reference/LICENSE:1-201 only), so there is no reference FFI
 * to cite line by line.  This header realises the contract of SURVEY.md section 8b, which
 * keeps the north-star entry point `batch_verify(commitments, zs, ys, proofs, srs)`
 * (BASELINE.json:5) behind a thin C ABI; every entry point below cites the spec line it
 * implements.  Plain pointers and sizes only; no torch or HIP types in any signature.
 *
 * Conventions:
 *   - Encodings are big-endian canonical.  Fr scalar: 32 B, value < r.
 *     G1: BLS12-381 96 B x||y, infinity = 0x40 || 95 zero bytes (ZCash uncompressed flags);
 *         BN254 64 B x||y, infinity = 64 zero bytes.
 *     G2: x.c1||x.c0||y.c1||y.c0 (192 B BLS12-381 / 128 B BN254), same infinity rules.
 *   - Points must be on the curve (checked: KZGMI_ERR_NOT_ON_CURVE).  Subgroup membership is
 *     checked only with KZGMI_FLAG_SUBGROUP_CHECK (the *_ex entry points, SURVEY.md 8f item
 *     1), which also accept compressed G1 inputs (KZGMI_FLAG_COMPRESSED):
 *       BLS12-381 48 B ZCash (0x80 compressed, 0x40 infinity, 0x20 larger y),
 *       BN254 32 B gnark-crypto (top bits 0b10 smaller y, 0b11 larger y, 0b01 infinity).
 *   - Return value 0 = OK, negative = error (see KZGMI_ERR_*).  Invalid input is an error,
 *     never "ok = 0".  kzgmi_last_error() gives a thread-local message.
 *   - Threading: one ctx per host thread; calls on one ctx are serialised by the caller.
 *   - Device-memory ordering: the library runs on its own non-blocking HIP streams, one per
 *     pipeline slot (+ one for host-buffer copies).  HIP gives streams GPU_MAX_HW_QUEUES hardware
 *     queues per stream priority (4 by default) and streams sharing a queue run one after
 *     another: when the slots outnumber the queues the slot streams cycle through the device's
 *     stream priorities (KZGMI_STREAM_PRIO=0/1 forces it off/on), which keeps 16 slots at 0.96
 *     of their 24-queue rate at the default 4 queues.  With a queue per slot, the batches'
 *     bucket accumulations also start in submission order (at most 2 -- 4 for small batches --
 *     at once; KZGMI_ACC_ORDER / KZGMI_ACC_ORDER_SMALL), so slots complete in the order they were
 *     submitted.  A caller that produced device inputs on
 *     another stream (e.g. a torch stream) must order the slot's next job after it --
 *     kzgmi_stream_wait(ctx, slot, stream) (no host sync), or synchronise that stream -- before
 *     the call that reads them.  Device outputs
 *     (partials, digests, generated points) are complete when the call, or the
 *     kzgmi_slot_wait / kzgmi_msm_wait that completes it, returns.  Device buffers passed to
 *     an async call must stay allocated until its wait returns.
 *   - Randomisers: r_i = int_be(SHA256(seed || le64(i))[0:16]) >> 1 (1 if zero); 127-bit,
 *     counter mode, so a shard [off, off+n) derives its own r_i with no communication.
 *     seed == NULL draws 32 bytes from the OS CSPRNG (verifier-private randomness).
 *   - Batch check: A = sum r_i pi_i; B = sum r_i C_i + sum (r_i z_i) pi_i - (sum r_i y_i) G1;
 *     accept iff e(A, [tau]_2) * e(-B, [1]_2) == 1.  n == 0 accepts.
 *   - The hot path runs only on the GPU: without a usable HIP device every compute entry
 *     point fails with KZGMI_ERR_DEVICE (there is no CPU fallback).
 */
#ifndef KZGMI_H
#define KZGMI_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum { KZGMI_BLS12_381 = 0, KZGMI_BN254 = 1 } kzgmi_curve;

/* ABI revision of this header.  2: kzgmi_srs_load gained the g1 argument (3rd position),
 * kzgmi_ctx_reserve / kzgmi_alloc_count / kzgmi_abi_version were added.  3: kzgmi_pairing
 * returns the standard e(P, Q) on BLS12-381 (was its cube).  4: kzgmi_ctx_create takes the
 * SURVEY.md 8b device list (the single-device form is kzgmi_ctx_create_device; the ABI-3
 * kzgmi_ctx_create_multi is gone), and the pipelined host-buffer entry
 * kzgmi_batch_verify_ex_async, the pinned-host helpers kzgmi_host_* and kzgmi_slot_signal were
 * added.  5: partial records carry their shard's error (KZGMI_ERR_SHARD; combines fail on a
 * marked record), kzgmi_stream_wait orders the slot's NEXT job, multi-device contexts pipeline
 * whole batches per device through the async entry points (kzgmi_slot_device).  A caller built
 * against another revision must not bind the library: compare with kzgmi_abi_version(). */
#define KZGMI_ABI_VERSION 5

#define KZGMI_OK 0
#define KZGMI_ERR_ARG (-1)
#define KZGMI_ERR_ENCODING (-2)
#define KZGMI_ERR_NOT_ON_CURVE (-3)
#define KZGMI_ERR_SCALAR (-4)
#define KZGMI_ERR_DEVICE (-5)
#define KZGMI_ERR_OOM (-6)
#define KZGMI_ERR_NOT_IN_SUBGROUP (-7)
#define KZGMI_ERR_SHARD (-8) /* a gathered partial record marks a shard that failed on its own device */

/* flags of the *_ex entry points */
#define KZGMI_FLAG_COMPRESSED 1u     /* commitments/proofs are compressed G1 encodings */
#define KZGMI_FLAG_SUBGROUP_CHECK 2u /* reject points outside the order-r subgroup (BLS12-381;
                                        BN254 G1 has cofactor 1, the flag is a no-op there) */
#define KZGMI_FLAG_POWERS 4u         /* r_i = r^i with r = int_be(seed32) < r supplied by the caller
                                        (e.g. the EIP-4844 verify_kzg_proof_batch challenge) */
#define KZGMI_FLAG_FIAT_SHAMIR 8u    /* deterministic randomisers from the inputs: a challenge r
                                        derived on the GPU -- leaf_i = SHA256("KZGMI_FS_LEAF_V1" ||
                                        be64(i) || C_i || pi_i || z_i || y_i) (points compressed),
                                        binary Merkle root over max(4096, next_pow2(n)) zero-padded
                                        leaf slots, r = int_be(SHA256("KZGMI_FS_ROOT_V1" || be64(n)
                                        || root)) mod r (1 if 0) -- then the counter-mode 127-bit
                                        r_i above with seed = be32(r); seed32 is ignored */
#define KZGMI_FLAG_TRUSTED_G1 16u    /* the caller guarantees every C_i / pi_i is in G1 (e.g. it was
                                        subgroup-checked when deserialised): lets BLS12-381 use the
                                        GLV endomorphism, which is exact only on G1 (kzgmi_set_glv).
                                        Results for inputs outside G1 are then unspecified. */

typedef struct kzgmi_ctx kzgmi_ctx; /* one GPU (or a device list), its streams and workspaces */
typedef struct kzgmi_srs kzgmi_srs; /* {G1, [1]_2, [tau]_2} + precomputed Miller lines */
typedef struct kzgmi_ck kzgmi_ck;   /* prover commit key: [tau^i]_1 + fixed-base tables */

/* Version string of the library build. */
const char* kzgmi_version(void);
/* KZGMI_ABI_VERSION the library was built with. */
int kzgmi_abi_version(void);
/* Thread-local description of the last error. */
const char* kzgmi_last_error(void);

/* SURVEY.md 8b kzgmi_ctx_create(out, device_ids, n_devices), plus the pipeline depth: one
 * context over a device list (one process driving several GPUs; a device id may repeat;
 * n_devices = 1 is the common single-GPU context).  device_ids[0] is the primary device: every
 * synchronous single-device entry point below runs there.  `pipeline_slots` >= 1 (at most 64) is
 * the number of independent workspaces for the async entry points (1 is enough for the
 * synchronous calls; over several devices see kzgmi_slot_device); each holds ~1.3 GiB at
 * n = 2^20.  With n_devices > 1 the synchronous host-buffer
 * entry points kzgmi_batch_verify / kzgmi_batch_verify_ex / kzgmi_msm_g1 split their input by
 * point range over all devices (balanced, in units of 4096), run the shards concurrently and
 * combine the partial sums on the primary; kzgmi_batch_verify_multi_device /
 * kzgmi_msm_g1_multi_device take shards already resident on each device.  The exchange is 2
 * (batch) or 1 (MSM) partial records per device, copied to the primary with hipMemcpyPeerAsync
 * (xGMI) on the primary after every shard completed; processes that own one GPU each instead
 * all-gather kzgmi_batch_partial_device records over RCCL.  Every device gets
 * ceil(pipeline_slots / n_devices) workspaces, and the async entry points run whole batches per
 * device (kzgmi_slot_device). */
int kzgmi_ctx_create(kzgmi_ctx** out, const int* device_ids, int n_devices, int pipeline_slots);
/* The n_devices = 1 case of kzgmi_ctx_create, by device id (>= 0). */
int kzgmi_ctx_create_device(kzgmi_ctx** out, int device_id, int pipeline_slots);
void kzgmi_ctx_destroy(kzgmi_ctx* ctx);
int kzgmi_ctx_num_devices(const kzgmi_ctx* ctx);
/* Multi-device context: the async entry points (kzgmi_*_async, kzgmi_slot_wait, kzgmi_msm_wait,
 * kzgmi_stream_wait, kzgmi_slot_signal) pipeline WHOLE batches per device -- caller slot `slot`
 * (0 <= slot < pipeline_slots) runs on device device_ids[slot % n_devices], which this returns;
 * device pointers passed to that slot must live there.  Each device holds
 * ceil(pipeline_slots / n_devices) slots; caller slots 0 .. n_devices-1 are the devices' first
 * slots, which the synchronous split calls use.  Single-device context: device_ids[0]. */
int kzgmi_slot_device(const kzgmi_ctx* ctx, int slot);

/* Size every pipeline slot's device workspace (and, on a multi-device context, each device's
 * shard workspace) for batches of up to n tuples of `curve` verified with `flags`
 * (KZGMI_FLAG_*), and create the profiling events, so that later batch calls of at most that
 * size and mode allocate nothing.  Workspaces otherwise grow on first use; a caller timing a
 * steady state calls this first.  No job may be in flight.  On a multi-device context each
 * peer is sized for its share of the library's own balanced split (what the host-buffer entry
 * points use): shards passed to kzgmi_batch_verify_multi_device that are larger than
 * ceil(n / n_devices) rounded up to 4096 still grow the peer's workspace on first use.  The
 * host-buffer entry points also use a per-slot device staging buffer (n x (2 G1 + 64) B) and,
 * for pageable inputs, a per-slot pinned ring (2 x 16 MiB): these are made on a slot's first
 * host-buffer call, so a timed steady state of host-buffer calls warms every slot once first. */
int kzgmi_ctx_reserve(kzgmi_ctx* ctx, kzgmi_curve curve, size_t n, uint32_t flags);
/* Process-wide number of device workspace allocations the library has made so far (a timed
 * region that leaves it unchanged allocated nothing). */
uint64_t kzgmi_alloc_count(void);

/* Order the next job issued on slot `slot` after all work enqueued so far on `hip_stream` (a
 * hipStream_t of the ctx's primary device, passed as void*; NULL = the null stream), without a
 * host sync.  Several calls before one job all apply. */
int kzgmi_stream_wait(kzgmi_ctx* ctx, int slot, void* hip_stream);
/* The other direction: order all work enqueued later on `hip_stream` (a hipStream_t of the
 * primary device; NULL = the null stream) after everything enqueued so far on slot `slot`,
 * without a host sync -- e.g. an RCCL all-gather of a kzgmi_batch_partial_device_async partial
 * issued on the caller's stream.  The slot's job still completes (and reports its errors) with
 * kzgmi_slot_wait. */
int kzgmi_slot_signal(kzgmi_ctx* ctx, int slot, void* hip_stream);

/* Page-locked host memory for the host-buffer entry points: input arrays that lie inside a
 * kzgmi_host_alloc block or a kzgmi_host_register'ed range are copied to HBM by DMA on the
 * slot's stream, asynchronously (PCIe at full rate, overlapped with other slots' kernels).
 * Other (pageable) host memory is first copied by the calling thread(s) into the slot's own
 * pinned staging ring.  kzgmi_host_register pins an existing allocation (hipHostRegister);
 * unregister/free only when no job reading it is in flight. */
int kzgmi_host_alloc(size_t bytes, void** out);
void kzgmi_host_free(void* p);
int kzgmi_host_register(void* p, size_t bytes);
int kzgmi_host_unregister(void* p);

/* SURVEY.md 8b kzgmi_srs_load (BASELINE.json:5 "srs" = {G1, [1]_2, [tau]_2}): host encodings
 * of the SRS's G1 element g1 (the base of the -t G1 term; validated, must be a G1 member
 * other than infinity; g1 == NULL means the standard generator), the G2 generator and
 * [tau]_2.  Precomputes the Miller-loop line coefficients on the device(s). */
int kzgmi_srs_load(kzgmi_ctx* ctx, kzgmi_curve curve, const uint8_t* g1, const uint8_t* g2,
                   const uint8_t* tau_g2, kzgmi_srs** out);
void kzgmi_srs_free(kzgmi_srs* srs);

/* BASELINE.json:5 batch_verify(commitments, zs, ys, proofs, srs) -- host buffers (copied to
 * HBM, i.e. the PCIe-inclusive path; see kzgmi_batch_verify_ex_async for how).  *ok_out = 1
 * accept, 0 reject.  From 2^17 tuples the copy overlaps the computation: the batch is copied in
 * point ranges and each range's work starts when its copy lands (slot 0; slots 0-1 for
 * compressed, subgroup-checked and powers-of-r batches, which must then be idle too; not with
 * Fiat-Shamir).  KZGMI_HOST_CHUNKS=1 in the environment before kzgmi_ctx_create turns it off.
 * Calls of at most 4096 MSM terms (a batch has 3n + 1; with GLV 2 (2n + 1)) take a one-wave-
 * per-term path instead of the bucket method (KZGMI_SMALL_TERMS=<terms> moves the limit). */
int kzgmi_batch_verify(kzgmi_ctx* ctx, const kzgmi_srs* srs, const uint8_t* commitments,
                       const uint8_t* zs, const uint8_t* ys, const uint8_t* proofs, size_t n,
                       const uint8_t* seed32, int* ok_out);

/* Same check with the four input arrays already resident in device memory (device
 * pointers on ctx's device).  Synchronous. */
int kzgmi_batch_verify_device(kzgmi_ctx* ctx, const kzgmi_srs* srs, const void* d_commitments,
                              const void* d_zs, const void* d_ys, const void* d_proofs, size_t n,
                              const uint8_t* seed32, int* ok_out);

/* Pipelined form: enqueue on workspace `slot` (0 <= slot < pipeline_slots) and return at
 * once; kzgmi_slot_wait() blocks until that slot's verdict is ready.  Independent batches
 * on different slots overlap on the GPU (latency-bound tails of one batch run beside the
 * bucket accumulation of the next). */
int kzgmi_batch_verify_device_async(kzgmi_ctx* ctx, const kzgmi_srs* srs, int slot,
                                    const void* d_commitments, const void* d_zs, const void* d_ys,
                                    const void* d_proofs, size_t n, const uint8_t* seed32);
int kzgmi_slot_wait(kzgmi_ctx* ctx, int slot, int* ok_out);

/* batch_verify with input-format / validation flags (KZGMI_FLAG_*).
 * flags = 0 is exactly kzgmi_batch_verify / kzgmi_batch_verify_device_async. */
int kzgmi_batch_verify_ex(kzgmi_ctx* ctx, const kzgmi_srs* srs, const uint8_t* commitments,
                          const uint8_t* zs, const uint8_t* ys, const uint8_t* proofs, size_t n,
                          const uint8_t* seed32, uint32_t flags, int* ok_out);
int kzgmi_batch_verify_device_ex_async(kzgmi_ctx* ctx, const kzgmi_srs* srs, int slot,
                                       const void* d_commitments, const void* d_zs,
                                       const void* d_ys, const void* d_proofs, size_t n,
                                       const uint8_t* seed32, uint32_t flags);
/* BASELINE.json:5 batch_verify from HOST buffers, pipelined: the H2D copy of the four arrays is
 * enqueued on slot `slot`'s stream ahead of the batch's kernels, so the copy of one batch runs
 * beside the kernels of the batches on the other slots; kzgmi_slot_wait() returns the verdict.
 * Arrays inside pinned memory (kzgmi_host_alloc / kzgmi_host_register) are DMA'd directly and
 * the call returns at once -- they must stay allocated and unmodified until the wait returns.
 * Pageable arrays are copied through the slot's pinned staging ring before the call returns
 * (they may be reused at once; the call then costs the host-side copy).  On a multi-device
 * context the whole batch runs on the slot's device (kzgmi_slot_device); kzgmi_batch_verify_ex
 * splits one batch over all devices instead.
 * kzgmi_batch_verify / kzgmi_batch_verify_ex are this on slot 0 followed by the wait. */
int kzgmi_batch_verify_ex_async(kzgmi_ctx* ctx, const kzgmi_srs* srs, int slot,
                                const uint8_t* commitments, const uint8_t* zs, const uint8_t* ys,
                                const uint8_t* proofs, size_t n, const uint8_t* seed32,
                                uint32_t flags);

/* Multi-device context (kzgmi_ctx_create with n_devices > 1): device d holds n_per_device[d] tuples
 * (global indices follow device order) at d_*[d], device pointers on device_ids[d].  flags as
 * kzgmi_batch_verify_ex; with KZGMI_FLAG_FIAT_SHAMIR every non-empty shard but the last must
 * hold a multiple of 4096 tuples.  Synchronous. */
int kzgmi_batch_verify_multi_device(kzgmi_ctx* ctx, const kzgmi_srs* srs, const void* const* d_commitments,
                                    const void* const* d_zs, const void* const* d_ys,
                                    const void* const* d_proofs, const size_t* n_per_device,
                                    const uint8_t* seed32, uint32_t flags, int* ok_out);

/* Fiat-Shamir challenge of KZGMI_FLAG_FIAT_SHAMIR for a device-resident batch (flags:
 * KZGMI_FLAG_COMPRESSED): r as 32 big-endian bytes. */
int kzgmi_fs_challenge_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_commitments,
                              const void* d_zs, const void* d_ys, const void* d_proofs, size_t n,
                              uint32_t flags, uint8_t* r_out);
/* Multi-GPU form: a shard [index_offset, index_offset + n) with index_offset % 4096 == 0
 * writes its ceil(n / 4096) subtree roots (32 B each) to d_out; gather all shards' roots in
 * order and derive r with kzgmi_fs_challenge_from_digests_device, then verify each shard
 * with kzgmi_batch_partial_device_async(..., flags 0, seed32 = be32(r)). */
int kzgmi_fs_chunk_digests_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_commitments,
                                  const void* d_zs, const void* d_ys, const void* d_proofs, size_t n,
                                  uint64_t index_offset, uint32_t flags, void* d_out);
int kzgmi_fs_challenge_from_digests_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_digests,
                                           size_t nchunks, uint64_t n_total, uint8_t* r_out);

/* Validate n device-resident G1 encodings (flags: KZGMI_FLAG_COMPRESSED,
 * KZGMI_FLAG_SUBGROUP_CHECK): 0 if all are valid, else the first error class found. */
int kzgmi_g1_validate_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_points, size_t n,
                             uint32_t flags);
/* Compress n device-resident uncompressed G1 encodings into d_out (n x 48 B / 32 B).  Input
 * utility for tests and benchmarks: no validation. */
int kzgmi_g1_compress_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_points, size_t n,
                             void* d_out);

/* Diagnostics: the combined points A and B of the last synchronous batch_verify on slot 0
 * (G1 encodings, 2 x G1 bytes), for bit-exact parity tests against the oracle. */
int kzgmi_last_combination(kzgmi_ctx* ctx, uint8_t* a_out, uint8_t* b_out);

/* SURVEY.md 8b kzgmi_msm_g1: sum k_i P_i, host buffers; out = G1 encoding. */
int kzgmi_msm_g1(kzgmi_ctx* ctx, kzgmi_curve curve, const uint8_t* points, const uint8_t* scalars,
                 size_t n, uint8_t* out);
/* Same with device-resident points/scalars (output to host). */
int kzgmi_msm_g1_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_points,
                        const void* d_scalars, size_t n, uint8_t* out);

/* Pipelined MSM (configs[1] throughput): enqueue on workspace `slot` and return at once;
 * kzgmi_msm_wait() blocks until that slot's result is ready and writes the G1 encoding.
 * MSMs on different slots overlap on the GPU exactly like the async batch verifications
 * (kzgmi_slot_wait also completes an MSM job, discarding the point). */
int kzgmi_msm_g1_device_async(kzgmi_ctx* ctx, kzgmi_curve curve, int slot, const void* d_points,
                              const void* d_scalars, size_t n);
int kzgmi_msm_wait(kzgmi_ctx* ctx, int slot, uint8_t* out);

/* ---- multi-GPU point-range sharding ----------------------------
 * A rank verifying tuples [index_offset, index_offset + n) of a global batch writes its
 * partial (A_k, B_k) as 2 opaque partial-point records (kzgmi_partial_bytes() each) to
 * device memory; the records are all-gathered over RCCL and any rank combines them.
 * A shard that fails validation on its own device (an error reported by its wait) still writes
 * its records, MARKED as failed; a shard rejected before anything ran (an error returned by the
 * enqueue call) is marked by the caller filling its records with 0xFF bytes.  Every combine
 * that reads a marked record fails -- with the shard's own error code, or KZGMI_ERR_SHARD -- so
 * no rank can accept a batch one of whose shards was rejected, and every rank still takes part
 * in the collective (kzgmi/distributed.py). */
size_t kzgmi_partial_bytes(kzgmi_curve curve);
/* Encode `count` device-resident partial records (e.g. a shard's A_k, B_k) as G1 encodings
 * (count x G1 bytes, host) -- for checking partials against a CPU reference. */
int kzgmi_partial_encode_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_records, size_t count,
                                uint8_t* out);
int kzgmi_batch_partial_device(kzgmi_ctx* ctx, const kzgmi_srs* srs, const void* d_commitments,
                               const void* d_zs, const void* d_ys, const void* d_proofs, size_t n,
                               uint64_t index_offset, const uint8_t* seed32, void* d_partial_out);
int kzgmi_batch_combine_device(kzgmi_ctx* ctx, const kzgmi_srs* srs, const void* d_partials,
                               int n_parts, int* ok_out);
/* Pipelined forms of the two calls above on workspace `slot`; kzgmi_slot_wait() completes
 * them (ok_out = 1 for a partial job, the verdict for a combine job).  A rank keeps several
 * shards in flight exactly like kzgmi_batch_verify_device_async. */
int kzgmi_batch_partial_device_async(kzgmi_ctx* ctx, const kzgmi_srs* srs, int slot,
                                     const void* d_commitments, const void* d_zs, const void* d_ys,
                                     const void* d_proofs, size_t n, uint64_t index_offset,
                                     const uint8_t* seed32, uint32_t flags, void* d_partial_out);
int kzgmi_batch_combine_device_async(kzgmi_ctx* ctx, const kzgmi_srs* srs, int slot,
                                     const void* d_partials, int n_parts);
int kzgmi_msm_partial_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_points,
                             const void* d_scalars, size_t n, void* d_partial_out);
int kzgmi_msm_combine_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_partials,
                             int n_parts, uint8_t* out);
/* sum k_i P_i over shards resident on each device of a multi-device context (see
 * kzgmi_batch_verify_multi_device); out = G1 encoding. */
int kzgmi_msm_g1_multi_device(kzgmi_ctx* ctx, kzgmi_curve curve, const void* const* d_points,
                              const void* const* d_scalars, const size_t* n_per_device, uint8_t* out);
/* Pipelined forms: the partial completes with kzgmi_slot_wait, the combine (sum of the
 * gathered records, encoded) with kzgmi_msm_wait. */
int kzgmi_msm_partial_device_async(kzgmi_ctx* ctx, kzgmi_curve curve, int slot, const void* d_points,
                                   const void* d_scalars, size_t n, void* d_partial_out);
int kzgmi_msm_combine_device_async(kzgmi_ctx* ctx, kzgmi_curve curve, int slot,
                                   const void* d_partials, int n_parts);

/* prover-side commitments with a fixed SRS base.  kzgmi_ck_load uploads
 * n G1 powers ([tau^i]_1, host encodings, validated) and precomputes 16 rows of 2^(16 w)-shifted
 * copies on the device (16 n points resident); kzgmi_commit then computes
 * sum_{i < m} coeff_i [tau^i]_1 (coefficients: m x 32 B canonical Fr, m <= n) as ONE bucket
 * set of 16-bit signed digits -- no per-window reduction, no window combination.  The key
 * must be freed before (or is detached by) kzgmi_ctx_destroy. */
int kzgmi_ck_load(kzgmi_ctx* ctx, kzgmi_curve curve, const uint8_t* g1_powers, size_t n, kzgmi_ck** out);
void kzgmi_ck_free(kzgmi_ck* ck);
int kzgmi_commit(kzgmi_ctx* ctx, const kzgmi_ck* ck, const uint8_t* coeffs, size_t m, uint8_t* out);
int kzgmi_commit_device(kzgmi_ctx* ctx, const kzgmi_ck* ck, const void* d_coeffs, size_t m,
                        uint8_t* out);
/* Pipelined form: enqueue on workspace `slot`; kzgmi_msm_wait(ctx, slot, out) returns the
 * commitment (G1 encoding). */
int kzgmi_commit_device_async(kzgmi_ctx* ctx, const kzgmi_ck* ck, int slot, const void* d_coeffs, size_t m);

/* Optimal-ate pairing e(P, Q) for P in G1, Q in G2: 12 Fp values in tower order, big-endian:
 * 576 B (BLS12-381) / 384 B (BN254).  Test/diagnostic utility.  (ABI 2 returned e(P, Q)^3 on
 * BLS12-381, the value the batch check's final exponentiation computes; ABI 3 scales P by
 * 3^-1 mod r first, so the result is the standard e(P, Q) -- for P outside G1 it is not.) */
int kzgmi_pairing(kzgmi_ctx* ctx, kzgmi_curve curve, const uint8_t* g1, const uint8_t* g2,
                  uint8_t* out);
/* (The 3^-1 scaling runs the library's MSM on one point with the GLV split forced off, so the
 * result does not depend on kzgmi_set_trusted_g1 / kzgmi_set_glv.) */

/* ---- synthetic-input generators (device side; used by bench.py and GPU tests) ---------
 * d_points_out[i] = k_i * G1 for device scalars k_i (32 B BE each). */
int kzgmi_gen_g1(kzgmi_ctx* ctx, kzgmi_curve curve, const void* d_scalars, size_t n,
                 void* d_points_out);
/* n valid opening tuples under a toy tau (32 B BE, < r): c_i, z_i, y_i = 253-bit values
 * int_be(SHA256(seed || le64(i) || tag)) & (2^253 - 1), tag = 'c','z','y';
 * q_i = (c_i - y_i)/(tau - z_i); C_i = c_i G1, pi_i = q_i G1.  Device outputs. */
int kzgmi_gen_tuples(kzgmi_ctx* ctx, kzgmi_curve curve, const uint8_t* tau32, const uint8_t* seed32,
                     size_t n, void* d_commitments, void* d_zs, void* d_ys, void* d_proofs);

/* [k]Q for a G2 point Q (host encodings; k = 32 B BE, < r): toy-SRS generation
 * ([tau]_2 from a known tau, SURVEY.md 2 "test-only toy-tau generator"). */
int kzgmi_g2_mul(kzgmi_ctx* ctx, kzgmi_curve curve, const uint8_t* g2, const uint8_t* k32, uint8_t* out);

/* Compute-roofline probe: Montgomery Fp multiplications per second on this GPU (many
 * independent products per thread, whole chip), written to *muls_per_s. */
int kzgmi_probe_fpmul(kzgmi_ctx* ctx, kzgmi_curve curve, double* muls_per_s);

/* GLV endomorphism phi(x, y) = (beta x, y) = [lambda] P.  Full Fr
 * scalars k are split as k = k0 + k1 lambda (|k0|, |k1| < 2^127) so each MSM runs 8 windows
 * over P and phi(P) instead of 16 over P: the same bucket additions, half the bucket sets to
 * reduce and half the window-combination doublings.  phi acts as [lambda] only on G1, so the
 * split is used where the points are G1 members: always on BN254 (cofactor 1); on BLS12-381
 * for batch calls with KZGMI_FLAG_SUBGROUP_CHECK or KZGMI_FLAG_TRUSTED_G1 and for MSMs after
 * kzgmi_set_trusted_g1(ctx, 1).  On G1 the results are identical either way.
 * kzgmi_set_glv switches the split off/on (msm: kzgmi_msm_g1*, batch: s_i, t and r^i of batch
 * verification; default both on) for A/B measurements.  Not allowed while jobs are in flight. */
int kzgmi_set_glv(kzgmi_ctx* ctx, int msm, int batch);
/* Declare that every point passed to kzgmi_msm_g1* on this context is in G1 (default 0). */
int kzgmi_set_trusted_g1(kzgmi_ctx* ctx, int on);
/* Split accumulation of a batch's two MSMs (latency): MSM#0's bucket sets accumulate in a first
 * launch and its reduction + window combination run on a side stream beside MSM#1's launch
 * (KZGMI_SPLIT_REV=0 in the environment at context creation: MSM#1's sets first instead).
 * mode -1 (default): synchronous kzgmi_batch_verify_device calls of >= 2^25 window entries whose
 * second MSM has more windows (no GLV) with no other slot in flight (async calls never split:
 * the first batch of a pipeline is alone too); 0: never;
 * 1: every two-MSM call.
 * Results are identical either way.  Not allowed while jobs are in flight. */
int kzgmi_set_split_acc(kzgmi_ctx* ctx, int mode);

/* ---- profiling -----------------------------------------------------------------------
 * When enabled, every batch / MSM call records HIP events around each phase on the stream
 * its kernels run on; kzgmi_get_phase_ms() returns the per-phase device time (ms) averaged
 * over all calls completed since profiling was (re)enabled, in the order of
 * kzgmi_phase_names() (comma-separated).  Enabling resets the averages.  On a multi-device
 * context the switch applies to every device and the times are the primary device's. */
int kzgmi_set_profiling(kzgmi_ctx* ctx, int on);
const char* kzgmi_phase_names(void);
int kzgmi_get_phase_ms(kzgmi_ctx* ctx, double* out, int max_n);

#ifdef __cplusplus
}
#endif
#endif /* KZGMI_H */
