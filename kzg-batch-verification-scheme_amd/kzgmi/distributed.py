"""Multi-GPU batch verification: point-range shards + one RCCL all-gather.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Rank k owns
tuples [offset_k, offset_k + n_k) of a global batch.  Randomisers are counter-mode in the
GLOBAL index (include/kzgmi.h), so every rank derives its own r_i with no communication and
the sharded check is bit-identical to the unsharded one.  Each rank computes its partial
(A_k, B_k) -- it folds its own -(sum r_i y_i) G1 into B_k -- and the 2-point partial
records (2 x kzgmi_partial_bytes) are all-gathered; every rank sums them and runs the
two-pairing check, so all ranks return the same verdict without a broadcast.

RCCL has no elliptic-curve reduction operator (rccl.h:448-454 lists sum/prod/max/min/avg),
so gather-then-add IS the collective; the payload is ~400 B per rank (latency-bound).

`ShardedPipeline` keeps `slots` global batches in flight per rank (async partial on slot
k % slots, then gather + pairing of the batch that used the slot before), so a rank runs
at the single-GPU pipelined rate plus one small all-gather per batch.

`backend` is anything with the methods used below (a `kzgmi.Context` on the GPU; the
CPU tests substitute a double built on the oracle to exercise this orchestration with gloo).

A shard that fails on its own rank (invalid encoding, off-curve point, subgroup check...) still
takes part in the collective: its partial record is marked failed -- by the device
(k_partial_out) or, for errors raised before anything ran, here (every byte 0xFF) -- so every
rank's combine reports an error (KZGMI_ERR_SHARD, or the shard's own code) instead of a
verdict, the failing rank re-raises its own error, and no rank can accept the batch.  Raising
before the all-gather instead would leave the other ranks blocked in it.

Stream order: the collectives run on torch's streams, kzgmi on its own.  Every
`kzgmi.Context` method that reads a device tensor first orders its slot's stream after
torch's current stream (kzgmi_stream_wait), and every kzgmi output read here (partial
records, subtree roots) is complete when the call or its wait() returns -- so gathered
buffers are never read before the all-gather has written them, whatever buffer the caching
allocator hands out.
"""
from __future__ import annotations

from typing import Tuple


FS_CHUNK = 4096  # Fiat-Shamir transcript subtree (csrc/fs.hpp): shard offsets must align to it

_COMM_STREAMS = {}


def comm_stream(device):
    """The side stream the eager schedules gather on: ONE per device for the process.  HIP maps
    streams onto GPU_MAX_HW_QUEUES hardware queues round-robin at creation; a stream that shares
    a queue with a slot stream blocks the slot behind its GPU-side wait for a partial (a run that
    made a new side stream per pipeline wrapped the 24 queues and serialised its MSMs), so the
    pipelines share this one."""
    import torch
    key = str(device)
    if key not in _COMM_STREAMS:
        _COMM_STREAMS[key] = torch.cuda.Stream(device=device)
    return _COMM_STREAMS[key]


def mark_failed(record):
    """Mark a partial record (device or CPU tensor) as a failed shard: every byte 0xFF
    (include/kzgmi.h: the combine then reports KZGMI_ERR_SHARD on every rank)."""
    record.fill_(0xFF)


# input-validation errors (KZGMI_ERR_ENCODING / NOT_ON_CURVE / SCALAR / NOT_IN_SUBGROUP) that a
# partial job's wait reports were found on the device, which wrote the record marked with the
# code itself: other ranks then report that code rather than KZGMI_ERR_SHARD
_DEVICE_MARKED = (-2, -3, -4, -7)


def _mark_unless_device_marked(record, err):
    if getattr(err, "code", None) not in _DEVICE_MARKED:
        mark_failed(record)


def shard_range(n_total: int, world: int, rank: int, align: int = 1) -> Tuple[int, int]:
    """Contiguous balanced split: (offset, count) of rank's tuples; offsets are multiples of
    `align` (the Fiat-Shamir mode needs align = 4096)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    units = (n_total + align - 1) // align
    base, extra = divmod(units, world)
    u0 = rank * base + min(rank, extra)
    u1 = u0 + base + (1 if rank < extra else 0)
    lo, hi = min(n_total, u0 * align), min(n_total, u1 * align)
    return lo, hi - lo


def fs_challenge_sharded(backend, curve: str, commitments, zs, ys, proofs, n_local: int, offset: int,
                         n_total: int, compressed: bool = False, group=None) -> int:
    """The Fiat-Shamir r of the whole (sharded) batch: each rank hashes its 4096-leaf subtrees,
    the subtree roots are all-gathered (one collective), every rank derives the same r.
    Shards must come from shard_range(..., align=4096)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    dev = backend.tensor_device()
    counts = [(shard_range(n_total, world, k, FS_CHUNK)[1] + FS_CHUNK - 1) // FS_CHUNK for k in range(world)]
    width = max(1, max(counts))
    local = torch.zeros(width * 32, dtype=torch.uint8, device=dev)
    if n_local:
        backend.fs_chunk_digests(curve, commitments, zs, ys, proofs, n_local, offset, local, compressed=compressed)
    gathered = torch.empty(world * width * 32, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(gathered, local, group=group)
    parts = [gathered[k * width * 32:(k * width + counts[k]) * 32] for k in range(world) if counts[k]]
    digests = torch.cat(parts)
    return backend.fs_challenge_from_digests(curve, digests, sum(counts), n_total)


def sharded_batch_verify(backend, srs, commitments, zs, ys, proofs, n_local: int, offset: int,
                         seed: bytes, group=None, fiat_shamir: bool = False, n_total: int = 0,
                         compressed: bool = False) -> bool:
    """Verify this rank's shard as part of a global batch; collective over `group`.

    commitments/zs/ys/proofs: this rank's shard (device tensors on the GPU path).
    fiat_shamir: the counter-mode r_i seeded with the whole batch's transcript challenge r
    (fs_challenge_sharded; shards from shard_range(n_total, world, rank, align=4096)); seed is
    ignored.
    Returns the global verdict on every rank.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    pb = backend.partial_bytes(srs.curve)
    dev = backend.tensor_device()
    local = torch.empty(2 * pb, dtype=torch.uint8, device=dev)
    err = None
    if fiat_shamir:
        r = fs_challenge_sharded(backend, srs.curve, commitments, zs, ys, proofs, n_local, offset, n_total,
                                 compressed=compressed, group=group)
    try:
        if fiat_shamir:
            backend.batch_partial_async(srs, 0, commitments, zs, ys, proofs, n_local, offset,
                                        r.to_bytes(32, "big"), local, compressed=compressed)
            backend.wait(0)
        else:
            backend.batch_partial(srs, commitments, zs, ys, proofs, n_local, offset, seed, local)
    except Exception as e:  # this shard failed: join the collective with a marked record
        err = e
        _mark_unless_device_marked(local, e)
    gathered = torch.empty(world * 2 * pb, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(gathered, local, group=group)
    try:
        ok = backend.batch_combine(srs, gathered, world)
    except Exception:
        if err is not None:
            raise err
        raise
    if err is not None:  # (a combine always reports a marked record)
        raise err
    return ok


class _PartialPipeline:
    """Shared schedule of ShardedPipeline / ShardedMsmPipeline: the shard partial of job k runs on
    slot k % slots, its record is all-gathered over `group`, and the gathered records are combined.
    Every rank must submit the same sequence of jobs (the all-gathers are collectives); results
    come back in submission order.

    Two schedules:
      - eager (a backend with `signal`, i.e. kzgmi.Context on a GPU; the default there): right
        after job k's partial is enqueued on slot s, its all-gather and its combine are enqueued
        too, ordered on the GPU -- a side stream waits for the slot (kzgmi_slot_signal), RCCL
        gathers on it, and the combine is chained on slot s itself behind that stream (a combine
        on a slot whose pending job is a partial).  The host never waits on a partial before
        issuing the collective; collecting slot s's result when it comes round again is the
        pipeline's only throttle.  The context needs `slots` workspaces;
      - deferred (otherwise, e.g. the CPU test double): when slot s comes round, its partial
        (job k - slots) is waited for on the host, all-gathered, and combined on lane j % lanes
        (context slots slots .. slots + lanes - 1), whose result is collected when the lane is
        reused.  The context needs slots + lanes workspaces.

    A shard that fails on this rank -- at enqueue or at its wait -- joins the all-gather with a
    marked record (module docstring): every rank's combine of that job then fails, and this
    rank re-raises its own error when the job's result is collected.

    submit() enqueues the new job and returns the results of the jobs that completed during the
    call; drain() completes everything still in flight.  If one of those jobs failed, its error
    is raised instead -- after the new job was enqueued and every other collected job completed,
    so all ranks stay in step -- with the call's results on the exception as `.results` (None at
    each failed job's place).
    """

    records = 1  # partial records per rank per job

    def __init__(self, backend, curve: str, slots: int, lanes: int, group=None, eager=None):
        import torch
        import torch.distributed as dist
        self.backend, self.group = backend, group
        self.slots, self.lanes = slots, lanes
        self.world = dist.get_world_size(group)
        rec = self.records * backend.partial_bytes(curve)
        self.dev = backend.tensor_device()
        on_gpu = getattr(self.dev, "type", str(self.dev)) == "cuda"
        self.eager = (on_gpu and hasattr(backend, "signal")) if eager is None else eager
        self.comm = comm_stream(self.dev) if self.eager and on_gpu else None  # CPU test doubles: no stream
        self.local = [torch.empty(rec, dtype=torch.uint8, device=self.dev) for _ in range(slots)]
        # one gather buffer per slot (eager) / lane (deferred): the combine reads it until the
        # slot / lane is reused
        nbuf = slots if self.eager else lanes
        self.gathered = [torch.empty(self.world * rec, dtype=torch.uint8, device=self.dev) for _ in range(nbuf)]
        self.pending = [False] * slots
        self.lane_pending = [False] * lanes
        self.err = {}   # context slot -> this rank's own shard error, re-raised when collected
        self.k = 0      # jobs submitted
        self.j = 0      # combines issued (deferred)

    # hooks
    def _partial_async(self, s, args):
        raise NotImplementedError

    def _combine_async(self, slot, gathered):
        raise NotImplementedError

    def _result(self, slot):
        raise NotImplementedError

    def _collect(self, slot: int):
        """The combined result of `slot`, or _Failed; this rank's own shard error wins over the
        marked-record error its combine reports."""
        err = self.err.pop(slot, None)
        try:
            res = self._result(slot)
        except Exception as e:
            return _Failed(err if err is not None else e)
        return res if err is None else _Failed(err)

    @staticmethod
    def _finish(out):
        failed = [r for r in out if isinstance(r, _Failed)]
        if failed:
            e = failed[0].err
            e.results = [None if isinstance(r, _Failed) else r for r in out]
            raise e
        return out

    def _collect_lane(self, lane: int, out):
        if self.lane_pending[lane]:
            self.lane_pending[lane] = False
            out.append(self._collect(self.slots + lane))

    def _gather_and_combine(self, s: int, out):
        import torch.distributed as dist
        err = self.err.pop(s, None)
        if err is not None:                                    # rejected at enqueue: nothing ran
            mark_failed(self.local[s])
        else:
            try:
                self.backend.wait(s)                           # shard partial ready
            except Exception as e:                             # failed shard: joins with a marked record
                err = e
                _mark_unless_device_marked(self.local[s], e)
        self.pending[s] = False
        lane = self.j % self.lanes
        self.j += 1
        self._collect_lane(lane, out)                          # result of the job `lanes` combines ago
        # the combine lane's stream is ordered after torch's current stream (which waits for the
        # collective) inside the combine call (kzgmi_stream_wait): no host sync
        dist.all_gather_into_tensor(self.gathered[lane], self.local[s], group=self.group)
        self._combine_async(self.slots + lane, self.gathered[lane])
        self.lane_pending[lane] = True
        if err is not None:
            self.err[self.slots + lane] = err

    def _enqueue_eager(self, s: int):
        import contextlib
        import torch
        import torch.distributed as dist
        with (torch.cuda.stream(self.comm) if self.comm is not None else contextlib.nullcontext()):
            self.backend.signal(s, self.comm)                  # the side stream waits for the partial
            if s in self.err:                                  # rejected at enqueue: nothing ran on the slot
                mark_failed(self.local[s])
            dist.all_gather_into_tensor(self.gathered[s], self.local[s], group=self.group)
            # chained on slot s, ordered after torch's current stream (= the side stream)
            self._combine_async(s, self.gathered[s])

    def _submit(self, args):
        s = self.k % self.slots
        self.k += 1
        done = []
        if self.pending[s]:
            self.pending[s] = False
            if self.eager:
                done.append(self._collect(s))                  # partial + gather + combine of job k - slots
            else:
                self._gather_and_combine(s, done)
        try:
            self._partial_async(s, args)
        except Exception as e:  # rejected before anything ran: the collective still happens
            self.err[s] = e
        self.pending[s] = True
        if self.eager:
            self._enqueue_eager(s)
        return self._finish(done)

    def drain(self):
        out = []
        for i in range(self.slots):
            s = (self.k + i) % self.slots                      # oldest first
            if self.pending[s]:
                self.pending[s] = False
                if self.eager:
                    out.append(self._collect(s))
                else:
                    self._gather_and_combine(s, out)
        if not self.eager:
            for i in range(self.lanes):
                self._collect_lane((self.j + i) % self.lanes, out)
        return self._finish(out)


class _Failed:
    def __init__(self, err):
        self.err = err


class ShardedPipeline(_PartialPipeline):
    """Several global batches in flight per rank (the multi-GPU form of the single-GPU slot
    pipeline; schedules in _PartialPipeline).  Each job is one batch: this rank's partial
    (A_k, B_k) of its shard, the all-gather of the 2-record partials, and the sum + pairing
    check (kzgmi_batch_combine_device_async); results are verdicts."""

    records = 2

    def __init__(self, backend, srs, slots: int = 3, lanes: int = 2, group=None, eager=None):
        self.srs = srs
        super().__init__(backend, srs.curve, slots, lanes, group, eager)

    def _partial_async(self, s, args):
        commitments, zs, ys, proofs, n_local, offset, seed = args
        self.backend.batch_partial_async(self.srs, s, commitments, zs, ys, proofs, n_local, offset, seed,
                                         self.local[s])

    def _combine_async(self, slot, gathered):
        self.backend.batch_combine_async(self.srs, slot, gathered, self.world)

    def _result(self, slot):
        return self.backend.wait(slot)

    def submit(self, commitments, zs, ys, proofs, n_local: int, offset: int, seed: bytes):
        return self._submit((commitments, zs, ys, proofs, n_local, offset, seed))


def sharded_msm(backend, curve: str, points, scalars, n_local: int, group=None) -> bytes:
    """sum_i k_i P_i over all ranks' point ranges; result (G1 encoding) on every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    pb = backend.partial_bytes(curve)
    dev = backend.tensor_device()
    local = torch.empty(pb, dtype=torch.uint8, device=dev)
    err = None
    try:
        backend.msm_partial(curve, points, scalars, n_local, local)
    except Exception as e:  # join the collective with a marked record (module docstring)
        err = e
        _mark_unless_device_marked(local, e)
    gathered = torch.empty(world * pb, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(gathered, local, group=group)
    try:
        out = backend.msm_combine(curve, gathered, world)
    except Exception:
        if err is not None:
            raise err
        raise
    if err is not None:
        raise err
    return out



class ShardedMsmPipeline(_PartialPipeline):
    """Several global MSMs in flight per rank (schedules in _PartialPipeline): the shard partial
    sum of MSM k (kzgmi_msm_partial_device_async), the all-gather of the 1-record partials, and
    their sum, encoded (kzgmi_msm_combine_device_async); results are G1 encodings, the same on
    every rank."""

    def __init__(self, backend, curve: str, slots: int = 3, lanes: int = 2, group=None, eager=None):
        self.curve = curve
        super().__init__(backend, curve, slots, lanes, group, eager)

    def _partial_async(self, s, args):
        points, scalars, n_local = args
        self.backend.msm_partial_async(self.curve, s, points, scalars, n_local, self.local[s])

    def _combine_async(self, slot, gathered):
        self.backend.msm_combine_async(self.curve, slot, gathered, self.world)

    def _result(self, slot):
        return self.backend.msm_wait(slot)

    def submit(self, points, scalars, n_local: int):
        return self._submit((points, scalars, n_local))
