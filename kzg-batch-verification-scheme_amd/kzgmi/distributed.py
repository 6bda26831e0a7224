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

`backend` is anything with the three methods used below (a `kzgmi.Context` on the GPU; the
CPU tests substitute a double built on the oracle to exercise this orchestration with gloo).
"""
from __future__ import annotations

from typing import Tuple


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split: (offset, count) of rank's tuples."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    base, extra = divmod(n_total, world)
    offset = rank * base + min(rank, extra)
    return offset, base + (1 if rank < extra else 0)


def sharded_batch_verify(backend, srs, commitments, zs, ys, proofs, n_local: int, offset: int,
                         seed: bytes, group=None) -> bool:
    """Verify this rank's shard as part of a global batch; collective over `group`.

    commitments/zs/ys/proofs: this rank's shard (device tensors on the GPU path).
    Returns the global verdict on every rank.
    """
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    pb = backend.partial_bytes(srs.curve)
    dev = backend.tensor_device()
    local = torch.empty(2 * pb, dtype=torch.uint8, device=dev)
    backend.batch_partial(srs, commitments, zs, ys, proofs, n_local, offset, seed, local)
    gathered = torch.empty(world * 2 * pb, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(gathered, local, group=group)
    return backend.batch_combine(srs, gathered, world)


def sharded_msm(backend, curve: str, points, scalars, n_local: int, group=None) -> bytes:
    """sum_i k_i P_i over all ranks' point ranges; result (G1 encoding) on every rank."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    pb = backend.partial_bytes(curve)
    dev = backend.tensor_device()
    local = torch.empty(pb, dtype=torch.uint8, device=dev)
    backend.msm_partial(curve, points, scalars, n_local, local)
    gathered = torch.empty(world * pb, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(gathered, local, group=group)
    return backend.msm_combine(curve, gathered, world)
