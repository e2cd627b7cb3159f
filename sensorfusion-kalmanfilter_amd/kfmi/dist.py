"""Multi-GPU sharding of independent filters: one process per GPU, torch.distributed
(RCCL over xGMI as backend 'nccl'; 'gloo' on CPU for tests).

Filters are independent (each reference combo runs from its own copy of (x, P),
kf_workers.py:29-30), so rank r owns the contiguous global filter range
``shard_range(B_global, r, world)`` and regenerates its own input streams from the
counter-based generator (kf_synth keyed by the GLOBAL filter index) — no scatter and no
collective in the time loop.  The only collective is the final reassembly of per-shard
results (``gather_shards``), plus scalar reductions for timing.
"""
from __future__ import annotations

import torch


def shard_range(total, rank, world):
    """(offset, count) of rank's contiguous slice; the first total % world ranks get one more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f'bad rank {rank} / world {world}')
    base, rem = divmod(int(total), world)
    count = base + (1 if rank < rem else 0)
    offset = rank * base + min(rank, rem)
    return offset, count


def shard_counts(total, world):
    return [shard_range(total, r, world)[1] for r in range(world)]


def gather_shards(local, total, group=None):
    """All-gather per-rank tensors whose LAST dim is the rank's filter slice into one tensor
    with last dim ``total`` on every rank (filter order = global order).  Uneven shards are
    padded to the largest one for the collective and trimmed afterwards."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    counts = shard_counts(total, world)
    width = max(counts)
    lead = tuple(local.shape[:-1])
    if local.shape[-1] != counts[dist.get_rank(group)]:
        raise ValueError(f'local shard has {local.shape[-1]} filters, expected {counts[dist.get_rank(group)]}')
    padded = local
    if local.shape[-1] != width:
        padded = torch.zeros(lead + (width,), dtype=local.dtype, device=local.device)
        padded[..., :local.shape[-1]] = local
    # gather along a new leading rank axis, then lay the shards side by side
    flat = padded.reshape(-1, width).contiguous()
    rows = flat.shape[0]
    out = torch.empty((world * rows, width), dtype=flat.dtype, device=flat.device)
    dist.all_gather_into_tensor(out, flat, group=group)
    out = out.reshape(world, rows, width)
    parts = [out[r, :, :counts[r]] for r in range(world)]
    return torch.cat(parts, dim=-1).reshape(lead + (total,))


def max_over_ranks(values, device, group=None):
    """Element-wise max of a list of floats over all ranks (timing: the slowest rank counts)."""
    import torch.distributed as dist
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(v) for v in t.tolist()]
