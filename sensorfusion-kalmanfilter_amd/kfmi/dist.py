"""Multi-GPU sharding of independent filters: one process per GPU, torch.distributed
(RCCL over xGMI as backend 'nccl'; 'gloo' on CPU for tests).

Filters are independent (each reference combo runs from its own copy of (x, P),
kf_workers.py:29-30), so rank r owns the contiguous global filter range
``shard_range(B_global, r, world)`` and regenerates its own input streams from the
counter-based generator (kf_synth keyed by the GLOBAL filter index) — no scatter and no
collective in the time loop.  The only collective is the final reassembly of per-shard
results (``gather_shards``), plus scalar reductions for timing.

The brute-force search (kf_workers.py:1218-1392) shards by subset class instead: the subsets
are split by their intersection with the first few candidates, each rank runs the
shared-prefix search over its classes, and two all-reduces pick the globally first acceptable
combination (``brute_force_search``).  ``brute_force_search_ranks`` shards one filter per
subset by combination rank, for searches whose prefix levels do not fit on the GPU.
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
    # gloo collectives take host tensors (a CUDA tensor only appears here under gloo in the
    # bench's one-GPU rehearsal, bench.py --dist-backend gloo); RCCL gathers in HBM
    home = flat.device
    if dist.get_backend(group) == 'gloo':
        flat = flat.cpu()
    rows = flat.shape[0]
    out = torch.empty((world * rows, width), dtype=flat.dtype, device=flat.device)
    dist.all_gather_into_tensor(out, flat, group=group)
    out = out.to(home).reshape(world, rows, width)
    parts = [out[r, :, :counts[r]] for r in range(world)]
    return torch.cat(parts, dim=-1).reshape(lead + (total,))


def decimated_steps(T, every):
    """Time steps kept by a trajectory decimated every ``every`` steps: every-1, 2 every-1, ...
    (the last step whenever every divides T); none for every <= 0."""
    return list(range(every - 1, T, every)) if every > 0 else []


def gather_run_outputs(x, logdet_last, traj=None, every=0, total=None, group=None):
    """Reassemble a sharded run on every rank (north_star: the RCCL all-gather "to reassemble
    the final trajectory array"; the brute-force parent's tuples carry each combination's
    trajectory, kf_workers.py:86, 1349-1371).  x [n, b] final states, logdet_last [b] last
    log-dets, traj [T, W, b] (optional) decimated to ``decimated_steps(T, every)``: all packed
    into one [rows, b] tensor and moved by ONE all-gather.  Returns dict(x [n, total], logdet
    [total], traj [R, W, total] or None, rows, bytes_per_rank) in global filter order."""
    b = x.shape[-1]
    total = b if total is None else int(total)
    parts = [x.reshape(-1, b), logdet_last.reshape(1, b)]
    steps = decimated_steps(traj.shape[0], every) if traj is not None else []
    if steps:
        parts.append(traj[steps[0]::every][:len(steps)].reshape(-1, b))
    packed = torch.cat(parts, dim=0).contiguous()
    full = gather_shards(packed, total, group=group)
    n = x.shape[0]
    out = dict(x=full[:n], logdet=full[n], traj=None, rows=packed.shape[0],
               bytes_per_rank=packed.numel() * packed.element_size())
    if steps:
        out['traj'] = full[n + 1:].reshape(len(steps), traj.shape[1], total)
    return out


def max_over_ranks(values, device, group=None):
    """Element-wise max of a list of floats over all ranks (timing: the slowest rank counts)."""
    import torch.distributed as dist
    if dist.get_backend(group) == 'gloo':
        device = 'cpu'
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return [float(v) for v in t.tolist()]


_NONE = (1 << 63) - 1


def search_classes(n, world, dtype='f64', mem_bytes=32 << 30, sym=False):
    """Shard plan of the shared-prefix search over ``world`` ranks: the subsets are split by their
    intersection with the first w candidates (2^w classes of 2^(n-w) subsets each, the same
    work each), class c going to rank c % world.  w = the larger of the rank rule (the fewest
    classes, at least one per rank, that deal out within 25 % of even: 2^w = world for a power of
    two, 8 classes for 3 ranks; at most n - 1; 0 for one rank) and the memory rule
    (ref15.search_class_width: a class's every size fits ``mem_bytes`` and the 2^28-parent cap),
    so no rank ever falls back to one filter per subset.  Returns w."""
    from . import ref15
    w = 0
    if world > 1:
        while w < n - 1 and ((1 << w) < world or -(-(1 << w) // world) * world * 4 > 5 * (1 << w)):
            w += 1
    return max(w, ref15.search_class_width(n, dtype, mem_bytes, sym))


def brute_force_search(events, start_idx=0, end_idx=None, R_threshold=None, initial_pt=None, initial_state=None,
                       max_combos_in_memory=1 << 22, dtype='f64', device=0, group=None, search_class=None,
                       finish=None, search_mem_bytes=32 << 30, consts=None):
    """run_brute_force_kalman_filter_no_sampling_min_usage sharded over the ranks of ``group``
    with the shared-prefix search (kf_search_combos): after the sizes that fit one call (the same
    on every rank) and, past those, bands of prefix classes dealt over the ranks
    (ref15.search_bands) while they are the fewer calls, the subsets are split into 2^w classes by
    their intersection with the first w candidates (``search_classes``: enough classes to deal
    out evenly over the ranks, each small enough for one search call); each rank searches its
    classes, keeping
    the first size with an acceptable subset and its first such subset in itertools order, and
    two all-reduces (MIN of the size, then MAX of the bit-reversed subset mask at that size) pick
    the same winner as the single-GPU search.  Every rank returns the reference's result dict
    (or None).  ``max_combos_in_memory`` is the reference's argument (unused: no per-subset batch).

    ``search_class(n_fixed, fixed_mask, k_max) -> (k, indices or None)`` / ``finish(k, indices)``
    replace the GPU evaluation (tests drive the reduction logic with the CPU oracle on gloo).
    consts: a ref15.ModelConsts (the reference's constants by default)."""
    from . import ref15
    if R_threshold is None:
        raise ValueError('R_threshold must be specified for brute force KF.')
    import torch.distributed as dist
    world = dist.get_world_size(group)
    st = ref15.brute_force_setup(events, start_idx, end_idx, initial_pt, initial_state, consts)
    if st is None:
        return None
    cand, xt, Pt, prev_time, target_end, ev, init = st
    n = len(cand)
    kf = None
    sym = False
    k_search = n
    if finish is None:
        def finish(k, idx):
            return ref15.brute_force_result(cand, k, None, xt, Pt, prev_time, target_end, dtype, device,
                                            indices=idx, consts=consts)
    if search_class is None:
        kf = ref15.BatchedKF('ref15', 1, dtype, device=device, params=ref15._params(consts))
        sym = kf.search_plan(init, n, k_max=1)['sym']
        k_search = ref15.search_levels(n, dtype, search_mem_bytes, sym)
        if k_search < n:
            # a search too large for one call (n = 40): first its sizes 1 .. k_search in one call,
            # the same on every rank (the reference's windows accept within them in milliseconds);
            # only if none is accepted, every size by class over the ranks
            try:
                k, idx = ref15.one_call_search(kf, ev, init, prev_time, target_end, R_threshold, k_search, dtype,
                                               search_mem_bytes, sym)
            except BaseException:
                kf.close()
                raise
            if k:
                kf.close()
                return finish(k, idx)

        def search_class(n_fixed, fixed_mask, k_max):
            k, idx, _, _ = kf.search_combos(ev, init, prev_time, target_end, R_threshold, k_max=k_max,
                                            n_fixed=n_fixed, fixed_mask=fixed_mask)
            return k, idx
    w = search_classes(n, world, dtype, search_mem_bytes, sym)
    try:
        won = None
        if kf is not None and k_search < n:
            # the next sizes by bands of prefix classes dealt over the ranks, while those are
            # fewer than the sharded fixed-pattern classes (ref15.search_past's order), then
            # every size by the latter
            for K, classes in ref15.search_bands(n, k_search, dtype, search_mem_bytes, sym, 1 << w):
                won = search_winner(search_class, n, 0, group, classes=classes, k_max=K)
                if won is not None:
                    break
        if won is None:
            won = search_winner(search_class, n, w, group)
    finally:
        if kf is not None:
            kf.close()
    return None if won is None else finish(*won)


def _tdev(group=None):
    import torch.distributed as dist
    return torch.device('cuda', torch.cuda.current_device()) if dist.get_backend(group) == 'nccl' else torch.device('cpu')


def rank_classes(w, rank, world):
    """The classes rank searches: c = rank, rank + world, ... of the 2^w, fewest fixed members
    first (ref15.class_order)."""
    from . import ref15
    return [c for c in ref15.class_order(w) if c % world == rank]


def search_winner(search_class, n, w, group=None, exhaustive=False, classes=None, k_max=None):
    """The cross-rank half of ``brute_force_search``: this rank searches its classes
    (``rank_classes``; or every world-th of ``classes``, e.g. ref15.prefix_classes' (n_fixed,
    mask) pairs) through ``search_class(n_fixed, c, k_max) -> (k, indices or None)``, keeping the
    smallest accepted size (up to ``k_max``) and, at it, the first subset in
    itertools.combinations order (ref15.class_search: not exhaustive, a class searches only the
    sizes that can still win on this rank); two all-reduces (MIN of the size, then MAX of the
    bit-reversed mask as two 32-bit halves) give every rank the global winner (k, indices), or
    None when no class accepted a subset."""
    import torch.distributed as dist

    from . import ref15
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    tdev = _tdev(group)
    mine = rank_classes(w, rank, world) if classes is None else list(classes)[rank::world]
    k_r, key_r = ref15.class_search(search_class, n, w, mine, exhaustive, k_max)
    if k_r is ref15.NO_SIZE:
        k_r = _NONE
    t = torch.tensor([k_r], dtype=torch.int64, device=tdev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    k_min = int(t.item())
    if k_min == _NONE:
        return None
    # keys are unsigned 64-bit: all-reduce them as two non-negative halves (high, then low)
    hi = torch.tensor([key_r >> 32 if k_r == k_min else -1], dtype=torch.int64, device=tdev)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    lo = torch.tensor([key_r & 0xFFFFFFFF if (k_r == k_min and key_r >> 32 == int(hi.item())) else -1],
                      dtype=torch.int64, device=tdev)
    dist.all_reduce(lo, op=dist.ReduceOp.MAX, group=group)
    mask = ref15.bitrev64((int(hi.item()) << 32) | int(lo.item()))
    return k_min, tuple(i for i in range(n) if (mask >> i) & 1)


def sum_counts(counts, group=None):
    """Element-wise sum over the ranks of a per-size count array (uint64 values < 2^63)."""
    import numpy as np
    import torch.distributed as dist
    t = torch.as_tensor(np.asarray(counts, dtype=np.int64), device=_tdev(group))
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return t.cpu().numpy()


def brute_force_search_ranks(events, start_idx=0, end_idx=None, R_threshold=None, initial_pt=None,
                             initial_state=None, max_combos_in_memory=1 << 22, dtype='f64', device=0, group=None,
                             first_valid=None, finish=None, consts=None):
    """run_brute_force_kalman_filter_no_sampling_min_usage sharded over the ranks of ``group``,
    one filter per subset: for k = 1..n, rank r scans combination ranks
    shard_range(C(n, k), r, world) on its GPU (kf_eval_combos), then an all-reduce MIN of the
    first acceptable rank (or "none") decides — the same winner as the single-GPU search (the
    first acceptable subset of the smallest size, in itertools.combinations order).  Every rank
    returns the reference's result dict (or None).  The per-subset cross-check of brute_force_search.

    ``first_valid(k, lo, hi)`` / ``finish(k, rank)`` replace the GPU evaluation (tests drive the
    reduction logic with the CPU oracle on gloo)."""
    import math

    import torch.distributed as dist

    from . import ref15
    if R_threshold is None:
        raise ValueError('R_threshold must be specified for brute force KF.')
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    st = ref15.brute_force_setup(events, start_idx, end_idx, initial_pt, initial_state, consts)
    if st is None:
        return None
    cand, xt, Pt, prev_time, target_end, ev, init = st
    n = len(cand)
    kf = None
    if first_valid is None:
        width = max(1, min(max_combos_in_memory, max(shard_range(math.comb(n, k), rank, world)[1]
                                                     for k in range(1, n + 1))))
        kf = ref15.BatchedKF('ref15', width, dtype, device=device, params=ref15._params(consts))

        def first_valid(k, lo, hi):
            return ref15.first_valid_rank(kf, ev, init, prev_time, target_end, k, lo, hi, R_threshold)
    if finish is None:
        def finish(k, r):
            return ref15.brute_force_result(cand, k, r, xt, Pt, prev_time, target_end, dtype, device, consts=consts)
    backend = dist.get_backend(group)
    tdev = torch.device('cuda', torch.cuda.current_device()) if backend == 'nccl' else torch.device('cpu')
    try:
        for k in range(1, n + 1):
            lo, cnt = shard_range(math.comb(n, k), rank, world)
            r = first_valid(k, lo, lo + cnt) if cnt else None
            t = torch.tensor([_NONE if r is None else int(r)], dtype=torch.int64, device=tdev)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
            best = int(t.item())
            if best != _NONE:
                return finish(k, best)
    finally:
        if kf is not None:
            kf.close()
    return None
