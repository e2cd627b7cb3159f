"""Multi-process (world_size 2, gloo, CPU) coverage of the filter-sharding path used by
bench.py on N GPUs: shard ranges, per-rank work on its own slice, and the final
all-gather reassembly.  The per-shard compute here is the CPU oracle (test
infrastructure); on the GPU box the same kfmi.dist code moves RCCL tensors."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kfmi import dist as kdist
from oracle import ref_kf


def test_shard_ranges_cover_exactly():
    for total in (0, 1, 7, 64, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            got = [kdist.shard_range(total, r, world) for r in range(world)]
            assert sum(c for _, c in got) == total
            off = 0
            for o, c in got:
                assert o == off
                off += c
            assert max(c for _, c in got) - min(c for _, c in got) <= 1
    with pytest.raises(ValueError):
        kdist.shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, T, out_q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(123)  # same global inputs on every rank
        model = ref_kf.CV3
        x0 = rng.normal(0, 100, (total, 6))
        u = rng.normal(0, 0.3, (T, 3, total))
        z = rng.normal(0, 30, (T, 3, total))
        off, cnt = kdist.shard_range(total, rank, world)
        sl = slice(off, off + cnt)
        tr, ld, x, _ = ref_kf.run_batch(model, x0[sl], model.P0(), np.full(T, 0.1), u[:, :, sl], z[:, :, sl], 1)
        local = torch.from_numpy(np.concatenate([x.T, ld[-1:]], axis=0))  # [n+1, cnt]
        full = kdist.gather_shards(local, total)
        slow = kdist.max_over_ranks([rank + 0.5, -rank], 'cpu')
        if rank == 0:
            trg, ldg, xg, _ = ref_kf.run_batch(model, x0, model.P0(), np.full(T, 0.1), u, z, 1)
            ref = np.concatenate([xg.T, ldg[-1:]], axis=0)
            out_q.put((np.abs(full.numpy() - ref).max(), slow))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('total', [10, 9])  # even and uneven shards
def test_gloo_world2_shard_and_gather(total):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, 6, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert [p.exitcode for p in procs] == [0, 0]
    err, slow = q.get(timeout=10)
    assert err < 1e-12
    assert slow == [1.5, 0.0]
