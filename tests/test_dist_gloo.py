"""Multi-process (world_size 2, 3 and 8, gloo, CPU) coverage of the filter-sharding path used by
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


# even and uneven shards at world 2; world 8 (config 4's rank count) with uneven shards and
# one rank holding no filter
@pytest.mark.parametrize('world,total', [(2, 10), (2, 9), (8, 21), (8, 7)])
def test_gloo_shard_and_gather(world, total):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, 6, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert [p.exitcode for p in procs] == [0] * world
    err, slow = q.get(timeout=10)
    assert err < 1e-12
    assert slow == [world - 0.5, 0.0]


def _traj_worker(rank, world, port, total, T, every, out_q):
    """gather_run_outputs: final x, last log-det and the trajectory decimated every `every`
    steps, one all-gather, against the unsharded oracle run."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(321)
        model = ref_kf.CV3
        x0 = rng.normal(0, 100, (total, 6))
        u = rng.normal(0, 0.3, (T, 3, total))
        z = rng.normal(0, 30, (T, 3, total))
        off, cnt = kdist.shard_range(total, rank, world)
        sl = slice(off, off + cnt)
        tr, ld, x, _ = ref_kf.run_batch(model, x0[sl], model.P0(), np.full(T, 0.1), u[:, :, sl], z[:, :, sl], 1)
        res = kdist.gather_run_outputs(torch.from_numpy(np.ascontiguousarray(x.T)), torch.from_numpy(ld[-1].copy()),
                                       torch.from_numpy(tr), every, total)
        if rank == 0:
            trg, ldg, xg, _ = ref_kf.run_batch(model, x0, model.P0(), np.full(T, 0.1), u, z, 1)
            steps = kdist.decimated_steps(T, every)
            errs = [np.abs(res['x'].numpy() - xg.T).max(), np.abs(res['logdet'].numpy() - ldg[-1]).max()]
            if steps:
                errs.append(np.abs(res['traj'].numpy() - trg[steps]).max())
            else:
                errs.append(0.0 if res['traj'] is None else np.inf)
            out_q.put((errs, res['rows'], len(steps)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world,total,T,every', [(2, 11, 8, 4), (3, 10, 9, 4), (3, 7, 6, 0), (2, 5, 5, 1)])
def test_gloo_gather_decimated_trajectory(world, total, T, every):
    """Uneven shards (11 over 2, 10 and 7 over 3), T not a multiple of every, no trajectory."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_traj_worker, args=(r, world, port, total, T, every, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert [p.exitcode for p in procs] == [0] * world
    errs, rows, nsteps = q.get(timeout=10)
    assert nsteps == len(range(every - 1, T, every)) if every else nsteps == 0
    assert rows == 6 + 1 + 6 * nsteps
    assert max(errs) == 0.0, errs  # the gather moves bits; the shards ran the same arithmetic


def test_decimated_steps():
    assert kdist.decimated_steps(256, 16) == list(range(15, 256, 16))
    assert kdist.decimated_steps(10, 4) == [3, 7]
    assert kdist.decimated_steps(10, 0) == []
    assert kdist.decimated_steps(3, 1) == [0, 1, 2]


def _bf_worker(rank, world, port, golden, thr, out_q):
    """kfmi.dist.brute_force_search on gloo with the oracle as the per-rank evaluator."""
    import sys
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    sys.path.insert(0, os.path.dirname(__file__))
    from golden_events import unpack_events
    from kfmi import ref15
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        g = np.load(golden)
        events = unpack_events(g)
        s, e = int(g['start']), int(g['end'])
        thr = float(g['threshold']) if thr is None else thr
        cand, xt, Pt, prev, end, _, _ = ref15.brute_force_setup(events, s, e, g['init_P'], tuple(g['init_state']))
        n = len(cand)
        scanned = []

        def first_valid(k, lo, hi):
            scanned.append((k, lo, hi))
            for r in range(lo, hi):
                combo = tuple(cand[i] for i in ref15.unrank_combination(n, k, r))
                res = ref_kf.evaluate_combo_chunk([combo], xt, Pt, prev, end)[0]
                if max(res[5]) < thr:
                    return r
            return None

        def finish(k, r):
            return ref15.unrank_combination(n, k, r)

        out = kdist.brute_force_search_ranks(events, s, e, R_threshold=thr, initial_pt=g['init_P'],
                                             initial_state=tuple(g['init_state']), first_valid=first_valid,
                                             finish=finish)
        out_q.put((rank, out, scanned, n))
    finally:
        dist.destroy_process_group()


def _bf_class_worker(rank, world, port, golden, thr, out_q):
    """kfmi.dist.brute_force_search (shared-prefix classes) on gloo with the oracle as the
    per-class search."""
    import sys
    from itertools import combinations
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    sys.path.insert(0, os.path.dirname(__file__))
    from golden_events import unpack_events
    from kfmi import ref15
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        g = np.load(golden)
        events = unpack_events(g)
        s, e = int(g['start']), int(g['end'])
        thr = float(g['threshold']) if thr is None else thr
        cand, xt, Pt, prev, end, _, _ = ref15.brute_force_setup(events, s, e, g['init_P'], tuple(g['init_state']))
        n = len(cand)
        searched = []

        def search_class(w, c, k_max=None):
            """first acceptable subset (smallest size, then itertools order) among those whose
            intersection with candidates 0..w-1 is the bit pattern c"""
            searched.append(c)
            fixed = [i for i in range(w) if (c >> i) & 1]
            subsets = [tuple(fixed) + t for kk in range(n - w + 1) for t in combinations(range(w, n), kk)]
            subsets = sorted((x for x in subsets if x), key=lambda x: (len(x), x))
            for x in subsets:
                res = ref_kf.evaluate_combo_chunk([tuple(cand[i] for i in x)], xt, Pt, prev, end)[0]
                if max(res[5]) < thr:
                    return len(x), x
            return 0, None

        def finish(k, idx):
            return list(idx)

        out = kdist.brute_force_search(events, s, e, R_threshold=thr, initial_pt=g['init_P'],
                                       initial_state=tuple(g['init_state']), search_class=search_class,
                                       finish=finish)
        out_q.put((rank, out, searched, n))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
@pytest.mark.parametrize('thr', [None, -27.0, -1e9])  # the reference's threshold; a looser one; nothing
def test_gloo_class_sharded_brute_force_search(golden_dir, thr, world):
    """Every rank returns the winner of the unsharded search (the first acceptable subset of the
    smallest size in itertools order), and the ranks' classes partition the 2^w classes."""
    from itertools import combinations
    from kfmi import ref15
    from golden_events import unpack_events
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    golden = os.path.join(golden_dir, 'ref15_bruteforce.npz')
    procs = [ctx.Process(target=_bf_class_worker, args=(r, world, port, golden, thr, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert [p.exitcode for p in procs] == [0] * world
    res = dict((r, (out, sc, n)) for r, out, sc, n in (q.get(timeout=10) for _ in range(world)))
    g = np.load(golden)
    n = res[0][2]
    w = kdist.search_classes(n, world)
    searched = sorted(c for r in res for c in res[r][1])
    assert len(set(searched)) == len(searched) and set(searched) <= set(range(1 << w))
    if thr is None:
        want = list(g['selected'])
    else:  # the unsharded search with the oracle
        events = unpack_events(g)
        cand, xt, Pt, prev, end, _, _ = ref15.brute_force_setup(events, int(g['start']), int(g['end']), g['init_P'],
                                                                tuple(g['init_state']))
        want = None
        for k in range(1, n + 1):
            for x in combinations(range(n), k):
                res_x = ref_kf.evaluate_combo_chunk([tuple(cand[i] for i in x)], xt, Pt, prev, end)[0]
                if max(res_x[5]) < thr:
                    want = list(x)
                    break
            if want:
                break
    assert all(res[r][0] == want for r in res)
    # a class goes unsearched only when its fixed members alone outnumber a size already accepted
    skipped = set(range(1 << w)) - set(searched)
    assert all(bin(c).count('1') > len(want) for c in skipped) if want else not skipped


@pytest.mark.parametrize('thr', [None, -1e9])  # the reference's threshold and winner; nothing acceptable
def test_gloo_world2_brute_force_search(golden_dir, thr):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    golden = os.path.join(golden_dir, 'ref15_bruteforce.npz')
    procs = [ctx.Process(target=_bf_worker, args=(r, 2, port, golden, thr, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    assert [p.exitcode for p in procs] == [0, 0]
    res = dict((r, (out, sc, n)) for r, out, sc, n in (q.get(timeout=10), q.get(timeout=10)))
    g = np.load(golden)
    want = list(g['selected']) if thr is None else None
    assert res[0][0] == want and res[1][0] == want          # every rank returns the same winner
    n = res[0][2]
    from math import comb
    for k in range(1, (len(want) if want else n) + 1):      # the two ranks split each size exactly
        spans = sorted((lo, hi) for r in (0, 1) for (kk, lo, hi) in res[r][1] if kk == k)
        assert spans[0][0] == 0 and spans[-1][1] == comb(n, k)      # (a rank with no ranks skips)
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def _winner_worker(rank, world, port, n, w, exhaustive, out_q):
    """kfmi.dist.search_winner / sum_counts on synthetic class results: each class reports the
    smallest size (up to the k_max it is given) at which it accepts and its first accepted subset
    (itertools order), from one random acceptance table shared by every rank; the reduction must
    give the global winner, and the searched sizes must stop where they can no longer win."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from itertools import combinations
        rng = np.random.default_rng(77)
        accept = {}
        for k in range(1, n + 1):
            for c in combinations(range(n), k):
                accept[c] = rng.random() < 0.02 * k
        counts = np.zeros(n + 1, np.int64)
        calls = []

        def search_class(n_fixed, fixed_mask, k_max=None):
            calls.append((fixed_mask, k_max))
            best = None
            for k in range(1, (n if k_max is None else k_max) + 1):
                for c in combinations(range(n), k):
                    if sum(1 << i for i in c if i < n_fixed) != fixed_mask or not accept[c]:
                        continue
                    counts[k] += 1
                    if best is None:
                        best = (k, c)
            return best if best else (0, None)
        won = kdist.search_winner(search_class, n, w, exhaustive=exhaustive)
        total = kdist.sum_counts(counts)
        k1 = next(k for k in range(1, n + 1) if any(accept[c] for c in combinations(range(n), k)))
        c1 = next(c for c in combinations(range(n), k1) if accept[c])
        # not exhaustive, no class searched a size that could no longer win on this rank
        assert exhaustive or all(k_max == n or k_max >= k1 for _, k_max in calls)
        if rank == 0:
            want = [0] + [sum(accept[c] for c in combinations(range(n), k)) for k in range(1, n + 1)]
            out_q.put((won, (k1, c1), list(total), want, len(calls)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('exhaustive', [True, False])
@pytest.mark.parametrize('world', [2, 3, 8])
def test_gloo_search_winner_and_counts(world, exhaustive):
    """The cross-rank half of the sharded search (the bench's bf rows at N > 1 time it):
    classes dealt round-robin over the ranks, MIN of the first accepted size, MAX of the
    bit-reversed mask — the same winner as one rank over every class; exhaustive, the counts
    summed over the ranks are every size's."""
    n = 9
    w = kdist.search_classes(n, world)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_winner_worker, args=(r, world, port, n, w, exhaustive, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert [p.exitcode for p in procs] == [0] * world
    won, want_won, total, want, _ = q.get(timeout=10)
    assert won == want_won
    if exhaustive:
        assert total == want


def _band_worker(rank, world, port, n, k_done, mem, out_q):
    """The sharded search past its one-call sizes (kfmi.dist.brute_force_search on the GPU):
    bands of prefix classes (ref15.search_bands) dealt over the ranks through search_winner,
    then the fixed-pattern classes — on a random acceptance table shared by every rank that
    accepts nothing up to k_done."""
    from itertools import combinations

    from kfmi import ref15
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        res = []
        for trial, rate in enumerate((0.2, 0.01, 0.0005)):
            rng = np.random.default_rng(100 + trial)
            order = [(k, x) for k in range(k_done + 1, n + 1) for x in combinations(range(n), k)
                     if rng.random() < rate * k]

            def search_class(nf, c, k_max):
                assert bin(c).count('1') < k_max <= n and c >> nf == 0
                return next(((k, x) for k, x in order if k <= k_max and sum(1 << i for i in x if i < nf) == c),
                            (0, None))
            w = kdist.search_classes(n, world, 'f64', mem, True)
            won = None
            for K, classes in ref15.search_bands(n, k_done, 'f64', mem, True, 1 << w):
                won = kdist.search_winner(search_class, n, 0, classes=classes, k_max=K)
                if won is not None:
                    break
            if won is None:
                won = kdist.search_winner(search_class, n, w)
            res.append((won, order[0] if order else None))
        if rank == 0:
            out_q.put(res)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_gloo_banded_search_winner(world):
    """Bands of prefix classes over the ranks give the reference's pick (the smallest accepted
    size past the one-call sizes, then the first subset in itertools order), as one rank does."""
    from kfmi import ref15
    n, k_done = 15, 2
    mem = next(m for m in range(8192, 1 << 30, 4096) if ref15.search_levels(n, 'f64', m, True) == k_done)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_band_worker, args=(r, world, port, n, k_done, mem, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
    assert [p.exitcode for p in procs] == [0] * world
    for won, want in q.get(timeout=10):
        assert won == want
