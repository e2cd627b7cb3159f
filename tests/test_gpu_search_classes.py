"""The class-decomposed brute-force search (kfmi.ref15.search_combos_classed) — needs an MI355X.

The reference's search (kf_workers.py:1218-1392) over n candidates takes every subset, 2^n - 1
of them; the reference's visualizing run brute-forces a window of n = 40
(kf_workers_visualizing.py:2293, 2340).  One kf_search_combos call holds its level buffers for
every size only up to n = 32 (the 2^28-parent cap and the 32 GiB budget), so a larger search runs
as 2^w classes — the subsets with one fixed intersection with candidates 0 .. w - 1 — one call
each, reduced to the reference's pick (smallest accepted size, then itertools order).

Checked here: at n = 25 and 28 the classes reproduce the whole search (every subset's score
through subset_max, winners and acceptance counts, exhaustive and not); at n = 40 the winner
equals one filter per subset (kf_eval_combos, first_valid_rank) at thresholds whose first
accepted size is 2 and is past the one-call search's sizes, and acceptance counts of sizes 1-4
equal the C oracle's (oracle/cpu_kf.c, one filter per subset); at n = 40, 48 and 64 the first
size past one call, searched by a band of prefix classes (ref15.search_past), gives one filter
per subset's winner.
"""
import math
from itertools import combinations

import numpy as np
import pytest
import torch

import bench
import kfmi
from kfmi import ref15
from oracle import ref_kf
from test_gpu_bench_parity import _combo_maxima

pytestmark = pytest.mark.gpu


def _thresholds(sm, q):
    """Thresholds just above the q-quantiles of the finite subset scores (a relative margin of
    1e-9 keeps every decision away from a score's last bits)."""
    vals = torch.sort(sm[torch.isfinite(sm)]).values
    return [float(vals[int(x * (len(vals) - 1))]) * (1 - 1e-9) + 1e-9 for x in q]


@pytest.mark.parametrize('n,ws,axis_sym', [(25, (1, 3, 6), 'auto'), (25, (4,), 'off'), (28, (3, 5), 'auto')])
def test_classed_search_equals_whole_search(n, ws, axis_sym):
    """Every class split gives the whole search's scores (subset_max, bit for bit), and at
    thresholds accepting nothing, 0.01 %, 2 % and half of the subsets its winner and acceptance
    counts, exhaustive and stopping at the first accepted size."""
    ev, init, _, t0, t_end = bench.bf_events(n)
    kf = kfmi.BatchedKF('ref15', 1, 'f64', options={'axis_sym': axis_sym})
    assert kf.search_plan(init, n)['sym'] == (axis_sym == 'auto')
    _, _, _, whole = kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True, subset_max=True)
    assert kf.search_info()['sym'] == (axis_sym == 'auto')
    thrs = [-1e30] + _thresholds(whole, (1e-4, 0.02, 0.5))
    for w in ws:
        k, idx, acc, sm = ref15.search_combos_classed(kf, ev, init, t0, t_end, -1e30, w, exhaustive=True,
                                                      subset_max=True)
        assert k == 0 and idx is None and not acc.any()
        assert torch.equal(sm.view(torch.int64), whole.view(torch.int64)), (n, w)
        del sm
        for thr in thrs:
            for exhaustive in (True, False):
                want = kf.search_combos(ev, init, t0, t_end, thr, exhaustive=exhaustive)
                got = ref15.search_combos_classed(kf, ev, init, t0, t_end, thr, w, exhaustive=exhaustive)
                assert got[:2] == want[:2], (n, w, thr, exhaustive, got[:2], want[:2])
                np.testing.assert_array_equal(got[2], want[2])
    kf.close()


def _n40_case():
    """The bench's 40 candidates (bf_events: 200 Hz IMU, a fix every 20th) with the target 5 s
    past the last one, so that each subset's score is its final predict's log-det, which falls
    with every update: the smallest score falls with the size well past the one-call sizes."""
    n = 40
    ev, init, Pw, t0, t_end = bench.bf_events(n)
    return n, ev, init, Pw, t0, t_end + 5.0


def _min_scores(kf, n, ev, init, t0, t_end, sizes):
    """Smallest per-subset score of each size (kf_eval_combos, one filter per subset)."""
    out = {}
    for k in sizes:
        total, best = math.comb(n, k), float('inf')
        for off in range(0, total, kf.batch):
            mx, _, _ = kf.eval_combos(ev, init, t0, t_end, k, combo_offset=off, logdets=False)
            best = min(best, float(mx[:min(kf.batch, total - off)].min()))
        out[k] = best
    return out


def test_n40_search_vs_per_subset():
    """The reference's n = 40 window: run_brute_force_kalman_filter_no_sampling_min_usage's
    winner (one call for sizes 1 .. k_search, then 256 classes) equals the first acceptable
    subset one filter per subset finds (first_valid_rank, kf_eval_combos over every size in
    combination order), at a threshold whose first accepted size is 2 and at one whose first
    accepted size is past k_search."""
    n, ev, init, Pw, t0, t_far = _n40_case()
    kfe = kfmi.BatchedKF('ref15', 1 << 22, 'f64')
    kfs = kfmi.BatchedKF('ref15', 1, 'f64')
    sym = kfs.search_plan(init, n)['sym']
    k_search = ref15.search_levels(n, 'f64', 32 << 30, sym)
    assert sym and k_search == 10 and ref15.search_class_width(n, 'f64', 32 << 30, sym) == 8
    mins = _min_scores(kfe, n, ev, init, t0, t_far, range(1, k_search + 1))
    print('n = 40 smallest score per size:', {k: round(v, 6) for k, v in mins.items()})
    L0 = float(np.linalg.slogdet(Pw)[1])
    m_lo = min(mins.values())
    assert mins[2] < mins[1] and m_lo > L0
    thr_lo = m_lo - 1e-9 * abs(m_lo)      # nothing of sizes 1 .. k_search scores below
    thr_2 = (mins[1] + mins[2]) / 2        # pairs first
    # the driver's steps on these arrays (its window's target is the last event's time, so the
    # far target is set here): sizes 1 .. k_search in one call, then every size by class
    w = ref15.search_class_width(n, 'f64', 32 << 30, sym)
    for thr, want_min in ((thr_2, 2), (thr_lo, k_search + 1)):
        k, idx, _, _ = kfs.search_combos(ev, init, t0, t_far, thr, k_max=k_search)
        if not k:
            k, idx, _, _ = ref15.search_combos_classed(kfs, ev, init, t0, t_far, thr, w)
        assert k == want_min if want_min == 2 else want_min <= k <= want_min + 1, (thr, k)
        r = None
        for kk in range(1, k + 1):
            r = ref15.first_valid_rank(kfe, ev, init, t0, t_far, kk, 0, math.comb(n, kk), thr)
            if r is not None:
                break
        assert r is not None and kk == k, (thr, kk, k)
        assert tuple(ref15.unrank_combination(n, k, r)) == idx, (thr, k, r, idx)
        # and against the C oracle (one filter per subset, the reference's dense step): the winner
        # scores below the threshold, and sampled subsets before it — 4096 of every smaller size
        # and 4096 of its size earlier in itertools order (ranks below r) — do not
        rng = np.random.default_rng(k)
        assert _combo_maxima(ev, Pw, t0, t_far, np.array([idx]))[0] < thr
        for kk2 in range(1, k + 1):
            hi = r if kk2 == k else math.comb(n, kk2)
            ranks = np.unique(rng.integers(0, hi, 4096)) if hi > 4096 else np.arange(hi)
            if not len(ranks):
                continue
            combos = np.array([ref15.unrank_combination(n, kk2, int(x)) for x in ranks])
            assert (_combo_maxima(ev, Pw, t0, t_far, combos) >= thr).all(), (thr, kk2)
        print(f'n = 40, threshold {thr:.9f}: winner of size {k}: {idx}')
    kfe.close()
    kfs.close()


@pytest.mark.parametrize('n', [40, 48, 64])
def test_sizes_past_one_call_by_prefix_bands(n):
    """Windows past one call's sizes up to kf_search_combos' limit of 64 candidates: with sizes
    1 .. k_search accepting nothing, the driver's next sizes run as bands of prefix classes
    (ref15.search_past: n = 40 size 11 in 40 classes, n = 48 size 9 in 48, n = 64 size 8 in 64,
    where the fixed-pattern classes that fit every size would be 256, 65,536 and 2^32).  The winner
    equals one filter per subset (first_valid_rank in combination order) and the C oracle's
    scores: the winner below the threshold, sampled subsets before it not."""
    ev, init, Pw, t0, t_end = bench.bf_events(n)
    t_far = t_end + 5.0
    kfe = kfmi.BatchedKF('ref15', 1 << 22, 'f64')
    kfs = kfmi.BatchedKF('ref15', 1, 'f64')
    sym = kfs.search_plan(init, n)['sym']
    k_lo = ref15.search_levels(n, 'f64', 32 << 30, sym)
    w = ref15.search_class_width(n, 'f64', 32 << 30, sym)
    K1, band1 = next(iter(ref15.search_bands(n, k_lo, 'f64', 32 << 30, sym, 1 << w)))
    assert sym and K1 == k_lo + 1 and len(band1) == n and len(band1) < 1 << w
    mins = _min_scores(kfe, n, ev, init, t0, t_far, range(1, k_lo + 1))
    m_lo = min(mins.values())
    thr = m_lo - 1e-9 * abs(m_lo)          # nothing of sizes 1 .. k_search scores below
    assert kfs.search_combos(ev, init, t0, t_far, thr, k_max=k_lo)[0] == 0
    calls = []

    def search_class(nf, c, k_max):
        calls.append((nf, c, k_max))
        k, idx, _, _ = kfs.search_combos(ev, init, t0, t_far, thr, k_max=k_max, n_fixed=nf, fixed_mask=c)
        return k, idx
    k, key = ref15.search_past(search_class, n, k_lo, w, 'f64', 32 << 30, sym)
    assert k is not ref15.NO_SIZE and k_lo < k <= k_lo + 2, k
    idx = tuple(i for i in range(n) if (ref15.bitrev64(key) >> i) & 1)
    assert all(nf < n and c >> nf == 0 for nf, c, _ in calls)
    if k == K1:
        assert len(calls) <= len(band1)    # the first band decided it
    r = ref15.first_valid_rank(kfe, ev, init, t0, t_far, k, 0, math.comb(n, k), thr)
    if k > K1:
        assert ref15.first_valid_rank(kfe, ev, init, t0, t_far, K1, 0, math.comb(n, K1), thr) is None
    assert r is not None and tuple(ref15.unrank_combination(n, k, r)) == idx, (k, r, idx)
    rng = np.random.default_rng(n)
    assert _combo_maxima(ev, Pw, t0, t_far, np.array([idx]))[0] < thr
    for kk in range(1, k + 1):
        hi = r if kk == k else math.comb(n, kk)
        ranks = np.unique(rng.integers(0, hi, 2048)) if hi > 2048 else np.arange(hi)
        if len(ranks):
            combos = np.array([ref15.unrank_combination(n, kk, int(x)) for x in ranks])
            assert (_combo_maxima(ev, Pw, t0, t_far, combos) >= thr).all(), kk
    print(f'n = {n}: sizes 1 .. {k_lo} in one call, winner of size {k} {idx} from {len(calls)} prefix classes')
    kfe.close()
    kfs.close()


def test_n40_counts_sizes_1_to_4_vs_oracle():
    """Acceptance counts of sizes 1-4 summed over the 256 classes of the n = 40 search (size cap
    4, exhaustive) equal the C oracle's per-subset scores' (every subset of sizes 1-4, 102,090),
    at thresholds through the size-1, size-2 and size-3 scores; the winner is the oracle's first."""
    n, ev, init, Pw, t0, t_far = _n40_case()
    kfs = kfmi.BatchedKF('ref15', 1, 'f64')
    w = ref15.search_class_width(n, 'f64', 32 << 30, kfs.search_plan(init, n)['sym'])
    small = {k: np.array(list(combinations(range(n), k))) for k in range(1, 5)}
    maxima = {k: _combo_maxima(ev, Pw, t0, t_far, c) for k, c in small.items()}
    for thr in (float(np.median(maxima[1])), float(np.quantile(maxima[2], 0.1)), float(np.median(maxima[3]))):
        want = [0] + [int((maxima[k] < thr).sum()) for k in range(1, 5)]
        assert sum(want) > 0
        k, idx, acc, _ = ref15.search_combos_classed(kfs, ev, init, t0, t_far, thr, w, exhaustive=True, k_max=4)
        assert [int(v) for v in acc[:5]] == want and not acc[5:].any(), (thr, list(acc[:5]), want)
        first = next(kk for kk in range(1, 5) if want[kk])
        assert k == first and idx == tuple(small[first][np.argmax(maxima[first] < thr)])
        # and not exhaustive: the same winner, counts up to it
        k2, idx2, acc2, _ = ref15.search_combos_classed(kfs, ev, init, t0, t_far, thr, w)
        assert (k2, idx2) == (k, idx) and [int(v) for v in acc2[:k + 1]] == want[:k + 1] and not acc2[k + 1:].any()
    kfs.close()


def test_n40_driver_winner_vs_reference_search():
    """run_brute_force_kalman_filter_no_sampling_min_usage over a 40-event window whose winner
    has two events equals the NumPy restatement of the reference's search (kf_workers.py:
    1218-1392, sizes 1 and 2 through the reference's own loop), records and all."""
    n = 40
    ev, init, Pw, t0, _ = bench.bf_events(n)
    t_last = float(ev[-1, 0])
    events = [(i, 'GPS', ev[i, 0], {'easting': ev[i, 2], 'northing': ev[i, 3], 'altitude': ev[i, 4]})
              if ev[i, 1] == 0 else (i, 'IMU', ev[i, 0], ['t', *ev[i, 2:]]) for i in range(n)]
    state0 = (t0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
    s1 = np.sort(_combo_maxima(ev, Pw, t0, t_last, np.arange(n)[:, None]))
    L0 = float(np.linalg.slogdet(Pw)[1])
    thr = (L0 + s1[0]) / 2
    ref = ref_kf.run_brute_force(events, 0, n, thr, Pw, state0)
    got = ref15.run_brute_force_kalman_filter_no_sampling_min_usage(events, 0, n, R_threshold=thr, initial_pt=Pw,
                                                                     initial_state=state0)
    sel = [e[0] for e in ref['selected_sensors']]
    assert len(sel) == 2 and [e[0] for e in got['selected_sensors']] == sel
    for key in ('log_determinants', 'final_state', 'trajectory'):
        a, b = np.asarray(got[key], np.float64), np.asarray(ref[key], np.float64)
        assert a.shape == b.shape and np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0)) <= 1e-6, key


@pytest.mark.parametrize('n,dtype', [(25, 'f64'), (28, 'f64'), (25, 'f32')])
def test_pair_launches_equal_single_levels(n, dtype):
    """KF_OPT_SEARCH_PAIR (auto; 2: every parent-major level paired parent-major; 3: every level
    child-major): two levels per launch (the first kept in LDS, never stored) give every subset's score bit for bit as one level per launch, and the same winners
    and acceptance counts, whole and by class, exhaustive and not; the launches are the Python
    mirror's (ref15.search_plan), and a pair launch stores half the level nodes."""
    ev, init, _, t0, t_end = bench.bf_events(n)
    res = {}
    for pair in ('auto', 'all', 'cm', 'off'):
        kf = kfmi.BatchedKF('ref15', 1, dtype, options={'search_pair': pair})
        _, _, _, sm = kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True, subset_max=True)
        info = kf.search_info()
        assert info['sym']
        plan, stored = ref15.search_plan(n, sym=True, pair=pair)
        assert info['level_launches'] + (1 if info['head_sizes'] else 0) == len(plan)
        out = [sm.cpu()]
        thrs = _thresholds(sm, (1e-4, 0.02, 0.5))
        for thr in thrs:
            for exhaustive in (True, False):
                out.append(kf.search_combos(ev, init, t0, t_end, thr, exhaustive=exhaustive)[:3])
                out.append(ref15.search_combos_classed(kf, ev, init, t0, t_end, thr, 3, exhaustive=exhaustive)[:3])
        res[pair] = (out, plan, stored)
        kf.close()
    key = torch.int64 if dtype == 'f64' else torch.int32
    b = res['off'][0]
    nodes = lambda st: sum(math.comb(n - 2, k) for k in st)  # noqa: E731
    for pair, kind in (('auto', 'pair'), ('all', 'pair'), ('cm', 'pair_cm')):
        a = res[pair][0]
        assert torch.equal(a[0].view(key), b[0].view(key)), pair
        for x, y in zip(a[1:], b[1:]):
            assert x[:2] == y[:2], pair
            np.testing.assert_array_equal(x[2], y[2])
        if pair == 'auto' and n < 28:  # no level of 2^22 parents: auto runs one level per launch
            assert res[pair][1] == res['off'][1]
            continue
        assert any(kd == kind for kd, _ in res[pair][1]), pair
        assert nodes(res[pair][2]) < 0.6 * nodes(res['off'][2]), pair


@pytest.mark.parametrize('case', ['golden_every_chain', 'custom_sym', 'custom_asym_f32'])
def test_classed_search_other_chains_and_constants(golden_dir, case):
    """The class split over the reference's own log (candidates out of time order, so negative
    dt skips) with every chain, and over caller constants (class_args) axis-symmetric and not, f64
    and f32: every subset's score bitwise the whole search's, and the whole search's winners and
    counts at three thresholds, exhaustive and not — the pair launches included where they run."""
    from test_gpu_ref15 import _search_case, _symmetric_consts
    n = 24
    if case == 'golden_every_chain':
        _, ev, init, t0, t_end = _search_case(golden_dir, n)
        dtype, params, opts = 'f64', None, {'axis_sym': 'off'}
    else:
        ev, init, _, t0, t_end = bench.bf_events(n)
        c = _symmetric_consts(11)
        if case == 'custom_asym_f32':
            q = c.q.copy()
            q[13] *= 1.5   # the y axis's acceleration noise: every chain
            c = ref15.ModelConsts('ref15', q=q, r_imu=c.r_imu, r_gps=c.r_gps, p0=c.p0)
        dtype, params, opts = ('f32' if case.endswith('f32') else 'f64'), c.params(), {'search_pair': 'all'}
    kf = kfmi.BatchedKF('ref15', 1, dtype, params=params, options=opts)
    _, _, _, whole = kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True, subset_max=True)
    assert kf.search_info()['sym'] == (case == 'custom_sym')
    key = torch.int64 if dtype == 'f64' else torch.int32
    for w in (2, 5):
        _, _, _, sm = ref15.search_combos_classed(kf, ev, init, t0, t_end, -1e30, w, exhaustive=True, subset_max=True)
        assert torch.equal(sm.view(key), whole.view(key)), (case, w)
        del sm
        for thr in _thresholds(whole, (1e-4, 0.02, 0.5)):
            for exhaustive in (True, False):
                want = kf.search_combos(ev, init, t0, t_end, thr, exhaustive=exhaustive)
                got = ref15.search_combos_classed(kf, ev, init, t0, t_end, thr, w, exhaustive=exhaustive)
                assert got[:2] == want[:2], (case, w, thr, exhaustive)
                np.testing.assert_array_equal(got[2], want[2])
    kf.close()
