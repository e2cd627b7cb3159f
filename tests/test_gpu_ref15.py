"""The reference's 15-state model on the GPU (KF_MODEL_REF15) vs the reference's own outputs
(tests/golden/ref15_*.npz) and the CPU oracle — needs an MI355X.

Tolerance (north_star): 1e-6 relative for fp64 (states normalised by max(|x|, 1), logdets by
max(|logdet|, 1)); the engine solves by LDL^T where the reference uses np.linalg.inv, and forms
(I-KH)P per chain (P = KR for the IMU's H = I chains; Joseph for the fp32 GPS fix), so agreement
is ~1e-10, not bitwise.
"""
import math
import os
from itertools import combinations

import numpy as np
import pytest
import torch

import kfmi
from golden_events import unpack_events
from kfmi import ref15
from oracle import ref_kf

pytestmark = pytest.mark.gpu
TOL = 1e-6


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0))) if a.size else 0.0


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def test_run_kalman_filter_full_cold(golden_dir):
    g = _load(golden_dir, 'ref15_full.npz')
    events = unpack_events(g)
    st, ld, P, prev = ref15.run_kalman_filter_full(events, 0, len(events))
    assert np.array(st).shape == g['cold_states'].shape
    assert _rel(st, g['cold_states']) <= TOL
    assert _rel(ld, g['cold_logdets']) <= TOL
    assert _rel(P, g['cold_P']) <= TOL
    assert prev == float(g['cold_prev_time'])


def test_run_kalman_filter_full_warm(golden_dir):
    g = _load(golden_dir, 'ref15_full.npz')
    events = unpack_events(g)
    s0 = int(g['warm_start'])
    st, ld, P, _ = ref15.run_kalman_filter_full(events, s0, s0 + 60, initial_pt=g['warm_init_P'],
                                                initial_state=tuple(g['warm_init_state']))
    assert _rel(st, g['warm_states']) <= TOL
    assert _rel(ld, g['warm_logdets']) <= TOL
    assert _rel(P, g['warm_P']) <= TOL


def test_adaptive_threshold(golden_dir):
    g = _load(golden_dir, 'ref15_full.npz')
    events = unpack_events(g)
    st, ld, P, prev, times = ref15.run_adaptive_threshold_kalman_filter(
        events, 0, len(events), R_threshold=float(g['adapt_threshold']))
    np.testing.assert_array_equal(np.array(times), g['adapt_times'])
    assert _rel(st, g['adapt_states']) <= TOL
    assert _rel(ld, g['adapt_logdets']) <= TOL
    assert _rel(P, g['adapt_P']) <= TOL


def test_combo_chunk_worker(golden_dir):
    g = _load(golden_dir, 'ref15_combos.npz')
    cand = unpack_events(g)
    chunk = [tuple(cand[i] for i in row if i >= 0) for row in g['combo_idx']]
    res = ref15.evaluate_combo_chunk(chunk, g['x0'], g['P0'], float(g['prev_time']), float(g['target_end']))
    assert len(res) == len(chunk)
    assert [len(r[5]) for r in res] == list(np.diff(g['offsets']))
    assert _rel([v for r in res for v in r[5]], g['logdet_flat']) <= TOL
    assert _rel([v for r in res for v in r[1]], g['traj_flat']) <= TOL
    assert _rel([r[3] for r in res], g['x_final']) <= TOL
    assert all(r[0] == 0 and r[4] is None and r[6] == len(r[2]) for r in res)


@pytest.mark.parametrize('mem', [32 << 30, 0, 200_000])
def test_brute_force_search(golden_dir, mem):
    """The reference's search result; mem = level-buffer budget of the shared-prefix search (0:
    every size one filter per subset; 200 kB: the first sizes by the search, the rest per subset)."""
    g = _load(golden_dir, 'ref15_bruteforce.npz')
    events = unpack_events(g)
    s, e = int(g['start']), int(g['end'])
    out = ref15.run_brute_force_kalman_filter_no_sampling_min_usage(
        events, s, e, R_threshold=float(g['threshold']), initial_pt=g['init_P'],
        initial_state=tuple(g['init_state']), search_mem_bytes=mem)
    cand = events[s:e]
    assert [cand.index(ev) for ev in out['selected_sensors']] == list(g['selected'])
    assert out['num_measurements_used'] == len(g['selected'])
    assert _rel(out['log_determinants'], g['log_determinants']) <= TOL
    assert _rel(out['final_state'], g['final_state']) <= TOL
    assert _rel(out['trajectory'], g['trajectory']) <= TOL
    # a threshold no subset meets -> None (kf_workers.py:1391-1392)
    assert ref15.run_brute_force_kalman_filter_no_sampling_min_usage(
        events, s, e, R_threshold=-1e9, initial_pt=g['init_P'], initial_state=tuple(g['init_state']),
        search_mem_bytes=mem) is None


def _search_case(golden_dir, n, swap=True):
    """n candidates after a warm start on the golden log; with ``swap`` two candidates are
    out of time order, so some subsets meet a negative dt (skipped, kf_workers.py:38-40)."""
    g = _load(golden_dir, 'ref15_full.npz')
    events = unpack_events(g)
    s0 = 100
    st, ld, P, prev = ref_kf.run_kalman_filter_full(events, 0, s0)
    cand = list(events[s0:s0 + n])
    if swap:
        cand[3], cand[6] = cand[6], cand[3]
    xt = np.zeros(15)
    xt[0:6] = st[-1][1:7]
    target = max(c[2] for c in cand)
    ev = np.array([[t, 0 if s == 'GPS' else 1, *ref15.event_payload(s, d)] for (_, s, t, d) in cand])
    init = np.concatenate([xt, ref15.to_blocks(P)])
    return cand, ev, init, st[-1][0], target


@pytest.mark.parametrize('head', ['on', 'off'])
@pytest.mark.parametrize('kernel', ['cm', 'pm'])
@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_search_subset_max_equals_eval_combos(golden_dir, dtype, kernel, head):
    """kf_search_combos (one event step per subset, from the stored prefix) gives every subset the
    max log-det the per-subset kernel gives (same operations in the same order), with either
    search kernel (child-major / parent-major levels), with the first levels in the one-launch
    head (KF_OPT_SEARCH_HEAD) or level by level."""
    n = 12
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    kf = kfmi.BatchedKF('ref15', 1, dtype, options={'search_kernel': kernel, 'search_head': head})
    kfound, win, acc, sm = kf.search_combos(ev, init, t0, target, threshold=-1e30, exhaustive=True, subset_max=True)
    kf.close()
    assert kfound == 0 and win is None and int(acc.sum()) == 0
    sm = sm.double().cpu().numpy()
    assert np.isnan(sm[0])  # the empty subset is not evaluated
    worst, exact, total = 0.0, 0, 0
    for k in range(1, n + 1):
        combos = list(combinations(range(n), k))
        kc = kfmi.BatchedKF('ref15', len(combos), dtype)
        mx, _, _ = kc.eval_combos(ev, init, t0, target, k, logdets=False)
        mx = mx.double().cpu().numpy()
        kc.close()
        masks = np.array([sum(1 << i for i in c) for c in combos])
        got = sm[masks]
        assert np.isfinite(got).all() and np.isfinite(mx).all()
        worst = max(worst, float(np.max(np.abs(got - mx) / np.maximum(np.abs(mx), 1.0))))
        exact += int((got == mx).sum())
        total += len(combos)
    assert total == 2 ** n - 1
    assert worst <= (1e-12 if dtype == 'f64' else 1e-6), (worst, exact, total)


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_search_acceptance_on_determinants_is_the_logs(golden_dir, dtype):
    """Without subset_max the search tests max(log_det) < R_threshold on determinants (a band
    around exp(threshold), the log taken only inside it).  At thresholds equal to subsets' own
    max log-dets, one ulp either side of them, and far outside every max, the per-size
    acceptance counts and the winner equal the ones the logs give (counted on the host from the
    same search's subset_max)."""
    n = 12
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    kf = kfmi.BatchedKF('ref15', 1, dtype)
    _, _, _, sm = kf.search_combos(ev, init, t0, target, -1e30, exhaustive=True, subset_max=True)
    sm = sm.cpu().numpy()
    size = np.array([bin(m).count('1') for m in range(1 << n)])
    vals = np.sort(sm[np.isfinite(sm)])
    npt = np.float64 if dtype == 'f64' else np.float32
    picks = [vals[0], vals[len(vals) // 3], vals[len(vals) // 2], vals[-1]]
    thresholds = [float(np.nextafter(npt(v), npt(d))) for v in picks for d in (-np.inf, np.inf)]
    thresholds += [float(v) for v in picks] + [float(vals[0]) - 50.0, float(vals[-1]) + 50.0, 2e5, -2e5]
    for thr in thresholds:
        k, win, acc, _ = kf.search_combos(ev, init, t0, target, thr, exhaustive=True)
        ok = sm < npt(thr)           # NaN never passes
        want = [int(np.sum(ok & (size == s))) for s in range(n + 1)]
        assert [int(a) for a in acc] == want, thr
        first = next((s for s in range(1, n + 1) if want[s]), 0)
        assert k == first, thr
        if first:
            masks = [m for m in range(1 << n) if size[m] == first and ok[m]]
            lex = min(tuple(i for i in range(n) if (m >> i) & 1) for m in masks)
            assert win == lex, thr
    kf.close()


def test_combo_inputs_reused_and_refreshed(golden_dir):
    """The handle keeps the last uploaded candidates and root on the device: a call with other
    inputs uploads them, a call with the same ones reuses them, also from another stream (which
    then waits for that upload), and kf_eval_combos shares the workspace.  Every result equals a
    fresh handle's, bit for bit."""
    n = 10
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    ev2 = ev.copy()
    ev2[[2, 5]] = ev2[[5, 2]]  # two candidates out of time order: other subsets skip a negative dt
    init2 = init.copy()
    init2[15] *= 1.5  # another root covariance

    def search(kf, e, i):
        _, _, _, sm = kf.search_combos(e, i, t0, target, threshold=-1e30, exhaustive=True, subset_max=True)
        return sm.cpu().numpy()

    def evals(kf, e, i):
        return kf.eval_combos(e, i, t0, target, 3, logdets=False)[0].cpu().numpy()

    fresh = {}
    for key, (e, i) in {'a': (ev, init), 'b': (ev2, init), 'c': (ev, init2)}.items():
        kf = kfmi.BatchedKF('ref15', 1, 'f64')
        fresh[key] = search(kf, e, i)
        kf.close()
    assert not np.array_equal(fresh['a'][1:], fresh['b'][1:]) and not np.array_equal(fresh['a'][1:], fresh['c'][1:])
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    for key, (e, i) in (('a', (ev, init)), ('a', (ev, init)), ('b', (ev2, init)), ('c', (ev, init2)), ('a', (ev, init))):
        np.testing.assert_array_equal(search(kf, e, i), fresh[key], err_msg=key)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        got = search(kf, ev, init)
    np.testing.assert_array_equal(got, fresh['a'])
    kf.close()
    # kf_eval_combos over the same workspace, interleaved with searches
    kc = kfmi.BatchedKF('ref15', math.comb(n, 3), 'f64')
    e_a, e_b = evals(kc, ev, init), evals(kc, ev2, init)
    np.testing.assert_array_equal(evals(kc, ev, init), e_a)
    kc.close()
    kc = kfmi.BatchedKF('ref15', math.comb(n, 3), 'f64')
    np.testing.assert_array_equal(evals(kc, ev2, init), e_b)
    kc.close()


@pytest.mark.parametrize('head', ['on', 'off'])
@pytest.mark.parametrize('kernel', ['cm', 'pm'])
@pytest.mark.parametrize('n,k_max', [(1, 1), (2, 2), (3, 3), (4, 4), (5, 5), (9, 3), (9, 8), (9, 9)])
def test_search_small_and_cut_levels(golden_dir, n, k_max, kernel, head):
    """Edge cases of the stored levels: with n <= 3 some levels have no stored parents (scored
    whole by the previous launch's tail); with k_max < n no subset larger than k_max is scored
    (the tail stops at k_max).  Every subset up to k_max gets the per-subset kernel's score."""
    cand, ev, init, t0, target = _search_case(golden_dir, n, swap=n > 6)
    kf = kfmi.BatchedKF('ref15', 1, 'f64', options={'search_kernel': kernel, 'search_head': head})
    kfound, win, acc, sm = kf.search_combos(ev, init, t0, target, threshold=-1e30, k_max=k_max, exhaustive=True,
                                            subset_max=True)
    kf.close()
    assert kfound == 0 and win is None and int(acc.sum()) == 0
    sm = sm.cpu().numpy()
    sizes = np.array([bin(m).count('1') for m in range(1 << n)])
    assert np.isnan(sm[sizes > k_max]).all() and np.isnan(sm[0])
    for k in range(1, k_max + 1):
        combos = list(combinations(range(n), k))
        kc = kfmi.BatchedKF('ref15', len(combos), 'f64')
        mx, _, _ = kc.eval_combos(ev, init, t0, target, k, logdets=False)
        mx = mx.cpu().numpy()
        kc.close()
        got = sm[np.array([sum(1 << i for i in c) for c in combos])]
        assert np.max(np.abs(got - mx) / np.maximum(np.abs(mx), 1.0)) <= 1e-12, k


@pytest.mark.parametrize('head', ['on', 'off'])
@pytest.mark.parametrize('kernel', ['cm', 'pm'])
@pytest.mark.parametrize('q', [0.0, 0.01, 0.3, 0.9])
def test_search_winner_matches_per_subset_search(golden_dir, q, kernel, head):
    """The search's winner and per-size accepted counts at thresholds across the distribution of
    subset scores equal the per-subset kernel's (first acceptable subset in itertools order of
    the smallest size)."""
    n = 11
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    kf = kfmi.BatchedKF('ref15', 1, 'f64', options={'search_kernel': kernel, 'search_head': head})
    _, _, _, sm = kf.search_combos(ev, init, t0, target, threshold=-1e30, exhaustive=True, subset_max=True)
    vals = np.sort(sm.cpu().numpy()[1:])
    thr = float(vals[int(q * (len(vals) - 1))]) + (1e-9 if q > 0 else -1.0)
    kfound, win, acc, _ = kf.search_combos(ev, init, t0, target, thr, exhaustive=True)
    k1, win1, _, _ = kf.search_combos(ev, init, t0, target, thr, exhaustive=False)
    kf.close()
    assert (k1, win1) == (kfound, win)
    want_k, want_combo = 0, None
    for k in range(1, n + 1):
        combos = list(combinations(range(n), k))
        kc = kfmi.BatchedKF('ref15', len(combos), 'f64')
        mx, _, _ = kc.eval_combos(ev, init, t0, target, k, logdets=False)
        ok = (mx < thr).cpu().numpy()
        kc.close()
        assert int(acc[k]) == int(ok.sum()), k
        if want_k == 0 and ok.any():
            want_k, want_combo = k, combos[int(np.argmax(ok))]
    assert (kfound, win) == (want_k, want_combo)
    if q == 0.0:
        assert kfound == 0


@pytest.mark.parametrize('n_fixed,fixed_mask', [(0, 0), (3, 0b101)])
def test_search_head_equals_level_search(golden_dir, n_fixed, fixed_mask):
    """The one-launch head (levels 1 .. K, one lane per subset from the root) and the level-by-level
    search give every subset the same max log-det, bit for bit, the same acceptance counts per
    size and the same winner, exhaustive and not, also on a class of a sharded search (fixed
    candidates); n = 18 (the head covers sizes 1 .. 7 there, the level kernels the rest)."""
    n = 18
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    out = {}
    for head in ('on', 'off'):
        kf = kfmi.BatchedKF('ref15', 1, 'f64', options={'search_head': head})
        _, _, _, sm = kf.search_combos(ev, init, t0, target, -1e30, exhaustive=True, subset_max=True,
                                       n_fixed=n_fixed, fixed_mask=fixed_mask)
        sm = sm.cpu().numpy()
        vals = np.sort(sm[np.isfinite(sm)])
        thr = float(vals[len(vals) // 50]) + 1e-9
        ex = kf.search_combos(ev, init, t0, target, thr, exhaustive=True, n_fixed=n_fixed, fixed_mask=fixed_mask)
        first = kf.search_combos(ev, init, t0, target, thr, exhaustive=False, n_fixed=n_fixed, fixed_mask=fixed_mask)
        kf.close()
        out[head] = (sm, ex, first)
    a, b = out['on'], out['off']
    np.testing.assert_array_equal(a[0], b[0])
    assert a[1][:2] == b[1][:2] and a[2][:2] == b[2][:2] and a[1][0] > 0
    np.testing.assert_array_equal(a[1][2], b[1][2])
    # not exhaustive: the counts stop at the first accepted size whichever way the levels ran
    np.testing.assert_array_equal(a[2][2], b[2][2])
    assert a[2][0] > 0 and not a[2][2][a[2][0] + 1:].any()


@pytest.mark.parametrize('dtype,sym,n_fixed,fixed_mask,consts', [('f64', False, 0, 0, 'reference'),
                                                                 ('f64', True, 0, 0, 'reference'),
                                                                 ('f64', True, 3, 0b101, 'reference'),
                                                                 ('f32', True, 0, 0, 'reference'),
                                                                 ('f32', False, 2, 0b10, 'reference'),
                                                                 ('f64', True, 0, 0, 'custom'),
                                                                 ('f32', False, 0, 0, 'custom')])
def test_search_end_equals_level_search(golden_dir, dtype, sym, n_fixed, fixed_mask, consts):
    """The end launch (the last sizes in one launch, each subset from its stored prefix) and the
    level-by-level search give every subset the same max log-det, bit for bit, the same counts
    per size and the same winner, exhaustive and not, with the head on; n = 18 (the end launch
    covers sizes 13 .. 18 of the free candidates there), every-chain and axis-symmetric nodes,
    f64 and f32, the reference's constants and a caller's, a whole search and a class of a
    sharded one."""
    n = 18
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    if sym:
        init = _axis_symmetric(init)
    params = _symmetric_consts(7).params() if consts == 'custom' else None
    out = {}
    for end in ('on', 'off'):
        kf = kfmi.BatchedKF('ref15', 1, dtype, params=params, options={'search_end': end})
        _, _, _, sm = kf.search_combos(ev, init, t0, target, -1e30, exhaustive=True, subset_max=True,
                                       n_fixed=n_fixed, fixed_mask=fixed_mask)
        info = kf.search_info()
        assert info['sym'] == sym
        sm = sm.cpu().numpy()
        res = [sm]
        for q in (0.02, 0.6, 0.97):
            thr = _gap_threshold(sm, q)
            res.append(kf.search_combos(ev, init, t0, target, thr, exhaustive=True, n_fixed=n_fixed,
                                        fixed_mask=fixed_mask))
            res.append(kf.search_combos(ev, init, t0, target, thr, exhaustive=False, n_fixed=n_fixed,
                                        fixed_mask=fixed_mask))
        out[end] = (res, info['level_launches'])
        kf.close()
    a, b = out['on'][0], out['off'][0]
    np.testing.assert_array_equal(a[0], b[0])
    assert np.isfinite(a[0][1:]).sum() > 0
    for x, y in zip(a[1:], b[1:]):
        assert x[:2] == y[:2]
        np.testing.assert_array_equal(x[2], y[2])
    # fewer launches (in a class of 15 free candidates the head leaves a single level, which the
    # end launch does not replace)
    assert out['on'][1] <= out['off'][1] and (n_fixed > 0 or out['on'][1] < out['off'][1])


@pytest.mark.parametrize('n', [4, 5, 9, 12, 18, 25])
def test_search_launch_bookkeeping(golden_dir, n):
    """kfmi.ref15's mirror of the launch plan (the bench's bytes and the PMC reduction use it)
    agrees with what kf_search_combos ran: the head's sizes and the launches of one search."""
    _, ev, init, t0, target = _search_case(golden_dir, n, swap=n > 6)
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    kf.search_combos(ev, init, t0, target, -1e30, exhaustive=True)
    info = kf.search_info()
    kf.close()
    assert info['head_sizes'] == ref15.search_head_size(n)
    assert info['level_launches'] + (1 if info['head_sizes'] else 0) == ref15.search_launches(n, sym=info['sym'])


def test_search_end_random_shapes(golden_dir):
    """The end launch against the level-by-level search over seeded shapes: n 6 .. 20, k_max
    below n, head on and off, every-chain and axis-symmetric nodes, fixed candidates; every
    subset's max log-det bit for bit and the counts per size."""
    rng = np.random.default_rng(2025)
    fused = 0
    for case in range(14):
        n = int(rng.integers(6, 21))
        k_max = int(rng.integers(max(2, n - 4), n + 1))
        head = ['on', 'off'][case % 2]
        sym = bool(case % 3)
        n_fixed = int(rng.integers(0, 3))
        fixed_mask = int(rng.integers(0, 1 << n_fixed)) if n_fixed else 0
        if k_max <= bin(fixed_mask).count('1'):
            k_max = n
        _, ev, init, t0, target = _search_case(golden_dir, n, swap=n > 6)
        if sym:
            init = _axis_symmetric(init)
        got = {}
        for end in ('on', 'off'):
            kf = kfmi.BatchedKF('ref15', 1, 'f64', options={'search_end': end, 'search_head': head})
            k, win, acc, sm = kf.search_combos(ev, init, t0, target, -1e30, k_max=k_max, exhaustive=True,
                                               subset_max=True, n_fixed=n_fixed, fixed_mask=fixed_mask)
            launches = kf.search_info()['level_launches']
            sm = sm.cpu().numpy()
            thr = _gap_threshold(sm, 0.3)
            r2 = kf.search_combos(ev, init, t0, target, thr, k_max=k_max, exhaustive=True, n_fixed=n_fixed,
                                  fixed_mask=fixed_mask)
            kf.close()
            got[end] = (sm, r2, launches)
        shape = (n, k_max, head, sym, n_fixed, fixed_mask)
        np.testing.assert_array_equal(got['on'][0], got['off'][0], err_msg=str(shape))
        assert got['on'][1][:2] == got['off'][1][:2], shape
        np.testing.assert_array_equal(got['on'][1][2], got['off'][1][2], err_msg=str(shape))
        fused += got['on'][2] < got['off'][2]
    assert fused >= 4  # the end launch ran in enough of the shapes


def _axis_symmetric(init):
    """init with the x axis's covariance blocks copied to the y and z axes."""
    out = np.array(init, dtype=np.float64)
    b = out[15:]
    for c in (1, 2):
        b[6 * c:6 * c + 6] = b[0:6]
        b[18 + 3 * c:18 + 3 * c + 3] = b[18:21]
    return out


def _symmetric_consts(seed):
    """Caller constants that are the same on the three axes (one value per state group)."""
    rng = np.random.default_rng(seed)
    g = lambda lo, hi: np.repeat(rng.uniform(lo, hi, 5), 3)  # noqa: E731 (pos, att, vel, rate, acc)
    return ref15.ModelConsts('ref15', q=g(0.01, 8.0), r_imu=g(0.02, 120.0), r_gps=np.full(3, rng.uniform(0.5, 9.0)),
                             p0=g(20.0, 2e4))


def _gap_threshold(vals, q):
    """A threshold near quantile q of the finite scores, midway in a gap between two consecutive
    ones of at least 1e-9 relative, so rounding-level differences cannot move a subset across it."""
    v = np.unique(vals[np.isfinite(vals)])
    i = int(q * (len(v) - 1))
    while i + 1 < len(v) and v[i + 1] - v[i] <= 1e-9 * max(abs(v[i]), 1.0):
        i += 1
    return float(0.5 * (v[i] + v[i + 1]))


@pytest.mark.parametrize('consts', ['reference', 'custom'])
@pytest.mark.parametrize('kernel,pm', [('cm', 'auto'), ('pm', 'lds'), ('pm', 'regs')])
@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_search_axis_symmetric_equals_every_chain(golden_dir, dtype, kernel, pm, consts):
    """KF_OPT_AXIS_SYM: with the same constants and root blocks on the three axes the search
    computes and stores one pva and one aw chain for the three of each.  Every subset's max
    log-det equals the every-chain search's to rounding (the three chains' copies of the same
    arithmetic are compiled separately there, and round alike in ~98 % of subsets, one ulp
    apart in the rest), and both equal the per-subset kernel's to 1e-12; the acceptance counts
    and the winner (exhaustive and not) are the same, on each search kernel, with the head and
    without, in both precisions."""
    n = 14
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    init = _axis_symmetric(init)
    params = _symmetric_consts(5).params() if consts == 'custom' else None
    tol = 1e-14 if dtype == 'f64' else 1e-6
    out = {}
    for sym in ('on', 'off'):
        res = []
        for head in ('on', 'off'):
            kf = kfmi.BatchedKF('ref15', 1, dtype, params=params,
                                options={'search_kernel': kernel, 'search_pm': pm, 'axis_sym': sym, 'search_head': head})
            _, _, _, sm = kf.search_combos(ev, init, t0, target, -1e30, exhaustive=True, subset_max=True)
            info = kf.search_info()
            sm = sm.double().cpu().numpy()
            assert info['sym'] == (sym == 'on') and (info['head_sizes'] > 0) == (head == 'on'), info
            res.append(sm)
            kf.close()
        out[sym] = res
    ref = out['off'][0]
    assert np.isnan(ref[0]) and np.isfinite(ref[1:]).all()
    for sm in out['on'] + out['off'][1:]:
        assert np.isnan(sm[0])
        assert np.max(np.abs(sm[1:] - ref[1:]) / np.maximum(np.abs(ref[1:]), 1.0)) <= tol
    for q in (0.02, 0.4):
        thr = _gap_threshold(ref[1:], q)
        got = {}
        for sym in ('on', 'off'):
            kf = kfmi.BatchedKF('ref15', 1, dtype, params=params,
                                options={'search_kernel': kernel, 'search_pm': pm, 'axis_sym': sym})
            ex = kf.search_combos(ev, init, t0, target, thr, exhaustive=True)
            first = kf.search_combos(ev, init, t0, target, thr, exhaustive=False)
            kf.close()
            got[sym] = (ex, first)
        (ea, fa), (eb, fb) = got['on'], got['off']
        assert ea[:2] == eb[:2] == fa[:2] == fb[:2] and ea[0] > 0, q
        np.testing.assert_array_equal(ea[2], eb[2])


def test_search_axis_symmetry_detected_exactly(golden_dir):
    """The axis-symmetric search runs only where it is exact: the handle's constants the same on
    the three axes and the root covariance's blocks equal bit for bit.  One ulp off in one block,
    or one axis's constant changed, and the search runs every chain (and agrees with the oracle
    as before)."""
    n = 9
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    sym_init = _axis_symmetric(init)
    off_init = sym_init.copy()
    off_init[15 + 6 + 2] = np.nextafter(off_init[15 + 6 + 2], np.inf)  # y axis, pva block entry (0, 2)
    c = _symmetric_consts(6)
    q = c.q.copy()
    q[13] *= 1.5  # the y axis's acceleration noise
    asym = ref15.ModelConsts('ref15', q=q, r_imu=c.r_imu, r_gps=c.r_gps, p0=c.p0)
    cases = [(None, sym_init, True), (None, off_init, False), (c.params(), sym_init, True),
             (asym.params(), sym_init, False)]
    for params, ini, want in cases:
        kf = kfmi.BatchedKF('ref15', 1, 'f64', params=params)
        kf.search_combos(ev, ini, t0, target, -1e30, exhaustive=True)
        assert kf.search_info()['sym'] == want
        kf.close()


@pytest.mark.parametrize('w', [1, 3])
def test_search_classes_partition_the_search(golden_dir, w):
    """The per-GPU shards of kfmi.dist.brute_force_search: searches restricted to the subsets
    with a fixed intersection with the first w candidates score each of their subsets as the
    whole search does, cover every subset exactly once, and their per-class winners combine
    (smallest size, then itertools order) into the whole search's winner."""
    n = 11
    cand, ev, init, t0, target = _search_case(golden_dir, n)
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    _, _, _, full = kf.search_combos(ev, init, t0, target, threshold=-1e30, exhaustive=True, subset_max=True)
    full = full.cpu().numpy()
    seen = np.zeros(1 << n, dtype=int)
    for c in range(1 << w):
        _, _, _, sm = kf.search_combos(ev, init, t0, target, -1e30, exhaustive=True, subset_max=True,
                                       n_fixed=w, fixed_mask=c)
        sm = sm.cpu().numpy()
        idx = np.flatnonzero(~np.isnan(sm))
        assert ((idx & ((1 << w) - 1)) == c).all()
        seen[idx] += 1
        assert np.max(np.abs(sm[idx] - full[idx]) / np.maximum(np.abs(full[idx]), 1.0)) <= 1e-12
    assert (seen[1:] == 1).all() and seen[0] == 0
    vals = np.sort(full[1:])
    for q in (0.0, 0.02, 0.5):
        thr = float(vals[int(q * (len(vals) - 1))]) + (1e-9 if q > 0 else -1.0)
        want = kf.search_combos(ev, init, t0, target, thr)[:2]
        got = (0, None)
        for c in range(1 << w):
            k, idx, _, _ = kf.search_combos(ev, init, t0, target, thr, n_fixed=w, fixed_mask=c)
            if k and (got[0] == 0 or (k, idx) < got):
                got = (k, idx)
        assert got == want, (q, got, want)
    kf.close()


@pytest.mark.parametrize('head', ['on', 'off'])
def test_search_stops_at_the_first_accepted_size(golden_dir, head):
    """Not exhaustive, levels are queued in groups between result peeks and a level queued past
    the first accepted size does nothing: for thresholds whose first accepted size runs over
    the sizes (and none), the size, the winner and the counts up to it equal the exhaustive
    search's, and the counts past it are 0."""
    n = 18
    _, ev, init, t0, target = _search_case(golden_dir, n)
    kf = kfmi.BatchedKF('ref15', 1, 'f64', options={'search_head': head})
    _, _, _, sm = kf.search_combos(ev, init, t0, target, threshold=-1e30, exhaustive=True, subset_max=True)
    sm = sm.cpu().numpy()
    sizes = np.array([bin(m).count('1') for m in range(1 << n)])
    seen = set()
    for s in list(range(1, n + 1)) + [None]:
        if s is None:
            thr = -1e30
        else:
            m = float(np.min(sm[sizes == s]))
            thr = m + abs(m) * 1e-9 + 1e-12
        want = kf.search_combos(ev, init, t0, target, thr, exhaustive=True)
        got = kf.search_combos(ev, init, t0, target, thr, exhaustive=False)
        kfound = want[0]
        seen.add(kfound)
        assert got[:2] == want[:2], (s, got[:2], want[:2])
        np.testing.assert_array_equal(got[2][:kfound + 1], want[2][:kfound + 1])
        if kfound:
            assert not got[2][kfound + 1:].any()
    kf.close()
    assert 0 in seen and len(seen) >= 4


def test_search_counters_carry_across_calls_and_streams(golden_dir):
    """The finish kernel hands each search's counters to the host and zeroes them for the next
    search on its stream: repeated searches, one on another stream, a non-exhaustive one that
    stops early and a refused call in between all report what a fresh handle reports; inside a
    graph capture the call is refused before it queues anything."""
    n = 11
    _, ev, init, t0, target = _search_case(golden_dir, n)
    fresh = kfmi.BatchedKF('ref15', 1, 'f64')
    _, _, _, sm = fresh.search_combos(ev, init, t0, target, threshold=-1e30, exhaustive=True, subset_max=True)
    thr = float(np.sort(sm.cpu().numpy()[1:])[600]) + 1e-9
    want = fresh.search_combos(ev, init, t0, target, thr, exhaustive=True)
    want_ne = fresh.search_combos(ev, init, t0, target, thr, exhaustive=False)
    fresh.close()
    assert want[0] > 0 and int(want[2].sum()) > 0

    def same(got, ref):
        assert got[:2] == ref[:2]
        np.testing.assert_array_equal(got[2], ref[2])

    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    side = torch.cuda.Stream()
    for _ in range(3):
        same(kf.search_combos(ev, init, t0, target, thr, exhaustive=True), want)
    with torch.cuda.stream(side):
        same(kf.search_combos(ev, init, t0, target, thr, exhaustive=True), want)
    same(kf.search_combos(ev, init, t0, target, thr, exhaustive=False), want_ne)
    with pytest.raises(kfmi.KFError):
        kf.search_combos(ev, init, t0, target, thr, k_max=n + 1)
    same(kf.search_combos(ev, init, t0, target, thr, exhaustive=True), want)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with pytest.raises(kfmi.KFError, match='capturable'):
        with torch.cuda.graph(g):
            kf.search_combos(ev, init, t0, target, thr, exhaustive=True)
    same(kf.search_combos(ev, init, t0, target, thr, exhaustive=True), want)
    kf.close()


def test_search_combos_rejects_bad_arguments():
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    ev = np.zeros((4, 11))
    ev[:, 0] = np.arange(4)
    init = np.zeros(42)
    with pytest.raises(kfmi.KFError):
        kf.search_combos(ev, init, 0.0, 4.0, 0.0, k_max=5)
    bad = ev.copy()
    bad[1, 1] = 7
    with pytest.raises(kfmi.KFError):
        kf.search_combos(bad, init, 0.0, 4.0, 0.0)
    big = np.tile(ev, (17, 1))  # 68 candidates: more than the 64-bit subset masks hold
    big[:, 0] = np.arange(len(big))
    with pytest.raises(kfmi.KFError):
        kf.search_combos(big, init, 0.0, 68.0, 0.0, k_max=1)
    with pytest.raises(kfmi.KFError):  # a fixed bit at or above n_fixed
        kf.search_combos(ev, init, 0.0, 4.0, 0.0, n_fixed=1, fixed_mask=2)
    with pytest.raises(kfmi.KFError):  # every candidate fixed
        kf.search_combos(ev, init, 0.0, 4.0, 0.0, n_fixed=4, fixed_mask=0)
    with pytest.raises(kfmi.KFError):  # k_max not above the fixed subset's size
        kf.search_combos(ev, init, 0.0, 4.0, 0.0, k_max=2, n_fixed=2, fixed_mask=3)
    kf.close()
    cv = kfmi.BatchedKF('cv3', 4, 'f64')
    with pytest.raises(ValueError):
        cv.search_combos(ev, init, 0.0, 4.0, 0.0)
    cv.close()


def test_eval_combos_rejects_logdets_past_4gib():
    """The k + 2 logdet rows share one buffer descriptor with a 32-bit range: 64 rows of 2^23
    f64 filters (exactly 4 GiB) are refused instead of wrapping; without records the launch runs."""
    B, n, k = 1 << 23, 64, 62
    ev = np.zeros((n, 11))
    ev[:, 0] = np.arange(n)
    ev[:, 1] = ref15.IMU
    init = np.concatenate([np.zeros(15), ref15.to_blocks(ref15.P0)])
    kf = kfmi.BatchedKF('ref15', B, 'f64')
    with pytest.raises(kfmi.KFError, match='4 GiB'):
        kf.eval_combos(ev, init, 0.0, float(n), k, logdets=True)
    mx, _, nrec = kf.eval_combos(ev, init, 0.0, float(n), k, logdets=False)
    assert torch.isfinite(mx[:math.comb(n, k)]).all() and int(nrec[0]) == k + 2  # P0, k events, final predict
    kf.close()


@pytest.mark.parametrize('n,k', [(10, 1), (10, 4), (12, 6)])
def test_eval_combos_kernel_vs_oracle(golden_dir, n, k):
    """Every k-subset of n candidates, unranked in-kernel, against the oracle's worker: record
    lists, max logdet and final state per subset (itertools.combinations order)."""
    g = _load(golden_dir, 'ref15_full.npz')
    events = unpack_events(g)
    s0 = 100
    st, ld, P, prev = ref_kf.run_kalman_filter_full(events, 0, s0)
    cand = events[s0:s0 + n]
    xt = np.zeros(15)
    xt[0:6] = st[-1][1:7]
    target = events[s0 + n - 1][2]
    ev = np.array([[t, 0 if s == 'GPS' else 1, *ref15.event_payload(s, d)] for (_, s, t, d) in cand])
    init = np.concatenate([xt, ref15.to_blocks(P)])
    total = math.comb(n, k)
    kf = kfmi.BatchedKF('ref15', total + 37, 'f64')  # a ragged tail of padding lanes
    mx, lds, nrec = kf.eval_combos(ev, init, st[-1][0], target, k)
    x, _ = kf.state()
    mx, lds, nrec, x = mx.cpu().numpy(), lds.cpu().numpy(), nrec.cpu().numpy(), x.cpu().numpy()
    st_lane = kf.status().cpu().numpy()
    assert (st_lane[:total] == 0).all() and (st_lane[total:] == 1).all()
    assert np.isnan(mx[total:]).all()
    ref = ref_kf.evaluate_combo_chunk(list(combinations(cand, k)), xt, P, st[-1][0], target)
    for f, r in enumerate(ref):
        assert nrec[f] == len(r[5])
        assert _rel(lds[:nrec[f], f], r[5]) <= TOL
        assert np.isnan(lds[nrec[f]:, f]).all()
        assert abs(mx[f] - max(r[5])) <= TOL * max(abs(max(r[5])), 1.0)
        assert _rel(x[:, f], r[3]) <= TOL


def test_run_events_random_batch_vs_oracle():
    """B independent filters on their own random GPS/IMU/predict-only/padding streams (ragged,
    irregular dt) against the oracle's dense 15x15 reference-order step."""
    rng = np.random.default_rng(7)
    B, T = 300, 40
    etype = rng.choice([0, 1, 1, 1, 2], size=(T, B)).astype(np.uint8)
    etype[30:, ::3] = 255                          # ragged ends
    dt = rng.uniform(0.0, 0.12, (T, B))
    pay = np.zeros((T, 9, B))
    pay[:, 0:3] = rng.normal(0, 20, (T, 3, B))    # GPS e, n, alt (and IMU angles for IMU)
    pay[:, 3:6] = rng.normal(0, 0.05, (T, 3, B))
    pay[:, 6:9] = rng.normal(0, 0.5, (T, 3, B))
    x0 = np.zeros((B, 15))
    x0[:, :3] = rng.normal(0, 20, (B, 3))
    kf = kfmi.BatchedKF('ref15', B, 'f64')
    kf.reset(torch.from_numpy(np.ascontiguousarray(x0.T)).cuda())
    tr, ld, up, _ = kf.run_events(etype, dt, pay, updated=True)
    tr, ld, up = tr.cpu().numpy(), ld.cpu().numpy(), up.cpu().numpy()
    x, Pb = kf.state()
    x, Pb = x.cpu().numpy(), Pb.cpu().numpy()
    assert (kf.status().cpu().numpy() == 0).all()
    for f in range(0, B, 7):
        xf, Pf = x0[f].copy(), ref_kf.P0_REF15.copy()
        for t in range(T):
            ty = etype[t, f]
            if ty == 255:
                pass
            elif ty == 2:
                F = ref_kf.F_ref15(dt[t, f])
                xf = F @ xf
                Pf = ref_kf.predict_covariance(Pf, F, ref_kf.Q_ref15(dt[t, f]))
            else:
                if ty == 0:
                    sdata = {'easting': pay[t, 0, f], 'northing': pay[t, 1, f], 'altitude': pay[t, 2, f]}
                else:
                    sdata = ['t', *pay[t, :, f]]
                xf, Pf = ref_kf.step15(xf, Pf, 'GPS' if ty == 0 else 'IMU', sdata, dt[t, f])
            assert _rel(tr[t, :, f], xf[:6]) <= TOL, (f, t)
            assert abs(ld[t, f] - np.linalg.slogdet(Pf)[1]) <= TOL * max(1.0, abs(np.linalg.slogdet(Pf)[1]))
            assert up[t, f] == (1 if ty in (0, 1) else 0)
        assert _rel(x[:, f], xf) <= TOL
        assert _rel(ref15.from_blocks(Pb[:, f]), Pf) <= TOL


def test_ref15_handle_rejects_cv_entry_points():
    from kfmi import _lib
    kf = kfmi.BatchedKF('ref15', 4, 'f64')
    assert _lib.lib().kf_predict(kf.handle, 0.1, None, None, None, None) == _lib.KF_EINVAL  # C ABI: cv only
    with pytest.raises(ValueError):
        kf.predict(0.1, u=np.zeros((3, 4)))
    with pytest.raises(ValueError):
        kfmi.BatchedKF('cv3', 4, 'f64').run_events(np.zeros((1, 4), np.uint8), np.zeros((1, 4)), np.zeros((1, 9, 4)))


# -- sensor scheduling (kf_workers.py:99-213, 826-957) ----------------------------------------

@pytest.mark.parametrize('f', [20, 50, 120])
def test_scheduled_greedy(golden_dir, f):
    g = _load(golden_dir, 'ref15_scheduled.npz')
    events = unpack_events(g)
    st, ld, P = ref15.run_kalman_filter_scheduled(events, 0, len(events), selection_method='greedy',
                                                  processing_frequency=f)
    assert np.array(st).shape == g[f'greedy{f}_states'].shape
    assert _rel(st, g[f'greedy{f}_states']) <= TOL
    assert _rel(ld, g[f'greedy{f}_logdets']) <= TOL
    assert _rel(P, g[f'greedy{f}_P']) <= TOL


def test_scheduled_random_and_warm(golden_dir):
    g = _load(golden_dir, 'ref15_scheduled.npz')
    events = unpack_events(g)
    np.random.seed(int(g['random50_seed']))
    st, ld, P = ref15.run_kalman_filter_scheduled(events, 0, len(events), selection_method='random',
                                                  processing_frequency=50)
    assert np.array(st).shape == g['random50_states'].shape
    assert _rel(st, g['random50_states']) <= TOL
    assert _rel(ld, g['random50_logdets']) <= TOL
    assert _rel(P, g['random50_P']) <= TOL
    st, ld, P = ref15.run_kalman_filter_scheduled(events, 60, 180, initial_pt=g['warm_init_P'],
                                                  initial_state=tuple(g['warm_init_state']),
                                                  selection_method='greedy', processing_frequency=100)
    assert np.array(st).shape == g['warm_states'].shape
    assert _rel(st, g['warm_states']) <= TOL
    assert _rel(ld, g['warm_logdets']) <= TOL
    assert _rel(P, g['warm_P']) <= TOL
    assert ref15.run_kalman_filter_scheduled(events, 0, 10, selection_method='bogus',
                                             processing_frequency=50) is None


def test_scheduler_gain(golden_dir):
    g = _load(golden_dir, 'ref15_scheduled.npz')
    S = g['sched_sigma']
    gain = ref15.scheduler_gain(S)
    assert _rel(gain, g['sched_gain']) <= TOL
    assert _rel(gain, np.trace(g['sched_cov_first'], axis1=2, axis2=3)) <= TOL
    full = ref15.scheduler_gain(S, full=True)
    assert _rel(full, np.trace(g['sched_cov_full'], axis1=2, axis2=3)) <= TOL


def test_sampling_sweep_one_launch(golden_dir):
    """Every processing frequency as its own filter in ONE kf_run_scheduled launch, against the
    reference's outputs (20/50/120 Hz) and the oracle (the rest)."""
    g = _load(golden_dir, 'ref15_scheduled.npz')
    events = unpack_events(g)
    freqs = [10, 20, 30, 40, 50, 60, 70, 80, 90, 100, 110, 120, 1000]
    out = ref15.sampling_sweep(events, freqs)
    for f in freqs:
        st, ld, P = out[f]
        if f in (20, 50, 120):
            rs, rl, rP = g[f'greedy{f}_states'], g[f'greedy{f}_logdets'], g[f'greedy{f}_P']
        else:
            rs, rl, rP = ref_kf.run_kalman_filter_scheduled(events, 0, len(events), selection_method='greedy',
                                                            processing_frequency=f)
        assert np.array(st).shape == np.array(rs).shape, f
        assert _rel(st, rs) <= TOL, f
        assert _rel(ld, rl) <= TOL, f
        assert _rel(P, rP) <= TOL, f


@pytest.mark.parametrize('seed,B', [(0, 48), (1, 48), (2, 128)])
def test_scheduled_random_streams_vs_oracle(seed, B):
    """kf_run_scheduled over independent random streams (a GPS fix at random positions, 200 Hz
    with jitter, ragged ends, every lane its own rate, so the lanes of a wave trigger at
    different events), each filter against the oracle's greedy driver (kf_workers.py:826-957)
    from the same warm start."""
    rng = np.random.default_rng(seed)
    T = 120  # B % 64 == 0 takes the LDS-staged kernel (chunks of 16 events, a ragged last one)
    t0 = 1697739278.761565
    rates = rng.choice([10, 20, 35, 50, 75, 120, 160, 400], B).astype(np.float64)
    etype = np.where(rng.random((T, B)) < 0.15, 0, 1).astype(np.uint8)
    tt = t0 + np.cumsum(rng.uniform(0.003, 0.007, (T, B)), axis=0)
    pay = rng.normal(0, 1, (T, 9, B))
    pay[:, 0:3] *= 0.05
    pay[:, 6:9] *= 0.3
    pay[:, 0:3] = np.where((etype == 0)[:, None, :], pay[:, 0:3] * 60, pay[:, 0:3])
    lens = rng.integers(T // 2, T + 1, B)
    for f in range(B):
        etype[lens[f]:, f] = 255
    x0 = np.zeros((15, B))
    x0[0:6] = rng.normal(0, 2, (6, B))
    Pblk = np.repeat(ref15.to_blocks(ref_kf.P0_REF15)[:, None], B, axis=1)
    kf = kfmi.BatchedKF('ref15', B, 'f64')
    kf.set_state(x0, Pblk)
    tr, ld, stt, ns = kf.run_scheduled(tt, etype, pay, np.full(B, t0), rates)
    tr, ld, stt, ns = (v.cpu().numpy() for v in (tr, ld, stt, ns))
    kf.close()
    for f in range(B):
        ev = [(0, 'GPS', t0, {'easting': 0.0, 'northing': 0.0, 'altitude': 0.0})]  # skipped (warm start)
        for i in range(lens[f]):
            if etype[i, f] == 0:
                ev.append((i + 1, 'GPS', tt[i, f], {'easting': pay[i, 0, f], 'northing': pay[i, 1, f],
                                                    'altitude': pay[i, 2, f]}))
            else:
                ev.append((i + 1, 'IMU', tt[i, f], ['t', *pay[i, :, f]]))
        rs, rl, _ = ref_kf.run_kalman_filter_scheduled(ev, 0, len(ev), ref_kf.P0_REF15.copy(),
                                                       (t0, *x0[0:6, f]), 'greedy', rates[f])
        n = int(ns[f])
        assert n == len(rs) - 1, f
        if n == 0:
            continue
        assert _rel(stt[:n, f], [r[0] for r in rs[1:]]) <= 1e-12, f
        assert _rel(tr[:n, :, f], np.array([r[1:7] for r in rs[1:]])) <= TOL, f
        assert _rel(ld[:n, f], rl[1:]) <= TOL, f


@pytest.mark.parametrize('B,records', [(48, False), (128, False), (128, True), (128, 'time')])
def test_scheduled_random_vs_oracle(B, records):
    """kf_run_scheduled_random (the random arm, kf_workers.py:826-957 with random_schedule
    :188-193) over random ragged streams with per-lane rates: each filter draws from its own
    column of generator outputs, and against the oracle's random driver drawing from a
    RandomState with the same seed it picks the same events (times bitwise) with the same states
    and log-dets, and reports exactly the outputs the oracle consumed.  B = 48: the fused kernel;
    B = 128: the pick and apply passes (payload rows and records).  A column too short for its
    filter's draws reports -1."""
    rng = np.random.default_rng(60 + B + {False: 0, True: 1, 'time': 2}[records])
    T = 120
    t0, rates, etype, tt, pay = _sched_streams(rng, B, T)
    W = 2 * T + 64
    words = np.stack([np.random.RandomState(1000 + f).randint(0, 1 << 32, size=W, dtype=np.uint32)
                      for f in range(B)], axis=1)
    x0 = np.zeros((15, B))
    x0[0:6] = rng.normal(0, 2, (6, B))
    Pblk = np.repeat(ref15.to_blocks(ref_kf.P0_REF15)[:, None], B, axis=1)
    opts = {'sched_rec_time': 'on'} if records == 'time' else None   # rec[9] = the event's time
    kf = kfmi.BatchedKF('ref15', B, 'f64', options=opts)
    kf.set_state(x0, Pblk)
    payload = _sched_records(pay, 12) if records else pay
    if records == 'time':
        payload[:, :, 9] = tt
    records = bool(records)
    tr, ld, stt, ns, used = (v.cpu().numpy() for v in kf.run_scheduled_random(tt, etype, payload, np.full(B, t0),
                                                                               rates, words, records=records))
    # the picks alone (kf_sched_random_picks): the same events, times and generator outputs
    pk, st2, ns2, used2 = (v.cpu().numpy() for v in kf.sched_random_picks(tt, etype, np.full(B, t0), rates, words))
    kf.close()
    np.testing.assert_array_equal(ns2, ns)
    np.testing.assert_array_equal(used2, used)
    for f in range(B):
        np.testing.assert_array_equal(st2[:ns[f], f], stt[:ns[f], f])
        np.testing.assert_array_equal(st2[:ns[f], f], tt[pk[:ns[f], f], f])
    for f in range(B):
        ev = [(0, 'GPS', t0, {'easting': 0.0, 'northing': 0.0, 'altitude': 0.0})]  # skipped (warm start)
        for i in range(T):
            if etype[i, f] == 255:
                break
            ev.append((i + 1, 'GPS', tt[i, f], {'easting': pay[i, 0, f], 'northing': pay[i, 1, f],
                                                'altitude': pay[i, 2, f]}) if etype[i, f] == 0
                      else (i + 1, 'IMU', tt[i, f], ['t', *pay[i, :, f]]))
        gen = np.random.RandomState(1000 + f)
        rs, rl, _ = ref_kf.run_kalman_filter_scheduled(ev, 0, len(ev), ref_kf.P0_REF15.copy(), (t0, *x0[0:6, f]),
                                                       'random', rates[f], rng_choice=gen.choice)
        after = gen.random_sample()
        check = np.random.RandomState(1000 + f)
        check.randint(0, 1 << 32, size=int(used[f]), dtype=np.uint32)
        assert check.random_sample() == after, f     # the outputs taken are the ones the oracle drew
        n = int(ns[f])
        assert n == len(rs) - 1, f
        if n == 0:
            continue
        np.testing.assert_array_equal(stt[:n, f], [r[0] for r in rs[1:]])
        assert _rel(tr[:n, :, f], np.array([r[1:7] for r in rs[1:]])) <= TOL, f
        assert _rel(ld[:n, f], rl[1:]) <= TOL, f
    # too few outputs: the filter stops at its last completed pick and reports -1
    kf = kfmi.BatchedKF('ref15', B, 'f64', options=opts)
    kf.set_state(x0, Pblk)
    out = kf.run_scheduled_random(tt, etype, payload, np.full(B, t0), rates, words[:3], records=records)
    kf.close()
    u3, n3 = out[4].cpu().numpy(), out[3].cpu().numpy()
    short = used > 3
    assert short.any() and (u3[short] == -1).all() and (u3[~short] == used[~short]).all()
    assert (n3[short] <= ns[short]).all() and (n3[~short] == ns[~short]).all()


def _sched_streams(rng, B, T):
    """Random scheduled-filter inputs as test_scheduled_random_streams_vs_oracle builds them."""
    t0 = 1697739278.761565
    rates = rng.choice([10, 20, 35, 50, 75, 120, 160, 400], B).astype(np.float64)
    etype = np.where(rng.random((T, B)) < 0.15, 0, 1).astype(np.uint8)
    tt = t0 + np.cumsum(rng.uniform(0.003, 0.007, (T, B)), axis=0)
    pay = rng.normal(0, 1, (T, 9, B))
    pay[:, 0:3] *= 0.05
    pay[:, 6:9] *= 0.3
    pay[:, 0:3] = np.where((etype == 0)[:, None, :], pay[:, 0:3] * 60, pay[:, 0:3])
    lens = rng.integers(T // 2, T + 1, B)
    for f in range(B):
        etype[lens[f]:, f] = 255
    return t0, rates, etype, tt, pay


@pytest.mark.parametrize('r_gps,dtype,nan', [(None, 'f64', False), (0.0, 'f64', False), (400.0, 'f64', False),
                                             (None, 'f32', False), (None, 'f64', True)])
def test_sched_two_pass_matches_fused_kernels(r_gps, dtype, nan):
    """KF_OPT_SCHED_KERNEL: the two-pass path (pick pass + apply pass, mispicks rerun by the fused
    kernel; one- and four-wave groups, KF_OPT_SCHED_GROUP; heaviest-first or batch wave order,
    KF_OPT_SCHED_ORDER) equals the fused LDS and register kernels, with the reference constants, with
    R_gps[0] == R_imu[0] (a tie: the pick pass cannot decide and every gain comparison is left to
    the covariance, so rounding sends filters down the fallback) and with R_gps > R_imu (GPS
    wins).  Same arithmetic in every kernel: 1e-12."""
    rng = np.random.default_rng(31)
    B, T = 192, 96
    t0, rates, etype, tt, pay = _sched_streams(rng, B, T)
    if nan:  # a NaN sample poisons its filter's state (the covariance never reads it)
        for f in (3, 70, 131):
            pay[20:50, :, f] = np.nan  # 30 events: longer than any window, so one is picked
    ref = ref15.ModelConsts('ref15')
    if r_gps is None:
        params = None
    else:
        rg = np.full(3, r_gps if r_gps else ref.r_imu[0])
        params = ref15.ModelConsts('ref15', r_gps=rg).params()
    out = {}
    arms = {'auto': {}, 'group1': {'sched_group': 'wave'}, 'one_launch': {'sched_kernel': 'one_launch'},
            'batch_order': {'sched_order': 'batch'}, 'fused': {'sched_kernel': 'fused'},
            'regs': {'sched_kernel': 'regs'}}
    # the same runs with the payload as one record per event (kf_run_scheduled_rec)
    rec_arms = {'rec_' + k: v for k, v in arms.items() if k != 'batch_order'}
    payt = pay.astype(np.float32) if dtype == 'f32' else pay
    recs = _sched_records(payt, 10 if dtype == 'f64' else 12)
    # f64 records carrying the event's time at rec[9] (KF_OPT_SCHED_REC_TIME): the apply pass
    # takes each pick's time from its record and writes sel_time itself
    recs_t = None
    if dtype == 'f64':
        recs_t = _sched_records(payt, 12)
        recs_t[:, :, 9] = tt
        rec_arms.update({'rect_' + k: dict(v, sched_rec_time='on') for k, v in arms.items() if k != 'batch_order'})
    for kern, opts in {**arms, **rec_arms}.items():
        kf = kfmi.BatchedKF('ref15', B, dtype, params=params, options=opts)
        if kern.startswith('rec'):
            res = kf.run_scheduled(tt, etype, recs_t if kern.startswith('rect_') else recs, np.full(B, t0), rates,
                                   records=True)
        else:
            res = kf.run_scheduled(tt, etype, payt, np.full(B, t0), rates)
        out[kern] = [v.cpu().numpy() for v in res] + [kf.status().cpu().numpy()]
        kf.close()
    for kern in rec_arms:  # the records change only where the values are read from: bitwise
        base = kern.split('_', 1)[1]
        for a, b in zip(out[base], out[kern]):
            if a.ndim == 1:
                np.testing.assert_array_equal(a, b, err_msg=kern)
        ns0 = out[base][3]
        for f in range(B):
            n = int(ns0[f])
            for a, b in zip(out[base][:3], out[kern][:3]):
                np.testing.assert_array_equal(a[:n, ..., f], b[:n, ..., f], err_msg=kern)
    tr, ld, stt, ns, st = out['auto']
    assert ns.min() > 0
    assert (st != 0).sum() == 0  # a NaN measurement leaves P (and so S) intact: NaN states only
    for f in ((3, 70, 131) if nan else ()):
        assert np.isnan(tr[:ns[f], :, f]).any(), f
    tol = 1e-12 if dtype == 'f64' else 1e-5  # f32: the same operations, the fp32 event's rounding
    for kern in ('group1', 'one_launch', 'batch_order', 'fused', 'regs'):
        t2, l2, s2, n2, st2 = out[kern]
        np.testing.assert_array_equal(ns, n2, err_msg=kern)
        np.testing.assert_array_equal(st, st2, err_msg=kern)
        for f in range(B):  # rows past n_sel are not written
            n = int(ns[f])
            np.testing.assert_array_equal(stt[:n, f], s2[:n, f], err_msg=kern)
            np.testing.assert_allclose(tr[:n, :, f], t2[:n, :, f], rtol=tol, atol=tol, err_msg=kern)
            np.testing.assert_allclose(ld[:n, f], l2[:n, f], rtol=tol, atol=tol, err_msg=kern)


def _sched_records(pay, rec):
    """[T, 9, B] payload rows -> [T, B, rec] records (kf_run_scheduled_rec), the pad slots NaN
    (never read)."""
    T, _, B = pay.shape
    r = np.full((T, B, rec), np.nan, dtype=pay.dtype)
    k = min(rec, 9)  # (a too-short record for the rejection test)
    r[:, :, :k] = pay.transpose(0, 2, 1)[:, :, :k]
    return r


def test_sched_records_reject_bad_layouts():
    """kf_run_scheduled_rec: a record shorter than 9 values, one whose byte length is not a
    multiple of 16, and records that are not 16-byte aligned are KF_EINVAL."""
    rng = np.random.default_rng(5)
    B, T = 64, 16
    t0, rates, etype, tt, pay = _sched_streams(rng, B, T)
    dev = torch.device('cuda', 0)
    kf = kfmi.BatchedKF('ref15', B, 'f64')
    for rec in (8, 9, 11):
        with pytest.raises(kfmi.KFError, match='rec_len'):
            kf.run_scheduled(tt, etype, _sched_records(pay, rec), np.full(B, t0), rates, records=True)
    buf = torch.zeros(T * B * 10 + 1, dtype=torch.float64, device=dev)
    mis = buf[1:].view(T, B, 10)  # 8 bytes past a 16-byte boundary
    mis.copy_(torch.as_tensor(_sched_records(pay, 10), device=dev))
    with pytest.raises(kfmi.KFError, match='aligned'):
        kf.run_scheduled(tt, etype, mis, np.full(B, t0), rates, records=True)
    kf.close()


@pytest.mark.parametrize('warm', [True, False])
def test_scheduled_replays_as_a_hip_graph(warm):
    """kf_run_scheduled captured into a hipGraph.  Warm: an eager call sized the two-pass
    workspace first, and the replay gives that call's outputs bitwise (pick pass, wave sort,
    apply pass, fallback).  Cold: no workspace can be allocated inside the capture, so the fused
    kernel runs, and the replay equals an eager two-pass run at 1e-12 (the kernels' agreement)."""
    rng = np.random.default_rng(41)
    B, T = 128, 80
    t0, rates, etype, tt, pay = _sched_streams(rng, B, T)
    dev = torch.device('cuda', 0)
    ttd, etd, payd = (torch.as_tensor(v, device=dev) for v in (tt, etype, pay))
    prev, frd = torch.full((B,), t0, dtype=torch.float64, device=dev), torch.as_tensor(rates, device=dev)
    x0 = torch.zeros(15, B, dtype=torch.float64, device=dev)
    P0b = torch.as_tensor(np.repeat(ref15.to_blocks(ref_kf.P0_REF15)[:, None], B, axis=1), device=dev)
    outs = (torch.empty(T, 6, B, dtype=torch.float64, device=dev), torch.empty(T, B, dtype=torch.float64, device=dev),
            torch.empty(T, B, dtype=torch.float64, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    def run(kf):
        kf.set_state(x0, P0b)
        for o, r in zip(outs, kf.run_scheduled(ttd, etd, payd, prev, frd)):
            o.copy_(r)

    ref_kf_ = kfmi.BatchedKF('ref15', B, 'f64')
    run(ref_kf_)
    torch.cuda.synchronize()
    eager = [o.cpu().numpy().copy() for o in outs]
    ref_kf_.close()
    kf = kfmi.BatchedKF('ref15', B, 'f64')
    if warm:
        run(kf)
        torch.cuda.synchronize()
    for o in outs:
        o.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run(kf)
    g.replay()
    torch.cuda.synchronize()
    got = [o.cpu().numpy() for o in outs]
    kf.close()
    np.testing.assert_array_equal(got[3], eager[3])
    for f in range(B):
        n = int(eager[3][f])
        np.testing.assert_array_equal(got[2][:n, f], eager[2][:n, f])
        if warm:
            np.testing.assert_array_equal(got[0][:n, :, f], eager[0][:n, :, f])
            np.testing.assert_array_equal(got[1][:n, f], eager[1][:n, f])
        else:
            np.testing.assert_allclose(got[0][:n, :, f], eager[0][:n, :, f], rtol=1e-12, atol=1e-12)
            np.testing.assert_allclose(got[1][:n, f], eager[1][:n, f], rtol=1e-12, atol=1e-12)


def test_scheduled_graph_survives_a_larger_eager_call():
    """A captured kf_run_scheduled keeps its workspace: an eager call with a longer stream on the
    same handle grows the workspace without freeing the one the graph writes, and a
    replay after it still gives the first call's outputs bitwise."""
    rng = np.random.default_rng(43)
    B, T = 128, 80
    t0, rates, etype, tt, pay = _sched_streams(rng, B, 3 * T)
    dev = torch.device('cuda', 0)
    ttd, etd, payd = (torch.as_tensor(v, device=dev) for v in (tt, etype, pay))
    prev, frd = torch.full((B,), t0, dtype=torch.float64, device=dev), torch.as_tensor(rates, device=dev)
    x0 = torch.zeros(15, B, dtype=torch.float64, device=dev)
    P0b = torch.as_tensor(np.repeat(ref15.to_blocks(ref_kf.P0_REF15)[:, None], B, axis=1), device=dev)
    outs = (torch.empty(T, 6, B, dtype=torch.float64, device=dev), torch.empty(T, B, dtype=torch.float64, device=dev),
            torch.empty(T, B, dtype=torch.float64, device=dev), torch.empty(B, dtype=torch.int32, device=dev))

    def run(kf, n):
        kf.set_state(x0, P0b)
        res = kf.run_scheduled(ttd[:n], etd[:n], payd[:n], prev, frd)
        if n == T:
            for o, r in zip(outs, res):
                o.copy_(r)

    kf = kfmi.BatchedKF('ref15', B, 'f64')
    run(kf, T)
    torch.cuda.synchronize()
    eager = [o.cpu().numpy().copy() for o in outs]
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run(kf, T)
    run(kf, 3 * T)           # grows the workspace: the captured one must stay alive
    torch.cuda.synchronize()
    for o in outs:
        o.zero_()
    g.replay()
    torch.cuda.synchronize()
    got = [o.cpu().numpy() for o in outs]
    # the graph is destroyed: its workspace can go (kf_release_retired), once
    del g
    assert kf.release_retired() > 0 and kf.release_retired() == 0
    run(kf, 3 * T)           # the grown workspace is still the handle's
    torch.cuda.synchronize()
    kf.close()
    np.testing.assert_array_equal(got[3], eager[3])
    live = np.arange(T)[:, None] < eager[3][None, :]
    for a, b in zip(got[:3], eager[:3]):
        m = live[:, None, :] if a.ndim == 3 else live
        np.testing.assert_array_equal(np.where(m, a, 0.0), np.where(m, b, 0.0))


def test_score_candidates_random_batch():
    """kf_score_candidates over a batch of random block-diagonal covariances vs the oracle's
    Scheduler.cov_matrix trace (first row and full)."""
    rng = np.random.default_rng(3)
    B = 130
    Ps = []
    for _ in range(B):
        P = np.zeros((15, 15))
        for idx in [(0, 6, 12), (1, 7, 13), (2, 8, 14), (3, 9), (4, 10), (5, 11)]:  # the axis chains
            A = rng.normal(size=(len(idx), len(idx)))
            P[np.ix_(idx, idx)] = A @ A.T + np.eye(len(idx)) * rng.uniform(0.1, 100)
        Ps.append(P)
    Ps = np.array(Ps)
    for full in (False, True):
        gain = ref15.scheduler_gain(Ps, full=full)
        for b in range(0, B, 5):
            for ti, s in enumerate(('GPS', 'IMU')):
                R = ref_kf.R_gps15() if s == 'GPS' else ref_kf.R_imu15()
                H = ref_kf.H_gps15() if s == 'GPS' else ref_kf.H_imu15()
                rows = list(range(1, R.shape[0] + 1)) if full else [1]
                want = np.trace(ref_kf.scheduler_cov_matrix(rows, Ps[b], R, H))
                assert abs(gain[b, ti] - want) <= TOL * max(1.0, abs(want)), (full, b, s)


def test_sharded_brute_force_single_rank(golden_dir):
    """kfmi.dist.brute_force_search with the GPU evaluator on a world-1 group gives the
    reference's winner (the gloo world-2 logic is covered in tests/test_dist_gloo.py)."""
    import socket
    import torch.distributed as dist
    from kfmi import dist as kdist
    g = _load(golden_dir, 'ref15_bruteforce.npz')
    events = unpack_events(g)
    s, e = int(g['start']), int(g['end'])
    sk = socket.socket()
    sk.bind(('127.0.0.1', 0))
    port = sk.getsockname()[1]
    sk.close()
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    try:
        out = kdist.brute_force_search(events, s, e, R_threshold=float(g['threshold']), initial_pt=g['init_P'],
                                       initial_state=tuple(g['init_state']))
    finally:
        dist.destroy_process_group()
    cand = events[s:e]
    assert [cand.index(ev) for ev in out['selected_sensors']] == list(g['selected'])
    assert _rel(out['log_determinants'], g['log_determinants']) <= TOL


def test_search_full_size_sampled_vs_per_subset():
    """The bench's full-size search (n = 25, all 2^25 - 1 subsets, exhaustive) against the
    per-subset kernel: every subset of the smallest and largest sizes, and a 4096-subset window
    of each middle size, compared through the search's subset_max (≤ 1e-12)."""
    rng = np.random.default_rng(2025)
    n = 25
    t0 = 1697739552.3362827
    ev = np.zeros((n, 11))
    ev[:, 0] = t0 + 0.005 * np.arange(1, n + 1)
    ev[:, 1] = 1
    ev[::20, 1] = 0
    ev[:, 2:5] = rng.normal(0, 0.05, (n, 3))
    ev[:, 5:8] = rng.normal(0, 0.01, (n, 3))
    ev[:, 8:11] = rng.normal(0, 0.3, (n, 3))
    ev[ev[:, 1] == 0, 2:5] = rng.normal(0, 3, (int((ev[:, 1] == 0).sum()), 3))
    Pw = np.diag([0.9, 0.9, 0.9, 0.02, 0.02, 0.02, 0.5, 0.5, 0.5, 0.05, 0.05, 0.05, 20.0, 20.0, 20.0])
    init = np.concatenate([np.zeros(15), ref15.to_blocks(Pw)])
    t_end = t0 + 0.005 * (n + 1)
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    kfound, _, acc, sm = kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True, subset_max=True)
    kf.close()
    assert kfound == 0 and int(acc.sum()) == 0
    sm = sm.cpu().numpy()
    assert np.isnan(sm[0]) and np.isfinite(sm[1:]).all()
    W = 4096
    for k in range(1, n + 1):
        total = math.comb(n, k)
        off = 0 if total <= W else int(rng.integers(0, total - W))
        cnt = min(W, total)
        kc = kfmi.BatchedKF('ref15', cnt, 'f64')
        mx, _, _ = kc.eval_combos(ev, init, t0, t_end, k, combo_offset=off, logdets=False)
        mx = mx.cpu().numpy()
        kc.close()
        masks = np.array([sum(1 << i for i in ref15.unrank_combination(n, k, off + r)) for r in range(cnt)])
        got = sm[masks]
        assert np.max(np.abs(got - mx) / np.maximum(np.abs(mx), 1.0)) <= 1e-12, k


# The ref15 / ref15f32 / sched rows at their bench sizes against the oracle (>= 4096 filters plus
# the wave and batch edges): tests/test_gpu_bench_parity.py


def test_scheduled_random_long_log_stream_route(tmp_path):
    """The random arm over a whole drive log (the config-1 CSVs, 50 Hz: ~146k picks, beyond
    kf_run_events' one-filter time-parallel threshold of 65,536 events, so its leading padding
    event goes through kf_run_stream): with np.random seeded alike the picks are the
    same, the states and log-dets equal the single filter's over the same picked events
    (parallel=False) at roundoff, and the global generator ends at the same place."""
    import bench
    from kfmi import ingest
    from kfmi.kf_workers import EventList
    gp, ip = bench.synth_log(bench.CONFIGS['1'], str(tmp_path))
    stream = ingest.ingest_arrays(ingest.read_csv(gp, 4), ingest.read_csv(ip, 11), device=0)
    ev = EventList(stream)
    out = []
    for par in (True, False):
        np.random.seed(3)
        st, ld, P = ref15.run_kalman_filter_scheduled(ev, None, None, None, None, 'random', 50.0, parallel=par)
        out.append((np.array(st), np.array(ld), P, np.random.random()))
    (s1, l1, P1, r1), (s2, l2, P2, r2) = out
    assert len(s1) == len(s2) > 65536 + 1 and r1 == r2
    np.testing.assert_array_equal(s1[:, 0], s2[:, 0])        # the picked times
    rel = lambda a, b: float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0)))  # noqa: E731
    assert rel(s1[:, 1:], s2[:, 1:]) <= 1e-9 and rel(l1, l2) <= 1e-9 and rel(P1, P2) <= 1e-9
