"""Host-side logic of kfmi.ref15 (no GPU): block packing of the 15x15 covariance and the
combination unranking used by the brute-force search."""
import math
from itertools import combinations

import numpy as np
import pytest

from golden_events import unpack_events
from kfmi import ref15


def test_blocks_roundtrip_on_reference_covariances(golden_dir):
    g = np.load(f'{golden_dir}/ref15_full.npz')
    for key in ('cold_P', 'warm_P', 'adapt_P', 'warm_init_P'):
        P = g[key]
        # the reference's simple-form update leaves P asymmetric by ~1 ulp; packing keeps i <= j
        Psym = np.triu(P) + np.triu(P, 1).T
        np.testing.assert_array_equal(ref15.from_blocks(ref15.to_blocks(P)), Psym)
        np.testing.assert_allclose(Psym, P, rtol=1e-14, atol=1e-17)
    np.testing.assert_array_equal(ref15.from_blocks(ref15.to_blocks(ref15.P0)), ref15.P0)


def test_blocks_reject_cross_chain_coupling():
    P = ref15.P0.copy()
    P[0, 1] = P[1, 0] = 1e-3   # pos_x <-> pos_y couples two chains
    with pytest.raises(ValueError):
        ref15.to_blocks(P)
    P = ref15.P0.copy()
    P[0, 6] = P[6, 0] = 5.0    # pos_x <-> vel_x is inside a chain: fine
    assert ref15.to_blocks(P)[1] == 5.0


@pytest.mark.parametrize('n,k', [(5, 1), (8, 3), (12, 6), (25, 12)])
def test_unrank_matches_itertools(n, k):
    total = math.comb(n, k)
    ranks = list(range(min(total, 300))) + [total // 2, total - 1]
    allc = None
    if total <= 5000:
        allc = list(combinations(range(n), k))
    for r in ranks:
        got = ref15.unrank_combination(n, k, r)
        if allc is not None:
            assert tuple(got) == allc[r]
        assert sorted(got) == got and len(set(got)) == k and got[-1] < n


def test_event_payload_layout(golden_dir):
    events = unpack_events(np.load(f'{golden_dir}/ref15_full.npz'))
    gps = next(e for e in events if e[1] == 'GPS')
    imu = next(e for e in events if e[1] == 'IMU')
    assert ref15.event_payload('GPS', gps[3])[:3] == [gps[3]['easting'], gps[3]['northing'], gps[3]['altitude']]
    assert ref15.event_payload('IMU', imu[3]) == [float(v) for v in imu[3][1:10]]


def test_empty_warm_window_returns_none(golden_dir):
    """A warm start over an empty window (start_idx >= end_idx) has no candidate: the
    reference's size loop never runs and it returns None (kf_workers.py:1325, 1391); so do the
    single-GPU search and both sharded searches, before any device work."""
    import socket

    import torch.distributed as dist

    from kfmi import dist as kdist
    events = unpack_events(np.load(f'{golden_dir}/ref15_bruteforce.npz'))
    st = (events[5][2], 1.0, 2.0, 3.0, 0.0, 0.0, 0.0)
    kw = dict(R_threshold=0.0, initial_pt=ref15.P0, initial_state=st)
    assert ref15.brute_force_setup(events, 10, 10, ref15.P0, st) is None
    assert ref15.run_brute_force_kalman_filter_no_sampling_min_usage(events, 10, 10, **kw) is None
    assert ref15.run_brute_force_kalman_filter_no_sampling_min_usage(events, 12, 10, **kw) is None
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    dist.init_process_group('gloo', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1)
    try:
        assert kdist.brute_force_search(events, 10, 10, **kw) is None
        assert kdist.brute_force_search_ranks(events, 10, 10, **kw) is None
    finally:
        dist.destroy_process_group()


def test_greedy_schedule_empty_queue_raises():
    """Scheduler.greedy_schedule on an empty queue: the reference ends in
    measurements.index(None), a ValueError (kf_workers.py:213)."""
    from kfmi.kf_workers import Scheduler
    with pytest.raises(ValueError, match='None is not in list'):
        Scheduler().greedy_schedule([], ref15.P0, None, None)


def test_euler_to_rotation_matrix_composition():
    """kf_workers.py:441-458: R = Rz(yaw) Ry(pitch) Rx(roll), a proper rotation."""
    from kfmi import kf_workers as kfw
    sf = object.__new__(kfw.KF_SensorFusion)  # host-only method: no GPU, no data
    a = 0.7
    np.testing.assert_allclose(sf.euler_to_rotation_matrix(0.0, 0.0, a),
                               [[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]], atol=1e-15)
    np.testing.assert_allclose(sf.euler_to_rotation_matrix(a, 0.0, 0.0),
                               [[1, 0, 0], [0, np.cos(a), -np.sin(a)], [0, np.sin(a), np.cos(a)]], atol=1e-15)
    R = sf.euler_to_rotation_matrix(0.1, -0.2, 0.3)
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-15)
    assert abs(np.linalg.det(R) - 1.0) < 1e-15
    # the x axis after a pitch then a yaw
    np.testing.assert_allclose(sf.euler_to_rotation_matrix(0.0, a, a) @ [1, 0, 0],
                               [np.cos(a) * np.cos(a), np.sin(a) * np.cos(a), -np.sin(a)], atol=1e-15)


# ------------------------------------------------------------------------------------------
# model constants (kf_params.ref_*): the class_args / getter replacements the engine accepts
# ------------------------------------------------------------------------------------------

def test_model_consts_reference_values():
    """kf_default_params for the reference models = the getters' constants (kf_workers.py:519-614,
    :651; hw5_2.py:233-304, :317-326); the reference's constants hand the handle no params."""
    from oracle import ref_kf
    c = ref15.ModelConsts('ref15')
    np.testing.assert_array_equal(c.Q(0.37), ref_kf.Q_ref15(0.37))
    np.testing.assert_array_equal(c.R_imu, ref_kf.R_imu15())
    np.testing.assert_array_equal(c.R_gps, ref_kf.R_gps15())
    np.testing.assert_array_equal(c.P0, ref_kf.P0_REF15)
    assert c.is_reference() and c.params() is None
    c8 = ref15.ModelConsts('ref8')
    np.testing.assert_array_equal(c8.Q(0.37), ref_kf.Q_ref8(0.37))
    np.testing.assert_array_equal(c8.R_imu, ref_kf.R_imu8())
    np.testing.assert_array_equal(c8.P0, ref_kf.P0_REF8)
    custom = ref15.ModelConsts('ref15', p0=np.r_[[1000.0] * 3, [100.0] * 9, [1000.0] * 3])  # KF_SensorFusion.ipynb:814
    p = custom.params()
    assert p is not None and list(p.ref_p0)[:3] == [1000.0] * 3 and list(p.ref_q)[:3] == [5.0] * 3


def test_model_consts_from_getters_accepts_diagonal_rejects_coupling():
    from kfmi import kf_workers as kw
    c = ref15.ModelConsts.from_matrices('ref15', F=kw._F, Q=kw._Q, H_gps=kw._H_GPS, H_imu=kw._H_IMU,
                                        R_gps=kw._R_GPS, R_imu=kw._R_IMU)
    assert c.is_reference()
    q2 = lambda dt: 2.0 * kw._Q(dt)
    c = ref15.ModelConsts.from_matrices('ref15', Q=q2, R_gps=np.diag([1.0, 2.0, 4.0]))
    np.testing.assert_array_equal(c.q, 2 * ref15.ModelConsts('ref15').q)
    np.testing.assert_array_equal(c.r_gps, [1.0, 2.0, 4.0])
    with pytest.raises(ValueError, match='off-diagonal'):
        R = np.diag([3.0, 3.0, 3.0])
        R[0, 1] = R[1, 0] = 0.5   # correlated GPS axes couple chains
        ref15.ModelConsts.from_matrices('ref15', R_gps=R)
    with pytest.raises(ValueError, match='diag'):
        ref15.ModelConsts.from_matrices('ref15', Q=lambda dt: kw._Q(dt) + np.eye(15) * 0.1)  # not q * dt
    with pytest.raises(ValueError, match='observation'):
        ref15.ModelConsts.from_matrices('ref15', H_gps=np.eye(15)[3:6])
    with pytest.raises(ValueError, match='transition'):
        ref15.ModelConsts.from_matrices('ref15', F=lambda dt: np.eye(15))
    with pytest.raises(ValueError):
        ref15.ModelConsts.from_matrices('ref15', R_imu=np.diag([0.0] + [1.0] * 14))


def test_class_args_worker_checks_formulas():
    from kfmi import kf_workers as kw
    bad = {'calculate_kalman_gain': lambda P, H, R: np.dot(P, H.T)}
    with pytest.raises(ValueError, match='calculate_kalman_gain'):
        kw._consts_of(bad)
    ok = {'predict_covariance': lambda P, F, Q: F @ P @ F.T + Q,
          'get_imu_measurement_noise_covariance_matrix': lambda: np.diag(np.arange(1.0, 16.0))}
    c = kw._consts_of(ok)
    np.testing.assert_array_equal(c.r_imu, np.arange(1.0, 16.0))


def legacy_choice_emulation(words, lens):
    """What kf_run_scheduled_random's legacy_choice does (kf_ref.hip), in Python: per window of
    n queued events, no output for n = 1, else outputs & (smallest 2^k - 1 >= n - 1) until one is
    <= n - 1.  Returns (draws, outputs taken)."""
    wp, out = 0, []
    for n in lens:
        rng = int(n) - 1
        if rng == 0:
            out.append(0)
            continue
        mask = rng
        for sh in (1, 2, 4, 8, 16):
            mask |= mask >> sh
        while True:
            v = int(words[wp]) & mask
            wp += 1
            if v <= rng:
                out.append(v)
                break
    return out, wp


def test_device_draws_reproduce_np_random_choice():
    """The random scheduled filter draws np.random.choice(len(queue)) on the device from the
    global generator's raw outputs (kfmi.ref15.legacy_words, read without advancing it); the
    masked rejection gives the reference's draws exactly (kf_workers.py:188-193), including queues
    of one (no draw) and sizes past 2^16, and advancing the generator by the outputs taken leaves
    it where the reference's calls leave it."""
    rng = np.random.default_rng(3)
    lens = np.r_[rng.integers(1, 300, 5000), [1, 1, 2, 65537, 3, 1 << 20, 1]]
    np.random.seed(77)
    words = ref15.legacy_words(3 * len(lens))
    got, taken = legacy_choice_emulation(words, lens)
    want = [np.random.choice(int(n)) for n in lens]
    after = np.random.random()
    assert got == want
    np.random.seed(77)
    np.testing.assert_array_equal(ref15.legacy_words(3 * len(lens)), words)   # reading does not advance
    np.random.randint(0, 1 << 32, size=taken, dtype=np.uint32)
    assert np.random.random() == after


def test_search_class_width_fits_every_size():
    """ref15.search_class_width: the fewest leading candidates whose 2^w classes kf_search_combos
    runs whole within the budget and the 2^28-parent cap — the reference's n = 40 window
    (kf_workers_visualizing.py:2293) takes 256 axis-symmetric classes of 32 free candidates,
    1024 every-chain classes of 30; n <= 30 needs none."""
    assert ref15.search_class_width(40, sym=True) == 8 and ref15.search_class_width(40) == 10
    for n in (12, 25, 30):
        assert ref15.search_class_width(n) == 0 and ref15.search_levels(n) == n
    for n in (33, 36, 40, 45):
        for sym in (False, True):
            w = ref15.search_class_width(n, sym=sym)
            assert ref15.search_levels(n - w, sym=sym) == n - w > ref15.search_levels(n - w + 1, sym=sym) - 1
            assert ref15.search_levels(n - w + 1, sym=sym) < n - w + 1       # one candidate fewer fixed: no
            m = n - w
            widest = max(math.comb(m - 2, k) for k in range(1, m - 1))
            assert 2 * ref15.search_level_bytes(widest, 'f64', sym) + 4096 <= 32 << 30
            assert all(math.comb(m - 2, k - 1) < 1 << 28 for k in range(2, m + 1))
    # the sharded plan never goes below the memory rule, nor below one class per rank dealt out
    # within 25 % of even
    from kfmi import dist as kdist
    assert kdist.search_classes(40, 8, sym=True) == 8 and kdist.search_classes(40, 1) == 10
    assert kdist.search_classes(25, 8) == 3 and kdist.search_classes(25, 1) == 0
    assert [kdist.search_classes(25, r) for r in (2, 3, 4, 5, 6, 7, 8, 16)] == [1, 3, 2, 3, 4, 5, 3, 4]
    for r in range(2, 33):
        c = 1 << kdist.search_classes(25, r)
        assert c >= r and -(-c // r) <= 1.25 * c / r


@pytest.mark.parametrize('w', [0, 1, 3, 5])
@pytest.mark.parametrize('exhaustive', [True, False])
def test_class_search_picks_the_reference_winner(w, exhaustive):
    """ref15.class_search over a random acceptance table: the smallest accepted size, then the
    first subset in itertools.combinations order (kf_workers.py:1325-1356), whatever the class
    order; not exhaustive, no class searches sizes that can no longer win and classes whose
    fixed members alone are too many are skipped."""
    n = 11
    rng = np.random.default_rng(5 + w)
    for trial in range(6):
        rate = [0.0, 0.001, 0.004, 0.02, 0.05, 0.2][trial]
        acc = {c: rng.random() < rate * len(c) for k in range(1, n + 1) for c in combinations(range(n), k)}
        calls = []

        def search_class(nf, c, k_max):
            calls.append((c, k_max))
            for k in range(1, k_max + 1):
                for x in combinations(range(n), k):
                    if sum(1 << i for i in x if i < nf) == c and acc[x]:
                        return k, x
            return 0, None
        want = next(((k, x) for k in range(1, n + 1) for x in combinations(range(n), k) if acc[x]), None)
        for order in (ref15.class_order(w), list(range(1 << w))[::-1]):
            calls.clear()
            k, key = ref15.class_search(search_class, n, w, order, exhaustive)
            got = None if k is ref15.NO_SIZE else (k, tuple(i for i in range(n) if (ref15.bitrev64(key) >> i) & 1))
            assert got == want, (w, trial, got, want)
            assert sorted(c for c, _ in calls) == (list(range(1 << w)) if exhaustive or want is None
                                                   else sorted(c for c, _ in calls))
            if not exhaustive and want:
                assert all(km >= want[0] for _, km in calls)
                assert all(bin(c).count('1') < km for c, km in calls)   # a class searched has a size to search


@pytest.mark.parametrize('w', [2, 4])
def test_class_search_size_cap(w):
    """class_search(k_max=K): the reference's pick among sizes 1..K only; no class is asked for
    more than one size past K, and none whose fixed members alone exceed K."""
    n = 10
    rng = np.random.default_rng(11)
    acc = {c: rng.random() < 0.01 * len(c) ** 2 for k in range(1, n + 1) for c in combinations(range(n), k)}
    for K in (1, 2, 3, 6):
        for exhaustive in (True, False):
            calls = []

            def search_class(nf, c, k_max):
                calls.append((c, k_max))
                for k in range(1, k_max + 1):
                    for x in combinations(range(n), k):
                        if sum(1 << i for i in x if i < nf) == c and acc[x]:
                            return k, x
                return 0, None
            want = next(((k, x) for k in range(1, K + 1) for x in combinations(range(n), k) if acc[x]), None)
            k, key = ref15.class_search(search_class, n, w, ref15.class_order(w), exhaustive, k_max=K)
            got = None if k is ref15.NO_SIZE else (k, tuple(i for i in range(n) if (ref15.bitrev64(key) >> i) & 1))
            assert got == want, (K, exhaustive, got, want)
            assert all(bin(c).count('1') <= K and km <= max(K, bin(c).count('1') + 1) for c, km in calls)


def _small_budget(n, want):
    """A level budget at which one call of n candidates holds sizes 1 .. want exactly."""
    for mem in range(8192, 1 << 30, 4096):
        if ref15.search_levels(n, 'f64', mem, True) == want:
            return mem
    raise AssertionError((n, want))


@pytest.mark.parametrize('n,k_done', [(13, 3), (14, 4), (15, 2), (16, 2)])
def test_prefix_classes_cover_every_subset_once(n, k_done):
    """ref15.prefix_classes: for the sizes up to K of a search whose one call holds sizes up to
    k_done, classes (n_fixed, prefix) that each fit one call for their sizes and hold every subset
    of sizes k_done + 1 .. K exactly once (the prefixes a split leaves out are of searched sizes);
    search_bands stops when they are no fewer than the fixed-pattern classes."""
    mem = _small_budget(n, k_done)
    for K in range(k_done + 1, min(n, 2 * k_done + 2)):
        classes, split = ref15.prefix_classes(n, K, 'f64', mem, True)
        assert split <= k_done and len(set(classes)) == len(classes)
        for nf, c in classes:
            p = bin(c).count('1')
            assert 0 <= nf < n and c >> nf == 0 and p < K
            assert ref15.search_levels(n - nf, 'f64', mem, True) >= min(K - p, n - nf)
        for k in range(1, K + 1):
            for x in combinations(range(n), k):
                m = sum(1 << i for i in x)
                hits = sum((m & ((1 << nf) - 1)) == c for nf, c in classes)
                assert hits == 1 or (k <= split and hits == 0), (K, x, hits)
    w = ref15.search_class_width(n, 'f64', mem, True)
    bands = list(ref15.search_bands(n, k_done, 'f64', mem, True, 1 << w))
    assert [K for K, _ in bands] == list(range(k_done + 1, k_done + 1 + len(bands)))
    assert all(len(c) < 1 << w for _, c in bands)


@pytest.mark.parametrize('n,k_done', [(12, 3), (13, 3), (15, 2), (16, 2)])
def test_search_past_picks_the_reference_winner(n, k_done):
    """ref15.search_past over random acceptance tables with nothing accepted up to k_done (what
    the one-call sizes found): the reference's pick — the smallest accepted size, then the first
    subset in itertools.combinations order — whether a band of prefix classes or the
    fixed-pattern classes decide it; every call is one kf_search_combos takes."""
    mem = _small_budget(n, k_done)
    w = ref15.search_class_width(n, 'f64', mem, True)
    rng = np.random.default_rng(n)
    for trial in range(8):
        rate = [0.0005, 0.002, 0.01, 0.05, 0.2, 0.0, 0.003, 0.02][trial]
        # the accepted subsets in the reference's order (size, then itertools order)
        order = [(k, x) for k in range(k_done + 1, n + 1) for x in combinations(range(n), k)
                 if rng.random() < rate * k]
        calls = []

        def search_class(nf, c, k_max):
            assert 0 <= nf < n and c >> nf == 0 and bin(c).count('1') < k_max <= n
            calls.append((nf, c, k_max))
            return next(((k, x) for k, x in order if k <= k_max and sum(1 << i for i in x if i < nf) == c),
                        (0, None))
        want = order[0] if order else None
        k, key = ref15.search_past(search_class, n, k_done, w, 'f64', mem, True)
        got = None if k is ref15.NO_SIZE else (k, tuple(i for i in range(n) if (ref15.bitrev64(key) >> i) & 1))
        assert got == want, (trial, got, want)
        if want and want[0] <= k_done + 2:  # decided by a band: no fixed-pattern class was searched
            bands = [K for K, _ in ref15.search_bands(n, k_done, 'f64', mem, True, 1 << w)]
            if want[0] in bands:
                assert all(nf != w or k_max <= want[0] for nf, _, k_max in calls)


def test_facade_reference_constants_read_once():
    """KF_SensorFusion._consts: with no getter replaced (class or instance) and the reference's
    P0, the drivers get the reference constants read once; a subclass getter, an instance
    getter or another P0 is read from the object each call, as before."""
    from kfmi import kf_workers as kfw

    def obj(cls=kfw.KF_SensorFusion):
        o = cls.__new__(cls)
        o.P0 = ref15.P0.copy()
        return o
    a = obj()
    c = a._consts()
    assert c.is_reference() and obj()._consts() is c

    class Sub(kfw.KF_SensorFusion):
        def get_gps_measurement_noise_covariance_matrix(self):
            return 5.0 * np.eye(3)
    assert not obj(Sub)._consts().is_reference()
    b = obj()
    b.P0[0, 0] = 7.0
    assert b._consts() is not c and not b._consts().is_reference()
    d = obj()
    d.get_process_noise_covariance_matrix = lambda dt: np.eye(15) * dt
    assert d._consts() is not c and not d._consts().is_reference()
