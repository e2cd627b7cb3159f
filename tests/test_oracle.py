"""Pin the CPU oracle (oracle/ref_kf.py) against the reference's own outputs.

The fixtures in tests/golden/ were produced by importing the reference
(tests/golden/make_golden.py); these tests need no GPU and no reference checkout.
"""
import os

import numpy as np
import pytest

from oracle import ref_kf
from golden_events import unpack_events

RTOL = 1e-12


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0)))


def test_kat_logdet_p0():
    # slogdet of kf_workers.py:651's P0 = 6 ln 1e4 + 9 ln 1e3
    ld = np.linalg.slogdet(ref_kf.P0_REF15)[1]
    assert abs(ld - 117.43183974269634) < 1e-12
    assert abs(ld - (6 * np.log(1e4) + 9 * np.log(1e3))) < 1e-12


def test_ref15_full_cold_start(golden_dir):
    g = _load(golden_dir, 'ref15_full.npz')
    events = unpack_events(g)
    st, ld, P, prev = ref_kf.run_kalman_filter_full(events, 0, len(events))
    assert np.array(st).shape == g['cold_states'].shape
    assert _rel(st, g['cold_states']) < RTOL
    assert _rel(ld, g['cold_logdets']) < RTOL
    assert _rel(P, g['cold_P']) < RTOL
    assert prev == float(g['cold_prev_time'])


def test_ref15_full_warm_start(golden_dir):
    g = _load(golden_dir, 'ref15_full.npz')
    events = unpack_events(g)
    s0 = int(g['warm_start'])
    st, ld, P, _ = ref_kf.run_kalman_filter_full(events, s0, s0 + 60, initial_pt=g['warm_init_P'].copy(),
                                                 initial_state=tuple(g['warm_init_state']))
    assert _rel(st, g['warm_states']) < RTOL
    assert _rel(ld, g['warm_logdets']) < RTOL
    assert _rel(P, g['warm_P']) < RTOL


def test_ref15_adaptive_threshold(golden_dir):
    g = _load(golden_dir, 'ref15_full.npz')
    events = unpack_events(g)
    st, ld, P, prev, times = ref_kf.run_adaptive_threshold(events, 0, len(events),
                                                           R_threshold=float(g['adapt_threshold']))
    assert _rel(st, g['adapt_states']) < RTOL
    assert _rel(ld, g['adapt_logdets']) < RTOL
    assert _rel(P, g['adapt_P']) < RTOL
    np.testing.assert_array_equal(np.array(times), g['adapt_times'])


def test_ref15_combo_worker(golden_dir):
    g = _load(golden_dir, 'ref15_combos.npz')
    cand = unpack_events(g)
    chunk = [tuple(cand[i] for i in row if i >= 0) for row in g['combo_idx']]
    res = ref_kf.evaluate_combo_chunk(chunk, g['x0'], g['P0'], float(g['prev_time']), float(g['target_end']))
    ld_flat = [v for r in res for v in r[5]]
    tr_flat = [v for r in res for v in r[1]]
    assert _rel(ld_flat, g['logdet_flat']) < RTOL
    assert _rel(tr_flat, g['traj_flat']) < RTOL
    assert _rel([r[3] for r in res], g['x_final']) < RTOL
    off = g['offsets']
    assert [len(r[5]) for r in res] == list(np.diff(off))


def test_ref8_full(golden_dir):
    g = _load(golden_dir, 'ref8_full.npz')
    events = unpack_events(g)
    st, _ = ref_kf.run_kalman_filter_8state(events)
    assert _rel(st, g['states']) < RTOL
    st, _ = ref_kf.run_kalman_filter_8state(unpack_events(g, 'ooo_'))
    assert _rel(st, g['ooo_states']) < RTOL


@pytest.mark.parametrize('prefix', ['', 'ooo_'])
def test_ref8_dead_reckoning(golden_dir, prefix):
    """hw5_2.run_dead_reckoning_for_IMU (hw5_2.py:382-436): the restatement against the
    reference's own output, in-order and out-of-order (a negative IMU-to-IMU dt) streams."""
    g = _load(golden_dir, 'ref8_full.npz')
    events = unpack_events(g, prefix)
    st, _ = ref_kf.run_dead_reckoning_8state(events)
    want = g[prefix + 'dr_states']
    assert len(st) == len(want) == sum(e[1] == 'IMU' for e in events)
    assert _rel(st, want) < RTOL


def test_ref15_run_kalman_filter_simple(golden_dir):
    g = _load(golden_dir, 'ref15_drivers.npz')
    events = unpack_events(g)
    st, covs = ref_kf.run_kalman_filter_simple(events, 0, len(events))
    assert _rel(st, g['simple_states']) < RTOL
    assert _rel(covs, g['simple_covs']) < RTOL
    s0, e0 = (int(v) for v in g['simple_win'])
    st, covs = ref_kf.run_kalman_filter_simple(events, s0, e0)
    assert _rel(st, g['simple_win_states']) < RTOL
    assert _rel(covs, g['simple_win_covs']) < RTOL


def test_ref15_no_update(golden_dir):
    g = _load(golden_dir, 'ref15_drivers.npz')
    events = unpack_events(g)
    st, ld, P, prev, mt = ref_kf.run_no_update(events, 0, len(events))
    assert _rel(st, g['noupd_states']) < RTOL
    assert _rel(ld, g['noupd_logdets']) < RTOL
    assert _rel(P, g['noupd_P']) < RTOL
    assert prev == float(g['noupd_prev'])
    np.testing.assert_array_equal(mt, g['noupd_mtimes'])
    st, ld, P, prev, mt = ref_kf.run_no_update(events, 60, 100, initial_pt=g['noupd_warm_P0'],
                                               initial_state=tuple(g['noupd_warm_state0']))
    assert _rel(st, g['noupd_warm_states']) < RTOL
    assert _rel(ld, g['noupd_warm_logdets']) < RTOL
    assert _rel(P, g['noupd_warm_P']) < RTOL
    assert mt == []


@pytest.mark.parametrize('d', [2, 3])
@pytest.mark.parametrize('k', [1, 5])
def test_cv_batch_and_loop(golden_dir, d, k):
    g = _load(golden_dir, 'cv_batch.npz')
    key = f'cv{d}_k{k}'
    model = ref_kf.CVModel(d)
    dt, u, z, x0, P0 = (g[f'{key}_{s}'] for s in ('dt', 'u', 'z', 'x0', 'P0'))
    np.testing.assert_array_equal(P0, model.P0())
    traj, ld, x, P = ref_kf.run_batch(model, x0, P0, dt, u, z, update_every=k)
    assert _rel(traj, g[f'{key}_traj']) < RTOL
    assert _rel(ld, g[f'{key}_logdet']) < RTOL
    assert _rel(P, g[f'{key}_Pfinal']) < RTOL
    for b in (0, x0.shape[0] - 1):
        tl, ll, _, Pl = ref_kf.run_filter_loop(model, x0[b], P0, dt, u[:, :, b], z[:, :, b], update_every=k)
        assert _rel(tl, g[f'{key}_traj'][:, :, b]) < RTOL
        assert _rel(ll, g[f'{key}_logdet'][:, b]) < RTOL
        assert _rel(Pl, g[f'{key}_Pfinal'][b]) < RTOL


def test_tri_pack_roundtrip():
    rng = np.random.default_rng(0)
    A = rng.normal(size=(5, 6, 6))
    P = A @ A.transpose(0, 2, 1)
    back = ref_kf.tri_unpack(ref_kf.tri_pack(P), 6)
    np.testing.assert_array_equal(back, P)


def test_batch_mask_skips_update():
    model = ref_kf.CV3
    rng = np.random.default_rng(1)
    B, T = 4, 6
    x0 = rng.normal(size=(B, 6))
    dt = np.full(T, 0.1)
    u = rng.normal(size=(T, 3, B))
    z = rng.normal(size=(T, 3, B))
    mask = np.ones((T, B), bool)
    mask[:, 2] = False
    tr, ld, _, _ = ref_kf.run_batch(model, x0, model.P0(), dt, u, z, 1, mask=mask)
    # a never-updated filter is pure prediction
    tr_pred, ld_pred, _, _ = ref_kf.run_batch(model, x0[2:3], model.P0(), dt, u[:, :, 2:3], z[:, :, 2:3],
                                              update_every=T + 1)
    np.testing.assert_allclose(tr[:, :, 2], tr_pred[:, :, 0], rtol=1e-14)
    np.testing.assert_allclose(ld[:, 2], ld_pred[:, 0], rtol=1e-14)


def test_ref15_bruteforce_search(golden_dir):
    g = _load(golden_dir, 'ref15_bruteforce.npz')
    events = unpack_events(g)
    s, e = int(g['start']), int(g['end'])
    out = ref_kf.run_brute_force(events, s, e, float(g['threshold']), g['init_P'], tuple(g['init_state']))
    cand = events[s:e]
    assert [cand.index(ev) for ev in out['selected_sensors']] == list(g['selected'])
    assert _rel(out['log_determinants'], g['log_determinants']) < RTOL
    assert _rel(out['final_state'], g['final_state']) < RTOL
    assert _rel(out['trajectory'], g['trajectory']) < RTOL


@pytest.mark.parametrize('f', [20, 50, 120])
def test_ref15_scheduled_greedy(golden_dir, f):
    g = _load(golden_dir, 'ref15_scheduled.npz')
    events = unpack_events(g)
    st, ld, P = ref_kf.run_kalman_filter_scheduled(events, 0, len(events), selection_method='greedy',
                                                   processing_frequency=f)
    assert np.array(st).shape == g[f'greedy{f}_states'].shape
    assert _rel(st, g[f'greedy{f}_states']) < RTOL
    assert _rel(ld, g[f'greedy{f}_logdets']) < RTOL
    assert _rel(P, g[f'greedy{f}_P']) < RTOL


def test_ref15_scheduled_random_and_warm(golden_dir):
    g = _load(golden_dir, 'ref15_scheduled.npz')
    events = unpack_events(g)
    np.random.seed(int(g['random50_seed']))
    st, ld, P = ref_kf.run_kalman_filter_scheduled(events, 0, len(events), selection_method='random',
                                                   processing_frequency=50)
    assert _rel(st, g['random50_states']) < RTOL
    assert _rel(ld, g['random50_logdets']) < RTOL
    st, ld, P = ref_kf.run_kalman_filter_scheduled(events, 60, 180, initial_pt=g['warm_init_P'],
                                                   initial_state=tuple(g['warm_init_state']),
                                                   selection_method='greedy', processing_frequency=100)
    assert _rel(st, g['warm_states']) < RTOL
    assert _rel(ld, g['warm_logdets']) < RTOL
    assert _rel(P, g['warm_P']) < RTOL


def test_scheduler_gain_and_cov_matrix(golden_dir):
    g = _load(golden_dir, 'ref15_scheduled.npz')
    for si, S in enumerate(g['sched_sigma']):
        for ti, s in enumerate(('GPS', 'IMU')):
            R = ref_kf.R_gps15() if s == 'GPS' else ref_kf.R_imu15()
            H = ref_kf.H_gps15() if s == 'GPS' else ref_kf.H_imu15()
            assert _rel(ref_kf.scheduler_gain(s, S), g['sched_gain'][si, ti]) < RTOL
            assert _rel(ref_kf.scheduler_cov_matrix([1], S, R, H), g['sched_cov_first'][si, ti]) < RTOL
            full = list(range(1, R.shape[0] + 1))
            assert _rel(ref_kf.scheduler_cov_matrix(full, S, R, H), g['sched_cov_full'][si, ti]) < RTOL


# ---- the C restatement (oracle/cpu_kf.c): the CPU baseline's engine, pinned here ---------

@pytest.fixture(scope='module')
def cpu_kf():
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(['make', '-C', os.path.join(root, 'oracle')], check=True, capture_output=True)
    from oracle import cpu_kf as ck
    return ck


@pytest.mark.parametrize('d', [2, 3])
@pytest.mark.parametrize('k', [1, 5])
def test_c_restatement_vs_goldens(golden_dir, cpu_kf, d, k):
    """The C port reproduces the reference-generated BASELINE goldens (cv_batch.npz)."""
    g = _load(golden_dir, 'cv_batch.npz')
    key = f'cv{d}_k{k}'
    dt, u, z, x0, P0 = (g[f'{key}_{s}'] for s in ('dt', 'u', 'z', 'x0', 'P0'))
    tr, ld, x, P = cpu_kf.cv_run(d, x0.T, P0, dt, u, z, k)   # irregular dt: a zero and a 1.7x step
    assert _rel(tr, g[f'{key}_traj']) < 1e-10
    assert _rel(ld, g[f'{key}_logdet']) < 1e-10
    assert _rel(P, g[f'{key}_Pfinal']) < 1e-10


def test_c_restatement_vs_numpy_oracle(cpu_kf):
    rng = np.random.default_rng(3)
    for d, k in ((2, 1), (3, 1), (3, 10)):
        model = ref_kf.CV2 if d == 2 else ref_kf.CV3
        B, T = 9, 40
        x0 = rng.normal(0, 100, (B, 2 * d))
        u = rng.normal(0, 0.3, (T, d, B))
        z = rng.normal(0, 30, (T // k, d, B))
        tr, ld, x, P = cpu_kf.cv_run(d, x0.T, model.P0(), 0.1, u, z, k)
        rt, rl, rx, rP = ref_kf.run_batch(model, x0, model.P0(), np.full(T, 0.1), u, z, k)
        assert _rel(tr, rt) < 1e-10 and _rel(ld, rl) < 1e-10 and _rel(P, rP) < 1e-10


def test_c_ref15_events_vs_numpy_oracle(cpu_kf):
    rng = np.random.default_rng(4)
    B, T = 7, 50
    etype = rng.choice([0, 1, 1, 2, 255], size=(T, B)).astype(np.uint8)
    dt = rng.uniform(0, 0.05, (T, B))
    pay = rng.normal(0, 1, (T, 9, B)) * np.array([20, 20, 20, .05, .05, .05, .5, .5, .5])[None, :, None]
    x0 = rng.normal(0, 5, (15, B))
    tr, ld = cpu_kf.ref15_events(etype, dt, pay, x0, ref_kf.P0_REF15)
    for f in range(B):
        x, P = x0[:, f].copy(), ref_kf.P0_REF15.copy()
        for t in range(T):
            ty = etype[t, f]
            if ty == 2:
                F = ref_kf.F_ref15(dt[t, f])
                x, P = F @ x, ref_kf.predict_covariance(P, F, ref_kf.Q_ref15(dt[t, f]))
            elif ty in (0, 1):
                sd = ({'easting': pay[t, 0, f], 'northing': pay[t, 1, f], 'altitude': pay[t, 2, f]} if ty == 0
                      else ['t', *pay[t, :, f]])
                x, P = ref_kf.step15(x, P, 'GPS' if ty == 0 else 'IMU', sd, dt[t, f])
            assert _rel(tr[t, :, f], x[:6]) < 1e-10
            assert abs(ld[t, f] - np.linalg.slogdet(P)[1]) < 1e-10 * max(1, abs(np.linalg.slogdet(P)[1]))


def test_hw5_2_facade_model_getters_match_the_oracle():
    """kfmi.hw5_2's host model getters (hw5_2.py:219-311) equal the oracle's 8-state model."""
    from kfmi import hw5_2 as khw5
    sf = object.__new__(khw5.KF_SensorFusion)  # host-only methods: no GPU, no data
    for dt in (0.0, 0.005, 0.1, 1.7):
        np.testing.assert_array_equal(sf.get_state_transition_matrix(dt), ref_kf.F_ref8(dt))
        np.testing.assert_array_equal(sf.get_process_noise_covariance_matrix(dt), ref_kf.Q_ref8(dt))
    np.testing.assert_array_equal(sf.get_gps_observation_matrix(), ref_kf.H_gps8())
    np.testing.assert_array_equal(sf.get_imu_observation_matrix(), ref_kf.H_imu8())
    np.testing.assert_array_equal(sf.get_gps_measurement_noise_covariance_matrix(), ref_kf.R_gps8())
    np.testing.assert_array_equal(sf.get_imu_measurement_noise_covariance_matrix(), ref_kf.R_imu8())
    rng = np.random.default_rng(3)
    A = rng.normal(size=(8, 8))
    P = A @ A.T + 8 * np.eye(8)
    H, R = ref_kf.H_gps8(), ref_kf.R_gps8()
    np.testing.assert_array_equal(sf.calculate_kalman_gain(P, H, R), ref_kf.calculate_kalman_gain(P, H, R))
    F, Q = ref_kf.F_ref8(0.1), ref_kf.Q_ref8(0.1)
    np.testing.assert_array_equal(sf.predict_covariance(P, F, Q), ref_kf.predict_covariance(P, F, Q))


def test_numpy_pool_runs_the_reference_loop_on_all_workers():
    """bench.py's all-core NumPy baseline (oracle/numpy_pool.py): every worker runs its own
    shard of filters through the reference-order loop and the rates add up."""
    from oracle import numpy_pool
    rng = np.random.default_rng(0)
    T, nf = 16, 6
    shards = [dict(d=3, x0=rng.normal(0, 100, (6, nf)), P0=ref_kf.CV3.P0(), R=None, dt=0.1, k=1, n=nf,
                   u=rng.normal(0, 0.3, (T, 3, nf)), z=rng.normal(0, 30, (T, 3, nf))) for _ in range(2)]
    out = numpy_pool.run('cv', shards, seconds=30.0)
    assert out['cores'] == 2 and out['filters'] == 2 * nf and out['units'] == 2 * nf * T
    assert out['value'] > 0
    assert numpy_pool.split(10, 3) == [(0, 4), (4, 7), (7, 10)]
    # the scheduled kind (its streams carry their own t0: the worker's clock must not be it)
    T, nf, t0 = 40, 3, 1697739278.761565
    et = np.ones((T, nf), np.uint8)
    et[9::10] = 0
    sched = [dict(et=et, t=t0 + 0.005 * np.arange(1, T + 1)[:, None] + np.zeros((1, nf)),
                  pay=rng.normal(0, 0.1, (T, 9, nf)), freq=np.array([20.0, 50.0, 120.0]), t0=t0, n=nf)
             for _ in range(2)]
    out = numpy_pool.run('sched', sched, seconds=30.0)
    assert out['filters'] == 2 * nf and out['units'] == 2 * nf * T
    assert 0 < out['seconds'] < 30 and out['value'] > 0


def _events_to_columns(events):
    """Event tuples -> one filter's columns: t [T, 1], etype [T, 1], payload [T, 9, 1]."""
    T = len(events)
    t, et, pay = np.zeros((T, 1)), np.zeros((T, 1), np.uint8), np.zeros((T, 9, 1))
    for i, (_, s, ti, sd) in enumerate(events):
        t[i, 0] = ti
        if s == 'GPS':
            pay[i, 0:3, 0] = sd['easting'], sd['northing'], sd['altitude']
        else:
            et[i, 0] = 1
            pay[i, :, 0] = sd[1:]
    return t, et, pay


@pytest.mark.parametrize('f', [20, 50, 120])
def test_c_ref15_sched_vs_goldens(golden_dir, cpu_kf, f):
    """oracle/cpu_kf.c's greedy scheduled driver reproduces the reference's own
    run_kalman_filter_scheduled outputs (ref15_scheduled.npz): the cold start as a warm start
    from the first fix (kf_workers.py:866-880), and the reference's warm-start window."""
    g = _load(golden_dir, 'ref15_scheduled.npz')
    events = unpack_events(g)
    first = next(i for i, e in enumerate(events) if e[1] == 'GPS')
    sd = events[first][3]
    x0 = np.array([[sd['easting']], [sd['northing']], [sd['altitude']], [0.0], [0.0], [0.0]])
    t, et, pay = _events_to_columns(events[first + 1:])
    st, tr, ld, ns = cpu_kf.ref15_sched(t, et, pay, [events[first][2]], [float(f)], ref_kf.P0_REF15, x0=x0)
    want = g[f'greedy{f}_states']
    n = int(ns[0])
    assert n == len(want) - 1
    assert _rel(st[:n, 0], want[1:, 0]) == 0.0
    assert _rel(tr[:n, :, 0], want[1:, 1:7]) < 1e-10
    assert _rel(ld[:n, 0], g[f'greedy{f}_logdets'][1:]) < 1e-10
    if f == 120:
        s0 = tuple(g['warm_init_state'])
        t, et, pay = _events_to_columns(events[61:180])
        st, tr, ld, ns = cpu_kf.ref15_sched(t, et, pay, [s0[0]], [100.0], g['warm_init_P'],
                                            x0=np.array(s0[1:7])[:, None])
        want = g['warm_states']
        n = int(ns[0])
        assert n == len(want) - 1
        assert _rel(tr[:n, :, 0], want[1:, 1:7]) < 1e-10
        assert _rel(ld[:n, 0], g['warm_logdets'][1:]) < 1e-10


def test_c_ref15_sched_vs_numpy_oracle(cpu_kf):
    """Random jittered streams, per-filter rates (window edges, empty-queue triggers, fixes and
    IMU samples queued together): every pick, time, state and log-det of the C driver equals
    the NumPy restatement's (oracle/ref_kf.run_kalman_filter_scheduled, greedy)."""
    rng = np.random.default_rng(11)
    B, T, t0 = 12, 120, 1697739278.761565
    et = (rng.random((T, B)) > 0.12).astype(np.uint8)
    t = t0 + np.cumsum(rng.uniform(0.001, 0.02, (T, B)), axis=0)
    pay = rng.normal(0, 1, (T, 9, B)) * np.array([20, 20, 20, .05, .05, .05, .5, .5, .5])[None, :, None]
    freq = rng.choice([5.0, 20.0, 50.0, 120.0, 400.0], B)
    x0 = rng.normal(0, 3, (6, B))
    st, tr, ld, ns = cpu_kf.ref15_sched(t, et, pay, np.full(B, t0), freq, ref_kf.P0_REF15, x0=x0, nthreads=2)
    for f in range(B):
        ev = [(0, 'GPS', t0, {'easting': 0.0, 'northing': 0.0, 'altitude': 0.0})]
        for i in range(T):
            ev.append((i + 1, 'GPS', t[i, f], {'easting': pay[i, 0, f], 'northing': pay[i, 1, f],
                                                'altitude': pay[i, 2, f]}) if et[i, f] == 0
                      else (i + 1, 'IMU', t[i, f], ['t', *pay[i, :, f]]))
        rs, rl, _ = ref_kf.run_kalman_filter_scheduled(ev, 0, len(ev), ref_kf.P0_REF15.copy(),
                                                       (t0, *x0[:, f]), 'greedy', float(freq[f]))
        n = int(ns[f])
        assert n == len(rs) - 1 and n > 3, f
        assert _rel(st[:n, f], [r[0] for r in rs[1:]]) == 0.0
        assert _rel(tr[:n, :, f], np.array([r[1:7] for r in rs[1:]])) < 1e-10
        assert _rel(ld[:n, f], rl[1:]) < 1e-10


def ref8_columns(events):
    """hw5_2.run_kalman_filter's stream (hw5_2.py:332-379) as one filter's columns: events from
    the first GPS fix on (that fix at dt = 0), dt = t - previous t with no dt < 0 guard."""
    first = next(i for i, e in enumerate(events) if e[1] == 'GPS')
    ev = events[first:]
    t, et, pay = _events_to_columns([(i, s, ti, sd) for (i, s, ti, sd) in ev])
    dt = t - np.r_[t[:1], t[:-1]]
    return et, dt, pay


@pytest.mark.parametrize('prefix', ['', 'ooo_'])
def test_c_ref8_events_vs_goldens(golden_dir, cpu_kf, prefix):
    """oracle/cpu_kf.c's 8-state model reproduces the reference's hw5_2.run_kalman_filter
    (ref8_full.npz, in-order and out-of-order streams) and the NumPy restatement's log-dets."""
    g = _load(golden_dir, 'ref8_full.npz')
    events = unpack_events(g, prefix)
    et, dt, pay = ref8_columns(events)
    tr, ld = cpu_kf.ref8_events(et, dt, pay, np.zeros((8, 1)), ref_kf.P0_REF8)
    want = g[prefix + 'states']
    assert tr.shape[0] == len(want) - 1
    assert _rel(tr[:, :, 0], want[1:]) < 1e-10
    x, P = np.zeros(8), ref_kf.P0_REF8.copy()
    for i in range(len(et)):
        s = 'GPS' if et[i, 0] == 0 else 'IMU'
        sd = {'easting': pay[i, 0, 0], 'northing': pay[i, 1, 0]} if s == 'GPS' else ['t', *pay[i, :, 0]]
        x, P = ref_kf.step8(x, P, s, sd, dt[i, 0])
        assert abs(ld[i, 0] - np.linalg.slogdet(P)[1]) < 1e-10 * max(1.0, abs(np.linalg.slogdet(P)[1]))


@pytest.mark.parametrize('prefix', ['', 'ooo_'])
def test_c_ref8_dead_reckoning_vs_goldens(golden_dir, cpu_kf, prefix):
    """oracle/cpu_kf.c's dead-reckoning walk (cpu_ref8_dead_reckoning) over the merged stream
    reproduces the reference's hw5_2.run_dead_reckoning_for_IMU (ref8_full.npz) and the NumPy
    restatement's log-dets."""
    g = _load(golden_dir, 'ref8_full.npz')
    events = unpack_events(g, prefix)
    t, et, pay = _events_to_columns(events)
    tr, ld = cpu_kf.ref8_dead_reckoning(et[:, 0], t[:, 0], pay[:, :, 0])
    want = g[prefix + 'dr_states']
    assert tr.shape == want.shape
    assert _rel(tr, want) < 1e-10
    x, P, prev, k = np.zeros(8), ref_kf.P0_REF8.copy(), None, 0
    for (_, s, ti, sd) in events:
        if s != 'IMU':
            continue
        x, P = ref_kf.step8(x, P, 'IMU', sd, ti - prev if prev is not None else 0.0)
        prev = ti
        assert abs(ld[k] - np.linalg.slogdet(P)[1]) < 1e-10 * max(1.0, abs(np.linalg.slogdet(P)[1]))
        k += 1
    assert k == len(ld)
