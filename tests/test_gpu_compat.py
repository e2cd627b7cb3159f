"""The drop-in modules kfmi.kf_workers / kfmi.hw5_2 used the way the reference's __main__ and
notebook use KF_SensorFusion (kf_workers.py:2256-2340), against the reference's goldens and
the oracle — needs an MI355X.  Tolerance: 1e-6 relative (north_star, fp64); ingest values as in
tests/test_gpu_ingest.py.
"""
import gzip
import os

import numpy as np
import pytest

from golden_events import unpack_events
from kfmi import hw5_2 as khw5
from kfmi import kf_workers as kfw
from oracle import ref_ingest, ref_kf

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0))) if a.size else 0.0


@pytest.fixture(scope='module')
def csvs(golden_dir, tmp_path_factory):
    d = tmp_path_factory.mktemp('compat')
    out = []
    for name in ('gps_synth.csv.gz', 'imu_synth.csv.gz'):
        p = d / name[:-3]
        with gzip.open(os.path.join(golden_dir, name), 'rt') as fi:
            p.write_text(fi.read())
        out.append(str(p))
    return out


def test_main_sequence(csvs, golden_dir, capsys):
    """load_data -> gps_to_modified_utm -> compute_imu_biases -> unbias_imu_data ->
    combine_sensor_data -> run_kalman_filter_full, as kf_workers.py:2256-2308 does."""
    g = np.load(os.path.join(golden_dir, 'ingest.npz'))
    sf = kfw.KF_SensorFusion(*csvs)
    sf.load_data()
    assert len(sf.gps_data) == 1500 and sf.gps_data[0][1] == 'nan'
    sf.gps_to_modified_utm()
    assert [u['time'] for u in sf.utm_data] == list(g['utm_time'])
    assert max(abs(u['easting'] - e) for u, e in zip(sf.utm_data, g['utm_easting'])) <= 1e-7
    bw, ba, fvi = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    assert fvi == int(g['first_valid_index'])
    np.testing.assert_array_equal(bw, g['gyro_bias'])
    np.testing.assert_array_equal(ba, g['accel_bias'])
    assert 'First valid GPS entry index: 300' in capsys.readouterr().out
    sf.unbias_imu_data(bw, ba)
    assert len(sf.unbias_imu_data) == 2500
    np.testing.assert_array_equal([r[4:10] for r in sf.unbias_imu_data[:50]], g['imu_values'][:50, 3:])
    # kf_workers.py:427-439 as the reference computes it, over the façade's rows
    rows = sf.unbias_imu_data[:fvi]
    ref_orient = tuple(np.mean([e[c] for e in rows]) for c in (1, 2, 3))
    assert sf.compute_stationary_orientation(fvi) == ref_orient
    R = sf.euler_to_rotation_matrix(*ref_orient)
    np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-15)
    sf.combine_sensor_data()
    ev = sf.indexed_sensor_data
    assert len(ev) == len(g['ev_time'])
    assert [e[1] == 'IMU' for e in ev[:400]] == list(g['ev_is_imu'][:400])
    st, ld, P, prev = sf.run_kalman_filter_full(start_idx=0, end_idx=len(ev))
    events, _, _ = ref_ingest.ingest(*csvs)
    rs, rl, rP, rprev = ref_kf.run_kalman_filter_full(events, 0, len(events))
    assert _rel(st, rs) <= 1e-6 and _rel(ld, rl) <= 1e-6 and _rel(P, rP) <= 1e-6 and prev == rprev
    assert sf.get_GT() is st
    assert len(sf._ground_truth_cov) == len(st)
    assert _rel(sf._ground_truth_cov[-1], rP) <= 1e-6
    # the adaptive driver on the façade's lazy event list
    s2, l2, P2, _, mt = sf.run_adaptive_threshold_kalman_filter(0, 600, R_threshold=float(np.median(rl)))
    r2, rl2, rP2, _, rmt = ref_kf.run_adaptive_threshold(events, 0, 600, R_threshold=float(np.median(rl)))
    assert _rel(s2, r2) <= 1e-6 and _rel(l2, rl2) <= 1e-6 and mt == rmt
    # GPS/IMU time ties make interp1d divide by zero in the reference too (NaN RMSE); the
    # metrics are post-processing of the outputs checked above
    m = sf.calculate_accuracy_metrics(s2)
    assert len(m['euclidean_errors']) == len(s2) and m['gt_start_time'] == s2[0][0]
    i = kfw.find_start_idx_for_time_offset(sf, -300.0)
    assert i == next(k for k, e in enumerate(events) if e[2] >= 1697739552.3362827 - 300.0)


def test_scheduler_facade(golden_dir):
    g = np.load(os.path.join(golden_dir, 'ref15_scheduled.npz'))
    sch = kfw.Scheduler()
    sf = kfw.KF_SensorFusion('', '')
    Rm = {'GPS': sf.get_gps_measurement_noise_covariance_matrix(), 'IMU': sf.get_imu_measurement_noise_covariance_matrix()}
    Hm = {'GPS': sf.get_gps_observation_matrix(), 'IMU': sf.get_imu_observation_matrix()}
    for si, S in enumerate(g['sched_sigma']):
        for ti, s in enumerate(('GPS', 'IMU')):
            assert _rel(sch.gain(('x', s), S, Rm, Hm), g['sched_gain'][si, ti]) <= 1e-6
            assert _rel(sch.cov_matrix([1], S, Rm[s], Hm[s]), g['sched_cov_first'][si, ti]) <= 1e-6
            full = list(range(1, Rm[s].shape[0] + 1))
            assert _rel(sch.cov_matrix(full, S, Rm[s], Hm[s]), g['sched_cov_full'][si, ti]) <= 1e-6
        q = [('a', 'IMU'), ('b', 'GPS'), ('c', 'IMU'), ('d', 'GPS')]
        want = ref_kf.greedy_schedule([(0, s, 0.0, None) for _, s in q], S)
        assert sch.greedy_schedule(q, S, Rm, Hm) == want
    # a caller's diagonal R is scored with its own constants (kf_workers.py:112-185 takes any
    # R); one that couples the axes is not (the engine's chains are independent)
    S0 = g['sched_sigma'][0]
    want = np.trace(ref_kf.scheduler_cov_matrix([1], S0, Rm['GPS'] * 2, Hm['GPS']))
    assert _rel(sch.gain(('x', 'GPS'), S0, {'GPS': Rm['GPS'] * 2}, Hm), want) <= 1e-6
    Rc = Rm['GPS'].astype(float)
    Rc[0, 1] = Rc[1, 0] = 0.5
    with pytest.raises(ValueError):
        sch.gain(('x', 'GPS'), S0, {'GPS': Rc}, Hm)
    with pytest.raises(ValueError):
        sch.gain(('x', 'GPS'), S0, {'GPS': Rm['GPS']}, {'GPS': np.eye(15)[3:6]})


def test_combo_worker_with_class_args(golden_dir):
    g = np.load(os.path.join(golden_dir, 'ref15_combos.npz'))
    cand = unpack_events(g)
    chunk = [tuple(cand[i] for i in row if i >= 0) for row in g['combo_idx']]
    sf = kfw.KF_SensorFusion('', '')
    class_args = {k: getattr(sf, k) for k in (
        'get_state_transition_matrix', 'get_process_noise_covariance_matrix', 'predict_covariance',
        'get_gps_observation_matrix', 'get_gps_measurement_noise_covariance_matrix',
        'get_imu_observation_matrix', 'get_imu_measurement_noise_covariance_matrix', 'calculate_kalman_gain')}
    res = kfw.evaluate_combo_chunk_worker(chunk, g['x0'], g['P0'], class_args, float(g['prev_time']),
                                          float(g['target_end']))
    assert _rel([v for r in res for v in r[5]], g['logdet_flat']) <= 1e-6
    # other diagonal constants run with those constants (the oracle worker with the same K) ...
    other = dict(class_args, get_gps_measurement_noise_covariance_matrix=lambda: np.diag([1, 1, 1]))
    res = kfw.evaluate_combo_chunk_worker(chunk, g['x0'], g['P0'], other, float(g['prev_time']),
                                          float(g['target_end']))
    K = dict(q=np.diag(ref_kf.Q_ref15(1.0)), r_imu=np.diag(ref_kf.R_imu15()), r_gps=np.ones(3),
             p0=np.diag(ref_kf.P0_REF15))
    want = ref_kf.evaluate_combo_chunk(chunk, g['x0'], g['P0'], float(g['prev_time']), float(g['target_end']), K=K)
    assert _rel([v for r in res for v in r[5]], [v for r in want for v in r[5]]) <= 1e-6
    # ... a coupled one is refused before any GPU work
    bad = dict(class_args, get_gps_measurement_noise_covariance_matrix=lambda: np.array(
        [[3.0, 1.0, 0.0], [1.0, 3.0, 0.0], [0.0, 0.0, 3.0]]))
    with pytest.raises(ValueError):
        kfw.evaluate_combo_chunk_worker(chunk, g['x0'], g['P0'], bad, 0.0, 1.0)


def test_hw5_2_sequence(csvs):
    sf = khw5.KF_SensorFusion(*csvs)
    sf.load_data()
    sf.gps_to_utm()
    assert all('altitude' not in u for u in sf.utm_data)
    bw, ba, fvi = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    sf.unbias_imu_data(bw, ba)
    rows = sf.unbias_imu_data[:fvi]
    assert sf.compute_stationary_orientation(fvi) == tuple(np.mean([e[c] for e in rows]) for c in (1, 2, 3))
    sf.combine_sensor_data()
    st = sf.run_kalman_filter()
    events, _, _ = ref_ingest.ingest(*csvs, with_altitude=False)
    rs, _ = ref_kf.run_kalman_filter_8state(events)
    assert np.array(st).shape == np.array(rs).shape
    assert _rel(st, rs) <= 1e-6
    # hw5_2.py:540: run_dead_reckoning_for_IMU over the same list (the rest of __main__, :543-546,
    # plots these two outputs)
    dr = sf.run_dead_reckoning_for_IMU()
    rdr, _ = ref_kf.run_dead_reckoning_8state(events)
    assert len(dr) == len(rdr) == sum(e[1] == 'IMU' for e in events)
    assert _rel(dr, rdr) <= 1e-6
    assert abs(sf.quaternion_to_euler(0.0, 0.0, 0.0, 1.0)[2]) == 0.0


@pytest.mark.parametrize('method', ['greedy', 'random'])
def test_scheduled_driver_on_the_ingested_list(csvs, method):
    """run_kalman_filter_scheduled on the façade's event list over the ingested stream (its
    windows read straight from the stream's arrays, no per-event tuples): cold start and a
    warm-start window, against the oracle's driver over the oracle's own ingest, with np.random
    seeded alike for the random arm; the global generator ends where the reference leaves it."""
    sf = kfw.KF_SensorFusion(*csvs)
    sf.load_data()
    sf.gps_to_modified_utm()
    bw, ba, _ = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    sf.unbias_imu_data(bw, ba)
    sf.combine_sensor_data()
    sf.set_processing_frequency(50)
    events, _, _ = ref_ingest.ingest(*csvs)
    P = ref_kf.P0_REF15 * 0.01
    for args in ((None, None, None, None), (400, 1500, P, (float(events[399][2]), 1.0, 2.0, 0.5, 0.0, 0.0, 0.1))):
        np.random.seed(11)
        st, ld, Pf = sf.run_kalman_filter_scheduled(*args, selection_method=method)
        after = np.random.random()
        np.random.seed(11)
        rs, rl, rP = ref_kf.run_kalman_filter_scheduled(events, *args, method, 50.0)
        assert np.random.random() == after
        assert len(st) == len(rs) > 10
        np.testing.assert_array_equal([s[0] for s in st], [r[0] for r in rs])
        assert _rel(st, rs) <= 1e-6 and _rel(ld, rl) <= 1e-6 and _rel(Pf, rP) <= 1e-6


def test_visualizing_pipeline_n40_window(csvs):
    """The reference's visualizing run (kf_workers_visualizing.py:2286-2340) on the synthetic
    log: the adaptive filter up to start_idx, then the brute-force search over the next
    start_offset = 40 events from its state and covariance — through the façade, against the
    oracle's restatement of the reference's adaptive driver and search, at thresholds whose
    winner has one and two events."""
    from kfmi import ref15
    sf = kfw.KF_SensorFusion(*csvs)
    sf.load_data()
    sf.gps_to_modified_utm()
    bw, ba, _ = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    sf.unbias_imu_data(bw, ba)
    sf.combine_sensor_data()
    events, _, _ = ref_ingest.ingest(*csvs)
    start_idx, start_offset, r_value = 1200, 40, -10.0
    st, ld, pt, _, _ = sf.run_adaptive_threshold_kalman_filter(end_idx=start_idx, R_threshold=r_value)
    rst, rld, rpt, _, _ = ref_kf.run_adaptive_threshold(events, 0, start_idx, R_threshold=r_value)
    assert _rel(st, rst) <= 1e-6 and _rel(pt, rpt) <= 1e-6
    # thresholds from the single events' scores over this window (one filter per subset on the GPU)
    cand, xt, Pt, prev, t_end, ev, init = ref15.brute_force_setup(events, start_idx, start_idx + start_offset,
                                                                  rpt, tuple(rst[-1]))
    assert len(cand) == start_offset
    import kfmi
    kf1 = kfmi.BatchedKF('ref15', 1024, 'f64')
    s1 = np.sort(kf1.eval_combos(ev, init, prev, t_end, 1, logdets=False)[0][:start_offset].cpu().numpy())
    s2 = np.sort(kf1.eval_combos(ev, init, prev, t_end, 2, logdets=False)[0][:780].cpu().numpy())
    kf1.close()
    cases = [((s1[2] + s1[3]) / 2, 1)]
    if s2[0] < s1[0]:   # some pair beats every single event: a winner of two events
        cases.append(((s2[0] + s1[0]) / 2, 2))
    print(f'visualizing window at {start_idx}: winner sizes checked {[k for _, k in cases]}')
    for thr, k_want in cases:
        got = sf.run_brute_force_kalman_filter_no_sampling_min_usage(start_idx=start_idx,
                                                                     end_idx=start_idx + start_offset,
                                                                     initial_pt=pt, initial_state=st[-1],
                                                                     R_threshold=thr)
        ref = ref_kf.run_brute_force(events, start_idx, start_idx + start_offset, thr, rpt, tuple(rst[-1]))
        sel = [e[0] for e in ref['selected_sensors']]
        assert len(sel) == k_want
        assert [e[0] for e in got['selected_sensors']] == sel
        for key in ('log_determinants', 'final_state', 'trajectory'):
            assert _rel(got[key], ref[key]) <= 1e-6, key


@pytest.mark.parametrize('warm', [False, True])
def test_monotone_drivers_on_the_device_stream(csvs, warm):
    """run_adaptive_threshold_kalman_filter and run_no_update_kalman_filter over the ingested
    event list run the window on the device (ref15.run_monotone_stream: kf_events_dt's
    KF_DT_MONOTONE rule, one kf_run_events launch); their results equal the event-list path's
    bit for bit (the same dt, the same launch), cold (first fix of the window) and warm, at a
    threshold that gates some updates; and the adaptive filter equals the NumPy restatement."""
    from kfmi import ref15
    sf = kfw.KF_SensorFusion(*csvs)
    sf.load_data()
    sf.gps_to_modified_utm()
    bw, ba, _ = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    sf.unbias_imu_data(bw, ba)
    sf.combine_sensor_data()
    ev = sf.indexed_sensor_data
    assert ref15._device_stream(ev) is not None
    plain = list(ev)
    kw = {}
    if warm:
        st, _, pt, _, _ = ref15.run_adaptive_threshold_kalman_filter(ev, end_idx=1200, R_threshold=-10.0)
        kw = dict(initial_pt=pt, initial_state=st[-1])
    for fn, args in ((ref15.run_adaptive_threshold_kalman_filter, dict(R_threshold=-10.0)),
                     (ref15.run_adaptive_threshold_kalman_filter, dict(R_threshold=float('-inf'))),
                     (ref15.run_no_update_kalman_filter, {})):
        a = fn(ev, 1200, 2600, **args, **kw)
        b = fn(plain, 1200, 2600, **args, **kw)
        assert len(a[0]) == len(b[0]) > 100
        np.testing.assert_array_equal(np.array(a[0]), np.array(b[0]))
        np.testing.assert_array_equal(a[1], b[1])
        np.testing.assert_array_equal(a[2], b[2])
        assert a[3] == b[3] and a[4] == b[4]
    gated = ref15.run_adaptive_threshold_kalman_filter(ev, 1200, 2600, R_threshold=-10.0, **kw)
    assert 0 < len(gated[4]) < len(gated[0])
    rs, rl, rP, rprev, rm = ref_kf.run_adaptive_threshold(plain, 1200, 2600, R_threshold=-10.0,
                                                          initial_pt=kw.get('initial_pt'),
                                                          initial_state=kw.get('initial_state'))
    assert _rel(gated[0], rs) <= 1e-9 and _rel(gated[1], rl) <= 1e-9 and gated[4] == list(rm)
