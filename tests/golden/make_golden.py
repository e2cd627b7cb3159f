"""Generate the golden vectors in tests/golden/ by running the REFERENCE itself.

Run in the build container only (it reads /root/reference, which never travels):

    python tests/golden/make_golden.py

The reference (IseanB/SensorFusion-KalmanFilter) is imported with empty stub modules
for ``numba`` (imported but unused, kf_workers.py:19) and ``utm`` (used only by the
ingest step gps_to_modified_utm, kf_workers.py:319, which these vectors bypass by
feeding pre-converted easting/northing). The imu_data.csv of the reference is absent
(.MISSING_LARGE_BLOBS), so every stream here is synthetic and seeded.

Fixtures written (inputs and the reference's outputs, nothing else):
  ref15_full.npz    run_kalman_filter_full (kf_workers.py:623-728), cold start + warm
                    start window, plus run_adaptive_threshold_kalman_filter (959-1058)
  ref15_combos.npz  evaluate_combo_chunk_worker (kf_workers.py:22-97) on k=1..3 subsets
  ref15_bruteforce.npz  run_brute_force_kalman_filter_no_sampling_min_usage (1218-1392)
  ref15_scheduled.npz   run_kalman_filter_scheduled (826-957), Scheduler.gain/cov_matrix (112-185)
  ref15_drivers.npz run_kalman_filter (kf_workers.py:738-824, states + per-step covariances)
                    and run_no_update_kalman_filter (1060-1160), cold and warm
  ref8_full.npz     hw5_2.run_kalman_filter (hw5_2.py:313-380) and run_dead_reckoning_for_IMU
                    (382-436), in-order and out-of-order streams
  ingest.npz        load_data_from_csv / gps_to_modified_utm / compute_imu_biases /
                    unbias_imu_data / combine_sensor_data (kf_workers.py:290-385) and
                    hw5_2.gps_to_utm (hw5_2.py:29-54) on synthetic GPS and IMU CSVs in the
                    reference's column layout (gps_synth.csv.gz, imu_synth.csv.gz; the
                    reference's own gps_data.csv is location data and is not copied, its
                    imu_data.csv is absent), with oracle.ref_ingest's restated projection
                    injected as utm.from_latlon
  cv_batch.npz      4/2 and 6/3 constant-velocity filters stepped with the reference's
                    own predict_covariance (kf_workers.py:546-549) and
                    calculate_kalman_gain (616-621), in the op order of 688-717
"""
import os
import sys
import types
from itertools import combinations

# the reference's brute force forks a multiprocessing.Pool(30): keep BLAS single-threaded so
# forked children cannot inherit a locked BLAS thread pool
for _v in ('OPENBLAS_NUM_THREADS', 'OMP_NUM_THREADS', 'MKL_NUM_THREADS'):
    os.environ[_v] = '1'

import numpy as np  # noqa: E402

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))
T0 = 1697739552.3362827  # first valid GPS stamp of gps_data.csv (KF_SensorFusion.ipynb:1331)


def import_reference():
    os.environ.setdefault('MPLBACKEND', 'Agg')
    for name in ('numba', 'utm'):
        if name not in sys.modules:
            mod = types.ModuleType(name)
            if name == 'numba':
                mod.jit = lambda *a, **k: (lambda f: f)
                mod.prange = range
            sys.modules[name] = mod
    sys.path.insert(0, REF)
    import kf_workers  # noqa: E402
    import hw5_2  # noqa: E402
    return kf_workers, hw5_2


def synth_events(seed, seconds=2.0, n_pre_imu=5, gps_hz=10.0, imu_hz=200.0, out_of_order=True):
    """A GPS(10 Hz)+IMU(200 Hz) stream shaped like combine_sensor_data's output
    (kf_workers.py:375-385): [(idx, 'GPS'|'IMU', t, payload)], sorted by t, GPS first
    on ties. IMU payload = [t_str, roll, pitch, yaw, wx, wy, wz, ax, ay, az]
    (kf_workers.py:367)."""
    rng = np.random.RandomState(seed)
    raw = []
    # true motion: gentle accelerating drive
    def truth(t):
        tau = t - T0
        p = np.array([3.0 * tau + 0.2 * tau ** 2, 1.5 * tau - 0.1 * tau ** 2, -32.6 + 0.05 * tau])
        return p
    t_imu = T0 - n_pre_imu / imu_hz
    while t_imu < T0 + seconds:
        acc = np.array([0.4, -0.2, 0.0]) + rng.normal(0, 0.05, 3)
        payload = [repr(t_imu), *(rng.normal(0, 0.02, 3)), *(rng.normal(0, 0.01, 3)), *acc]
        raw.append(('IMU', t_imu, payload))
        t_imu += 1.0 / imu_hz + rng.uniform(-1e-4, 1e-4)
    t_gps = T0
    first = True
    while t_gps < T0 + seconds:
        p = truth(t_gps)
        if first:
            z = p.copy()
            z[:2] = 0.0  # first fix is the UTM origin (kf_workers.py:327-328)
            first = False
        else:
            z = p + rng.normal(0, np.sqrt(3.0), 3)
        raw.append(('GPS', t_gps, {'time': t_gps, 'easting': float(z[0]), 'northing': float(z[1]),
                                   'zone_number': 19, 'zone_letter': 'T', 'altitude': float(z[2])}))
        t_gps += 1.0 / gps_hz + rng.uniform(-2e-3, 2e-3)
    # stable sort with GPS entries first (kf_workers.py:378-384 appends GPS before IMU)
    raw.sort(key=lambda e: (e[1], 0 if e[0] == 'GPS' else 1))
    events = [(i, *e) for i, e in enumerate(raw)]
    if out_of_order:
        # exercise the dt<0 guard (kf_workers.py:683-685): swap two IMU entries late in the run
        j = len(events) * 3 // 4
        while events[j][1] != 'IMU' or events[j + 1][1] != 'IMU':
            j += 1
        a, b = events[j], events[j + 1]
        events[j], events[j + 1] = (a[0], b[1], b[2], b[3]), (b[0], a[1], a[2], a[3])
    return events


def pack_events(events):
    N = len(events)
    etype = np.zeros(N, np.int8)
    et = np.zeros(N)
    gps = np.full((N, 3), np.nan)
    imu = np.full((N, 9), np.nan)
    for k, (_, s, t, d) in enumerate(events):
        et[k] = t
        if s == 'GPS':
            gps[k] = [d['easting'], d['northing'], d['altitude']]
        else:
            etype[k] = 1
            imu[k] = d[1:10]
    return dict(ev_type=etype, ev_t=et, ev_gps=gps, ev_imu=imu)


def ref15_full(kfw):
    events = synth_events(seed=11)
    sf = kfw.KF_SensorFusion('gps.csv', 'imu.csv')
    sf.indexed_sensor_data = events
    st, ld, P, prev = sf.run_kalman_filter_full(start_idx=0, end_idx=len(events))
    out = pack_events(events)
    out.update(cold_states=np.array(st), cold_logdets=np.array(ld), cold_P=np.array(P),
               cold_prev_time=np.array(prev))
    # warm-start window, as the experiment loop does (kf_workers.py:2316-2323)
    s0 = len(events) // 3
    st_a, ld_a, P_a, _ = sf.run_kalman_filter_full(start_idx=0, end_idx=s0)
    st_w, ld_w, P_w, prev_w = sf.run_kalman_filter_full(start_idx=s0, end_idx=s0 + 60,
                                                        initial_pt=P_a, initial_state=st_a[-1])
    out.update(warm_start=np.array(s0), warm_init_P=np.array(P_a), warm_init_state=np.array(st_a[-1]),
               warm_states=np.array(st_w), warm_logdets=np.array(ld_w), warm_P=np.array(P_w))
    # adaptive threshold variant (kf_workers.py:959-1058)
    thr = float(np.median(ld))
    st_g, ld_g, P_g, prev_g, times_g = sf.run_adaptive_threshold_kalman_filter(
        start_idx=0, end_idx=len(events), R_threshold=thr)
    out.update(adapt_threshold=np.array(thr), adapt_states=np.array(st_g),
               adapt_logdets=np.array(ld_g), adapt_P=np.array(P_g), adapt_times=np.array(times_g))
    np.savez_compressed(os.path.join(OUT, 'ref15_full.npz'), **out)
    print('ref15_full:', len(events), 'events; final logdet', ld[-1])


def ref15_combos(kfw):
    events = synth_events(seed=12, seconds=0.3, out_of_order=False)
    sf = kfw.KF_SensorFusion('gps.csv', 'imu.csv')
    sf.indexed_sensor_data = events
    # warm start from a short full run, then 9 candidate measurements as in
    # run_brute_force_kalman_filter_no_sampling_min_usage (kf_workers.py:1256-1263)
    st, ld, P, prev = sf.run_kalman_filter_full(start_idx=0, end_idx=20)
    cand = events[20:29]
    target_end = events[28][2]
    xt = np.zeros(15)
    xt[0:6] = st[-1][1:7]
    class_args = {
        'get_state_transition_matrix': sf.get_state_transition_matrix,
        'get_process_noise_covariance_matrix': sf.get_process_noise_covariance_matrix,
        'predict_covariance': sf.predict_covariance,
        'get_gps_observation_matrix': sf.get_gps_observation_matrix,
        'get_gps_measurement_noise_covariance_matrix': sf.get_gps_measurement_noise_covariance_matrix,
        'get_imu_observation_matrix': sf.get_imu_observation_matrix,
        'get_imu_measurement_noise_covariance_matrix': sf.get_imu_measurement_noise_covariance_matrix,
        'calculate_kalman_gain': sf.calculate_kalman_gain,
    }
    chunk = [c for k in (1, 2, 3) for c in combinations(cand, k)]
    res = kfw.evaluate_combo_chunk_worker(chunk, xt, P, class_args, prev, target_end)
    assert len(res) == len(chunk)
    # ragged outputs -> flat + offsets
    combo_pos = [[cand.index(e) for e in c] for c in chunk]
    ld_flat, ld_off, tr_flat = [], [0], []
    for r in res:
        ld_flat.extend(r[5])
        tr_flat.extend(r[1])
        ld_off.append(len(ld_flat))
    out = pack_events(cand)
    ci = np.full((len(chunk), 3), -1, np.int32)
    for i, c in enumerate(combo_pos):
        ci[i, :len(c)] = c
    out.update(x0=xt, P0=np.array(P), prev_time=np.array(prev), target_end=np.array(target_end),
               combo_idx=ci, logdet_flat=np.array(ld_flat), offsets=np.array(ld_off),
               traj_flat=np.array(tr_flat), x_final=np.array([r[3] for r in res]))
    np.savez_compressed(os.path.join(OUT, 'ref15_combos.npz'), **out)
    print('ref15_combos:', len(chunk), 'combos')


def ref15_bruteforce(kfw):
    """run_brute_force_kalman_filter_no_sampling_min_usage (kf_workers.py:1218-1392) on a small
    warm-started window; R_threshold placed between the best k=1 and best k=2 subsets so the
    answer needs two measurements."""
    from itertools import combinations as comb
    events = synth_events(seed=15, seconds=0.4, out_of_order=False)
    sf = kfw.KF_SensorFusion('gps.csv', 'imu.csv')
    sf.indexed_sensor_data = events
    st, ld, P, prev = sf.run_kalman_filter_full(start_idx=0, end_idx=30)
    start, end = 30, 38
    cand = events[start:end]
    xt = np.zeros(15)
    xt[0:6] = st[-1][1:7]
    class_args = {name: getattr(sf, name) for name in (
        'get_state_transition_matrix', 'get_process_noise_covariance_matrix', 'predict_covariance',
        'get_gps_observation_matrix', 'get_gps_measurement_noise_covariance_matrix',
        'get_imu_observation_matrix', 'get_imu_measurement_noise_covariance_matrix', 'calculate_kalman_gain')}
    best = {}
    for k in (1, 2):
        res = kfw.evaluate_combo_chunk_worker(list(comb(cand, k)), xt, P, class_args, st[-1][0], events[end - 1][2])
        best[k] = min(max(r[5]) for r in res)
    assert best[2] < best[1], best
    thr = 0.5 * (best[1] + best[2])
    out = sf.run_brute_force_kalman_filter_no_sampling_min_usage(
        start_idx=start, end_idx=end, R_threshold=thr, initial_pt=P, initial_state=st[-1])
    assert out is not None and out['num_measurements_used'] == 2
    sel = [cand.index(e) for e in out['selected_sensors']]
    o = pack_events(events)
    o.update(start=np.array(start), end=np.array(end), init_P=np.array(P), init_state=np.array(st[-1]),
             threshold=np.array(thr), selected=np.array(sel), final_state=np.array(out['final_state']),
             log_determinants=np.array(out['log_determinants']), trajectory=np.array(out['trajectory']))
    np.savez_compressed(os.path.join(OUT, 'ref15_bruteforce.npz'), **o)
    print('ref15_bruteforce: selected', sel, 'threshold', thr)


def ref15_scheduled(kfw):
    """run_kalman_filter_scheduled (kf_workers.py:826-957): greedy selection at several
    processing rates, random selection with the global numpy RNG seeded, and the Scheduler's
    gain / cov_matrix (kf_workers.py:112-185) on a few covariances."""
    events = synth_events(seed=16, seconds=1.2, out_of_order=False)
    sf = kfw.KF_SensorFusion('gps.csv', 'imu.csv')
    sf.indexed_sensor_data = events
    o = pack_events(events)
    for f in (20, 50, 120):
        sf.set_processing_frequency(f)
        st, ld, P = sf.run_kalman_filter_scheduled(start_idx=0, end_idx=len(events), selection_method='greedy')
        o.update({f'greedy{f}_states': np.array(st), f'greedy{f}_logdets': np.array(ld), f'greedy{f}_P': np.array(P)})
    sf.set_processing_frequency(50)
    np.random.seed(1234)
    st, ld, P = sf.run_kalman_filter_scheduled(start_idx=0, end_idx=len(events), selection_method='random')
    o.update(random50_seed=np.array(1234), random50_states=np.array(st), random50_logdets=np.array(ld),
             random50_P=np.array(P))
    # warm-start scheduled window
    st0, _, P0w, _ = sf.run_kalman_filter_full(start_idx=0, end_idx=60)
    sf.set_processing_frequency(100)
    st, ld, P = sf.run_kalman_filter_scheduled(start_idx=60, end_idx=180, initial_pt=P0w, initial_state=st0[-1],
                                               selection_method='greedy')
    o.update(warm_init_P=np.array(P0w), warm_init_state=np.array(st0[-1]), warm_states=np.array(st),
             warm_logdets=np.array(ld), warm_P=np.array(P))
    # Scheduler.gain / cov_matrix on covariances met along the run
    sch = kfw.Scheduler()
    Rm = {'GPS': sf.get_gps_measurement_noise_covariance_matrix(), 'IMU': sf.get_imu_measurement_noise_covariance_matrix()}
    Hm = {'GPS': sf.get_gps_observation_matrix(), 'IMU': sf.get_imu_observation_matrix()}
    sig = [P0w, P, np.diag([10000.0] * 3 + [1000.0] * 9 + [10000.0] * 3)]
    gains = [[sch.gain(('x', s), S, Rm, Hm, device='cpu') for s in ('GPS', 'IMU')] for S in sig]
    covs = [[sch.cov_matrix([1], S, Rm[s], Hm[s], device='cpu') for s in ('GPS', 'IMU')] for S in sig]
    full = [[sch.cov_matrix(list(range(1, Rm[s].shape[0] + 1)), S, Rm[s], Hm[s], device='cpu')
             for s in ('GPS', 'IMU')] for S in sig]
    o.update(sched_sigma=np.array(sig), sched_gain=np.array(gains), sched_cov_first=np.array(covs),
             sched_cov_full=np.array(full))
    np.savez_compressed(os.path.join(OUT, 'ref15_scheduled.npz'), **o)
    print('ref15_scheduled:', len(events), 'events; greedy120', len(o['greedy120_states']), 'selections')


def ref15_drivers(kfw):
    events = synth_events(seed=17, seconds=1.0)
    sf = kfw.KF_SensorFusion('gps.csv', 'imu.csv')
    sf.indexed_sensor_data = events
    out = pack_events(events)
    # run_kalman_filter: zero initial state, starts at the window's first GPS (kf_workers.py:738-824)
    st, covs = sf.run_kalman_filter(0, len(events))
    out.update(simple_states=np.array(st, dtype=np.float64), simple_covs=np.array(covs, dtype=np.float64))
    s0, e0 = 37, 140   # a window that starts between GPS fixes
    st, covs = sf.run_kalman_filter(s0, e0)
    out.update(simple_win=np.array([s0, e0]), simple_win_states=np.array(st, dtype=np.float64),
               simple_win_covs=np.array(covs, dtype=np.float64))
    # run_no_update_kalman_filter: predictions only (kf_workers.py:1060-1160), cold and warm
    st, ld, P, prev, mt = sf.run_no_update_kalman_filter(start_idx=0, end_idx=len(events))
    out.update(noupd_states=np.array(st), noupd_logdets=np.array(ld), noupd_P=np.array(P),
               noupd_prev=np.array(prev), noupd_mtimes=np.array(mt))
    st_a, _, P_a, _ = sf.run_kalman_filter_full(start_idx=0, end_idx=60)
    st, ld, P, prev, mt = sf.run_no_update_kalman_filter(start_idx=60, end_idx=100, initial_pt=P_a,
                                                         initial_state=st_a[-1])
    out.update(noupd_warm_P0=np.array(P_a), noupd_warm_state0=np.array(st_a[-1]), noupd_warm_states=np.array(st),
               noupd_warm_logdets=np.array(ld), noupd_warm_P=np.array(P), noupd_warm_prev=np.array(prev))
    np.savez_compressed(os.path.join(OUT, 'ref15_drivers.npz'), **out)
    print('ref15_drivers:', len(events), 'events')


def ref8_full(h5):
    events = synth_events(seed=13, seconds=1.5, out_of_order=False)
    sf = h5.KF_SensorFusion('gps.csv', 'imu.csv')
    sf.indexed_sensor_data = events
    st = sf.run_kalman_filter()
    out = pack_events(events)
    out.update(states=np.array(st, dtype=np.float64))
    # run_dead_reckoning_for_IMU (hw5_2.py:382-436) over the same list: IMU events only (the
    # leading ones before the first fix included), x0 = 0, first dt 0, no initial record
    out.update(dr_states=np.array(sf.run_dead_reckoning_for_IMU(), dtype=np.float64))
    # an out-of-order stream: hw5_2 has no dt < 0 guard, it predicts over the negative dt
    ev2 = synth_events(seed=18, seconds=0.8, out_of_order=True)
    sf.indexed_sensor_data = ev2
    st2 = sf.run_kalman_filter()
    out.update({'ooo_' + k: v for k, v in pack_events(ev2).items()})
    out.update(ooo_states=np.array(st2, dtype=np.float64))
    out.update(ooo_dr_states=np.array(sf.run_dead_reckoning_for_IMU(), dtype=np.float64))
    np.savez_compressed(os.path.join(OUT, 'ref8_full.npz'), **out)
    print('ref8_full:', len(events), 'events')


def synth_gps_csv(path, n=1500, n_lead_nan=300, t0=1697739278.761565, seed=22):
    """A synthetic GPS CSV in the layout of hw5_1.py's exporter (time, latitude, longitude,
    altitude; 'nan' strings while there is no fix).  A ~10 Hz drive around an arbitrary point
    (lat 40.0, lon -75.0), shaped like a real log: a block of leading no-fix rows, interior
    dropouts, and rows where only the altitude is 'nan' (kf_workers.py:310 drops them,
    hw5_2.py:35 keeps them) or the longitude is 'NaN'."""
    import gzip
    rng = np.random.RandomState(seed)
    t = t0
    lat, lon, alt = 40.0, -75.0, 12.5
    rows = []
    for i in range(n):
        if i < n_lead_nan or (i % 211 == 3):
            rows.append([repr(t), 'nan', 'nan', 'nan'])
        elif i % 173 == 7:
            rows.append([repr(t), repr(lat), repr(lon), 'nan'])
        elif i % 389 == 11:
            rows.append([repr(t), repr(lat), 'NaN', repr(alt)])
        else:
            rows.append([repr(t), repr(lat), repr(lon), repr(alt)])
        if i >= n_lead_nan:
            lat += 1e-6 * (3.0 + rng.normal(0, 0.3))
            lon += 1e-6 * (2.0 + rng.normal(0, 0.3))
            alt += rng.normal(0, 0.05)
        t += 0.1 + rng.uniform(-0.005, 0.005)
    with gzip.open(path, 'wt', newline='') as f:
        f.write('time,latitude,longitude,altitude\n')
        for r in rows:
            f.write(','.join(r) + '\n')


def synth_imu_csv(path, t0=1697739278.7381794, n=2500, hz=20.0, seed=21, gps_times=()):
    """A synthetic IMU CSV with the column layout of hw5_1.py's exporter (time, orientation
    x y z w, angular_velocity x y z, linear_acceleration x y z).  Exercises: yaw across +-pi,
    exact gimbal-lock rows (|sinp| >= 1), time stamps equal to GPS stamps (ties go GPS first),
    and biases of the size the notebook prints (KF_SensorFusion.ipynb:1331)."""
    import gzip
    rng = np.random.RandomState(seed)
    rows = []
    t = t0
    gps_times = list(gps_times)
    for i in range(n):
        r, p, y = rng.normal(0, 0.05), rng.normal(-0.05, 0.02), -np.pi + 2 * np.pi * i / n
        cr, sr, cp, sp, cy, sy = np.cos(r / 2), np.sin(r / 2), np.cos(p / 2), np.sin(p / 2), np.cos(y / 2), np.sin(y / 2)
        q = [sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
             cr * cp * cy + sr * sp * sy]
        if i == 17:
            q = [0.0, float(np.sqrt(0.5)), 0.0, float(np.sqrt(0.5))]   # pitch = +90 deg
        if i == 18:
            q = [0.0, -0.7071067811865476, 0.0, 0.7071067811865476]  # pitch = -90 deg
        w = rng.normal([-0.0017, -0.0075, -0.036], 0.002)
        a = rng.normal([-0.52, 0.0086, -9.53], 0.05)
        stamp = t
        if gps_times and i % 53 == 5:
            stamp = gps_times[(i * 7) % len(gps_times)]  # exact tie with a GPS stamp
        rows.append([repr(float(stamp)), *(repr(float(v)) for v in q), *(repr(float(v)) for v in w),
                     *(repr(float(v)) for v in a)])
        t += 1.0 / hz + rng.uniform(-1e-4, 1e-4)
    with gzip.open(path, 'wt', newline='') as f:
        f.write('time,orientation_x,orientation_y,orientation_z,orientation_w,angular_velocity_x,'
                'angular_velocity_y,angular_velocity_z,linear_acceleration_x,linear_acceleration_y,'
                'linear_acceleration_z\n')
        for r in rows:
            f.write(','.join(r) + '\n')


def ingest(kfw, h5):
    import gzip
    import shutil
    import tempfile
    sys.path.insert(0, os.path.dirname(os.path.dirname(OUT)))
    from oracle import ref_ingest
    sys.modules['utm'].from_latlon = ref_ingest.utm_from_latlon   # restated projection
    tmp = tempfile.mkdtemp()
    gps_gz = os.path.join(OUT, 'gps_synth.csv.gz')
    synth_gps_csv(gps_gz)
    gps_csv = os.path.join(tmp, 'gps.csv')
    with gzip.open(gps_gz, 'rt') as fi, open(gps_csv, 'w') as fo:
        fo.write(fi.read())
    with open(gps_csv) as f:
        gps_times = [float(l.split(',')[0]) for l in f.readlines()[301:]]
    imu_gz = os.path.join(OUT, 'imu_synth.csv.gz')
    synth_imu_csv(imu_gz, gps_times=gps_times)
    imu_csv = os.path.join(tmp, 'imu.csv')
    with gzip.open(imu_gz, 'rt') as fi, open(imu_csv, 'w') as fo:
        fo.write(fi.read())
    sf = kfw.KF_SensorFusion(gps_csv, imu_csv)
    sf.load_data()
    sf.gps_to_modified_utm()
    bw, ba, fvi = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    sf.unbias_imu_data(bw, ba)
    sf.combine_sensor_data()
    u = sf.utm_data
    unb = sf.unbias_imu_data
    ev = sf.indexed_sensor_data
    gps_pos = {id(g): k for k, g in enumerate(u)}
    imu_pos = {id(e): k for k, e in enumerate(unb)}
    out = dict(
        utm_time=np.array([g['time'] for g in u]),
        utm_easting=np.array([g['easting'] for g in u]), utm_northing=np.array([g['northing'] for g in u]),
        utm_altitude=np.array([g['altitude'] for g in u]), utm_zone_number=np.array([g['zone_number'] for g in u]),
        utm_zone_letter=np.array([ord(g['zone_letter']) for g in u]),
        gyro_bias=np.asarray(bw), accel_bias=np.asarray(ba), first_valid_index=np.array(fvi),
        imu_values=np.array([[float(v) for v in e[1:10]] for e in unb]),
        ev_is_imu=np.array([e[1] == 'IMU' for e in ev]), ev_time=np.array([e[2] for e in ev]),
        ev_src=np.array([gps_pos[id(e[3])] if e[1] == 'GPS' else imu_pos[id(e[3])] for e in ev]))
    h = h5.KF_SensorFusion(gps_csv, imu_csv)
    h.load_data()
    h.gps_to_utm()
    out.update(hw5_utm_time=np.array([g['time'] for g in h.utm_data]),
               hw5_utm_easting=np.array([g['easting'] for g in h.utm_data]),
               hw5_utm_northing=np.array([g['northing'] for g in h.utm_data]),
               hw5_has_altitude=np.array(any('altitude' in g for g in h.utm_data)))
    np.savez_compressed(os.path.join(OUT, 'ingest.npz'), **out)
    shutil.rmtree(tmp)
    print('ingest:', len(u), 'fixes,', len(unb), 'imu rows,', len(ev), 'events; first_valid_index', fvi)


def cv_batch(kfw):
    """4/2 and 6/3 constant-velocity filters stepped with the reference's own
    predict_covariance / calculate_kalman_gain, in the op order of kf_workers.py:688-717.
    The control term G u is the 15-state model's acceleration column applied to the IMU
    acceleration (kf_workers.py:501-509)."""
    sf = kfw.KF_SensorFusion('gps.csv', 'imu.csv')
    rng = np.random.RandomState(14)
    out = {}
    for d, p0p, p0v in ((2, 1000.0, 100.0), (3, 10000.0, 1000.0)):
        n = 2 * d
        for k, T, dt0 in ((1, 48, 0.1), (5, 60, 0.01)):
            B = 6
            dt = np.full(T, dt0)
            dt[3] = 0.0  # a zero-length step, like the re-processed initial GPS fix
            dt[7] = dt0 * 1.7
            u = rng.normal(0, 0.3, (T, d, B))
            z = rng.normal(0, 50.0, (T // k, d, B)) + np.linspace(0, 30, T // k)[:, None, None]
            x0 = np.zeros((B, n))
            x0[:, :d] = rng.uniform(-1000, 1000, (B, d))
            x0[:, d:] = rng.normal(0, 10, (B, d))
            P0 = np.diag([p0p] * d + [p0v] * d)
            traj = np.zeros((T, n, B))
            logdet = np.zeros((T, B))
            Pf = np.zeros((B, n, n))
            H = np.eye(n)[:d]
            R = np.diag([3.0] * d)
            for b in range(B):
                xt = x0[b].copy()
                Pt = P0.copy()
                for t in range(T):
                    h = dt[t]
                    F = np.eye(n)
                    G = np.zeros((n, d))
                    for i in range(d):
                        F[i, d + i] = h
                        G[i, i] = 0.5 * h ** 2
                        G[d + i, i] = h
                    Qt = np.diag([5.0 * h] * d + [1.0 * h] * d)
                    xt = np.dot(F, xt) + np.dot(G, u[t, :, b])
                    Pt = sf.predict_covariance(Pt, F, Qt)
                    if (t + 1) % k == 0:
                        K = sf.calculate_kalman_gain(Pt, H, R)
                        y = np.array(z[t // k, :, b]) - np.dot(H, xt)
                        xt = xt + np.dot(K, y)
                        Pt = np.dot(np.eye(n) - np.dot(K, H), Pt)
                    traj[t, :, b] = xt
                    logdet[t, b] = np.linalg.slogdet(Pt)[1]
                Pf[b] = Pt
            key = f'cv{d}_k{k}'
            out.update({f'{key}_dt': dt, f'{key}_u': u, f'{key}_z': z, f'{key}_x0': x0,
                        f'{key}_P0': P0, f'{key}_traj': traj, f'{key}_logdet': logdet,
                        f'{key}_Pfinal': Pf})
    np.savez_compressed(os.path.join(OUT, 'cv_batch.npz'), **out)
    print('cv_batch written')


if __name__ == '__main__':
    # python tests/golden/make_golden.py [generator ...]   (default: all)
    kfw, h5 = import_reference()
    gens = {'ref15_full': lambda: ref15_full(kfw), 'ref15_combos': lambda: ref15_combos(kfw),
            'ref15_bruteforce': lambda: ref15_bruteforce(kfw), 'ref15_scheduled': lambda: ref15_scheduled(kfw),
            'ref15_drivers': lambda: ref15_drivers(kfw), 'ref8_full': lambda: ref8_full(h5),
            'ingest': lambda: ingest(kfw, h5), 'cv_batch': lambda: cv_batch(kfw)}
    for name in (sys.argv[1:] or list(gens)):
        gens[name]()
    # analytic known answer: slogdet(P0) of kf_workers.py:651 = 6 ln 1e4 + 9 ln 1e3
    print('KAT logdet(P0) =', np.linalg.slogdet(np.diag([1e4] * 3 + [1e3] * 9 + [1e4] * 3))[1])
