"""The reference models with a caller's constants (kf_params.ref_*) and
Scheduler.cov_matrix for any row subset S (item 6), on the GPU against the CPU oracle fed the
same constants (oracle/ref_kf.py's K) — needs an MI355X.

The reference hard-codes its noise constants in getters (kf_workers.py:519-614, P0 :651;
hw5_2.py:233-304, :317-326) that a class_args dict of callables replaces (kf_workers.py:
1242-1251); the notebook's brute force uses P0 = diag(1000 x 3, 100 x 9, 1000 x 3)
(KF_SensorFusion.ipynb:814).  Tolerances as test_gpu_ref15.py: 1e-6 relative (fp64), the
agreement being ~1e-10 (Joseph + LDL^T vs (I-KH)P + inv).
"""
import os

import numpy as np
import pytest
import torch

import kfmi
from golden_events import unpack_events
from kfmi import kf_workers as kw
from kfmi import ref15
from oracle import ref_kf

pytestmark = pytest.mark.gpu
TOL = 1e-6
NOTEBOOK_P0 = np.r_[[1000.0] * 3, [100.0] * 9, [1000.0] * 3]  # KF_SensorFusion.ipynb:814


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0))) if a.size else 0.0


def _custom(model='ref15', seed=3, **over):
    rng = np.random.default_rng(seed)
    n, g = (15, 3) if model == 'ref15' else (8, 2)
    kw_ = dict(q=rng.uniform(0.01, 8.0, n), r_imu=rng.uniform(0.02, 120.0, n), r_gps=rng.uniform(0.5, 9.0, g),
               p0=rng.uniform(20.0, 2e4, n))
    kw_.update(over)
    return ref15.ModelConsts(model, **kw_)


def _streams(B, T, seed):
    rng = np.random.default_rng(seed)
    etype = rng.choice([0, 1, 1, 1], size=(T, B)).astype(np.uint8)
    dt = rng.uniform(0.0, 0.05, (T, B))
    pay = rng.normal(0, 1, (T, 9, B)) * np.array([20, 20, 20, 0.05, 0.05, 0.05, 0.5, 0.5, 0.5])[None, :, None]
    return etype, dt, pay


def _oracle_events(step, x0, P0, etype, dt, pay, f, K):
    x, P = x0.copy(), P0.copy()
    tr, ld = [], []
    for t in range(etype.shape[0]):
        if etype[t, f] == 0:
            sd = {'easting': pay[t, 0, f], 'northing': pay[t, 1, f], 'altitude': pay[t, 2, f]}
            x, P = step(x, P, 'GPS', sd, dt[t, f], K)
        else:
            x, P = step(x, P, 'IMU', ['t', *pay[t, :, f]], dt[t, f], K)
        tr.append(x[:6] if len(x) == 15 else x[:3])
        ld.append(np.linalg.slogdet(P)[1])
    return np.array(tr), np.array(ld)


@pytest.mark.parametrize('model', ['ref15', 'ref8'])
@pytest.mark.parametrize('kernel', ['lane', 'lds', 'chain'])
def test_events_with_custom_constants_vs_oracle(model, kernel):
    """kf_run_events on every kernel variant with the caller's Q, R_imu, R_gps and P0 (the handle's
    kf_reset puts the custom P0), against the oracle's step with the same constants."""
    B, T = 256, 24
    c = _custom(model, seed=11)
    etype, dt, pay = _streams(B, T, seed=12)
    n = 15 if model == 'ref15' else 8
    kf = kfmi.BatchedKF(model, B, 'f64', params=c.params(), options={'events_kernel': kernel})
    x0 = np.zeros((n, B))
    x0[0:2] = pay[0, 0:2] * 3.0
    kf.reset(torch.from_numpy(x0).cuda())
    tr, ld, _, _ = kf.run_events(etype, dt, pay)
    tr, ld = tr.cpu().numpy(), ld.cpu().numpy()
    kf.close()
    step = ref_kf.step15 if model == 'ref15' else ref_kf.step8
    K = c.oracle()
    worst = 0.0
    for f in range(0, B, 17):
        otr, old = _oracle_events(step, x0[:, f], c.P0, etype, dt, pay, f, K)
        worst = max(worst, _rel(tr[:, :, f], otr), _rel(ld[:, f], old))
    assert worst <= TOL, worst
    # and they differ from the reference constants' run (the constants reached the kernels)
    kr = kfmi.BatchedKF(model, B, 'f64', options={'events_kernel': kernel})
    kr.reset(torch.from_numpy(x0).cuda())
    _, ld_ref, _, _ = kr.run_events(etype, dt, pay)
    assert _rel(ld_ref.cpu().numpy(), ld) > 1e-3
    kr.close()


def test_reference_constants_as_params_are_the_default_kernels():
    """kf_params holding exactly the reference's constants select the kernels compiled with its
    literals: bit-identical to a handle without params."""
    B, T = 512, 16
    etype, dt, pay = _streams(B, T, seed=4)
    p = kfmi.default_params('ref15')                   # the reference's values, passed explicitly
    outs = []
    for params in (None, p):
        kf = kfmi.BatchedKF('ref15', B, 'f64', params=params)
        tr, ld, _, _ = kf.run_events(etype, dt, pay)
        outs.append((tr.cpu().numpy(), ld.cpu().numpy()))
        kf.close()
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


def test_invalid_constants_rejected():
    p = kfmi.default_params('ref15')
    p.ref_r_imu[4] = 0.0
    with pytest.raises(kfmi.KFError):
        kfmi.BatchedKF('ref15', 8, 'f64', params=p)
    p = kfmi.default_params('ref15')
    p.ref_q[0] = float('nan')
    with pytest.raises(kfmi.KFError):
        kfmi.BatchedKF('ref15', 8, 'f64', params=p)


def _search_case(golden_dir, n):
    g = np.load(os.path.join(golden_dir, 'ref15_full.npz'))
    events = unpack_events(g)
    st, _, P, _ = ref_kf.run_kalman_filter_full(events, 0, 100)
    cand = list(events[100:100 + n])
    xt = np.zeros(15)
    xt[0:6] = st[-1][1:7]
    ev = np.array([[t, 0 if s == 'GPS' else 1, *ref15.event_payload(s, d)] for (_, s, t, d) in cand])
    return cand, ev, xt, P, st[-1][0], max(c[2] for c in cand)


def test_combos_and_search_with_custom_constants(golden_dir):
    """kf_eval_combos and the shared-prefix search with the notebook's P0 and custom R: every
    subset's max log-det equals the per-subset kernel's, and sampled subsets the oracle worker's."""
    from itertools import combinations
    c = _custom(seed=5, p0=NOTEBOOK_P0)
    n = 9
    cand, ev, xt, P, t0, target = _search_case(golden_dir, n)
    init = np.concatenate([xt, ref15.to_blocks(P)])
    kf = kfmi.BatchedKF('ref15', 1, 'f64', params=c.params())
    _, _, _, sm = kf.search_combos(ev, init, t0, target, threshold=-1e30, exhaustive=True, subset_max=True)
    sm = sm.cpu().numpy()
    kf.close()
    K = c.oracle()
    for k in (1, 3, 6, 9):
        combos = list(combinations(range(n), k))
        kc = kfmi.BatchedKF('ref15', len(combos), 'f64', params=c.params())
        mx, _, _ = kc.eval_combos(ev, init, t0, target, k, logdets=False)
        mx = mx.cpu().numpy()
        kc.close()
        masks = np.array([sum(1 << i for i in cc) for cc in combos])
        assert _rel(sm[masks], mx) <= 1e-12
        for j in range(0, len(combos), max(1, len(combos) // 5)):
            res = ref_kf.evaluate_combo_chunk([tuple(cand[i] for i in combos[j])], xt, P, t0, target, K=K)[0]
            assert abs(mx[j] - max(res[5])) / max(1.0, abs(max(res[5]))) <= TOL


def test_brute_force_class_args_and_notebook_p0(golden_dir):
    """evaluate_combo_chunk_worker with a class_args dict whose getters return other diagonal
    constants (kf_workers.py:1242-1251), against the oracle worker with the same constants."""
    cand, ev, xt, P, t0, target = _search_case(golden_dir, 8)
    c = _custom(seed=9)
    class_args = {'get_state_transition_matrix': kw._F, 'get_process_noise_covariance_matrix': c.Q,
                  'get_gps_observation_matrix': lambda: kw._H_GPS.copy(),
                  'get_imu_observation_matrix': lambda: kw._H_IMU.copy(),
                  'get_gps_measurement_noise_covariance_matrix': lambda: c.R_gps,
                  'get_imu_measurement_noise_covariance_matrix': lambda: c.R_imu,
                  'predict_covariance': lambda Pt, F, Q: np.dot(np.dot(F, Pt), F.T) + Q,
                  'calculate_kalman_gain': lambda Pn, H, R: np.dot(np.dot(Pn, H.T),
                                                                   np.linalg.inv(np.dot(np.dot(H, Pn), H.T) + R))}
    chunk = [tuple(cand[i] for i in idx) for idx in ((0,), (1, 4), (0, 2, 5, 7), tuple(range(8)))]
    got = kw.evaluate_combo_chunk_worker(chunk, xt, P, class_args, t0, target)
    want = ref_kf.evaluate_combo_chunk(chunk, xt, P, t0, target, K=c.oracle())
    assert len(got) == len(want)
    for a, b in zip(got, want):
        assert _rel(a[5], b[5]) <= TOL and _rel([s[1:] for s in a[1]], [s[1:] for s in b[1]]) <= TOL
        assert _rel(a[3], b[3]) <= TOL


def test_facade_subclass_getters_and_p0(golden_dir):
    """KF_SensorFusion whose getters a subclass replaced (diagonal Q, R) and whose cold-start P0 is
    the notebook's: run_kalman_filter_full and the adaptive driver equal the oracle's drivers with
    the same constants."""
    g = np.load(os.path.join(golden_dir, 'ref15_full.npz'))
    events = unpack_events(g)
    c = _custom(seed=21, p0=NOTEBOOK_P0)

    class Tuned(kw.KF_SensorFusion):
        def get_process_noise_covariance_matrix(self, dt):
            return c.Q(dt)

        def get_gps_measurement_noise_covariance_matrix(self):
            return c.R_gps

        def get_imu_measurement_noise_covariance_matrix(self):
            return c.R_imu

    sf = Tuned('gps.csv', 'imu.csv')
    sf.P0 = np.diag(NOTEBOOK_P0)
    sf.indexed_sensor_data = events
    st, ld, P, prev = sf.run_kalman_filter_full(0, len(events))
    ost, old, oP, oprev = ref_kf.run_kalman_filter_full(events, 0, len(events), K=c.oracle())
    assert _rel(st, ost) <= TOL and _rel(ld, old) <= TOL and _rel(P, oP) <= TOL and prev == oprev

    class Coupled(kw.KF_SensorFusion):
        def get_gps_measurement_noise_covariance_matrix(self):
            return np.array([[3.0, 1.0, 0.0], [1.0, 3.0, 0.0], [0.0, 0.0, 3.0]])

    sc = Coupled('gps.csv', 'imu.csv')
    sc.indexed_sensor_data = events
    with pytest.raises(ValueError, match='off-diagonal'):
        sc.run_kalman_filter_full(0, len(events))


def test_scheduled_with_custom_constants_flips_the_greedy_pick(golden_dir):
    """With R_gps > R_imu[pos_x] the GPS candidate's posterior trace is the larger one, so the
    greedy scheduler picks fixes (the reference constants pick IMU samples): the engine's
    scheduled driver follows the constants, as the oracle's."""
    g = np.load(os.path.join(golden_dir, 'ref15_full.npz'))
    events = unpack_events(g)
    c = _custom(seed=2, r_gps=np.array([400.0, 400.0, 400.0]))
    for f in (20.0, 50.0):
        st, ld, P = ref15.run_kalman_filter_scheduled(events, 0, len(events), selection_method='greedy',
                                                      processing_frequency=f, consts=c)
        ost, old, oP = ref_kf.run_kalman_filter_scheduled(events, 0, len(events), selection_method='greedy',
                                                          processing_frequency=f, K=c.oracle())
        assert len(st) == len(ost)
        assert [s[0] for s in st] == [s[0] for s in ost]     # the same picks
        assert _rel(st, ost) <= TOL and _rel(ld, old) <= TOL and _rel(P, oP) <= TOL


def test_stream_parallel_with_custom_constants():
    """kf_run_stream (time-parallel, covariance maps with the caller's Q and R) equals the single
    filter with the same constants."""
    rng = np.random.default_rng(8)
    T = 70000
    et = np.ones(T, np.uint8)
    et[::20] = 0
    dt = np.full(T, 0.005)
    pay = np.zeros((T, 9))
    pay[:, 0:3] = rng.normal(0, 0.05, (T, 3))
    pay[:, 3:6] = rng.normal(0, 0.01, (T, 3))
    pay[:, 6:9] = rng.normal(0, 0.3, (T, 3))
    pay[et == 0, 0:3] = rng.normal(0, 3, (int((et == 0).sum()), 3))
    # the reference's constants rescaled (a tuned filter): the covariance recursion still forgets
    # its start within the maps' window, so the chunked records stand (the device check decides;
    # an unphysical choice would fail it and the sequential fallback would write the records)
    ref = ref15.ModelConsts('ref15')
    c = ref15.ModelConsts('ref15', q=ref.q * 1.5, r_imu=ref.r_imu * 0.7, r_gps=[2.0, 2.5, 4.0], p0=NOTEBOOK_P0)
    x0 = np.zeros(15)
    dev = torch.device('cuda', 0)
    tr, ld, x, P, _ = ref15.run_stream_parallel(torch.as_tensor(et, device=dev), torch.as_tensor(dt, device=dev),
                                                torch.as_tensor(pay, device=dev), x0, ref15.to_blocks(c.P0),
                                                consts=c)
    assert ref15.parallel_check['ok'] and ref15.parallel_check['chunks'] > 1, ref15.parallel_check
    kf = kfmi.BatchedKF('ref15', 1, 'f64', params=c.params())
    kf.set_state(x0[:, None], ref15.to_blocks(c.P0)[:, None])
    str_, sld, _, _ = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], sequential=True)
    assert _rel(tr.cpu().numpy(), str_[:, :, 0].cpu().numpy()) <= 1e-9
    assert _rel(ld.cpu().numpy(), sld[:, 0].cpu().numpy()) <= 1e-9
    kf.close()


@pytest.mark.parametrize('sensor', ['GPS', 'IMU'])
def test_scheduler_cov_matrix_any_rows_vs_oracle(sensor):
    """Scheduler.cov_matrix(S, Sigma, R, H) for random row subsets S and a caller's diagonal R
    (kf_workers.py:121-138) against the oracle's restatement."""
    rng = np.random.default_rng(17)
    sch = kw.Scheduler()
    H = kw._H_GPS if sensor == 'GPS' else kw._H_IMU
    m = H.shape[0]
    R = np.diag(rng.uniform(0.1, 60.0, m))
    for trial in range(12):
        A = [rng.normal(size=(3, 3)) for _ in range(3)] + [rng.normal(size=(2, 2)) for _ in range(3)]
        Sigma = np.zeros((15, 15))
        for ch, blk in enumerate(A):
            idx = [ch, 6 + ch, 12 + ch] if ch < 3 else [ch, ch + 6]
            Sigma[np.ix_(idx, idx)] = blk @ blk.T + np.eye(len(idx)) * rng.uniform(0.5, 50)
        k = int(rng.integers(1, m + 1))
        S = sorted(rng.choice(np.arange(1, m + 1), size=k, replace=False).tolist())
        got = sch.cov_matrix(S, Sigma, R, H)
        want = ref_kf.scheduler_cov_matrix(S, Sigma, R, H)
        assert np.max(np.abs(got - want) / np.maximum(np.abs(want), 1.0)) <= 1e-10, (S, trial)
    with pytest.raises(IndexError):
        sch.cov_matrix([m + 1], Sigma, R, H)


def test_hw5_2_facade_with_custom_constants(golden_dir):
    """hw5_2's 8-state driver with a subclass's diagonal constants vs the oracle's step8."""
    from kfmi import hw5_2
    g = np.load(os.path.join(golden_dir, 'ref8_full.npz'))
    events = unpack_events(g)
    c = _custom('ref8', seed=41)

    class Tuned8(hw5_2.KF_SensorFusion):
        def get_process_noise_covariance_matrix(self, dt):
            return c.Q(dt)

        def get_imu_measurement_noise_covariance_matrix(self):
            return c.R_imu

        def get_gps_measurement_noise_covariance_matrix(self):
            return c.R_gps

    sf = Tuned8('gps.csv', 'imu.csv')
    sf.P0 = c.P0
    sf.indexed_sensor_data = events
    got = sf.run_kalman_filter()
    x, P, want, started, prev = np.zeros(8), c.P0.copy(), [(0.0, 0.0, 0.0)], False, None
    for (_, stype, t, sdata) in events:
        if stype == 'GPS' and not started:
            started, prev = True, t
        if not started:
            continue
        x, P = ref_kf.step8(x, P, stype, sdata, t - prev, c.oracle())
        want.append((x[0], x[1], x[2]))
        prev = t
    assert _rel(got, want) <= TOL
