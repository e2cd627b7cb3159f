"""The reference's remaining drivers on the engine vs the reference's own outputs — needs an
MI355X: run_kalman_filter (kf_workers.py:738-824, per-step covariances),
run_no_update_kalman_filter (1060-1160) and hw5_2's 8-state filter (KF_MODEL_REF8,
hw5_2.py:313-380), plus a random batched REF8 stream against the oracle's dense step.

Tolerance (north_star): 1e-6 relative for fp64, normalised by max(|ref|, 1).
"""
import os

import numpy as np
import pytest
import torch

import kfmi
from golden_events import unpack_events
from kfmi import ref8, ref15
from oracle import ref_kf

pytestmark = pytest.mark.gpu
TOL = 1e-6


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0))) if a.size else 0.0


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


def test_run_kalman_filter_states_and_covariances(golden_dir):
    g = _load(golden_dir, 'ref15_drivers.npz')
    events = unpack_events(g)
    st, covs = ref15.run_kalman_filter(events, 0, len(events))
    assert np.array(st).shape == g['simple_states'].shape
    assert _rel(st, g['simple_states']) <= TOL
    assert np.array(covs).shape == g['simple_covs'].shape
    assert _rel(covs, g['simple_covs']) <= TOL
    s0, e0 = (int(v) for v in g['simple_win'])
    st, covs = ref15.run_kalman_filter(events, s0, e0)
    assert _rel(st, g['simple_win_states']) <= TOL
    assert _rel(covs, g['simple_win_covs']) <= TOL


def test_run_no_update_kalman_filter(golden_dir):
    g = _load(golden_dir, 'ref15_drivers.npz')
    events = unpack_events(g)
    st, ld, P, prev, mt = ref15.run_no_update_kalman_filter(events, 0, len(events))
    assert np.array(st).shape == g['noupd_states'].shape
    assert _rel(st, g['noupd_states']) <= TOL
    assert _rel(ld, g['noupd_logdets']) <= TOL
    assert _rel(P, g['noupd_P']) <= TOL
    assert prev == float(g['noupd_prev'])
    np.testing.assert_array_equal(mt, g['noupd_mtimes'])
    st, ld, P, prev, mt = ref15.run_no_update_kalman_filter(events, 60, 100, initial_pt=g['noupd_warm_P0'],
                                                            initial_state=tuple(g['noupd_warm_state0']))
    assert _rel(st, g['noupd_warm_states']) <= TOL
    assert _rel(ld, g['noupd_warm_logdets']) <= TOL
    assert _rel(P, g['noupd_warm_P']) <= TOL
    assert prev == float(g['noupd_warm_prev']) and mt == []
    # no GPS fix in a cold window -> None (kf_workers.py:1103-1105)
    first_gps = next(i for i, e in enumerate(events) if e[1] == 'GPS')
    if first_gps > 1:
        assert ref15.run_no_update_kalman_filter(events, 0, first_gps) is None


@pytest.mark.parametrize('prefix', ['', 'ooo_'])
def test_ref8_run_kalman_filter(golden_dir, prefix):
    g = _load(golden_dir, 'ref8_full.npz')
    events = unpack_events(g, prefix)
    st = ref8.run_kalman_filter(events)
    assert np.array(st).shape == g[prefix + 'states'].shape
    assert _rel(st, g[prefix + 'states']) <= TOL


def test_ref8_random_batch_vs_oracle():
    """B independent REF8 filters on random GPS/IMU/predict/padding streams with irregular dt,
    against the oracle's dense 8x8 reference-order step (hw5_2.py:336-366)."""
    rng = np.random.default_rng(8)
    B, T = 257, 36
    etype = rng.choice([0, 1, 1, 2], size=(T, B)).astype(np.uint8)
    etype[28:, ::4] = 255
    dt = rng.uniform(0.0, 0.1, (T, B))
    pay = np.zeros((T, 9, B))
    pay[:, 0:3] = rng.normal(0, 20, (T, 3, B))
    pay[:, 3:6] = rng.normal(0, 0.05, (T, 3, B))
    pay[:, 6:9] = rng.normal(0, 0.5, (T, 3, B))
    x0 = rng.normal(0, 5, (B, 8))
    kf = kfmi.BatchedKF('ref8', B, 'f64')
    kf.reset(torch.from_numpy(np.ascontiguousarray(x0.T)).cuda())
    tr, ld, up, cv = kf.run_events(etype, dt, pay, updated=True, cov=True)
    tr, ld, cv = tr.cpu().numpy(), ld.cpu().numpy(), cv.cpu().numpy()
    x, Pb = kf.state()
    x, Pb = x.cpu().numpy(), Pb.cpu().numpy()
    assert tr.shape == (T, 3, B) and cv.shape == (T, 15, B)
    assert (kf.status().cpu().numpy() == 0).all()
    for f in range(0, B, 5):
        xf, Pf = x0[f].copy(), ref8.P0.copy()
        for t in range(T):
            ty = etype[t, f]
            if ty == 2:
                F = ref_kf.F_ref8(dt[t, f])
                xf = F @ xf
                Pf = ref_kf.predict_covariance(Pf, F, ref_kf.Q_ref8(dt[t, f]))
            elif ty in (0, 1):
                sdata = ({'easting': pay[t, 0, f], 'northing': pay[t, 1, f]} if ty == 0
                         else ['t', *pay[t, :, f]])
                xf, Pf = ref_kf.step8(xf, Pf, 'GPS' if ty == 0 else 'IMU', sdata, dt[t, f])
            assert _rel(tr[t, :, f], xf[:3]) <= TOL, (f, t)
            assert _rel(ref15.from_blocks(cv[t, :, f]), Pf) <= TOL, (f, t)
            ref_ld = np.linalg.slogdet(Pf)[1]
            assert abs(ld[t, f] - ref_ld) <= TOL * max(1.0, abs(ref_ld))
        assert _rel(x[:, f], xf) <= TOL
        assert _rel(ref15.from_blocks(Pb[:, f]), Pf) <= TOL


def test_ref8_handle_rejects_ref15_only_entry_points():
    from kfmi import _lib
    kf = kfmi.BatchedKF('ref8', 4, 'f64')
    assert _lib.lib().kf_update(kf.handle, None, None, None, None) == _lib.KF_EINVAL
    for call in (lambda: kf.score_candidates([0]), lambda: kf.eval_combos(np.zeros((2, 11)), np.zeros(42), 0, 1, 1)):
        with pytest.raises(ValueError):
            call()


def _events_run(model, kernel, etype, dt, pay, x0, P0b, threshold=None, dtype='f64', records=True):
    B = etype.shape[1]
    kf = kfmi.BatchedKF(model, B, dtype, options={'events_kernel': kernel})
    npd = np.float64 if dtype == 'f64' else np.float32
    kf.set_state(np.ascontiguousarray(x0.T, npd), np.ascontiguousarray(P0b.T, npd))
    tr, ld, up, cv = kf.run_events(etype, dt, np.ascontiguousarray(pay, npd), updated=records, cov=records,
                                   threshold=threshold)
    x, Pb = kf.state()
    out = [None if v is None else v.double().cpu().numpy() if v.is_floating_point() else v.cpu().numpy()
           for v in (tr, ld, up, cv, x, Pb, kf.status())]
    kf.close()
    return out


@pytest.mark.parametrize('model', ['ref15', 'ref8'])
@pytest.mark.parametrize('gated', [False, True])
def test_chain_kernel_matches_lane_kernel(model, gated):
    """The chain-parallel kernel (one lane per axis chain, used below 16384 filters) against the
    lane-per-filter kernel on the same random streams: states, covariance records and update
    decisions agree to rounding, logdets to the summation-order difference."""
    rng = np.random.default_rng(21 if model == 'ref15' else 22)
    n = 15 if model == 'ref15' else 8
    B, T = 133, 48
    etype = rng.choice([0, 1, 1, 1, 2], size=(T, B)).astype(np.uint8)
    etype[40:, ::5] = 255
    dt = rng.uniform(0.0, 0.05, (T, B))
    pay = np.zeros((T, 9, B))
    pay[:, 0:3] = rng.normal(0, 20, (T, 3, B))
    pay[:, 3:6] = rng.normal(0, 0.05, (T, 3, B))
    pay[:, 6:9] = rng.normal(0, 0.5, (T, 3, B))
    x0 = rng.normal(0, 5, (B, n))
    P0 = ref15.P0 if model == 'ref15' else ref8.P0
    P0b = np.repeat(ref15.to_blocks(P0)[None], B, 0)
    P0b[7] = -P0b[7]                                   # one non-positive-definite filter
    thr = None
    if gated:  # a threshold inside the run's own logdet range, so the gate both applies and skips
        ld = _events_run(model, 'lane', etype, dt, pay, x0, P0b)[1]
        thr = float(np.median(ld[np.isfinite(ld)]))
    lane = _events_run(model, 'lane', etype, dt, pay, x0, P0b, thr)
    chain = _events_run(model, 'chain', etype, dt, pay, x0, P0b, thr)
    for name, a, b in zip(('traj', 'logdet', 'updated', 'cov', 'x', 'P', 'status'), lane, chain):
        ok = np.isfinite(a)
        np.testing.assert_array_equal(ok, np.isfinite(b), err_msg=name)
        if name in ('updated', 'status'):
            np.testing.assert_array_equal(a, b, err_msg=name)
        else:
            assert _rel(b[ok], a[ok]) <= 1e-12, name
    assert lane[6][7] == kfmi.KF_ENOTSPD and (lane[6][np.arange(B) != 7] == 0).all()
    if gated:
        assert 0 < lane[2].mean() < 1                   # the gate both applied and skipped updates


def test_per_step_calls_on_reference_models():
    """predict / update(sensor='gps') / step('imu') / logdet on a ref15 handle reproduce the
    oracle's dense per-event steps (the reference's per-call shape, kf_workers.py:688-717)."""
    rng = np.random.default_rng(31)
    B = 70
    kf = kfmi.BatchedKF('ref15', B, 'f64')
    x0 = rng.normal(0, 5, (B, 15))
    kf.reset(torch.from_numpy(np.ascontiguousarray(x0.T)).cuda())
    xs = [x0[f].copy() for f in range(B)]
    Ps = [ref_kf.P0_REF15.copy() for _ in range(B)]
    ld0 = kf.logdet().cpu().numpy()
    assert np.allclose(ld0, np.linalg.slogdet(ref_kf.P0_REF15)[1], rtol=1e-12)
    for k in range(12):
        dt = rng.uniform(0.001, 0.05, B)
        if k % 3 == 0:
            ld = kf.predict(None, dt_per_filter=dt, logdet=True).cpu().numpy()
            for f in range(B):
                F = ref_kf.F_ref15(dt[f])
                xs[f] = F @ xs[f]
                Ps[f] = ref_kf.predict_covariance(Ps[f], F, ref_kf.Q_ref15(dt[f]))
        elif k % 3 == 1:
            z = rng.normal(0, 20, (3, B))
            mask = (rng.random(B) > 0.2).astype(np.uint8)
            ld = kf.update(z, mask=mask, sensor='gps').cpu().numpy()
            for f in range(B):
                if mask[f]:
                    xs[f], Ps[f] = ref_kf.step15(xs[f], Ps[f], 'GPS', {'easting': z[0, f], 'northing': z[1, f],
                                                                        'altitude': z[2, f]}, 0.0)
        else:
            imu = np.concatenate([rng.normal(0, 0.05, (6, B)), rng.normal(0, 0.5, (3, B))])
            ld = kf.step('imu', dt, imu).cpu().numpy()
            for f in range(B):
                xs[f], Ps[f] = ref_kf.step15(xs[f], Ps[f], 'IMU', ['t', *imu[:, f]], dt[f])
        for f in range(0, B, 3):
            ref = np.linalg.slogdet(Ps[f])[1]
            assert abs(ld[f] - ref) <= TOL * max(1.0, abs(ref)), (k, f)
    x, Pb = kf.state()
    x, Pb = x.cpu().numpy(), Pb.cpu().numpy()
    for f in range(B):
        assert _rel(x[:, f], xs[f]) <= TOL
        assert _rel(ref15.from_blocks(Pb[:, f]), Ps[f]) <= TOL
    with pytest.raises(ValueError):
        kf.update(np.zeros((3, B)), sensor='imu')


@pytest.mark.parametrize('kernel', ['lane', 'chain'])
def test_ref15_fp32_events_vs_fp64_oracle(kernel):
    """fp32 handle (north_star: 1e-3 relative in fp32) against the fp64 oracle fed the same
    fp32-rounded inputs, on realistic 200 Hz IMU + 10 Hz GPS streams."""
    import os as _os
    rng = np.random.default_rng(41)
    B, T = 96, 200
    etype = np.ones((T, B), np.uint8)
    etype[::20] = 0
    dt = np.full((T, B), 0.005)
    pay = np.zeros((T, 9, B))
    pay[:, 0:3] = rng.normal(0, 0.05, (T, 3, B))
    pay[:, 3:6] = rng.normal(0, 0.01, (T, 3, B))
    pay[:, 6:9] = rng.normal(0, 0.3, (T, 3, B))
    gps = etype == 0
    pay[:, 0:3] = np.where(gps[:, None, :], rng.normal(0, 3, (T, 3, B)), pay[:, 0:3])
    pay32 = pay.astype(np.float32)
    kf = kfmi.BatchedKF('ref15', B, 'f32', options={'events_kernel': kernel})
    tr, ld, _, _ = kf.run_events(etype, dt, pay32)
    tr, ld = tr.double().cpu().numpy(), ld.double().cpu().numpy()
    kf.close()
    worst_x = worst_l = 0.0
    for f in range(0, B, 11):
        x, P = np.zeros(15), ref_kf.P0_REF15.copy()
        for t in range(T):
            p = pay32[t, :, f].astype(np.float64)
            if etype[t, f] == 0:
                x, P = ref_kf.step15(x, P, 'GPS', {'easting': p[0], 'northing': p[1], 'altitude': p[2]}, dt[t, f])
            else:
                x, P = ref_kf.step15(x, P, 'IMU', ['t', *p], dt[t, f])
            ref_ld = np.linalg.slogdet(P)[1]
            worst_x = max(worst_x, np.linalg.norm(tr[t, :, f] - x[:6]) / max(np.linalg.norm(x[:6]), 1.0))
            worst_l = max(worst_l, abs(ld[t, f] - ref_ld) / max(abs(ref_ld), 1.0))
    assert worst_x <= 1e-3 and worst_l <= 1e-3, (worst_x, worst_l)


@pytest.mark.parametrize('model', ['ref15', 'ref8'])
@pytest.mark.parametrize('dtype', ['f64', 'f32'])
@pytest.mark.parametrize('records,gated', [(True, False), (False, False), (True, True)])
@pytest.mark.parametrize('B', [1040, 4096])
def test_lds_kernel_matches_lane_kernel(model, dtype, records, gated, B):
    """ref_events_lds_kernel (inputs staged through LDS by DMA; the default when B % 16 == 0)
    against the register-input kernel on the same streams: the same per-event arithmetic, so
    states, records, gate decisions and statuses agree to rounding.  B = 1040 leaves the last
    wave with 16 live lanes (its dead lanes still move their share of every DMA)."""
    rng = np.random.default_rng(41 + B + (dtype == 'f32'))
    n = 15 if model == 'ref15' else 8
    T = 37
    etype = rng.choice([0, 1, 1, 1, 2], size=(T, B)).astype(np.uint8)
    etype[30:, ::7] = 255
    dt = rng.uniform(0.0, 0.05, (T, B))
    pay = np.zeros((T, 9, B))
    pay[:, 0:3] = rng.normal(0, 20, (T, 3, B))
    pay[:, 3:6] = rng.normal(0, 0.05, (T, 3, B))
    pay[:, 6:9] = rng.normal(0, 0.5, (T, 3, B))
    x0 = rng.normal(0, 5, (B, n))
    P0 = ref15.P0 if model == 'ref15' else ref8.P0
    P0b = np.repeat(ref15.to_blocks(P0)[None], B, 0)
    P0b[B - 3] = -P0b[B - 3]                            # a non-positive-definite filter in the last wave
    thr = None
    if gated:
        ld = _events_run(model, 'lane', etype, dt, pay, x0, P0b, dtype=dtype)[1]
        thr = float(np.median(ld[np.isfinite(ld)]))
    lane = _events_run(model, 'lane', etype, dt, pay, x0, P0b, thr, dtype, records)
    lds = _events_run(model, 'lds', etype, dt, pay, x0, P0b, thr, dtype, records)
    tol = 1e-12 if dtype == 'f64' else 1e-5
    for name, a, b in zip(('traj', 'logdet', 'updated', 'cov', 'x', 'P', 'status'), lane, lds):
        if a is None:
            assert b is None, name
            continue
        ok = np.isfinite(a)
        np.testing.assert_array_equal(ok, np.isfinite(b), err_msg=name)
        if name in ('updated', 'status'):
            np.testing.assert_array_equal(a, b, err_msg=name)
        else:
            assert _rel(b[ok], a[ok]) <= tol, name
    assert lds[6][B - 3] == kfmi.KF_ENOTSPD and (lds[6][np.arange(B) != B - 3] == 0).all()
    if gated:
        assert 0 < lds[2].mean() < 1
