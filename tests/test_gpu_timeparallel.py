"""One filter over a long event stream, parallel over time (kfmi.ref15.run_stream_parallel) —
needs an MI355X.

The chunked run must give the single-filter run's records: the covariance warm-up reaches the
sequential covariance and the chunk maps are affine, so agreement is at roundoff (checked at
1e-9 relative in f64, the north_star's 1e-6 against the oracle); f32 against f64 at 1e-3.
"""
import numpy as np
import pytest
import torch

import kfmi
from kfmi import ingest, ref15
from oracle import cpu_kf, ref_kf

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0)))


def _stream(T, seed=1, gps_every=20, keep=0.7, skips=0):
    """A 200 Hz IMU stream with ~10 Hz GPS fixes (some missing) along a drive; ``skips`` events
    become NONE (the driver's dt < 0 rule)."""
    rng = np.random.default_rng(seed)
    et = np.ones(T, np.uint8)
    gi = np.arange(0, T, gps_every)
    gi = gi[rng.random(len(gi)) < keep]
    et[gi] = ref15.GPS
    et[0] = ref15.GPS
    if skips:
        et[rng.choice(np.arange(1, T), skips, replace=False)] = ref15.NONE
    dt = np.full(T, 0.005)
    dt[0] = 0.0
    t = np.arange(T) * 0.005
    pos = np.stack([300 + 3.3 * t, -200 + 2.2 * t, 0.05 * np.cumsum(rng.normal(0, 0.1, T))], 1)
    pay = np.zeros((T, 9))
    g = et == 0
    pay[g, 0:3] = pos[g] + rng.normal(0, 1.5, (int(g.sum()), 3))
    i = ~g
    pay[i, 0] = rng.normal(0, 0.02, int(i.sum()))
    pay[i, 1] = rng.normal(-0.05, 0.01, int(i.sum()))
    pay[i, 2] = np.cumsum(rng.normal(0, 2e-4, T))[i]
    pay[i, 3:6] = rng.normal(0, 0.01, (int(i.sum()), 3))
    pay[i, 6:9] = rng.normal(0, 0.3, (int(i.sum()), 3))
    x0 = np.zeros(15)
    x0[0:3] = pay[0, 0:3]
    return et, dt, pay, x0


def _sequential(et, dt, pay, x0, dtype='f64'):
    kf = kfmi.BatchedKF('ref15', 1, dtype)
    npd = np.float64 if dtype == 'f64' else np.float32
    kf.set_state(x0[:, None].astype(npd), ref15.to_blocks(ref15.P0)[:, None].astype(npd))
    tr, ld, _, _ = kf.run_events(et[:, None], dt[:, None], pay[:, :, None].astype(npd))
    x, P = kf.state()
    out = tr[:, :, 0].double().cpu().numpy(), ld[:, 0].double().cpu().numpy(), x[:, 0].double().cpu().numpy(), \
        P[:, 0].double().cpu().numpy()
    kf.close()
    return out


def _parallel(et, dt, pay, x0, **kw):
    dev = torch.device('cuda', 0)
    r = ref15.run_stream_parallel(torch.as_tensor(et, device=dev), torch.as_tensor(dt, device=dev),
                                  torch.as_tensor(pay, device=dev), x0, ref15.to_blocks(ref15.P0), **kw)
    if r is None:
        return None
    tr, ld, x, P, _ = r
    return tr.double().cpu().numpy(), ld.double().cpu().numpy(), x.double().cpu().numpy(), P.double().cpu().numpy()


@pytest.mark.parametrize('T,chunk,skips', [(60000, None, 0), (45001, 777, 50), (5000, 256, 3)])
def test_parallel_equals_single_filter(T, chunk, skips):
    """Records, final state and covariance equal the one-filter run; ragged last chunk, NONE
    events, and (T = 5000) chunks whose warm-up window reaches the stream start (exact)."""
    et, dt, pay, x0 = _stream(T, seed=T, skips=skips)
    seq = _sequential(et, dt, pay, x0)
    par = _parallel(et, dt, pay, x0, chunk=chunk)
    assert par is not None, ref15.parallel_check
    assert ref15.parallel_check['cov_gap'] == 0.0  # the warm-up reached the covariance bitwise
    for a, b in zip(par, seq):
        assert a.shape == b.shape
        assert _rel(a, b) <= 1e-9


def test_parallel_vs_oracle():
    """The reference's step (oracle/cpu_kf.c, dense 15x15, its op order) over the whole stream."""
    et, dt, pay, x0 = _stream(30000, seed=7)
    tr, ld, _, _ = _parallel(et, dt, pay, x0, chunk=512)
    rt, rl = cpu_kf.ref15_events(et[:, None], dt[:, None], pay[:, :, None], x0[:, None], ref_kf.P0_REF15, nthreads=4)
    assert _rel(tr, rt[:, :, 0]) <= 1e-6
    assert _rel(ld, rl[:, 0]) <= 1e-6


def test_parallel_f32():
    et, dt, pay, x0 = _stream(40000, seed=3)
    seq = _sequential(et, dt, pay, x0)
    par = _parallel(et, dt, pay, x0, dtype='f32')
    assert par is not None, ref15.parallel_check
    assert _rel(par[0], seq[0]) <= 1e-3 and _rel(par[1], seq[1]) <= 1e-3


def test_short_warmup_is_refused():
    """A warm-up too short for the covariance to converge fails the check (None: the caller
    falls back to one filter) instead of returning wrong records."""
    et, dt, pay, x0 = _stream(20000, seed=5)
    assert _parallel(et, dt, pay, x0, chunk=1000, warmup=16) is None
    assert ref15.parallel_check['reason'] == 'covariance warm-up did not converge'


def test_run_full_stream_parallel_matches_single_filter():
    """run_kalman_filter_full's device driver picks the chunked run for a long window; same
    outputs as parallel=False."""
    et, dt, pay, x0 = _stream(70000, seed=11)
    dev = torch.device('cuda', 0)
    t = 1.7e9 + np.cumsum(dt)
    n = len(et)
    stream = ingest.EventStream(etype=torch.as_tensor(et, device=dev), t=torch.as_tensor(t, device=dev),
                                payload=torch.as_tensor(pay, device=dev),
                                src=torch.zeros(n, dtype=torch.int32, device=dev),
                                zone_number=torch.zeros(n, dtype=torch.int8, device=dev),
                                zone_letter=torch.zeros(n, dtype=torch.uint8, device=dev),
                                first_valid_index=0, gyro_bias=np.zeros(3), accel_bias=np.zeros(3),
                                utm_origin=np.zeros(2), n_fixes=int((et == 0).sum()), n_imu=int((et == 1).sum()))
    a = ref15.run_full_stream(stream, 0, n, parallel=True, parallel_min_events=1000)
    b = ref15.run_full_stream(stream, 0, n, parallel=False)
    assert np.array_equal(a[0], b[0])
    for u, v in zip(a[1:4], b[1:4]):
        assert _rel(u, v) <= 1e-9
    assert a[4] == b[4]
