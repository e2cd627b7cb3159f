"""One filter over a long event stream, parallel over time (kf_run_stream through
kfmi.ref15.run_stream_parallel, BatchedKF.run_stream and kf_run_events' own route) — needs an
MI355X.

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


def _sequential(et, dt, pay, x0, dtype='f64', model='ref15'):
    """The single filter (kf_run_events_seq: never the stream route)."""
    kf = kfmi.BatchedKF(model, 1, dtype)
    npd = np.float64 if dtype == 'f64' else np.float32
    P0 = ref15.to_blocks(ref15.P0) if model == 'ref15' else kf.state()[1].double().cpu().numpy()[:, 0]
    kf.set_state(x0[:, None].astype(npd), P0[:, None].astype(npd))
    tr, ld, up, cv = kf.run_events(et[:, None], dt[:, None], pay[:, :, None].astype(npd), updated=True, cov=True,
                                   sequential=True)
    x, P = kf.state()
    out = tuple(v.double().cpu().numpy() for v in (tr[:, :, 0], ld[:, 0], x[:, 0], P[:, 0], cv[:, :, 0], up[:, 0]))
    kf.close()
    return out


def _parallel(et, dt, pay, x0, **kw):
    dev = torch.device('cuda', 0)
    tr, ld, x, P, _ = ref15.run_stream_parallel(torch.as_tensor(et, device=dev), torch.as_tensor(dt, device=dev),
                                                torch.as_tensor(pay, device=dev), x0, ref15.to_blocks(ref15.P0), **kw)
    return tr.double().cpu().numpy(), ld.double().cpu().numpy(), x.double().cpu().numpy(), P.double().cpu().numpy()


@pytest.mark.parametrize('final_pass', [False, True])
@pytest.mark.parametrize('T,chunk,skips,warmup', [(60000, None, 0, None), (45001, 777, 50, None),
                                                  (5000, 256, 3, 2560), (30001, 300, 7, -3)])
def test_parallel_equals_single_filter(T, chunk, skips, warmup, final_pass):
    """Records, final state and covariance equal the one-filter run, with the records taken
    from the map pass (default) or from a final pass over the true starts; the covariance
    warm-up by linear-fractional maps (default), by events (T = 5000: chunks whose warm-up
    reaches the stream start are exact) and by maps plus one chunk of events; ragged last
    chunk, NONE events."""
    et, dt, pay, x0 = _stream(T, seed=T, skips=skips)
    seq = _sequential(et, dt, pay, x0)
    par = _parallel(et, dt, pay, x0, chunk=chunk, warmup=warmup, options={'stream_final': int(final_pass)})
    chk = ref15.parallel_check
    assert chk['ok'] and chk['chunks'] > 1, chk
    assert chk['cov_gap'] <= 1e-12  # the warm-up reached the covariance (to roundoff)
    if final_pass:
        assert chk['state_gap'] <= 1e-9  # every chunk's end state meets its successor's start
    else:
        assert np.isnan(chk['state_gap'])  # records from the maps: no state seam is measured
    for a, b in zip(par, seq):
        assert a.shape == b.shape
        assert _rel(a, b) <= 1e-9


def test_parallel_vs_oracle():
    """The reference's step (oracle/cpu_kf.c, dense 15x15, its op order) over the whole stream."""
    et, dt, pay, x0 = _stream(30000, seed=7)
    tr, ld, _, _ = _parallel(et, dt, pay, x0, chunk=512)
    assert ref15.parallel_check['ok']
    rt, rl = cpu_kf.ref15_events(et[:, None], dt[:, None], pay[:, :, None], x0[:, None], ref_kf.P0_REF15, nthreads=4)
    assert _rel(tr, rt[:, :, 0]) <= 1e-6
    assert _rel(ld, rl[:, 0]) <= 1e-6


def test_parallel_f32():
    et, dt, pay, x0 = _stream(40000, seed=3)
    seq = _sequential(et, dt, pay, x0)
    par = _parallel(et, dt, pay, x0, dtype='f32')
    assert ref15.parallel_check['ok'], ref15.parallel_check
    assert _rel(par[0], seq[0]) <= 1e-3 and _rel(par[1], seq[1]) <= 1e-3


def test_short_warmup_falls_back():
    """A warm-up too short for the covariance to converge fails the device check; the
    sequential fallback then rewrites every record: the output is still the single filter's."""
    et, dt, pay, x0 = _stream(20000, seed=5)
    seq = _sequential(et, dt, pay, x0)
    par = _parallel(et, dt, pay, x0, chunk=1000, warmup=16)
    chk = ref15.parallel_check
    assert not chk['ok'] and chk['cov_gap'] > 1e-12, chk
    for a, b in zip(par, seq):
        assert np.array_equal(a, b)


def test_nan_fix_falls_back():
    """A NaN fix mid-stream poisons the state from there on (the covariance is unaffected): the
    chunk maps carry the NaN, the state seam check fails, and the fallback gives the single
    filter's records, NaN and all."""
    et, dt, pay, x0 = _stream(30000, seed=9)
    g = np.nonzero(et == ref15.GPS)[0]
    pay[g[len(g) // 2], 0] = np.nan
    seq = _sequential(et, dt, pay, x0)
    par = _parallel(et, dt, pay, x0, chunk=300)
    assert not ref15.parallel_check['ok']
    assert np.isnan(par[0][-1]).any()
    for a, b in zip(par, seq):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize('final_pass', [False, True])
def test_records_updated_cov_ref8(final_pass):
    """Every record kf_run_events writes (traj, logdet, updated, covariance) and the 8-state
    model, through the C ABI route kf_run_events takes by itself for T >= 65536."""
    T = 70000
    et, dt, pay, x0 = _stream(T, seed=13, skips=20)
    for model in ('ref15', 'ref8'):
        n = 15 if model == 'ref15' else 8
        xs = np.zeros(n)
        xs[0:2] = x0[0:2]
        seq = _sequential(et, dt, pay, xs, model=model)
        kf = kfmi.BatchedKF(model, 1, 'f64', options={'stream_final': int(final_pass)})
        kf.set_state(xs[:, None], kf.state()[1].double().cpu().numpy())
        tr, ld, up, cv = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], updated=True, cov=True)
        chk = kf.stream_check()
        assert chk['ok'] and chk['chunks'] > 1, chk
        x, P = kf.state()
        par = tuple(v.double().cpu().numpy() for v in (tr[:, :, 0], ld[:, 0], x[:, 0], P[:, 0], cv[:, :, 0], up[:, 0]))
        kf.close()
        for a, b in zip(par, seq):
            assert a.shape == b.shape
            assert _rel(a, b) <= 1e-9


def _symmetric_params(model, seed):
    """Caller constants that are the same on every axis (REF15: per state group; REF8: x and y)."""
    rng = np.random.default_rng(seed)
    if model == 'ref15':
        g = lambda lo, hi: np.repeat(rng.uniform(lo, hi, 5), 3)  # noqa: E731 (pos, att, vel, rate, acc)
        q, ri, p0 = g(0.01, 8.0), g(0.02, 120.0), g(20.0, 2e4)
        rg = np.full(3, rng.uniform(0.5, 9.0))
    else:
        def g(lo, hi):  # [x, y, theta, vx, vy, theta_dot, ax, ay]
            a, t, v, w, c = rng.uniform(lo, hi, 5)
            return np.array([a, a, t, v, v, w, c, c])
        q, ri, p0 = g(0.01, 8.0), g(0.02, 120.0), g(20.0, 2e4)
        rg = np.full(2, rng.uniform(0.5, 9.0))
    return ref15.ModelConsts(model, q=q, r_imu=ri, r_gps=rg, p0=p0).params()


@pytest.mark.parametrize('consts', ['reference', 'custom'])
@pytest.mark.parametrize('model', ['ref15', 'ref8'])
@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_axis_symmetric_maps_equal_every_chain(model, dtype, consts):
    """KF_OPT_AXIS_SYM: with the reference's constants (the same on every axis) the stream
    computes the covariance maps of one pva and one aw chain for all; the maps of the others are
    the same arithmetic on the same numbers, so every record, the final state and covariance and
    the device check equal the every-chain run's bit for bit."""
    T = 70000
    et, dt, pay, x0 = _stream(T, seed=21, skips=10)
    n = 15 if model == 'ref15' else 8
    outs = []
    for sym in ('on', 'off'):
        kf = kfmi.BatchedKF(model, 1, dtype, options={'axis_sym': sym},
                            params=_symmetric_params(model, 17) if consts == 'custom' else None)
        P0 = kf.state()[1].cpu().numpy()
        xs = np.zeros((n, 1), P0.dtype)
        xs[0:2, 0] = x0[0:2]
        kf.set_state(xs, P0)
        tr, ld, up, cv = kf.run_events(et[:, None], dt[:, None], pay[:, :, None].astype(P0.dtype), updated=True,
                                       cov=True)
        chk = kf.stream_check()
        assert chk['ok'] and chk['chunks'] > 1, chk
        x, P = kf.state()
        outs.append((tuple(v.cpu().numpy() for v in (tr, ld, up, cv, x, P)), chk['cov_gap']))
        kf.close()
    for a, b in zip(outs[0][0], outs[1][0]):
        np.testing.assert_array_equal(a, b)
    assert outs[0][1] == outs[1][1]


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


@pytest.mark.parametrize('warmup', [-1, 2048])
def test_repeated_runs_on_one_handle(warmup):
    """The check words (verdict, gaps, the scan's block counter) are re-initialised by every
    call: a second run_stream on the same handle (its workspace reused) passes its checks and
    gives the same records (covariance maps, and an event warm-up)."""
    et, dt, pay, x0 = _stream(20000, seed=17)
    dev = torch.device('cuda', 0)
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    P0b = ref15.to_blocks(ref15.P0)[:, None]
    outs = []
    for _ in range(2):
        kf.set_state(x0[:, None], P0b)
        tr, ld, _, _ = kf.run_stream(torch.as_tensor(et, device=dev), torch.as_tensor(dt, device=dev),
                                     torch.as_tensor(pay, device=dev), chunk=200, warmup=warmup)
        chk = kf.stream_check()
        assert chk['ok'] and chk['chunks'] > 1, chk
        outs.append((tr.cpu().numpy(), ld.cpu().numpy()))
    kf.close()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)


def test_many_chunks_multi_round_scan():
    """More chunks than one scan round holds (256 x 256 tiles): 1.1M events in chunks of 16 give
    68,750 chunks, so the tile-start scan carries over two rounds; records, final state and
    covariance equal the single filter's."""
    et, dt, pay, x0 = _stream(1_100_000, seed=23, skips=100)
    seq = _sequential(et, dt, pay, x0)
    par = _parallel(et, dt, pay, x0, chunk=16)
    chk = ref15.parallel_check
    assert chk['ok'] and chk['chunks'] > 65536, chk
    for a, b in zip(par, seq):
        assert a.shape == b.shape
        assert _rel(a, b) <= 1e-9


def test_many_tiles_top_scan():
    """Far more chunks than one scan round of tiles (2.2M events in chunks of 8: 275,000 chunks,
    1,075 tiles, five rounds of the top kernel, kf_ref.hip phase 3, instead of every starts block
    redoing its prefix): records, final state and covariance equal the single filter's."""
    et, dt, pay, x0 = _stream(2_200_000, seed=31, skips=40)
    seq = _sequential(et, dt, pay, x0)
    par = _parallel(et, dt, pay, x0, chunk=8)
    chk = ref15.parallel_check
    assert chk['ok'] and chk['chunks'] > 256 * 1024, chk
    for a, b in zip(par, seq):
        assert a.shape == b.shape
        assert _rel(a, b) <= 1e-9


def test_stream_run_replays_as_a_hip_graph():
    """kf_run_stream's launches (after a first eager call has sized the workspace) capture into a
    hipGraph as they are — no host synchronisation or allocation — and the replay gives the
    eager run's records and final state."""
    et, dt, pay, x0 = _stream(40000, seed=29, skips=30)
    dev = torch.device('cuda', 0)
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    P0b = torch.as_tensor(ref15.to_blocks(ref15.P0)[:, None], device=dev)
    x0d = torch.as_tensor(x0[:, None], device=dev)
    etd, dtd, payd = (torch.as_tensor(v, device=dev) for v in (et, dt, pay))
    T = len(et)
    tr, ld = kf.empty(T, 6, 1), kf.empty(T, 1)

    def run():
        kf.set_state(x0d, P0b)
        out = kf.run_stream(etd, dtd, payd)
        tr.copy_(out[0])
        ld.copy_(out[1])

    run()
    torch.cuda.synchronize()
    eager = (tr.cpu().numpy().copy(), ld.cpu().numpy().copy(), kf.state()[0].cpu().numpy())
    assert kf.stream_check()['ok']
    tr.zero_()
    ld.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    g.replay()
    torch.cuda.synchronize()
    replay = (tr.cpu().numpy(), ld.cpu().numpy(), kf.state()[0].cpu().numpy())
    for a, b in zip(replay, eager):
        np.testing.assert_array_equal(a, b)
    assert kf.stream_check()['ok']
    kf.close()



def test_gated_stream_route_replays_as_a_hip_graph():
    """The gated one-filter route with the look-ahead fallback (r_value = -10: the seam check
    fails, the chunked pass updated ~3 % of events) captured into a hipGraph after an eager call:
    the device choice and both queued fallback kernels replay as they are, and the replay gives
    the eager records, flags and final state."""
    et, dt, pay, x0 = _stream(70000, seed=11)
    dev = torch.device('cuda', 0)
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    P0b = torch.as_tensor(ref15.to_blocks(ref15.P0)[:, None], device=dev)
    x0d = torch.as_tensor(x0[:, None], device=dev)
    etd, dtd, payd = (torch.as_tensor(v, device=dev) for v in (et[:, None], dt[:, None], pay[:, :, None]))
    T = len(et)
    tr, ld = kf.empty(T, 6, 1), kf.empty(T, 1)
    up = torch.empty(T, 1, dtype=torch.uint8, device=dev)

    def run():
        kf.set_state(x0d, P0b)
        out = kf.run_events(etd, dtd, payd, updated=True, threshold=-10.0)
        tr.copy_(out[0])
        ld.copy_(out[1])
        up.copy_(out[2])

    run()
    torch.cuda.synchronize()
    eager = (tr.cpu().numpy().copy(), ld.cpu().numpy().copy(), up.cpu().numpy().copy(), kf.state()[0].cpu().numpy())
    chk = kf.stream_check()
    assert not chk['ok'] and chk['fallback'] == 'gated', chk
    tr.zero_()
    ld.zero_()
    up.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        run()
    g.replay()
    torch.cuda.synchronize()
    replay = (tr.cpu().numpy(), ld.cpu().numpy(), up.cpu().numpy(), kf.state()[0].cpu().numpy())
    for a, b in zip(replay, eager):
        np.testing.assert_array_equal(a, b)
    assert kf.stream_check()['fallback'] == 'gated'
    kf.close()

def _gated(et, dt, pay, x0, thr, sequential):
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    kf.set_state(x0[:, None], ref15.to_blocks(ref15.P0)[:, None])
    tr, ld, up, cv = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], updated=True, cov=True, threshold=thr,
                                   sequential=sequential)
    chk = None if sequential else kf.stream_check()
    x, P = kf.state()
    out = tuple(v.double().cpu().numpy() for v in (tr[:, :, 0], ld[:, 0], x[:, 0], P[:, 0], cv[:, :, 0]))
    flags = up[:, 0].cpu().numpy()
    kf.close()
    return out, flags, chk


@pytest.mark.parametrize('offset,absolute,stands,fallback', [(0.5, None, True, None), (1.0, None, True, None),
                                                             (2.0, None, False, 'chain'), (None, -30.0, False, 'chain'),
                                                             (None, -20.0, False, 'gated'),
                                                             (None, -10.0, False, 'gated')])
def test_gated_route_equals_single_filter(offset, absolute, stands, fallback):
    """kf_run_events' route for one long GATED filter (the adaptive threshold, kf_workers.py:
    959-1058): chunk starts from 2048 events of warm-up that apply the gate, every pass gated.
    Where the gate blocks few updates (thresholds 0.5 / 1.0 above the median record: 2 % / 7 %
    blocked) the warm-up meets the covariance and the chunked records stand; where it blocks many
    (2.0 above: 20 %; -30: 58 %; -20: 89 %; the reference's r_value = -10: 97 %) the gated
    covariance's sawtooth keeps the phase it started with, the seam check fails and the
    sequential fallback rewrites every record: the chain kernel (bitwise the sequential filter)
    or, where the chunked pass updated at most 1 event in 8, the look-ahead kernel (flags equal,
    records to rounding).  Either way: the sequential gated filter's records, update flags and
    final state."""
    et, dt, pay, x0 = _stream(70000, seed=11)
    base, _, _ = _gated(et, dt, pay, x0, None, True)
    thr = absolute if offset is None else float(np.median(base[1])) + offset
    seq, f_seq, _ = _gated(et, dt, pay, x0, thr, True)
    par, f_par, chk = _gated(et, dt, pay, x0, thr, False)
    assert chk['chunks'] > 1 and chk['warmup'] == 2048 and chk['ok'] == stands, chk
    assert chk['fallback'] == fallback, chk
    assert 0 < f_seq.mean() < 1 or offset == 0.5
    np.testing.assert_array_equal(f_par, f_seq)
    for a, b in zip(par, seq):
        assert a.shape == b.shape and _rel(a, b) <= 1e-9
    if fallback == 'chain':
        for a, b in zip(par, seq):
            assert np.array_equal(a, b)   # the fallback is the sequential kernel


def _one_gated(et, dt, pay, x0, thr, kernel, dtype='f64'):
    kf = kfmi.BatchedKF('ref15', 1, dtype, options={'events_kernel': kernel})
    kf.set_state(x0[:, None], ref15.to_blocks(ref15.P0)[:, None])
    tr, ld, up, cv = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], updated=True, cov=True, threshold=thr,
                                   sequential=True)
    x, P = kf.state()
    out = tuple(v.double().cpu().numpy() for v in (tr[:, :, 0], ld[:, 0], x[:, 0], P[:, 0], cv[:, :, 0]))
    flags, st = up[:, 0].cpu().numpy(), int(kf.status().sum().item())
    kf.close()
    return out, flags, st


@pytest.mark.parametrize('T,thr,skips', [(1, -10.0, 0), (7, -10.0, 0), (9, -10.0, 0), (300, -10.0, 0),
                                         (5000, -10.0, 300), (70000, -10.0, 0), (70000, -20.0, 0),
                                         (70000, -30.0, 0), (70000, -36.4, 0), (70000, 50.0, 0)])
def test_lookahead_gated_kernel_equals_chain(T, thr, skips):
    """KF_OPT_EVENTS_KERNEL = 4 (ref_chain_gated_kernel, one wave, opt-in): eight events of
    closed-form predicts ahead of the gate (additive F, Q(dt)·dt), the first event
    whose gate opens taken by the chain kernel's step.  Against the chain kernel's sequential
    gated filter (= 2) from 3 % (the reference's r_value = -10) to 98 % of events updated, a
    gate that never opens (50) and NONE events inside the look-ahead: flags equal, records and
    final state within 1e-9 relative (measured <= 1.8e-12: the closed form sums the predicts in
    another order), status equal."""
    et, dt, pay, x0 = _stream(max(T, 64), seed=11, skips=skips)
    et, dt, pay = et[:T], dt[:T], pay[:T]
    g, fg, sg = _one_gated(et, dt, pay, x0, thr, 'gated')
    c, fc, sc = _one_gated(et, dt, pay, x0, thr, 'chain')
    assert sg == sc == 0
    np.testing.assert_array_equal(fg, fc)
    for a, b in zip(g, c):
        assert a.shape == b.shape and _rel(a, b) <= 1e-9


def test_lookahead_gated_kernel_is_f64_only():
    """In f32 the closed-form predicts round differently enough to move gate decisions (8 of
    70,000 flags at r_value = -10, profiles/r06_lookahead/ab_f32.log), so option 4 keeps the
    default kernel there: bitwise the chain kernel's records."""
    et, dt, pay, x0 = _stream(3000, seed=11)
    pay, x0 = pay.astype(np.float32), x0.astype(np.float32)

    def run(kernel):
        kf = kfmi.BatchedKF('ref15', 1, 'f32', options={'events_kernel': kernel})
        kf.set_state(x0[:, None], ref15.to_blocks(ref15.P0).astype(np.float32)[:, None])
        out = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], updated=True, cov=True, threshold=-10.0,
                            sequential=True)
        out = [v.cpu().numpy() for v in out]
        kf.close()
        return out
    for a, b in zip(run('gated'), run('chain')):
        assert np.array_equal(a, b)


@pytest.mark.parametrize('consts', ['reference', 'custom'])
@pytest.mark.parametrize('model', ['ref15', 'ref8'])
def test_lookahead_gated_kernel_models_and_constants(model, consts):
    """The look-ahead kernel on both reference models, with the reference's constants (the
    compiled literals) and a caller's (kf_params: its CUSTOM instantiation reads Q, R, P0 from
    the handle), against the chain kernel: flags equal, records within 1e-9 relative.  The
    threshold sits far enough above the ungated filter's log-dets that most updates are blocked
    (2-50 % applied) and the look-ahead runs are long."""
    T = 20000
    et, dt, pay, x0 = _stream(T, seed=31, skips=40)
    n = 15 if model == 'ref15' else 8
    params = _symmetric_params(model, 5) if consts == 'custom' else None

    def run(kernel, thr):
        kf = kfmi.BatchedKF(model, 1, 'f64', options={'events_kernel': kernel}, params=params)
        P0 = kf.state()[1].cpu().numpy()
        xs = np.zeros((n, 1))
        xs[0:2, 0] = x0[0:2]
        kf.set_state(xs, P0)
        tr, ld, up, cv = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], updated=True, cov=True,
                                       threshold=thr, sequential=True)
        x, P = kf.state()
        out = tuple(v.double().cpu().numpy() for v in (tr, ld, cv, x, P))
        flags, st = up.cpu().numpy(), int(kf.status().sum().item())
        kf.close()
        return out, flags, st
    base, _, _ = run('chain', None)
    for above in (40.0, 20.0, 10.0, 5.0, 2.5):  # the gate opens above the threshold: from rare to frequent
        thr = float(np.median(base[1])) + above
        c, fc, sc = run('chain', thr)
        if fc.mean() >= 0.02:
            break
    assert 0.02 <= fc.mean() < 0.5, (above, fc.mean())
    g, fg, sg = run('gated', thr)
    assert sg == sc == 0
    np.testing.assert_array_equal(fg, fc)
    for a, b in zip(g, c):
        assert a.shape == b.shape and _rel(a, b) <= 1e-9
