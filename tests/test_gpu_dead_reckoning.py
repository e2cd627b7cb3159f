"""hw5_2.run_dead_reckoning_for_IMU (hw5_2.py:382-436) on the GPU — needs an MI355X.

The 8-state filter over the IMU events alone (fixes skipped, first dt 0, x0 = 0), against the
reference's own outputs (tests/golden/ref8_full.npz: in-order and out-of-order streams) through
both routes of kfmi.ref8.run_dead_reckoning — the reference's event list (host-built stream, one
kf_run_events launch) and an EventStream (kf_events_select + kf_events_dt on the device) — and,
over the bench's whole synthetic drive log (616,322 IMU rows, the time-parallel kf_run_stream
route), against the C oracle's walk of the oracle's own ingest (oracle/cpu_kf.c
cpu_ref8_dead_reckoning, pinned to the goldens by test_oracle.py).  Tolerance: 1e-6 relative
(north_star, fp64).
"""
import numpy as np
import pytest
import torch

import bench
from golden_events import unpack_events
from kfmi import _lib, ingest, ref8
from oracle import cpu_kf, ref_ingest, ref_kf

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0))) if a.size else 0.0


def _stream_from_golden(g, prefix):
    """An EventStream holding a golden's merged events (as kf_ingest lays them out)."""
    et = np.asarray(g[prefix + 'ev_type'], np.uint8)
    t = np.asarray(g[prefix + 'ev_t'], np.float64)
    pay = np.zeros((len(t), 9))
    pay[et == 0, 0:3] = g[prefix + 'ev_gps'][et == 0]
    pay[et == 1] = g[prefix + 'ev_imu'][et == 1]
    d = torch.device('cuda', 0)
    n = len(t)
    return ingest.EventStream(torch.from_numpy(et).to(d), torch.from_numpy(t).to(d), torch.from_numpy(pay).to(d),
                              torch.arange(n, dtype=torch.int32, device=d), torch.zeros(n, dtype=torch.int8, device=d),
                              torch.zeros(n, dtype=torch.uint8, device=d), 0, np.zeros(3), np.zeros(3), np.zeros(2),
                              int((et == 0).sum()), int((et == 1).sum()), True)


@pytest.mark.parametrize('prefix', ['', 'ooo_'])
def test_dead_reckoning_vs_reference_golden(golden_dir, prefix):
    g = np.load(f'{golden_dir}/ref8_full.npz')
    want = g[prefix + 'dr_states']
    events = unpack_events(g, prefix)
    st = ref8.run_dead_reckoning(events)
    assert np.array(st).shape == want.shape
    assert _rel(st, want) <= 1e-6
    st2, P2 = ref8.run_dead_reckoning(_stream_from_golden(g, prefix), return_covariance=True)
    assert np.array(st2).shape == want.shape
    assert _rel(st2, want) <= 1e-6
    _, rP = ref_kf.run_dead_reckoning_8state(events)
    assert _rel(P2, rP) <= 1e-6


def _stream_of_list(events):
    """An EventStream over a reference event list (fixes: easting, northing, altitude)."""
    et = np.array([0 if e[1] == 'GPS' else 1 for e in events], np.uint8)
    t = np.array([e[2] for e in events], np.float64)
    pay = np.array([ref8.event_payload(e[1], e[3]) for e in events], np.float64).reshape(len(events), 9)
    d = torch.device('cuda', 0)
    n = len(t)
    return ingest.EventStream(torch.from_numpy(et).to(d), torch.from_numpy(t).to(d), torch.from_numpy(pay).to(d),
                              torch.arange(n, dtype=torch.int32, device=d), torch.zeros(n, dtype=torch.int8, device=d),
                              torch.zeros(n, dtype=torch.uint8, device=d), 0, np.zeros(3), np.zeros(3), np.zeros(2),
                              int((et == 0).sum()), int((et == 1).sum()), True)


def test_dead_reckoning_edge_cases(golden_dir):
    """Logs with no IMU event (no estimates, P0 back), a single IMU event (dt 0: one update from
    P0), fixes before the first IMU event (they never move the previous time), through both
    routes against the oracle's walk; and the golden log forced through the time-parallel route
    (kf_run_stream at its shortest chunks) against the reference's outputs."""
    g = np.load(f'{golden_dir}/ref8_full.npz')
    events = unpack_events(g, '')
    gps = [e for e in events if e[1] == 'GPS']
    imu_idx = [i for i, e in enumerate(events) if e[1] == 'IMU']
    first_imu = imu_idx[0]
    cases = {
        'gps_only': gps[:5],
        'one_imu': [events[first_imu]],
        'fixes_first': gps[:3] + [e for e in events if e[1] == 'IMU'][:7] + gps[3:5],
    }
    for name, ev in cases.items():
        want, wP = ref_kf.run_dead_reckoning_8state(ev)
        for route in (ev, _stream_of_list(ev)):
            st, P = ref8.run_dead_reckoning(route, return_covariance=True)
            assert len(st) == len(want), name
            assert _rel(st, want) <= 1e-6, name
            assert _rel(P, wP) <= 1e-6, name
    want = g['dr_states']
    st = ref8.run_dead_reckoning(_stream_from_golden(g, ''), parallel_min_events=1)
    assert np.array(st).shape == want.shape
    assert _rel(st, want) <= 1e-6


@pytest.mark.parametrize('n,p_keep', [(1, 1.0), (2047, 0.5), (2048, 1.0), (2049, 0.0), (4_500_001, 0.97)])
def test_events_select_sizes(n, p_keep):
    """kf_events_select over one tile and its edges, none and all kept, and more tiles than
    blocks (several tiles per block): every kept event's time, payload row and position, in
    order, through the raw C ABI with each output alone too."""
    import ctypes
    rng = np.random.default_rng(n)
    et = np.where(rng.random(n) < p_keep, 1, 0).astype(np.uint8)
    d = torch.device('cuda', 0)
    et_d = torch.from_numpy(et).to(d)
    t_d = torch.arange(n, dtype=torch.float64, device=d) * 0.5
    pay_d = torch.arange(9 * n, dtype=torch.float64, device=d).reshape(n, 9)
    k_want = np.nonzero(et == 1)[0]
    lib = _lib.lib()
    for outs in ('all', 't', 'payload', 'src'):
        t_o = torch.full((max(len(k_want), 1),), -1.0, dtype=torch.float64, device=d)
        p_o = torch.full((max(len(k_want), 1), 9), -1.0, dtype=torch.float64, device=d)
        s_o = torch.full((max(len(k_want), 1),), -1, dtype=torch.int32, device=d)
        kept = ctypes.c_int64(-1)
        ptr = lambda x, name: ctypes.c_void_p(x.data_ptr()) if outs in ('all', name) else None  # noqa: E731
        rc = lib.kf_events_select(n, ctypes.c_void_p(et_d.data_ptr()), ctypes.c_void_p(t_d.data_ptr()),
                                  ctypes.c_void_p(pay_d.data_ptr()), 1, ptr(t_o, 't'), ptr(p_o, 'payload'),
                                  ptr(s_o, 'src'), ctypes.byref(kept),
                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0, _lib.last_error()
        assert kept.value == len(k_want)
        m = len(k_want)
        if outs in ('all', 't'):
            np.testing.assert_array_equal(t_o[:m].cpu().numpy(), k_want * 0.5)
        if outs in ('all', 'payload'):
            np.testing.assert_array_equal(p_o[:m].cpu().numpy(), (9 * k_want[:, None] + np.arange(9)).astype(float))
        if outs in ('all', 'src'):
            np.testing.assert_array_equal(s_o[:m].cpu().numpy(), k_want)


def test_events_select_refuses_capture():
    """kf_events_select synchronises to return its count, so inside a hipGraph capture it
    returns KF_EINVAL before queuing anything: the capture stays valid, the graph (holding a
    torch op captured around the refused call) replays, and the next eager call works."""
    import ctypes
    d = torch.device('cuda', 0)
    n = 5000
    et_d = (torch.arange(n, device=d) % 3 == 0).to(torch.uint8)
    t_d = torch.arange(n, dtype=torch.float64, device=d)
    t_o = torch.empty(n, dtype=torch.float64, device=d)
    lib = _lib.lib()
    kept = ctypes.c_int64(-1)
    x = torch.zeros(4, device=d)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        x += 1
        rc = lib.kf_events_select(n, ctypes.c_void_p(et_d.data_ptr()), ctypes.c_void_p(t_d.data_ptr()), None, 1,
                                  ctypes.c_void_p(t_o.data_ptr()), None, None, ctypes.byref(kept),
                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
        x += 1
    assert rc == _lib.KF_EINVAL and 'capturable' in _lib.last_error() and kept.value == 0
    g.replay()
    torch.cuda.synchronize()
    assert float(x[0]) == 2.0
    rc = lib.kf_events_select(n, ctypes.c_void_p(et_d.data_ptr()), ctypes.c_void_p(t_d.data_ptr()), None, 1,
                              ctypes.c_void_p(t_o.data_ptr()), None, None, ctypes.byref(kept),
                              ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0 and kept.value == (n + 2) // 3
    np.testing.assert_array_equal(t_o[:kept.value].cpu().numpy(), np.arange(0, n, 3, dtype=float))


def test_dead_reckoning_select_and_dt():
    """kf_events_select keeps one type in stream order; kf_events_dt with prev0 = NaN gives the
    first event dt 0 (hw5_2.py:401, 407) and the rest raw differences (no guard)."""
    rng = np.random.default_rng(3)
    n = 100_003
    et = rng.choice([0, 1, 1, 1], n).astype(np.uint8)
    t = np.cumsum(rng.uniform(0.0, 0.01, n)) + 1.7e9
    t[500], t[501] = t[501], t[500]
    pay = rng.normal(size=(n, 9))
    d = torch.device('cuda', 0)
    s = ingest.EventStream(torch.from_numpy(et).to(d), torch.from_numpy(t).to(d), torch.from_numpy(pay).to(d),
                           torch.arange(n, dtype=torch.int32, device=d), torch.zeros(n, dtype=torch.int8, device=d),
                           torch.zeros(n, dtype=torch.uint8, device=d), 0, np.zeros(3), np.zeros(3), np.zeros(2),
                           int((et == 0).sum()), int((et == 1).sum()), True)
    for ty in (0, 1, 7):
        ts, ps, src = ingest.select_events(s, ty)
        k = np.nonzero(et == ty)[0]
        np.testing.assert_array_equal(src.cpu().numpy(), k)
        np.testing.assert_array_equal(ts.cpu().numpy(), t[k])
        np.testing.assert_array_equal(ps.cpu().numpy(), pay[k])
    ts, _, _ = ingest.select_events(s, 1)
    dt, eo = ingest.events_dt(ts, float('nan'), _lib.KF_DT_RAW)
    th = t[et == 1]
    np.testing.assert_array_equal(dt.cpu().numpy(), np.r_[0.0, np.diff(th)])
    assert (eo.cpu().numpy() == _lib.KF_EVENT_IMU).all()
    with pytest.raises(_lib.KFError):
        ingest.events_dt(ts, float('nan'), _lib.KF_DT_MONOTONE)


def test_dead_reckoning_whole_log_vs_oracle(tmp_path):
    """The bench's whole synthetic drive log (config 1ref8's CSVs: 30,758 GPS rows, 616,322 IMU
    rows) ingested on the device as hw5_2 does (no altitude), dead-reckoned through the
    time-parallel route, against the C oracle's walk of the oracle's own ingest, every IMU
    event."""
    cfg = bench.CONFIGS['1ref8']
    gp, ip = bench.synth_log(cfg, str(tmp_path))
    stream = ingest.ingest_arrays(ingest.read_csv(gp, 4), ingest.read_csv(ip, 11), with_altitude=False, device=0)
    st, P = ref8.run_dead_reckoning(stream, return_covariance=True)
    chk = dict(ref8.dead_reckoning_check)
    assert chk['ok'] and chk['chunks'] > 1000, chk
    assert len(st) == stream.n_imu == cfg['n_imu']
    events, _, _ = ref_ingest.ingest(gp, ip, with_altitude=False)
    et = np.array([0 if e[1] == 'GPS' else 1 for e in events], np.uint8)
    th = np.array([e[2] for e in events])
    ph = np.zeros((len(events), 9))
    ph[et == 1] = [e[3][1:10] for e in events if e[1] == 'IMU']
    rt, _ = cpu_kf.ref8_dead_reckoning(et, th, ph)
    assert rt.shape == (len(st), 3)
    assert _rel(st, rt) <= 1e-6
