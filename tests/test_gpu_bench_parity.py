"""The SURVEY §8(d) parity gate at the bench rows' full sizes, against the oracle — needs an MI355X.

Each test runs a bench row's own workload (the generators bench.py times: ``ref15_streams``,
``sched_streams``, ``bf_events``, ``synth_log``) through the C ABI at the size the bench
measures, and checks it against the CPU oracle on >= 4096 filters spread over the batch plus
the wave and batch edges, every step: ``||x - x_ref||_2 / max(||x_ref||_2, 1)`` and
``|dlogdet| / max(|logdet_ref|, 1)`` <= 1e-6 in fp64, <= 1e-3 in fp32 (the fp64 oracle fed the
same fp32-rounded inputs).

The oracle here is ``oracle/cpu_kf.c`` (the reference's dense 15x15 step in its op order, C,
OpenMP): its event step is pinned to the NumPy restatement by
``test_oracle.py::test_c_ref15_events_vs_numpy_oracle`` and its scheduled driver to the
reference's own outputs by ``test_oracle.py::test_c_ref15_sched_vs_goldens``; the brute-force
winner is also checked against the NumPy restatement of the reference's search
(``oracle/ref_kf.run_brute_force``), and config 1 is ingested by the oracle's restatement of the
reference's ingest (``oracle/ref_ingest``), independently of the device ingest.
"""
import math
from itertools import combinations

import numpy as np
import pytest
import torch

import bench
import kfmi
from kfmi import _lib, ingest, ref15
from oracle import cpu_kf, ref_ingest, ref_kf

pytestmark = pytest.mark.gpu

F64_TOL, F32_TOL = 1e-6, 1e-3


def sample_filters(B, n=4096, seed=0):
    """n filters spread over the batch (one per stratum of B / n), plus the first and last
    waves whole and both sides of the wave boundaries at B/4, B/2 and 3B/4."""
    rng = np.random.default_rng(seed)
    edges = [np.arange(0, min(64, B)), np.arange(max(0, B - 64), B)]
    for q in (B // 4, B // 2, 3 * B // 4):
        w = q - q % 64
        edges.append(np.arange(max(0, w - 2), min(B, w + 2)))
    if B <= n:
        strata = np.arange(B)
    else:
        bounds = np.linspace(0, B, n + 1).astype(np.int64)
        strata = bounds[:-1] + (rng.random(n) * (bounds[1:] - bounds[:-1])).astype(np.int64)
    return np.unique(np.concatenate([strata] + edges))


def parity(traj, ld, rtraj, rld):
    """§8(d) per filter per step: (state error, logdet error); traj [T, W, F], ld [T, F]."""
    return ref_kf.parity_errors(np.asarray(traj, np.float64), np.asarray(ld, np.float64), rtraj, rld)


@pytest.mark.parametrize('config', ['ref15', 'ref15f32'])
def test_ref15_bench_size_vs_oracle(config):
    """The ref15 / ref15f32 rows (2^20 filters x 256 events, the LDS-staged event kernel):
    4096 + edge filters, every event, against the C oracle."""
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[config]
    B, T, k, dt = cfg['B'], cfg['T'], cfg['k'], cfg['dt']
    kf = kfmi.BatchedKF('ref15', B, cfg['dtype'])
    etype, dts, pay = bench.ref15_streams(B, T, dt, k, bench.SEED, dev, kf.torch_dtype)
    tr, ld, _, _ = kf.run_events(etype, dts, pay)
    assert int((kf.status() != 0).sum()) == 0
    kf.close()
    idx = sample_filters(B)
    it = torch.as_tensor(idx, device=dev)
    tr, ld = tr[:, :, it].double().cpu().numpy(), ld[:, it].double().cpu().numpy()
    et, dd, pa = etype[:, it].cpu().numpy(), dts[:, it].cpu().numpy(), pay[:, :, it].double().cpu().numpy()
    del etype, dts, pay
    rt, rl = cpu_kf.ref15_events(et, dd, pa, np.zeros((15, len(idx))), ref_kf.P0_REF15)
    ex, el = parity(tr, ld, rt, rl)
    tol = F64_TOL if cfg['dtype'] == 'f64' else F32_TOL
    assert ex <= tol and el <= tol, (len(idx), ex, el)


def test_sched_bench_size_vs_oracle():
    """The sched row (2^20 filters x 256 events, rates 10..120 Hz, the two passes over the
    bench's 10-double payload records, each pick's time read from rec[9]): the payload rows give
    every output bitwise, and 4096 + edge filters match the oracle's greedy driver pick for pick."""
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS['sched']
    B, T, k, dt = cfg['B'], cfg['T'], cfg['k'], cfg['dt']
    tt, etype, pay, freq, prev = bench.sched_streams(B, T, dt, k, cfg['rates'], 64, bench.SEED, dev)
    kf = kfmi.BatchedKF('ref15', B, 'f64', options=cfg['opts'])
    recs = torch.zeros(T, B, 10, dtype=torch.float64, device=dev)
    recs[:, :, :9] = pay.transpose(1, 2)
    recs[:, :, 9] = tt
    out = kf.run_scheduled(tt, etype, recs, prev, freq, records=True)
    del recs
    assert int((kf.status() != 0).sum()) == 0
    kf.close()
    kf = kfmi.BatchedKF('ref15', B, 'f64')
    rows = kf.run_scheduled(tt, etype, pay, prev, freq)
    kf.close()
    ns = out[3]
    assert torch.equal(ns, rows[3])
    live = torch.arange(T, device=dev)[:, None] < ns[None, :].long()  # rows past n_sel are not written
    for a, b in zip(out[:3], rows[:3]):
        m = live[:, None, :] if a.dim() == 3 else live
        assert torch.equal(torch.where(m, a, 0.0), torch.where(m, b, 0.0))
    del rows
    idx = sample_filters(B)
    it = torch.as_tensor(idx, device=dev)
    tr, ld, st, ns = (v[..., it].cpu().numpy() for v in out)
    t_h, e_h, p_h, f_h, pv_h = (v[..., it].cpu().numpy() for v in (tt, etype, pay, freq, prev))
    rst, rtr, rld, rns = cpu_kf.ref15_sched(t_h, e_h, p_h, pv_h, f_h, ref_kf.P0_REF15)
    np.testing.assert_array_equal(ns, rns)
    assert ns.min() > 0
    live = np.arange(T)[:, None] < ns[None, :]
    np.testing.assert_array_equal(np.where(live, st, 0.0), rst)   # the same events picked
    ex, el = parity(np.where(live[:, None, :], tr, 0.0), np.where(live, ld, 0.0), rtr, rld)
    assert ex <= F64_TOL and el <= F64_TOL, (ex, el)


def _combo_maxima(ev, Pw, t0, t_end, combos):
    """The reference worker's score per subset (kf_workers.py:22-97): max of the log-dets of the
    start covariance, every applied event and the final predict to t_end (:74-82), through the C
    oracle, one filter per subset.  combos: [C, k] sorted candidate indices."""
    combos = np.asarray(combos)
    nc, k = combos.shape
    et = np.full((k + 1, nc), 255, np.uint8)
    et[:k] = ev[combos.T, 1].astype(np.uint8)
    tt = ev[combos.T, 0]
    dd = np.zeros((k + 1, nc))
    dd[0] = tt[0] - t0
    dd[1:k] = np.diff(tt, axis=0)
    fin = tt[-1] < t_end - 1e-8
    et[k, fin] = 2
    dd[k] = np.where(fin, t_end - tt[-1], 0.0)
    pp = np.zeros((k + 1, 9, nc))
    pp[:k] = np.transpose(ev[combos.T, 2:], (0, 2, 1))
    _, ld = cpu_kf.ref15_events(et, dd, pp, np.zeros((15, nc)), Pw)
    return np.maximum(ld.max(axis=0), np.linalg.slogdet(Pw)[1])


def _unrank_lex(n, k, ranks):
    return np.array([ref15.unrank_combination(n, k, int(r)) for r in ranks])


def test_bf_full_size_subset_maxima_vs_oracle():
    """The bf row (n = 25 candidates, all 2^25 - 1 subsets, the shared-prefix search, exhaustive):
    every subset of sizes 1-4 and 21-25 and 4096 spread subsets of every other size, plus each
    size's first and last subset, scored as the oracle's per-subset worker scores them."""
    n = bench.CONFIGS['bf']['n']
    ev, init, Pw, t0, t_end = bench.bf_events(n)
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    kfound, _, acc, sm = kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True, subset_max=True)
    kf.close()
    assert kfound == 0 and int(acc.sum()) == 0
    sm = sm.cpu().numpy()
    assert np.isnan(sm[0]) and np.isfinite(sm[1:]).all()
    rng = np.random.default_rng(25)
    worst, checked = 0.0, 0
    for k in range(1, n + 1):
        total = math.comb(n, k)
        if total <= 20000:
            combos = np.array(list(combinations(range(n), k)))
        else:
            ranks = np.unique(np.r_[0, total - 1, np.linspace(0, total - 1, 4096).astype(np.int64)
                                    + rng.integers(0, total // 4096, 4096)].clip(0, total - 1))
            combos = _unrank_lex(n, k, ranks)
        want = _combo_maxima(ev, Pw, t0, t_end, combos)
        got = sm[(1 << combos).sum(axis=1)]
        err = float(np.max(np.abs(got - want) / np.maximum(np.abs(want), 1.0)))
        assert err <= F64_TOL, (k, err)
        worst = max(worst, err)
        checked += len(combos)
    assert checked > 80000
    print(f'bf subset maxima: {checked} subsets, worst rel {worst:.2e}')


def test_bf_full_size_winner_vs_oracle():
    """The reference's brute-force search over the bf row's 25 candidates (warm start, target =
    the last candidate's time, kf_workers.py:1218-1392) at thresholds that put the winner at
    size 1 (not the first subset) and at size 2: the device driver (the search, then the
    winner's records) equals the NumPy restatement of the reference's search; and at those
    thresholds the exhaustive search's acceptance count of every size up to 4 equals the oracle's."""
    n = bench.CONFIGS['bf']['n']
    ev, init, Pw, t0, _ = bench.bf_events(n)
    t_last = float(ev[-1, 0])
    events = [(i, 'GPS', ev[i, 0], {'easting': ev[i, 2], 'northing': ev[i, 3], 'altitude': ev[i, 4]})
              if ev[i, 1] == 0 else (i, 'IMU', ev[i, 0], ['t', *ev[i, 2:]]) for i in range(n)]
    state0 = (t0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
    small = {k: np.array(list(combinations(range(n), k))) for k in range(1, 5)}
    maxima = {k: _combo_maxima(ev, Pw, t0, t_last, c) for k, c in small.items()}
    L0 = np.linalg.slogdet(Pw)[1]
    s1 = np.sort(maxima[1])
    assert s1[0] > L0 + 0.1           # every single event's final predict ends above the start
    thresholds = [(s1[3] + s1[4]) / 2, (L0 + s1[0]) / 2]
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    for thr, want_k in zip(thresholds, (1, 2)):
        ref = ref_kf.run_brute_force(events, 0, n, thr, Pw, state0)
        got = ref15.run_brute_force_kalman_filter_no_sampling_min_usage(events, 0, n, R_threshold=thr, initial_pt=Pw,
                                                                         initial_state=state0)
        sel = [e[0] for e in ref['selected_sensors']]
        assert len(sel) == want_k
        assert [e[0] for e in got['selected_sensors']] == sel
        assert got['num_measurements_used'] == ref['num_measurements_used']
        for key in ('log_determinants', 'final_state', 'trajectory'):
            a, b = np.asarray(got[key], np.float64), np.asarray(ref[key], np.float64)
            assert a.shape == b.shape and np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0)) <= F64_TOL, key
        # the exhaustive search walks every size; acceptance counts of sizes 1..4 vs the oracle's
        _, win, acc, _ = kf.search_combos(ev, init, t0, t_last, thr, exhaustive=True)
        assert win == tuple(sel)
        for k in range(1, 5):
            assert int(acc[k]) == int((maxima[k] < thr).sum()), (thr, k)
        first = next(k for k in range(1, 5) if (maxima[k] < thr).any())
        assert first == want_k and tuple(small[first][np.argmax(maxima[first] < thr)]) == tuple(sel)
    kf.close()


@pytest.mark.parametrize('config', ['1', '1ref8'])
def test_config1_whole_log_vs_oracle(tmp_path, config):
    """BASELINE config 1 at its full size: the bench's synthetic drive log (30,758 GPS rows,
    616,322 IMU rows), ingested on the device, dt by kf_events_dt, ONE filter through
    kf_run_stream (the time-parallel route the bench times) — run_kalman_filter_full's 15-state
    filter (config 1) or hw5_2.run_kalman_filter's 8-state one (1ref8); against the oracle's own
    ingest of the same CSVs (oracle/ref_ingest) and the reference's dense step in C on one
    filter, every one of the ~583k events."""
    dev = torch.device('cuda', 0)
    cfg = bench.CONFIGS[config]
    ref8 = cfg['model'] == 'ref8'
    n_state, width = (8, 3) if ref8 else (15, 6)
    gp, ip = bench.synth_log(cfg, str(tmp_path))
    stream = ingest.ingest_arrays(ingest.read_csv(gp, 4), ingest.read_csv(ip, 11), with_altitude=not ref8, device=0)
    first = int(torch.nonzero(stream.etype == _lib.KF_EVENT_GPS)[0, 0])
    T = len(stream) - first
    t_ev, e_ev, pay = (v[first:].contiguous() for v in (stream.t, stream.etype, stream.payload))
    x0 = torch.zeros(n_state, 1, dtype=torch.float64, device=dev)
    if not ref8:
        x0[0:3, 0] = pay[0, 0:3]
    kf = kfmi.BatchedKF(cfg['model'], 1, 'f64')
    kf.reset(x0)
    dt, et = ingest.events_dt(t_ev, float(t_ev[0]), _lib.KF_DT_RAW if ref8 else _lib.KF_DT_FULL, e_ev)
    tr, ld, _, _ = kf.run_stream(et, dt, pay)
    chk = kf.stream_check()
    kf.close()
    assert chk['ok'] and chk['chunks'] > 1000, chk
    assert tr.shape == (T, width, 1)
    tr, ld = tr.cpu().numpy(), ld.cpu().numpy()
    # the oracle: the reference's ingest restated, then the driver's loop from the first fix
    # (kf_workers.py:655-686 / hw5_2.py:332-340: the fix processed at dt = 0; the full driver
    # skips a dt < 0 event, hw5_2 predicts over it)
    events, _, _ = ref_ingest.ingest(gp, ip, with_altitude=not ref8)
    f0 = next(i for i, e in enumerate(events) if e[1] == 'GPS')
    events = events[f0:]
    assert len(events) == T
    th = np.array([e[2] for e in events])
    eh = np.array([0 if e[1] == 'GPS' else 1 for e in events], np.uint8)
    ph = np.zeros((T, 9))
    g = eh == 0
    ph[g, 0:2] = [[e[3]['easting'], e[3]['northing']] for e in events if e[1] == 'GPS']
    if not ref8:
        ph[g, 2] = [e[3]['altitude'] for e in events if e[1] == 'GPS']
    ph[~g] = [e[3][1:10] for e in events if e[1] == 'IMU']
    np.testing.assert_array_equal(eh, e_ev.cpu().numpy())
    dh = th - np.r_[th[0], th[:-1]]
    xh = np.zeros((n_state, 1))
    if ref8:
        rt, rl = cpu_kf.ref8_events(eh[:, None], dh[:, None], ph[:, :, None], xh, ref_kf.P0_REF8, nthreads=1)
    else:
        eh[dh < 0] = 255
        xh[0:3, 0] = ph[0, 0:3]
        rt, rl = cpu_kf.ref15_events(eh[:, None], dh[:, None], ph[:, :, None], xh, ref_kf.P0_REF15, nthreads=1)
    ex, el = parity(tr, ld, rt, rl)
    assert ex <= F64_TOL and el <= F64_TOL, (ex, el)
