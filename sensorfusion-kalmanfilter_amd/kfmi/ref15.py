"""The reference's 15-state GPS+IMU drivers on the engine (KF_MODEL_REF15).

Same names, arguments and return layouts as the reference's methods on KF_SensorFusion, with
the event list (``indexed_sensor_data``, built by combine_sensor_data, kf_workers.py:375-385:
``[(idx, 'GPS'|'IMU', t, payload), ...]``) passed explicitly:

    run_kalman_filter_full                               kf_workers.py:623-728
    run_adaptive_threshold_kalman_filter                 kf_workers.py:959-1058
    evaluate_combo_chunk (evaluate_combo_chunk_worker)   kf_workers.py:22-97
    run_brute_force_kalman_filter_no_sampling_min_usage  kf_workers.py:1218-1392
    run_kalman_filter_scheduled                          kf_workers.py:826-957
    run_kalman_filter (states + per-step covariances)    kf_workers.py:738-824
    run_no_update_kalman_filter                          kf_workers.py:1060-1160
    scheduler_gain / scheduler_cov_trace (Scheduler)     kf_workers.py:112-185
    sampling_sweep (the driver behind sampling_sweep/kf_plot_{10..120}.png)

Host code here only selects events and differences their time stamps in fp64 with the
reference's rules (first-GPS start, negative-dt skips); every predict/update/logdet runs in the
HIP kernels (kf_run_events, kf_eval_combos).  Covariances cross the boundary as 15x15 NumPy
arrays (the reference's format) and are stored block-packed on the GPU: they must be
block-diagonal over the axis chains (pos,vel,acc) and (att,rate), which every covariance the
reference itself produces is, exactly (see csrc/kf_ref15.hip).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib
from .engine import BatchedKF

GPS, IMU, PREDICT, NONE = _lib.KF_EVENT_GPS, _lib.KF_EVENT_IMU, _lib.KF_EVENT_PREDICT, _lib.KF_EVENT_NONE

def _block_rows(pva, aw):
    rows = []
    for blk in pva:
        rows += [(blk[a], blk[b]) for a in range(3) for b in range(a, 3)]
    for blk in aw:
        rows += [(blk[a], blk[b]) for a in range(2) for b in range(a, 2)]
    return rows


# block-packed row r -> (i, j) of the dense covariance, per model (csrc/kf_ref.hip, include/kf.h)
_LAYOUT = {
    # n: (rows, model name) — REF15 chains (pos, vel, acc)_i = (i, 6+i, 12+i), (att, rate)_i = (3+i, 9+i)
    15: (_block_rows([(0, 6, 12), (1, 7, 13), (2, 8, 14)], [(3, 9), (4, 10), (5, 11)]), 'ref15'),
    # REF8 (hw5_2.py:219-231): (x, vx, ax), (y, vy, ay), (theta, theta_dot)
    8: (_block_rows([(0, 3, 6), (1, 4, 7)], [(2, 5)]), 'ref8'),
}
_BY_ROWS = {len(r): n for n, (r, _) in _LAYOUT.items()}
_MASK = {}
for _n, (_rows, _) in _LAYOUT.items():
    _MASK[_n] = np.zeros((_n, _n), bool)
    for _i, _j in _rows:
        _MASK[_n][_i, _j] = _MASK[_n][_j, _i] = True
_ROWS = _LAYOUT[15][0]

# reference P0 (kf_workers.py:651)
P0 = np.diag([10000.0] * 3 + [1000.0] * 3 + [1000.0] * 3 + [1000.0] * 3 + [10000.0] * 3)

# H of the models (kf_workers.py:551-579, hw5_2.py:258-278): the engine's update selects these rows
_H = {15: (np.eye(15)[:3], np.eye(15)), 8: (np.eye(8)[:2], np.eye(8))}


class ModelConsts:
    """Diagonal noise constants of a reference model (include/kf.h kf_params.ref_*): Q rates,
    R_imu, R_gps and P0 per state, in the model's state order.  The reference hard-codes them in
    its getters (kf_workers.py:519-614, P0 :651; hw5_2.py:233-304, P0 :317-326) and lets a
    caller replace the getters through its class_args dict (kf_workers.py:1242-1251); any
    diagonal choice keeps the covariance block-diagonal over the axis chains, which the engine
    stores.  ``ModelConsts('ref15')`` is the reference's."""

    def __init__(self, model='ref15', q=None, r_imu=None, r_gps=None, p0=None):
        from .engine import default_params
        if model not in ('ref15', 'ref8'):
            raise ValueError(f'ModelConsts: {model!r} is not a reference model')
        self.model = model
        self.n = 15 if model == 'ref15' else 8
        d = default_params(model)
        n, g = self.n, 3 if model == 'ref15' else 2

        def vec(v, ref, k, name):
            a = np.array(ref[:k] if v is None else v, dtype=np.float64).reshape(-1)
            if a.shape != (k,):
                raise ValueError(f'ModelConsts: {name} needs {k} values, got {a.shape}')
            return a
        self.q = vec(q, d.ref_q, n, 'q')
        self.r_imu = vec(r_imu, d.ref_r_imu, n, 'r_imu')
        self.r_gps = vec(r_gps, d.ref_r_gps, g, 'r_gps')
        self.p0 = vec(p0, d.ref_p0, n, 'p0')

    @property
    def P0(self):
        return np.diag(self.p0)

    def Q(self, dt):
        return np.diag(self.q * dt)

    @property
    def R_gps(self):
        return np.diag(self.r_gps)

    @property
    def R_imu(self):
        return np.diag(self.r_imu)

    def is_reference(self):
        return self == ModelConsts(self.model)

    def __eq__(self, other):
        return isinstance(other, ModelConsts) and self.model == other.model and all(
            np.array_equal(getattr(self, k), getattr(other, k)) for k in ('q', 'r_imu', 'r_gps', 'p0'))

    def params(self):
        """kf_params for BatchedKF(model, ..., params=...), or None for the reference's."""
        if self.is_reference():
            return None
        p = _lib.kf_params()
        for name, v in (('ref_q', self.q), ('ref_r_imu', self.r_imu), ('ref_r_gps', self.r_gps),
                        ('ref_p0', self.p0)):
            arr = getattr(p, name)
            for i, x in enumerate(v):
                arr[i] = float(x)
        return p

    def oracle(self):
        """The same constants as oracle/ref_kf.py's K argument (tests)."""
        return dict(q=self.q, r_imu=self.r_imu, r_gps=self.r_gps, p0=self.p0)

    @classmethod
    def from_matrices(cls, model='ref15', F=None, Q=None, H_gps=None, H_imu=None, R_gps=None, R_imu=None, P0=None):
        """Constants from the reference's getters or a caller's replacements (the class_args
        callables, kf_workers.py:1242-1251): F(dt), Q(dt) callables, H / R matrices, P0.  Any
        argument may be None (the reference's).  The engine runs the reference's F and H (a
        kinematic chain per axis) with Q = diag(q dt) and diagonal R, P0: anything else — a
        different F or H, a Q not of that form, an R or P0 with an off-diagonal entry — raises
        ValueError, before any GPU work."""
        c = cls(model)
        n = c.n
        if F is not None:
            from .kf_workers import _F
            from .hw5_2 import _F8
            ref_f = _F if n == 15 else _F8
            for dt in (0.5, 0.0123, 2.0):
                if not np.array_equal(np.asarray(F(dt), np.float64), ref_f(dt)):
                    raise ValueError('ModelConsts: the state transition is not the reference model\'s F(dt) '
                                     '(the engine\'s kernels run its kinematic chains)')
        for name, Hm, ref in (('H_gps', H_gps, _H[n][0]), ('H_imu', H_imu, _H[n][1])):
            if Hm is not None and not (np.shape(Hm) == ref.shape and np.array_equal(np.asarray(Hm, np.float64), ref)):
                raise ValueError(f'ModelConsts: {name} is not the reference model\'s observation matrix')

        def diag_of(M, k, name):
            M = np.asarray(M, np.float64)
            if M.shape != (k, k):
                raise ValueError(f'ModelConsts: {name} must be {k}x{k}, got {M.shape}')
            if np.any(M - np.diag(np.diag(M))):
                raise ValueError(f'ModelConsts: {name} has off-diagonal entries; the engine takes diagonal '
                                 f'noise and initial covariances (block-diagonal P over the axis chains)')
            return np.diag(M).copy()
        if Q is not None:
            q = diag_of(Q(1.0), n, 'Q(1)')
            for dt in (0.5, 0.0123, 2.0):
                if not np.allclose(diag_of(Q(dt), n, f'Q({dt})'), q * dt, rtol=1e-12, atol=0.0):
                    raise ValueError('ModelConsts: Q(dt) is not diag(q * dt), the reference\'s form '
                                     '(kf_workers.py:519-544)')
            c.q = q
        if R_gps is not None:
            c.r_gps = diag_of(R_gps, 3 if n == 15 else 2, 'R_gps')
        if R_imu is not None:
            c.r_imu = diag_of(R_imu, n, 'R_imu')
        if P0 is not None:
            c.p0 = diag_of(P0, n, 'P0')
        if np.any(c.q < 0) or np.any(c.r_gps <= 0) or np.any(c.r_imu <= 0) or np.any(c.p0 <= 0):
            raise ValueError('ModelConsts: Q rates must be >= 0 and R, P0 variances > 0')
        return c


def _params(consts):
    return consts.params() if consts is not None else None


def _p0(consts):
    return consts.P0 if consts is not None else P0


def to_blocks(P):
    """n x n (or [..., n, n]) covariance of REF15 (n = 15) or REF8 (n = 8) -> block-packed
    [..., 27 | 15]; raises ValueError if it couples different axis chains (the engine stores only
    the chain blocks)."""
    P = np.asarray(P, dtype=np.float64)
    n = P.shape[-1]
    if n not in _LAYOUT or P.shape[-2] != n:
        raise ValueError(f'expected a [..., 15, 15] or [..., 8, 8] covariance, got {P.shape}')
    off = np.abs(P[..., ~_MASK[n]])
    if off.size and off.max() > 0.0:
        raise ValueError(f'covariance couples different axis chains (max |off-block| = {off.max():g}); '
                         f'KF_MODEL_{_LAYOUT[n][1].upper()} stores the (pos,vel,acc)/(att,rate) blocks only')
    return np.stack([P[..., i, j] for i, j in _LAYOUT[n][0]], axis=-1)


def from_blocks(b):
    """block-packed [..., 27 | 15] -> 15x15 | 8x8 symmetric."""
    b = np.asarray(b, dtype=np.float64)
    n = _BY_ROWS[b.shape[-1]]
    P = np.zeros(b.shape[:-1] + (n, n))
    for r, (i, j) in enumerate(_LAYOUT[n][0]):
        P[..., i, j] = b[..., r]
        P[..., j, i] = b[..., r]
    return P


def event_payload(stype, sdata):
    """The 9 payload values of one reference event (kf_workers.py:331, 367; hw5_2.py:54 stores
    no altitude, which its 8-state model never reads)."""
    if stype == 'GPS':
        return [sdata['easting'], sdata['northing'], sdata.get('altitude', 0.0), 0, 0, 0, 0, 0, 0]
    return [float(v) for v in sdata[1:10]]


def _run_streams(streams, x0, P0b, dtype='f64', device=0, threshold=None, model='ref15', cov=False, consts=None,
                 kf=None):
    """Run one event list per filter in ONE kf_run_events launch.

    streams: list (per filter) of [(type, dt, payload9)]; each stream is preceded by a NONE
    event so row 0 of the outputs holds the initial state and logdet.  x0 [B, n] and P0b
    [B, rows] are the initial states.  Returns traj [T, W, B], logdet [T, B], updated [T, B],
    x [n, B], P blocks [rows, B], status [B] (and cov [T, rows, B] with cov=True) as NumPy
    arrays.  consts: a ModelConsts (None = the reference's constants).  kf: a handle of this
    model, batch, dtype and constants to run on (kept open), instead of a new one."""
    B = len(streams)
    T = 1 + max((len(s) for s in streams), default=0)
    etype = np.full((T, B), NONE, np.uint8)
    dt = np.zeros((T, B))
    pay = np.zeros((T, 9, B))
    for f, s in enumerate(streams):
        for t, (ty, d, p) in enumerate(s, start=1):
            etype[t, f] = ty
            dt[t, f] = d
            pay[t, :, f] = p
    own = kf is None
    if own:
        kf = BatchedKF(model, B, dtype, device=device, params=_params(consts))
    npd = np.float64 if dtype == 'f64' else np.float32
    kf.set_state(np.ascontiguousarray(np.asarray(x0, np.float64).T.astype(npd)),
                 np.ascontiguousarray(np.asarray(P0b, np.float64).T.astype(npd)))
    tr, ld, up, cv = kf.run_events(etype, dt, pay.astype(npd), updated=True, threshold=threshold, cov=cov)
    x, Pb = kf.state()
    st = kf.status()
    torch.cuda.synchronize(kf.device)
    out = (tr.double().cpu().numpy(), ld.double().cpu().numpy(), up.cpu().numpy(), x.double().cpu().numpy(),
           Pb.double().cpu().numpy(), st.cpu().numpy())
    if cov:
        out += (cv.double().cpu().numpy(),)
    if own:
        kf.close()
    return out


def _window(events, start_idx, end_idx):
    if start_idx is None or start_idx < 0:
        start_idx = 0
    if end_idx is None or end_idx > len(events):
        end_idx = len(events)
    return start_idx, end_idx


def _cold_start(events, start_idx, stop):
    """First GPS fix in events[start_idx:stop]: (x0, t0, absolute index) or None
    (kf_workers.py:655-666)."""
    for i, (_, stype, t, sdata) in enumerate(events[start_idx:stop]):
        if stype == 'GPS':
            x = np.zeros(15)
            x[0], x[1], x[2] = sdata['easting'], sdata['northing'], sdata['altitude']
            return x, t, start_idx + i
    return None


def run_kalman_filter_full(events, start_idx=None, end_idx=None, initial_pt=None, initial_state=None,
                           print_output=False, dtype='f64', device=0, consts=None):
    """kf_workers.py:623-728 on the GPU: returns (states, logdets, P, prev_time) in the
    reference's layout (states = [(t, x, y, z, roll, pitch, yaw), ...]).  ``events`` is the
    reference's event list or a kfmi.ingest.EventStream (then the whole window runs from HBM:
    run_full_stream, with the lists built from its arrays)."""
    from .ingest import EventStream
    if isinstance(events, EventStream):
        r = run_full_stream(events, start_idx, end_idx, initial_pt, initial_state, dtype, consts=consts)
        if r is None:
            return [], [], []
        t, traj, ld, P, prev = r
        states = [(float(t[i]), *traj[i]) for i in range(len(t))]
        if print_output:
            print(f'Full Kalman Filter (GPU): processed {len(t) - 1} measurements')
        return states, [float(v) for v in ld], P, prev
    if not events:
        return [], [], []
    start_idx, end_idx = _window(events, start_idx, end_idx)
    x0 = np.zeros(15)
    if initial_pt is not None and initial_state is not None:
        P = np.asarray(initial_pt, np.float64)
        x0[0:6] = initial_state[1:7]
        prev = initial_state[0]
        start_off = start_idx
    else:
        P = _p0(consts)
        cs = _cold_start(events, start_idx, end_idx + 1)
        if cs is None:
            return [], [], []
        x0, prev, start_off = cs
    stream, times = [], []
    for (_, stype, t, sdata) in events[start_off:end_idx]:
        dt = t - prev
        if dt < 0:  # kf_workers.py:683-685
            prev = t
            continue
        stream.append((GPS if stype == 'GPS' else IMU, dt, event_payload(stype, sdata)))
        times.append(t)
        prev = t
    tr, ld, _, x, Pb, st = _run_streams([stream], x0[None], to_blocks(P)[None], dtype, device, consts=consts)
    states = [(initial_state[0] if (initial_pt is not None and initial_state is not None) else
               events[start_off][2], *tr[0, :, 0])]
    states += [(t, *tr[i + 1, :, 0]) for i, t in enumerate(times)]
    logdets = [float(v) for v in ld[:len(times) + 1, 0]]
    if print_output:
        print(f'Full Kalman Filter (GPU): processed {len(times)} measurements from index {start_off} to {end_idx}')
    return states, logdets, from_blocks(Pb[:, 0]), prev


def run_full_stream(stream, start_idx=None, end_idx=None, initial_pt=None, initial_state=None, dtype='f64',
                    cov=False, parallel=True, parallel_min_events=1 << 16, consts=None):
    """run_kalman_filter_full (kf_workers.py:623-728) over an EventStream window, entirely on
    the device: cold-start fix search, per-event dt with the driver's dt < 0 rule
    (kf_events_dt, KF_DT_FULL) and one single-filter kf_run_events launch — or, for windows of
    at least ``parallel_min_events`` events, kf_run_stream (chunks of the window as filters of
    one launch, checked on the device, with the single filter as its fallback).  Returns NumPy
    (t [R], traj [R, 6], logdet [R], P 15x15, prev_time) with R = 1 + processed events (plus
    the block-packed per-record covariances [R, 27] with cov=True), or None when a cold window
    holds no fix."""
    from .ingest import events_dt
    n = len(stream)
    start_idx = 0 if start_idx is None or start_idx < 0 else int(start_idx)
    end_idx = n if end_idx is None or end_idx > n else int(end_idx)
    dev = stream.t.device
    x0 = np.zeros(15)
    if initial_pt is not None and initial_state is not None:
        P = np.asarray(initial_pt, np.float64)
        x0[0:6] = initial_state[1:7]
        prev0 = float(initial_state[0])
        start_off = start_idx
        t_first = prev0
    else:
        P = _p0(consts)
        win = stream.etype[start_idx:min(end_idx + 1, n)]  # the reference searches [start, end] (:655)
        hit = torch.nonzero(win == GPS)
        if hit.numel() == 0:
            return None
        start_off = start_idx + int(hit[0, 0])
        p = stream.payload[start_off].cpu().numpy()
        x0[0:3] = p[0:3]
        prev0 = float(stream.t[start_off])
        t_first = prev0
    T = max(end_idx - start_off, 0)
    kf = BatchedKF('ref15', 1, dtype, device=dev.index or 0, params=_params(consts))
    npd = np.float64 if dtype == 'f64' else np.float32
    kf.set_state(x0[:, None].astype(npd), to_blocks(P)[:, None].astype(npd))
    t = stream.t[start_off:start_off + T]
    dt, et = events_dt(t, prev0, _lib.KF_DT_FULL, stream.etype[start_off:start_off + T])
    pay = stream.payload[start_off:start_off + T]
    if dtype != 'f64':
        pay = pay.float()
    # a NONE event first records the initial state and logdet (states[0], logdets[0])
    et = torch.cat([torch.full((1,), NONE, dtype=torch.uint8, device=dev), et])
    dt = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev), dt])
    pay = torch.cat([torch.zeros(1, 9, dtype=pay.dtype, device=dev), pay])
    if parallel and T + 1 >= parallel_min_events:
        tr, ld, _, cv = kf.run_stream(et, dt, pay, cov=cov)
    else:
        # parallel=False: the single filter even where kf_run_events would route it over time
        tr, ld, _, cv = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], cov=cov, sequential=not parallel)
    x, Pb = kf.state()
    keep = et != NONE
    keep[0] = True
    t_all = torch.cat([torch.full((1,), t_first, dtype=torch.float64, device=dev), t])
    prev = float(t[-1]) if T else prev0
    out = (t_all[keep].cpu().numpy(), tr[keep, :, 0].double().cpu().numpy(), ld[keep, 0].double().cpu().numpy(),
           from_blocks(Pb[:, 0].double().cpu().numpy()), prev)
    if cov:
        out += (cv[keep, :, 0].double().cpu().numpy(),)
    kf.close()
    return out


# --------------------------------------------------------------------------------------------
# One filter over a long stream, parallel over time (run_kalman_filter_full's own use: one
# filter over a whole drive log, kf_workers.py:623-728)
# --------------------------------------------------------------------------------------------

# the checks of the last run_stream_parallel call (diagnostics)
parallel_check = {}


def run_stream_parallel(et, dt, pay, x0, P0b, chunk=None, warmup=None, dtype='f64', cov=False, options=None,
                        consts=None):
    """One filter over a long event stream, parallel over time (kf_run_stream): et [T] uint8,
    dt [T] float64 (the driver's dt rule already applied), pay [T, 9] on the device; x0 [15], P0b
    [27] block-packed initial state.  Returns (traj [T, 6], logdet [T], x [15], P blocks [27],
    cov [T, 27] or None) on the device.  The chunked records stand only if the device checks
    pass (warm-up covariances meet their predecessors' end covariances, chunk end states meet
    the next starts, no chunk filter failed); otherwise the library's sequential fallback has
    rewritten them.  ``parallel_check`` holds the verdict and the measured gaps.  ``options``:
    BatchedKF options of the handle (e.g. stream_final='on')."""
    dev = et.device
    npd = torch.float64 if dtype == 'f64' else torch.float32
    kf = BatchedKF('ref15', 1, dtype, device=dev.index or 0, options=options, params=_params(consts))
    try:
        kf.set_state(torch.as_tensor(np.asarray(x0, np.float64).reshape(15, 1), dtype=npd, device=dev),
                     torch.as_tensor(np.asarray(P0b, np.float64).reshape(27, 1), dtype=npd, device=dev))
        tr, ld, _, cv = kf.run_stream(et, dt, pay.to(npd), cov=cov, chunk=chunk or 0,
                                      warmup=-1 if warmup is None else warmup)
        x, P = kf.state()
        parallel_check.clear()
        parallel_check.update(kf.stream_check())
        return tr[:, :, 0], ld[:, 0], x[:, 0], P[:, 0], (cv[:, :, 0] if cov else None)
    finally:
        kf.close()


def _device_stream(events):
    """The kfmi.ingest.EventStream behind ``events`` (the stream itself, or an event list over
    one: kfmi.kf_workers.EventList after combine_sensor_data), or None for a plain list."""
    from .ingest import EventStream
    if isinstance(events, EventStream):
        return events
    s = getattr(events, 's', None)
    return s if isinstance(s, EventStream) else None


def run_monotone_stream(stream, start_idx=None, end_idx=None, initial_pt=None, initial_state=None, dtype='f64',
                        consts=None, threshold=None, predict_only=False):
    """The adaptive-threshold (``threshold``, kf_workers.py:959-1058) and no-update
    (``predict_only``, :1060-1160) drivers over an EventStream window, on the device: the cold
    start's first fix in [start, end) (:990-1000), the drivers' dt rule — a dt < 0 event is skipped
    without advancing the previous time (kf_events_dt KF_DT_MONOTONE) — and one single-filter
    kf_run_events launch (the gate on logdet(P_pred) needs the filter's own history, so it runs in
    time order).  The Python loop over the event list it replaces built a tuple and three array
    entries per event (0.49 s for the 82,570 events up to the visualizing run's start).  Returns
    NumPy (t [R], traj [R, 6], logdet [R], P 15x15, previous_time, measurement_times) with R = 1 +
    processed events, or None when a cold window holds no fix."""
    from .ingest import events_dt
    n = len(stream)
    start_idx = 0 if start_idx is None or start_idx < 0 else int(start_idx)
    end_idx = n if end_idx is None or end_idx > n else int(end_idx)
    dev = stream.t.device
    x0 = np.zeros(15)
    mtimes = []
    if initial_pt is not None and initial_state is not None:
        P = np.asarray(initial_pt, np.float64)
        x0[0:6] = initial_state[1:7]
        prev0 = float(initial_state[0])
        start_off = start_idx
    else:
        P = _p0(consts)
        hit = torch.nonzero(stream.etype[start_idx:end_idx] == GPS)
        if hit.numel() == 0:
            return None
        start_off = start_idx + int(hit[0, 0])
        x0[0:3] = stream.payload[start_off, 0:3].double().cpu().numpy()
        prev0 = float(stream.t[start_off])
        mtimes.append(prev0)
    T = max(end_idx - start_off, 0)
    t = stream.t[start_off:start_off + T]
    dt, et = events_dt(t, prev0, _lib.KF_DT_MONOTONE, stream.etype[start_off:start_off + T])
    if predict_only:
        et = torch.where(et != NONE, torch.full_like(et, PREDICT), et)
        pay = torch.zeros(T, 9, dtype=torch.float64, device=dev)
    else:
        pay = stream.payload[start_off:start_off + T].double()
    if dtype != 'f64':
        pay = pay.float()
    # a NONE event first records the initial state and logdet (states[0], logdets[0])
    et = torch.cat([torch.full((1,), NONE, dtype=torch.uint8, device=dev), et])
    dt = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev), dt])
    pay = torch.cat([torch.zeros(1, 9, dtype=pay.dtype, device=dev), pay])
    kf = BatchedKF('ref15', 1, dtype, device=dev.index or 0, params=_params(consts))
    try:
        npd = np.float64 if dtype == 'f64' else np.float32
        kf.set_state(x0[:, None].astype(npd), to_blocks(P)[:, None].astype(npd))
        tr, ld, up, _ = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], updated=True,
                                      threshold=None if threshold is None else float(threshold))
        x, Pb = kf.state()
        keep = et != NONE
        keep[0] = True
        t_all = torch.cat([torch.full((1,), prev0, dtype=torch.float64, device=dev), t.double()])
        upd = up[:, 0].bool() & keep
        upd[0] = False
        tk = t_all[keep]
        prev = float(tk[-1]) if tk.numel() > 1 else prev0
        out = (tk.cpu().numpy(), tr[keep, :, 0].double().cpu().numpy(), ld[keep, 0].double().cpu().numpy(),
               from_blocks(Pb[:, 0].double().cpu().numpy()), prev, mtimes + t_all[upd].cpu().tolist())
    finally:
        kf.close()
    return out


def _stream_states(t, traj):
    """[(t, x, y, z, roll, pitch, yaw), ...] from run_*_stream's arrays."""
    return list(zip(t.tolist(), *traj.T.tolist()))


def run_adaptive_threshold_kalman_filter(events, start_idx=None, end_idx=None, R_threshold=None,
                                         initial_pt=None, initial_state=None, print_output=False,
                                         dtype='f64', device=0, consts=None):
    """kf_workers.py:959-1058 on the GPU: the update is applied only when logdet(P_pred) >
    R_threshold.  Returns (states, logdets, P, previous_time, measurement_times).  Over an
    ingested stream (or an event list over one) the window never leaves the device
    (run_monotone_stream)."""
    if R_threshold is None:
        R_threshold = -float('inf')
    ds = _device_stream(events)
    if ds is not None:
        r = run_monotone_stream(ds, start_idx, end_idx, initial_pt, initial_state, dtype, consts,
                                threshold=float(R_threshold))
        if r is None:
            return None
        t, traj, ld, P, prev, mtimes = r
        if print_output:
            print(f'Adaptive Kalman Filter (GPU): processed {len(t) - 1} events')
        return _stream_states(t, traj), ld.tolist(), P, prev, mtimes
    start_idx, end_idx = _window(events, start_idx, end_idx)
    x0 = np.zeros(15)
    mtimes = []
    if initial_pt is not None and initial_state is not None:
        P = np.asarray(initial_pt, np.float64)
        x0[0:6] = initial_state[1:7]
        prev = initial_state[0]
        start_off = start_idx
    else:
        P = _p0(consts)
        cs = _cold_start(events, start_idx, end_idx)
        if cs is None:
            return None
        x0, prev, start_off = cs
        mtimes.append(prev)
    t_first = prev
    stream, times = [], []
    for (_, stype, t, sdata) in events[start_off:end_idx]:
        dt = t - prev
        if dt < 0:
            # kf_workers.py:1013-1015 assigns an unused name, so previous_time is NOT advanced
            continue
        stream.append((GPS if stype == 'GPS' else IMU, dt, event_payload(stype, sdata)))
        times.append(t)
        prev = t
    tr, ld, up, x, Pb, st = _run_streams([stream], x0[None], to_blocks(P)[None], dtype, device,
                                         threshold=float(R_threshold), consts=consts)
    states = [(t_first, *tr[0, :, 0])] + [(t, *tr[i + 1, :, 0]) for i, t in enumerate(times)]
    logdets = [float(v) for v in ld[:len(times) + 1, 0]]
    mtimes += [t for i, t in enumerate(times) if up[i + 1, 0]]
    if print_output:
        print(f'Adaptive Kalman Filter (GPU): processed {len(times)} events from index {start_off} to {end_idx}')
    return states, logdets, from_blocks(Pb[:, 0]), prev, mtimes


def run_kalman_filter(events, start_idx, end_idx, dtype='f64', device=0, consts=None):
    """kf_workers.py:738-824 on the GPU: x0 = 0, the reference's P0, the window's events from
    its first GPS fix on (that fix at dt = 0), no dt < 0 guard.  Returns (states,
    covariances) — states[0] = (0, 0, 0, 0, 0, 0, 0) and one 15x15 covariance per record, the
    per-step covariances coming from kf_run_events' cov stream."""
    stream, times = [], []
    prev = None
    for (_, stype, t, sdata) in events[start_idx:end_idx]:
        if stype == 'GPS' and prev is None:
            prev = t
        if prev is None:
            continue
        stream.append((GPS if stype == 'GPS' else IMU, t - prev, event_payload(stype, sdata)))
        times.append(t)
        prev = t
    tr, _, _, _, _, _, cv = _run_streams([stream], np.zeros((1, 15)), to_blocks(_p0(consts))[None], dtype, device,
                                         cov=True, consts=consts)
    states = [(0, *tr[0, :, 0])] + [(t, *tr[i + 1, :, 0]) for i, t in enumerate(times)]
    covs = list(from_blocks(cv[:len(times) + 1, :, 0]))
    return states, covs


def run_no_update_kalman_filter(events, start_idx=None, end_idx=None, R_threshold=None, initial_pt=None,
                                initial_state=None, print_output=False, dtype='f64', device=0, consts=None):
    """kf_workers.py:1060-1160 on the GPU: the window as KF_EVENT_PREDICT events (every update
    of the reference's loop is commented out), logdet after each.  A dt < 0 event is skipped
    without advancing the previous time (:1113-1116).  Returns (states, logdets, P,
    previous_time, measurement_times), or None when no GPS fix starts a cold window.  Over an
    ingested stream the window never leaves the device (run_monotone_stream)."""
    ds = _device_stream(events)
    if ds is not None:
        r = run_monotone_stream(ds, start_idx, end_idx, initial_pt, initial_state, dtype, consts, predict_only=True)
        if r is None:
            return None
        t, traj, ld, P, prev, mtimes = r
        if print_output:
            print(f'No-update Kalman Filter (GPU): {len(t) - 1} predictions')
        return _stream_states(t, traj), ld.tolist(), P, prev, mtimes
    start_idx, end_idx = _window(events, start_idx, end_idx)
    x0 = np.zeros(15)
    mtimes = []
    if initial_pt is not None and initial_state is not None:
        P = np.asarray(initial_pt, np.float64)
        x0[0:6] = initial_state[1:7]
        prev = initial_state[0]
        start_off = start_idx
    else:
        P = _p0(consts)
        cs = _cold_start(events, start_idx, end_idx)
        if cs is None:
            return None
        x0, prev, start_off = cs
        mtimes.append(prev)
    t_first = prev
    stream, times = [], []
    for (_, stype, t, sdata) in events[start_off:end_idx]:
        dt = t - prev
        if dt < 0:
            continue
        stream.append((PREDICT, dt, [0.0] * 9))
        times.append(t)
        prev = t
    tr, ld, _, _, Pb, _ = _run_streams([stream], x0[None], to_blocks(P)[None], dtype, device, consts=consts)
    states = [(t_first, *tr[0, :, 0])] + [(t, *tr[i + 1, :, 0]) for i, t in enumerate(times)]
    logdets = [float(v) for v in ld[:len(times) + 1, 0]]
    if print_output:
        print(f'No-update Kalman Filter (GPU): {len(times)} predictions from index {start_off} to {end_idx}')
    return states, logdets, from_blocks(Pb[:, 0]), prev, mtimes


def _combo_stream(combo, prev_time, target_end):
    """Event stream of one combination with the worker's rules (kf_workers.py:36-82)."""
    s, times = [], []
    cur = prev_time
    for (_, stype, t, sdata) in combo:
        dt = t - cur
        if dt < 0:
            continue
        s.append((GPS if stype == 'GPS' else IMU, dt, event_payload(stype, sdata)))
        times.append(t)
        cur = t
    if cur < target_end - 1e-8:
        s.append((PREDICT, target_end - cur, [0.0] * 9))
        times.append(target_end)
    return s, times


def evaluate_combo_chunk(chunk, xt, Pt, prev_time, target_end_time, dtype='f64', device=0, consts=None, kf=None):
    """evaluate_combo_chunk_worker (kf_workers.py:22-97) for a whole chunk in ONE launch, one
    filter per combination.  Returns [(0, traj, combo, x_final, None, log_det, k), ...].  kf: a
    'ref15' handle of len(chunk) filters with these constants to run on (_run_streams)."""
    if not chunk:
        return []
    built = [_combo_stream(c, prev_time, target_end_time) for c in chunk]
    B = len(chunk)
    tr, ld, _, x, Pb, st = _run_streams([b[0] for b in built], np.broadcast_to(np.asarray(xt, np.float64), (B, 15)),
                                        np.broadcast_to(to_blocks(Pt), (B, 27)), dtype, device, consts=consts, kf=kf)
    results = []
    for f, (combo, (s, times)) in enumerate(zip(chunk, built)):
        if st[f] != 0:  # the worker skips a combination that raised (kf_workers.py:88-91)
            continue
        n = len(times)
        traj = [(prev_time, *tr[0, :, f])] + [(t, *tr[i + 1, :, f]) for i, t in enumerate(times)]
        results.append((0, traj, combo, x[:, f].copy(), None, [float(v) for v in ld[:n + 1, f]], len(combo)))
    return results


def unrank_combination(n, k, r):
    """The r-th k-subset of range(n) in itertools.combinations order."""
    out, a = [], 0
    for j in range(k):
        while True:
            c = math.comb(n - a - 1, k - j - 1)
            if r < c:
                break
            r -= c
            a += 1
        out.append(a)
        a += 1
    return out


def brute_force_setup(events, start_idx=0, end_idx=None, initial_pt=None, initial_state=None, consts=None):
    """The search's inputs as kf_workers.py:1262-1310 sets them up: (candidates, x0, P0,
    prev_time, target_end, events [n, 11], init [42]), or None when there is no candidate: a
    cold window without a starting fix (:1303-1305), or an empty warm-start window, where the
    reference's size loop (:1325) never runs and it returns None (:1391-1392)."""
    if start_idx is None or start_idx < 0:
        start_idx = 0
    if end_idx is None or end_idx > len(events):
        end_idx = len(events)
    xt = np.zeros(15)
    if initial_pt is not None and initial_state is not None:
        Pt = np.asarray(initial_pt, np.float64)
        xt[0:6] = initial_state[1:7]
        prev_time = initial_state[0]
        cand = list(events[start_idx:end_idx])
    else:
        Pt = _p0(consts)
        cand, prev_time, started = [], None, False
        for (idx, stype, t, sdata) in events[start_idx:end_idx + 1]:  # the reference's +1 slice
            if not started and stype == 'GPS':
                xt[0], xt[1], xt[2] = sdata['easting'], sdata['northing'], sdata['altitude']
                started, prev_time = True, t
            if started:
                cand.append((idx, stype, t, sdata))
    if not cand:
        return None
    target_end = events[end_idx - 1][2]
    n = len(cand)
    if n > 64:
        raise ValueError(f'{n} candidate events: the GPU search supports at most 64 (2^64 subsets)')
    ev = np.zeros((n, 11))
    for i, (_, stype, t, sdata) in enumerate(cand):
        ev[i, 0] = t
        ev[i, 1] = GPS if stype == 'GPS' else IMU
        ev[i, 2:] = event_payload(stype, sdata)
    return cand, xt, Pt, prev_time, target_end, ev, np.concatenate([xt, to_blocks(Pt)])


def first_valid_rank(kf, ev, init, prev_time, target_end, k, lo, hi, threshold):
    """Smallest combination rank r in [lo, hi) of the k-subsets whose max log-determinant is
    below threshold (the reference's acceptance test, kf_workers.py:1353), or None; kf_eval_combos
    launches of kf.batch lanes."""
    width = kf.batch
    for off in range(lo, hi, width):
        cnt = min(width, hi - off)
        mx, _, _ = kf.eval_combos(ev, init, prev_time, target_end, k, combo_offset=off, logdets=False)
        ok = mx[:cnt] < threshold
        if bool(ok.any()):
            return off + int(torch.argmax(ok.to(torch.int8)).item())
    return None


def brute_force_result(cand, k, r, xt, Pt, prev_time, target_end, dtype='f64', device=0, indices=None, consts=None,
                       kf=None):
    """The reference's result dict (kf_workers.py:1358-1367) for combination rank r of size k
    (or the candidate ``indices`` of the subset); kf: a one-filter handle to run it on (the
    search's)."""
    idx = unrank_combination(len(cand), k, r) if indices is None else indices
    combo = tuple(cand[i] for i in idx)
    metric, traj, combo, x_bf, P_bf, log_det, used = evaluate_combo_chunk([combo], xt, Pt, prev_time, target_end,
                                                                          dtype, device, consts, kf=kf)[0]
    return {'selected_sensors': combo, 'final_state': x_bf, 'final_covariance': P_bf, 'trajectory': traj,
            'accuracy_metric': metric, 'log_determinants': log_det, 'num_measurements_used': used}


def search_level_bytes(nodes, dtype, sym=False):
    """Device bytes of one kf_search_combos level buffer (node blocks of 64, kf_internal.h; an
    axis-symmetric search's nodes hold 10 rows instead of 28, KF_OPT_AXIS_SYM; then the running
    max's exponent, the time and the mask: 20 B)."""
    w = 8 if dtype == 'f64' else 4
    return (nodes + 63) // 64 * 64 * ((10 if sym else 28) * w + 20)


SEARCH_HEAD_STEPS = 400000  # kf_capi.cpp kSearchHeadSteps
SEARCH_END_STEPS = 200000   # kf_capi.cpp kSearchEndSteps


def search_head_size(n, k_max=None):
    """The sizes 1 .. K kf_search_combos runs in its one-launch head (kf_capi.cpp: the largest K
    <= n - 2, below k_max, whose subsets' event steps from the root sum_k k C(n, k) stay within
    kSearchHeadSteps; 0 = no head, for n < 5 or K < 2).  Bookkeeping for the bench's bytes."""
    k_max = n if k_max is None else k_max
    if n < 5:
        return 0
    K, steps = 0, 0
    for k in range(1, min(n - 2, k_max - 1) + 1):
        steps += k * math.comb(n, k)
        if steps > SEARCH_HEAD_STEPS:
            break
        K = k
    return K if K >= 2 else 0


def search_end_size(n, k_max=None, head=True):
    """The first size k_end0 of kf_search_combos' end launch (kf_capi.cpp: sizes k_end0 .. k_max
    in one launch from level k_end0 - 1's stored nodes), k_max + 1 for none: the smallest k0 with
    sum_{k >= k0} (k - k0 + 1) C(n, k) within kSearchEndSteps, 2 <= k0 <= min(k_max - 1, n - 2),
    above the head's sizes, n - k0 + 1 <= 6.  Bookkeeping for the bench's bytes."""
    k_max = n if k_max is None else k_max
    K = search_head_size(n, k_max) if head else 0
    k_first = K + 1 if K else 1
    end = k_max + 1
    k0 = min(k_max - 1, n - 2)
    while k0 >= 2 and k0 > k_first and n - k0 + 1 <= 6:
        if sum((k - k0 + 1) * math.comb(n, k) for k in range(k0, k_max + 1)) > SEARCH_END_STEPS:
            break
        end = k0
        k0 -= 1
    return end


SEARCH_CM_PARENTS = 200000  # kf_capi.cpp kSearchChildMajorParents: levels with more parents run parent-major
SEARCH_PAIR_PARENTS = 1 << 22  # kf_capi.cpp kSearchPairParents: KF_OPT_SEARCH_PAIR = 0 pairs levels with as many


def _pair_policy(pair):
    """(least parents of a parent-major pair, child-major pairs for the rest?) of a
    KF_OPT_SEARCH_PAIR value, or None for no pairs (kf_capi.cpp)."""
    pair = {'auto': 0, 'off': 1, 'all': 2, 'cm': 3, True: 0, False: 1}.get(pair, pair)
    if pair == 1:
        return None
    pm_min = {0: SEARCH_PAIR_PARENTS, 2: 0, 3: None}.get(pair, int(pair))
    return pm_min, pair == 3


def search_plan(n, k_max=None, sym=False, pair='auto'):
    """kf_search_combos' launches over n free candidates, exhaustive (kf_capi.cpp): the head
    (sizes 1 .. K, if any), then per level k with stored parents a level launch or — axis-
    symmetric, level k + 1 below the end launch's sizes (KF_OPT_SEARCH_PAIR = pair) — one pair
    launch for levels k and k + 1: parent-major ('pair') for a parent-major level (more than
    SEARCH_CM_PARENTS parents) of at least the policy's parent count (SEARCH_PAIR_PARENTS by
    default), child-major ('pair_cm') otherwise; then the end launch (if any).  Returns
    (launches [(kind, k)], stored levels: the levels whose nodes a launch writes and the next one
    reads, once each)."""
    k_max = n if k_max is None else k_max
    K = search_head_size(n, k_max)
    end = search_end_size(n, k_max)
    pol = _pair_policy(pair) if sym else None
    launches, stored = [], []
    if K:
        launches.append(('head', K))
        stored.append(K)
    k = K + 1 if K else 1
    while k <= k_max:
        if k == end:
            launches.append(('end', k))
            break
        par = 1 if k == 1 else math.comb(n - 2, k - 1)
        if par and pol is not None and k >= 2 and k + 1 <= k_max and k + 1 < end:
            pm_pair = par > SEARCH_CM_PARENTS and pol[0] is not None and par >= pol[0]
            if pm_pair or pol[1]:
                launches.append(('pair' if pm_pair else 'pair_cm', k))
                if k + 1 < k_max:
                    stored.append(k + 1)
                k += 2
                continue
        if par:
            launches.append(('level', k))
            if k < k_max:
                stored.append(k)
        k += 1
    return launches, stored


def search_launches(n, k_max=None, sym=False, pair='auto'):
    """Kernel launches of one kf_search_combos over n free candidates (search_plan)."""
    return len(search_plan(n, k_max, sym, pair)[0])


def search_stored_levels(n, k_max=None, sym=False, pair='auto'):
    """The levels whose nodes one kf_search_combos writes once and reads once as parents
    (search_plan): the head's last size, each level launch's below k_max, each pair launch's
    second level; the end launch stores none."""
    return search_plan(n, k_max, sym, pair)[1]


def search_levels(n, dtype='f64', mem_bytes=32 << 30, sym=False):
    """Largest k_max for which kf_search_combos' level buffers (two of the widest stored level:
    the C(n - 2, k) subsets of size k < k_max whose largest candidate is <= n - 3) fit in
    ``mem_bytes`` and every level stays below 2^28 stored parents (n = free candidates; sym:
    the axis-symmetric search's 10-row nodes, kf_search_plan says which the handle runs)."""
    k_max, widest = 0, 0
    for k in range(1, n + 1):
        if k > 1:
            par = math.comb(n - 2, k - 1)
            if par >= 1 << 28:
                break
            widest = max(widest, par)
        if 2 * search_level_bytes(widest, dtype, sym) + 4096 > mem_bytes:
            break
        k_max = k
    return k_max


def search_class_width(n, dtype='f64', mem_bytes=32 << 30, sym=False):
    """The fewest leading candidates w whose fixed intersections split the search of n
    candidates into 2^w classes that kf_search_combos runs whole: a class has n - w free
    candidates, and every size of it fits ``mem_bytes`` and the 2^28-parent cap
    (search_levels(n - w) = n - w).  n = 40, f64, 32 GiB: 8 axis-symmetric (the widest stored
    level C(30, 15) nodes, 2 x 15.5 GB), 10 with every chain."""
    for w in range(n):
        if search_levels(n - w, dtype, mem_bytes, sym) >= n - w:
            return w
    return max(n - 1, 0)


NO_SIZE = None


def bitrev64(v):
    return int(f'{v & ((1 << 64) - 1):064b}'[::-1], 2)


def class_order(w):
    """The classes of candidates 0 .. w - 1, fewest fixed members first (the classes that can hold
    the smallest sizes; a search that is not exhaustive skips the rest once they cannot win)."""
    return sorted(range(1 << w), key=lambda c: (bin(c).count('1'), c))


def prefix_classes(n, k_max, dtype='f64', mem_bytes=32 << 30, sym=False, limit=None):
    """Classes for the sizes up to ``k_max`` of a search whose levels do not fit one call, when
    the fixed-pattern classes that fit every size (search_class_width) would be too many (n = 64:
    2^32).  A class is a prefix P, its members fixed and its free candidates those after max(P):
    kf_search_combos(n_fixed = max(P) + 1, fixed_mask = P), the subsets P + S, S within
    max(P) + 1 .. n - 1.  From the whole search (P empty), a class whose free sizes up to
    k_max - |P| do not fit one call (search_levels) is split by its next member f into the
    classes P + {f}, f = max(P) + 1 .. n - 1, which hold every subset of the class but P itself
    (the last, P + {n - 1}, as the class of P with the one free candidate n - 1).  Returns
    ([(n_fixed, fixed_mask)], fewest fixed members first, and the largest |P| of a split class —
    that subset is in no class: its size must have been searched already), or None past
    ``limit`` classes.  n = 64, 32 GiB: 64 classes for sizes up to 8, 532 up to 9, 2623 up to 10."""
    import functools
    levels = functools.lru_cache(None)(lambda m: search_levels(m, dtype, mem_bytes, sym))
    out, split = [], [-1]

    def rec(a, mask, p):
        if limit is not None and len(out) > limit:
            return
        if a == n:  # P + {n - 1}: the class of P over the one free candidate n - 1
            out.append((n - 1, mask & ~(1 << (n - 1))))
            return
        if levels(n - a) >= min(k_max - p, n - a):
            out.append((a, mask))
            return
        split[0] = max(split[0], p)
        for f in range(a, n):
            rec(f + 1, mask | (1 << f), p + 1)
    rec(0, 0, 0)
    if limit is not None and len(out) > limit:
        return None
    out.sort(key=lambda x: (bin(x[1]).count('1'), x[0], x[1]))
    return out, split[0]


def search_bands(n, k_done, dtype='f64', mem_bytes=32 << 30, sym=False, max_classes=None):
    """The size bands of a search too large for one call whose sizes 1 .. k_done accepted
    nothing: yields (K, prefix classes of the sizes up to K) for K = k_done + 1, k_done + 2, ...
    while those are fewer than ``max_classes`` (the fixed-pattern classes that search every
    size, which then finish the search: 256 at n = 40) and every subset a split leaves out has a
    size already searched (<= k_done).  Each band searches its sizes again below K; a band holds
    ~(n - K) / K times the subsets of the one before, so the repeats cost a fraction of the last."""
    for K in range(k_done + 1, n + 1):
        got = prefix_classes(n, K, dtype, mem_bytes, sym, limit=max_classes)
        if got is None:
            return
        classes, split = got
        if (max_classes is not None and len(classes) >= max_classes) or split > k_done:
            return
        yield K, classes


SEARCH_FIRST_BYTES = 1 << 30  # the first one-call pass's level buffers (one_call_search)


def one_call_search(kf, ev, init, prev_time, target_end, threshold, k_search, dtype='f64', mem_bytes=32 << 30,
                    sym=False):
    """The sizes 1 .. k_search in one kf_search_combos call each pass, stopping at the first
    accepted size: first the sizes whose level buffers fit SEARCH_FIRST_BYTES, then, if none was
    accepted, all k_search (which searches the first ones again).  A handle's level buffers are
    sized by the call's k_max and freed with the handle, and at n = 40 the sizes up to 10 take
    2 x 16 GB that a box took up to ~0.7 s to map and free per window; the reference's windows
    accept within the first pass's sizes (7 at n = 40, 1 GiB).  Returns (k, indices) or (0, None)."""
    n = int(np.asarray(ev).shape[0])
    k_first = min(k_search, search_levels(n, dtype, min(mem_bytes, SEARCH_FIRST_BYTES), sym))
    k, idx = 0, None
    for k_max in sorted({k_first, k_search} - {0}):
        k, idx, _, _ = kf.search_combos(ev, init, prev_time, target_end, threshold, k_max=k_max)
        if k:
            break
    return k, idx


def search_past(search_class, n, k_done, w, dtype='f64', mem_bytes=32 << 30, sym=False):
    """The reference's pick (class_search's (k, key)) in a search of n candidates whose sizes
    1 .. k_done accepted nothing and whose levels do not fit one call: the next sizes by bands of
    prefix classes (search_bands) while those are fewer than the 2^w classes that fit every size
    (search_class_width; n = 40: 40 classes for size 11, 151 up to 12, then the 256), then every
    size by the latter.  ``search_class(n_fixed, fixed_mask, k_max)`` as class_search's."""
    for K, classes in search_bands(n, k_done, dtype, mem_bytes, sym, 1 << w):
        k, key = class_search(search_class, n, 0, classes, False, K)
        if k is not NO_SIZE:
            return k, key
    return class_search(search_class, n, w, class_order(w))


def class_search(search_class, n, w, classes, exhaustive=False, k_max=None):
    """Runs ``search_class(n_fixed, c, k_max) -> (k, indices or None)`` for each class in turn and
    keeps the reference's pick among them (kf_workers.py:1325-1356): the smallest accepted size
    and, at it, the first subset in itertools.combinations order, i.e. the largest bit-reversed
    mask.  A class is a bit pattern c (the subsets whose intersection with candidates 0 .. w - 1
    is c, n_fixed = w) or a pair (n_fixed, c) (prefix_classes).  Returns (k, key) or
    (NO_SIZE, 0).  Not exhaustive, a class searches only the sizes that can still win: up to
    the best size so far (skipped when its fixed members alone exceed it; one size above when
    they make exactly it, the least k_max kf_search_combos takes).  ``k_max`` caps the sizes
    searched (the reference's loop over sizes 1 .. n, :1325, cut short)."""
    k_r, key_r = NO_SIZE, 0
    cap = n if k_max is None else int(k_max)
    for item in classes:
        nf, c = item if isinstance(item, tuple) else (w, item)
        k_base = bin(c).count('1')
        lim = cap
        if not exhaustive and k_r is not NO_SIZE:
            lim = min(lim, k_r)
        if k_base > lim:
            continue
        k, idx = search_class(nf, c, min(n, max(lim, k_base + 1)))
        if k and idx is not None and k <= cap:
            key = bitrev64(sum(1 << i for i in idx))
            if k_r is NO_SIZE or k < k_r or (k == k_r and key > key_r):
                k_r, key_r = k, key
    return k_r, key_r


def search_combos_classed(kf, ev, init, prev_time, target_end, threshold, w, exhaustive=False, subset_max=False,
                          classes=None, k_max=None):
    """kf.search_combos over sizes 1 .. k_max (default n) of the n candidates as 2^w class
    searches run one after another on this handle's GPU (``class_search``; w from
    ``search_class_width`` when the whole search does not fit one call).  Returns
    search_combos' (k_found, winner indices or None, accepted count per size [n + 1],
    subset_max [2^n] or None): the same winner and counts as one call over those sizes of every
    subset (not exhaustive: counts past k_found are 0)."""
    n = int(np.asarray(ev).shape[0])
    acc = np.zeros(n + 1, dtype=np.uint64)
    sm = None
    if subset_max:
        sm = kf.empty(1 << n)
        sm.fill_(float('nan'))

    def search_class(nf, c, k_max):
        k, idx, a, _ = kf.search_combos(ev, init, prev_time, target_end, threshold, k_max=k_max,
                                        exhaustive=exhaustive, subset_max=sm if sm is not None else False,
                                        n_fixed=nf, fixed_mask=c)
        acc[:len(a)] += a
        return k, idx
    k, key = class_search(search_class, n, w, class_order(w) if classes is None else classes, exhaustive, k_max)
    if k_max is not None:
        acc[int(k_max) + 1:] = 0   # a class whose fixed members make k_max searched one size more
    if k is NO_SIZE:
        return 0, None, acc, sm
    if not exhaustive:
        acc[k + 1:] = 0
    mask = bitrev64(key)
    return k, tuple(i for i in range(n) if (mask >> i) & 1), acc, sm


def run_brute_force_kalman_filter_no_sampling_min_usage(events, start_idx=0, end_idx=None, R_threshold=None,
                                                       initial_pt=None, initial_state=None,
                                                       max_combos_in_memory=1 << 22, dtype='f64', device=0,
                                                       search_mem_bytes=32 << 30, consts=None):
    """kf_workers.py:1218-1392 on the GPU: for k = 1..n, evaluate every k-subset of the candidate
    events and return the first subset, in itertools.combinations order, whose max
    log-determinant is below R_threshold — the reference's result dict — or None.  The subsets
    run as the shared-prefix search (kf_search_combos: one event step per subset): the sizes
    whose level buffers fit ``search_mem_bytes`` in one call (k_search), then, if none of those
    was accepted, class searches one after another (search_past): bands of the next sizes by
    prefix classes while they are the fewer calls, then every size as the 2^w fixed-pattern
    classes (n = 40, the reference's visualizing window, kf_workers_visualizing.py:2293, 2340:
    size 11 in 40 prefix classes, sizes up to 12 in 151, then 256 classes of 32 free
    candidates; n = 64: sizes up to 8 in 64 classes, 9 in 532, 10 in 2623).  ``max_combos_in_memory`` is the reference's argument; the
    search needs no per-subset batch.  One filter per subset stays available as
    ``first_valid_rank`` (kf_eval_combos).  Multi-GPU: kfmi.dist.brute_force_search."""
    if R_threshold is None:
        raise ValueError('R_threshold must be specified for brute force KF.')
    st = brute_force_setup(events, start_idx, end_idx, initial_pt, initial_state, consts)
    if st is None:
        return None
    cand, xt, Pt, prev_time, target_end, ev, init = st
    n = len(cand)
    kf = BatchedKF('ref15', 1, dtype, device=device, params=_params(consts))
    try:
        sym = kf.search_plan(init, n, k_max=1)['sym']
        k_search = search_levels(n, dtype, search_mem_bytes, sym)
        k, idx = one_call_search(kf, ev, init, prev_time, target_end, R_threshold, k_search, dtype,
                                 search_mem_bytes, sym)
        if not k and k_search < n:
            def search_class(nf, c, k_max):
                kk, ii, _, _ = kf.search_combos(ev, init, prev_time, target_end, R_threshold, k_max=k_max,
                                                n_fixed=nf, fixed_mask=c)
                return kk, ii
            w = search_class_width(n, dtype, search_mem_bytes, sym)
            kr, key = search_past(search_class, n, k_search, w, dtype, search_mem_bytes, sym)
            if kr is not NO_SIZE:
                mask = bitrev64(key)
                k, idx = kr, tuple(i for i in range(n) if (mask >> i) & 1)
        if not k:
            return None
        return brute_force_result(cand, k, None, xt, Pt, prev_time, target_end, dtype, device, indices=idx,
                                  consts=consts, kf=kf)
    finally:
        kf.close()


# --------------------------------------------------------------------------------------------
# Sensor scheduling (kf_workers.py:99-213, 826-957)
# --------------------------------------------------------------------------------------------

def scheduler_gain(covariances, types=('GPS', 'IMU'), full=False, dtype='f64', device=0, consts=None):
    """Scheduler.gain (kf_workers.py:174-185) for a batch: covariances [B, 15, 15] (block-diagonal)
    -> [B, len(types)] traces of the posterior covariance after a candidate of each type
    (full=False: the reference's cov_matrix(S=[1]); full=True: every row of the sensor),
    computed in one kf_score_candidates launch."""
    Ps = np.asarray(covariances, np.float64)
    if Ps.ndim == 2:
        Ps = Ps[None]
    B = Ps.shape[0]
    kf = BatchedKF('ref15', B, dtype, device=device, params=_params(consts))
    npd = np.float64 if dtype == 'f64' else np.float32
    kf.set_state(np.zeros((15, B), npd), np.ascontiguousarray(to_blocks(Ps).T.astype(npd)))
    g = kf.score_candidates([GPS if s == 'GPS' else IMU for s in types], full=full)
    out = g.double().cpu().numpy().T
    kf.close()
    return out


def _host_stream(events):
    """The host arrays behind an event list that views an ingested stream (kfmi.kf_workers
    .EventList over kf_ingest's output), or None for a plain list of tuples."""
    h = getattr(events, 'h', None)
    return h if isinstance(h, dict) and {'t', 'etype', 'payload'} <= set(h) else None


def _scheduled_window_events(events, start_idx, end_idx, initial_pt, initial_state, consts=None):
    """Start state and candidate events exactly as run_kalman_filter_scheduled sets them up
    (kf_workers.py:828-877).  Returns (x0, P, prev_time, candidates) or None; candidates is the
    list of event tuples, or for an event list over an ingested stream the (lo, hi) index range
    of the candidates in its arrays (no per-event Python)."""
    if start_idx is None or start_idx < 0:
        start_idx = 0
    if end_idx is None or end_idx > len(events):
        end_idx = len(events)
    x0 = np.zeros(15)
    h = _host_stream(events)
    if initial_state is not None:
        P = np.asarray(initial_pt, np.float64)
        x0[0:6] = initial_state[1:7]
        start_off, prev = start_idx, initial_state[0]
    elif h is not None:
        P = _p0(consts)
        fixes = np.nonzero(h['etype'][start_idx:end_idx] == GPS)[0]
        if not len(fixes):
            return None
        start_off = start_idx + int(fixes[0])
        x0[0:3] = h['payload'][start_off, 0:3]
        prev = float(h['t'][start_off])
    else:
        P = _p0(consts)
        cs = _cold_start(events, start_idx, end_idx)
        if cs is None:
            return None
        x0, prev, start_off = cs
    if end_idx == -1:
        end_idx = len(events)
    if h is not None:
        return x0, P, prev, (start_off + 1, max(start_off + 1, end_idx))
    return x0, P, prev, list(events[start_off + 1:end_idx])


def _stream_arrays(cands, B=1, events=None):
    """Candidate events as one filter's streams repeated over B columns: t [T, B], etype [T, B],
    payload [T, 9, B] (T >= 1: an empty window is one padding event).  cands: event tuples, or
    an index range into the ingested arrays of ``events`` (_scheduled_window_events)."""
    if isinstance(cands, tuple):
        h = _host_stream(events)
        lo, hi = cands
        T = hi - lo
        t = np.zeros((max(T, 1), B))
        et = np.full((max(T, 1), B), NONE, np.uint8)
        pay = np.zeros((max(T, 1), 9, B))
        t[:T] = h['t'][lo:hi, None]
        et[:T] = h['etype'][lo:hi, None]
        pay[:T] = h['payload'][lo:hi, :, None]
        return t, et, pay, T
    T = len(cands)
    t = np.zeros((max(T, 1), B))
    et = np.full((max(T, 1), B), NONE, np.uint8)
    pay = np.zeros((max(T, 1), 9, B))
    for i, (_, stype, ti, sdata) in enumerate(cands):
        t[i, :] = ti
        et[i, :] = GPS if stype == 'GPS' else IMU
        pay[i, :, :] = np.asarray(event_payload(stype, sdata))[:, None]
    return t, et, pay, T


def legacy_words(n):
    """The next n raw 32-bit outputs of NumPy's global legacy generator (np.random's
    MT19937), without advancing it: what kf_run_scheduled_random draws np.random.choice from."""
    rs = np.random.RandomState()
    rs.set_state(np.random.get_state())
    return rs.randint(0, 1 << 32, size=n, dtype=np.uint32)


def run_kalman_filter_scheduled(events, start_idx=None, end_idx=None, initial_pt=None, initial_state=None,
                                selection_method=None, processing_frequency=None, print_output=False,
                                dtype='f64', device=0, consts=None, parallel=True):
    """kf_workers.py:826-957 on the GPU.  'greedy': windowing, Scheduler scoring and the filter
    all run in kf_run_scheduled; 'random': the same in kf_run_scheduled_random, each pick
    np.random.choice over the queue drawn on the device from the global NumPy generator's outputs
    in the reference's order (the generator advances by the outputs drawn).  Returns (states,
    logdets, P).  parallel=False: the random arm's picked events run as the single filter even
    where kf_run_events would take the time-parallel route (a long log; tests)."""
    if selection_method not in ('random', 'greedy'):
        print("Invalid selection_method. Choose either 'random' or 'greedy'.")
        return None
    w = _scheduled_window_events(events, start_idx, end_idx, initial_pt, initial_state, consts)
    if w is None:
        return None, None
    x0, P, prev0, cands = w
    f = float(processing_frequency)
    if selection_method == 'greedy':
        kf = BatchedKF('ref15', 1, dtype, device=device, params=_params(consts))
        npd = np.float64 if dtype == 'f64' else np.float32
        kf.set_state(x0[:, None].astype(npd), to_blocks(P)[:, None].astype(npd))
        t, et, pay, _ = _stream_arrays(cands, events=events)
        tr, ld, stt, ns = kf.run_scheduled(t, et, pay.astype(npd), np.array([prev0]), f)
        # the handle's initial logdet comes from a zero-event pass of the same kernels
        ld0 = _run_streams([[]], x0[None], to_blocks(P)[None], dtype, device, consts=consts)[1][0, 0]
        n = int(ns[0])
        tr, ld, stt = tr.double().cpu().numpy(), ld.double().cpu().numpy(), stt.cpu().numpy()
        xf, Pb = kf.state()
        Pf = from_blocks(Pb[:, 0].double().cpu().numpy())
        kf.close()
        states = [(prev0, *x0[:6])] + [(stt[i, 0], *tr[i, :, 0]) for i in range(n)]
        logdets = [float(ld0)] + [float(v) for v in ld[:n, 0]]
    else:
        # random_schedule (kf_workers.py:188-193): each window's np.random.choice is drawn on the
        # device from the global generator's next outputs, in the reference's order (the windows
        # follow the picks); the global generator then advances by the outputs the run took
        # the picks (windows + draws, kf_sched_random_picks: no filter state needed), then the
        # picked events through the event engine, which runs one long filter parallel over time
        kf = BatchedKF('ref15', 1, dtype, device=device, params=_params(consts))
        npd = np.float64 if dtype == 'f64' else np.float32
        t, et, pay, n_cand = _stream_arrays(cands, events=events)
        dev = kf.device
        td, etd = torch.as_tensor(t, device=dev), torch.as_tensor(et, device=dev)
        n_words = 2 * n_cand + 64
        while True:
            pick, stt, ns, used = kf.sched_random_picks(td, etd, np.array([prev0]), f,
                                                        legacy_words(n_words)[:, None])
            taken = int(used[0])
            if taken >= 0:
                break
            n_words *= 4  # the column ran out (rejections beyond 2 outputs per window): draw again
        np.random.randint(0, 1 << 32, size=taken, dtype=np.uint32)
        n = int(ns[0])
        sel = pick[:n, 0].long()
        st_d = stt[:n, 0]
        prev_d = torch.cat([torch.tensor([prev0], dtype=torch.float64, device=dev), st_d[:-1]])
        # a leading padding event: row 0 of the records holds the start state and its log-det
        ev_t = torch.cat([torch.tensor([NONE], dtype=torch.uint8, device=dev), etd[sel, 0]])
        ev_dt = torch.cat([torch.zeros(1, dtype=torch.float64, device=dev), st_d - prev_d])
        paydev = torch.as_tensor(pay[:, :, 0].astype(npd), device=dev)
        ev_p = torch.cat([torch.zeros(1, 9, dtype=paydev.dtype, device=dev), paydev[sel]])
        kf.set_state(x0[:, None].astype(npd), to_blocks(P)[:, None].astype(npd))
        tr, ld, _, _ = kf.run_events(ev_t[:, None], ev_dt[:, None], ev_p[:, :, None].contiguous(),
                                     sequential=not parallel)
        tr, ld, stt = tr.double().cpu().numpy(), ld.double().cpu().numpy(), st_d.cpu().numpy()
        _, Pb = kf.state()
        Pf = from_blocks(Pb[:, 0].double().cpu().numpy())
        kf.close()
        states = [(prev0, *x0[:6])] + [(stt[i], *tr[i + 1, :, 0]) for i in range(n)]
        logdets = [float(v) for v in ld[:n + 1, 0]]
    if print_output:
        print(f'{selection_method.capitalize()} Scheduled Kalman Filter (GPU): processed {len(states) - 1} measurements')
    return states, logdets, Pf


def sampling_sweep(events, frequencies, start_idx=None, end_idx=None, initial_pt=None, initial_state=None,
                   dtype='f64', device=0, consts=None):
    """The greedy scheduled filter at every processing frequency in ONE kf_run_scheduled launch
    (one filter per frequency) — the experiment behind the reference's
    sampling_sweep/kf_plot_{10..120}.png.  Returns {f: (states, logdets, P)}."""
    w = _scheduled_window_events(events, start_idx, end_idx, initial_pt, initial_state, consts)
    if w is None:
        return {}
    x0, P, prev0, cands = w
    freqs = np.asarray(frequencies, np.float64)
    B = len(freqs)
    npd = np.float64 if dtype == 'f64' else np.float32
    kf = BatchedKF('ref15', B, dtype, device=device, params=_params(consts))
    kf.set_state(np.repeat(x0[:, None], B, 1).astype(npd), np.repeat(to_blocks(P)[:, None], B, 1).astype(npd))
    t, et, pay, _ = _stream_arrays(cands, B, events=events)
    tr, ld, stt, ns = kf.run_scheduled(t, et, pay.astype(npd), np.full(B, prev0), freqs)
    ld0 = _run_streams([[]], x0[None], to_blocks(P)[None], dtype, device, consts=consts)[1][0, 0]
    tr, ld, stt, ns = tr.double().cpu().numpy(), ld.double().cpu().numpy(), stt.cpu().numpy(), ns.cpu().numpy()
    _, Pb = kf.state()
    Pb = Pb.double().cpu().numpy()
    kf.close()
    out = {}
    for b, f in enumerate(frequencies):
        n = int(ns[b])
        states = [(prev0, *x0[:6])] + [(stt[i, b], *tr[i, :, b]) for i in range(n)]
        out[f] = (states, [float(ld0)] + [float(v) for v in ld[:n, b]], from_blocks(Pb[:, b]))
    return out
