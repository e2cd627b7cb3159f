"""CPU oracle for the batched KF predict/update path — TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product: only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it.
The shipped path (``kfmi``) never imports it and fails loudly without its HIP
library.

What it restates (all citations are into the reference, IseanB/SensorFusion-KalmanFilter):

* 15-state GPS+IMU model of ``kf_workers.py``:
  F(dt) ``kf_workers.py:493-517``, Q(dt) ``519-544``, ``predict_covariance`` ``546-549``,
  H_gps ``551-558``, H_imu ``560-579``, R_gps ``581-585``, R_imu ``587-614``,
  ``calculate_kalman_gain`` ``616-621``.
* 8-state legacy model of ``hw5_2.py``: F ``219-231``, Q ``233-251``, H ``258-278``,
  R ``280-304``, P0 ``317-326``.
* the per-event step in the reference's op order (``kf_workers.py:688-717``):
  ``x = F x``; ``P = (F P) F^T + Q``; ``K = (P H^T) inv((H P) H^T + R)``;
  ``y = Z - H x``; ``x = x + K y``; ``P = (I - K H) P``; ``slogdet(P)``.
* drivers: ``run_kalman_filter_full`` (``kf_workers.py:623-728``),
  ``evaluate_combo_chunk_worker`` (``kf_workers.py:22-97``),
  ``run_adaptive_threshold_kalman_filter`` (``kf_workers.py:959-1058``),
  ``hw5_2.run_kalman_filter`` (``hw5_2.py:313-380``).
* the BASELINE configs' 4-state/2-meas and 6-state/3-meas constant-velocity models
  (SURVEY.md §8a): restrictions of the two reference models to [pos, vel] with the
  IMU acceleration as control input ``u`` (``x = F x + G u``).  Same step function,
  same op order, same noise constants (``kf_workers.py:521,523,583,651``,
  ``hw5_2.py:235,237,282,317-326``).

Pinning: ``tests/golden/*.npz`` were produced by importing the reference itself
in the build container (``tests/golden/make_golden.py``); ``tests/test_oracle.py``
checks this module against them to <=1e-12 relative.
"""
from __future__ import annotations

import numpy as np

# --------------------------------------------------------------------------------------
# Model matrices
# --------------------------------------------------------------------------------------

# Q = diag(q * dt) noise rates, kf_workers.py:521-525 (position 5, orientation 0.05,
# velocity 1, angular velocity 0.1, acceleration 2).
_Q15 = np.array([5.0] * 3 + [0.05] * 3 + [1.0] * 3 + [0.1] * 3 + [2.0] * 3)
# R_imu diagonal, kf_workers.py:589-613.
_RIMU15 = np.array([50.0] * 3 + [0.05] * 3 + [10.0] * 3 + [0.1] * 3 + [100.0] * 3)
# P0, kf_workers.py:651.
P0_REF15 = np.diag([10000.0] * 3 + [1000.0] * 3 + [1000.0] * 3 + [1000.0] * 3 + [10000.0] * 3)

# 8-state model [x, y, theta, vx, vy, theta_dot, ax, ay] (hw5_2.py:219-304).
_Q8 = np.array([5.0, 5.0, 0.05, 1.0, 1.0, 0.1, 2.0, 2.0])
_RIMU8 = np.array([50.0, 50.0, 0.05, 10.0, 10.0, 0.1, 100.0, 100.0])
P0_REF8 = np.diag([1000.0, 1000.0, 100.0, 100.0, 100.0, 100.0, 1000.0, 1000.0])


def F_ref15(dt):
    """kf_workers.py:493-517 — pos += v dt + a dt^2/2, att += w dt, v += a dt."""
    F = np.eye(15)
    for i in range(3):
        F[i, 6 + i] = dt
        F[i, 12 + i] = 0.5 * dt ** 2
        F[3 + i, 9 + i] = dt
        F[6 + i, 12 + i] = dt
    return F


def Q_ref15(dt):
    """kf_workers.py:519-544."""
    return np.diag(_Q15 * dt)


def H_gps15():
    """kf_workers.py:551-558 (rows 0..2 of I15, integer dtype as in the reference)."""
    return np.eye(15, dtype=np.int64)[0:3]


def H_imu15():
    """kf_workers.py:560-579."""
    return np.eye(15, dtype=np.int64)


def R_gps15():
    """kf_workers.py:581-585 (integer diag(3,3,3), promoted on use)."""
    return np.diag([3, 3, 3])


def R_imu15():
    """kf_workers.py:587-614."""
    return np.diag(_RIMU15)


def F_ref8(dt):
    """hw5_2.py:219-231."""
    F = np.eye(8)
    F[0, 3] = dt
    F[0, 6] = 0.5 * dt ** 2
    F[1, 4] = dt
    F[1, 7] = 0.5 * dt ** 2
    F[2, 5] = dt
    F[3, 6] = dt
    F[4, 7] = dt
    return F


def Q_ref8(dt):
    """hw5_2.py:233-251."""
    return np.diag(_Q8 * dt)


def H_gps8():
    """hw5_2.py:258-264."""
    return np.eye(8, dtype=np.int64)[0:2]


def H_imu8():
    """hw5_2.py:266-278."""
    return np.eye(8, dtype=np.int64)


def R_gps8():
    """hw5_2.py:280-284."""
    return np.diag([3, 3])


def R_imu8():
    """hw5_2.py:286-304."""
    return np.diag(_RIMU8)


class CVModel:
    """Constant-velocity kinematic model with ``d`` axes: state [p_1..p_d, v_1..v_d].

    The BASELINE.json 4/2 (d=2) and 6/3 (d=3) configs:
    F = [[I, dt I], [0, I]] (the pos/vel block of ``kf_workers.py:501-509``),
    G = [[dt^2/2 I], [dt I]] (the acceleration column of the same rows, acceleration
    moved from state to control), Q = diag(q_pos dt I, q_vel dt I)
    (``kf_workers.py:521,523``), H = [I 0] (``kf_workers.py:551-558``),
    R = r_gps I (``kf_workers.py:583``).
    """

    def __init__(self, d, q_pos=5.0, q_vel=1.0, r_gps=3.0, p0_pos=None, p0_vel=None, r_full=None):
        self.d = d
        # r_full: a d x d measurement noise in place of r_gps I (the class_args override of
        # get_gps_measurement_noise_covariance_matrix, kf_workers.py:581-585, 1242-1251)
        self.r_full = None if r_full is None else np.array(r_full, dtype=np.float64)
        self.n = 2 * d
        self.m = d
        self.c = d
        self.q_pos = float(q_pos)
        self.q_vel = float(q_vel)
        self.r_gps = float(r_gps)
        if p0_pos is None:
            # 6/3: kf_workers.py:651 (1e4 pos, 1e3 vel); 4/2: hw5_2.py:317-326 (1000, 100).
            p0_pos = 10000.0 if d == 3 else 1000.0
        if p0_vel is None:
            p0_vel = 1000.0 if d == 3 else 100.0
        self.p0_pos = float(p0_pos)
        self.p0_vel = float(p0_vel)

    def F(self, dt):
        F = np.eye(self.n)
        for i in range(self.d):
            F[i, self.d + i] = dt
        return F

    def G(self, dt):
        G = np.zeros((self.n, self.c))
        for i in range(self.d):
            G[i, i] = 0.5 * dt ** 2
            G[self.d + i, i] = dt
        return G

    def Q(self, dt):
        return np.diag([self.q_pos * dt] * self.d + [self.q_vel * dt] * self.d)

    def H(self):
        return np.eye(self.n)[: self.d]

    def R(self):
        return self.r_full.copy() if self.r_full is not None else np.diag([self.r_gps] * self.d)

    def P0(self):
        return np.diag([self.p0_pos] * self.d + [self.p0_vel] * self.d)


CV2 = CVModel(2)
CV3 = CVModel(3)


# --------------------------------------------------------------------------------------
# Step primitives, reference op order
# --------------------------------------------------------------------------------------

def predict_covariance(Pt, F, Qt):
    """kf_workers.py:546-549: P_next = (F P) F^T + Q."""
    return np.dot(np.dot(F, Pt), F.T) + Qt


def calculate_kalman_gain(P, H, R):
    """kf_workers.py:616-621: K = (P H^T) inv((H P) H^T + R)."""
    S = np.dot(np.dot(H, P), H.T) + R
    return np.dot(np.dot(P, H.T), np.linalg.inv(S))


def update(x, P, H, R, Z):
    """kf_workers.py:708-711 (simple-form covariance update, as in the reference)."""
    K = calculate_kalman_gain(P, H, R)
    y = np.array(Z) - np.dot(H, x)
    x = x + np.dot(K, y)
    P = np.dot(np.eye(P.shape[0]) - np.dot(K, H), P)
    return x, P


def imu_pseudo_measurement15(x_pred, sdata, dt):
    """kf_workers.py:699-704 — Z built from the *predicted* state and the raw IMU payload.

    ``sdata`` = [t_str, roll, pitch, yaw, wx, wy, wz, ax, ay, az] (kf_workers.py:367).
    """
    ax, ay, az = sdata[7], sdata[8], sdata[9]
    Vx, Vy, Vz = x_pred[6] + ax * dt, x_pred[7] + ay * dt, x_pred[8] + az * dt
    X, Y, Z_pos = x_pred[0] + Vx * dt, x_pred[1] + Vy * dt, x_pred[2] + Vz * dt
    roll, pitch, yaw = sdata[1], sdata[2], sdata[3]
    ang_x, ang_y, ang_z = sdata[4], sdata[5], sdata[6]
    return [X, Y, Z_pos, roll, pitch, yaw, Vx, Vy, Vz, ang_x, ang_y, ang_z, ax, ay, az]


def imu_pseudo_measurement8(x_pred, sdata, dt):
    """hw5_2.py:362-370."""
    Vx = x_pred[3] + sdata[7] * dt
    Vy = x_pred[4] + sdata[8] * dt
    X = x_pred[0] + Vx * dt
    Y = x_pred[1] + Vy * dt
    theta = sdata[3]
    theta_dot = sdata[6]
    ax = sdata[7]
    ay = sdata[8]
    return [X, Y, theta, Vx, Vy, theta_dot, ax, ay]


def consts_matrices(K, n):
    """Custom diagonal constants K = dict(q, r_imu, r_gps, p0) per state (the class_args override
    of the model getters, kf_workers.py:1242-1251) -> (Q(dt), R_gps, R_imu, P0)."""
    q = np.asarray(K['q'], np.float64)[:n]
    return (lambda dt: np.diag(q * dt)), np.diag(np.asarray(K['r_gps'], np.float64)), \
        np.diag(np.asarray(K['r_imu'], np.float64)[:n]), np.diag(np.asarray(K['p0'], np.float64)[:n])


def step15(x, P, stype, sdata, dt, K=None):
    """One event of ``run_kalman_filter_full`` (kf_workers.py:688-711); K: custom diagonal
    constants (consts_matrices) instead of the reference's getters."""
    F = F_ref15(dt)
    if K is None:
        Qt, Rg, Ri = Q_ref15(dt), R_gps15(), R_imu15()
    else:
        Qf, Rg, Ri, _ = consts_matrices(K, 15)
        Qt = Qf(dt)
    x = np.dot(F, x)
    P = predict_covariance(P, F, Qt)
    if stype == 'GPS':
        H, R = H_gps15(), Rg
        Z = [sdata['easting'], sdata['northing'], sdata['altitude']]
    else:
        Z = imu_pseudo_measurement15(x, sdata, dt)
        H, R = H_imu15(), Ri
    return update(x, P, H, R, Z)


# --------------------------------------------------------------------------------------
# Reference drivers (event-list form, same tuple layout as the reference)
# --------------------------------------------------------------------------------------

def run_kalman_filter_full(events, start_idx=0, end_idx=None, initial_pt=None, initial_state=None, K=None):
    """kf_workers.py:623-728. ``events`` = [(idx, 'GPS'|'IMU', t, payload), ...] as built by
    ``combine_sensor_data`` (kf_workers.py:375-385). Returns (states, logdets, P, prev_time)."""
    if end_idx is None or end_idx > len(events):
        end_idx = len(events)
    xt = np.zeros(15)
    if initial_pt is not None and initial_state is not None:
        Pt = initial_pt
        xt[0:6] = initial_state[1:7]
        prev_time = initial_state[0]
        start_off = start_idx
    else:
        Pt = P0_REF15.copy() if K is None else consts_matrices(K, 15)[3]
        start_off = -1
        prev_time = None
        for i, (_, stype, t, sdata) in enumerate(events[start_idx:end_idx + 1]):
            if stype == 'GPS':
                xt[0] = sdata['easting']
                xt[1] = sdata['northing']
                xt[2] = sdata['altitude']
                prev_time = t
                start_off = start_idx + i
                break
        if start_off == -1:
            return [], [], []
    states = [(prev_time, *xt[:6])]
    logdets = [np.linalg.slogdet(Pt)[1]]
    # the initialising GPS event is processed again at dt=0 (kf_workers.py:681)
    for (_, stype, t, sdata) in events[start_off:end_idx]:
        dt = t - prev_time
        if dt < 0:  # kf_workers.py:683-685
            prev_time = t
            continue
        xt, Pt = step15(xt, Pt, stype, sdata, dt, K)
        states.append((t, *xt[:6]))
        logdets.append(np.linalg.slogdet(Pt)[1])
        prev_time = t
    return states, logdets, Pt, prev_time


def run_kalman_filter_simple(events, start_idx, end_idx):
    """kf_workers.py:738-824: x0 = 0 and the reference's integer P0 (:744-760), skip events
    until the window's first GPS (whose dt is 0), no dt < 0 guard.  Returns (states,
    covariances) with states[0] = (0, 0, ...) and one covariance per record."""
    xt = np.zeros(15, dtype=np.int64)
    Pt = P0_REF15.astype(np.int64)
    states = [(0, *xt[:6])]
    covs = [Pt.copy()]
    started = False
    prev = None
    for (_, stype, t, sdata) in events[start_idx:end_idx]:
        if stype == 'GPS' and not started:
            started = True
            prev = t
        if not started:
            continue
        dt = t - prev if prev is not None else 0
        xt, Pt = step15(xt, Pt, stype, sdata, dt)
        states.append((t, *xt[:6]))
        covs.append(Pt.copy())
        prev = t
    return states, covs


def run_no_update(events, start_idx=None, end_idx=None, initial_pt=None, initial_state=None):
    """kf_workers.py:1060-1160: the adaptive driver's loop with every update commented out —
    predictions only, logdet after each.  A dt < 0 event is skipped WITHOUT advancing the
    previous time (:1113-1116 assigns an unused name).  Returns (states, logdets, P,
    previous_time, measurement_times) or None when no GPS starts the window."""
    if start_idx is None or start_idx < 0:
        start_idx = 0
    if end_idx is None or end_idx > len(events):
        end_idx = len(events)
    xt = np.zeros(15)
    mtimes = []
    if initial_pt is not None and initial_state is not None:
        Pt = initial_pt
        xt[0:6] = initial_state[1:7]
        prev = initial_state[0]
        start_off = start_idx
    else:
        Pt = P0_REF15.copy()
        start_off = -1
        for i, (_, stype, t, sdata) in enumerate(events[start_idx:end_idx]):
            if stype == 'GPS':
                xt[0], xt[1], xt[2] = sdata['easting'], sdata['northing'], sdata['altitude']
                prev = t
                start_off = start_idx + i
                mtimes.append(t)
                break
        if start_off == -1:
            return None
    states = [(prev, *xt[:6])]
    logdets = [np.linalg.slogdet(Pt)[1]]
    for (_, stype, t, sdata) in events[start_off:end_idx]:
        dt = t - prev
        if dt < 0:
            continue
        F = F_ref15(dt)
        xt = np.dot(F, xt)
        Pt = predict_covariance(Pt, F, Q_ref15(dt))
        states.append((t, *xt[:6]))
        logdets.append(np.linalg.slogdet(Pt)[1])
        prev = t
    return states, logdets, Pt, prev, mtimes


def evaluate_combo_chunk(chunk, xt, Pt, prev_time, target_end_time, K=None):
    """kf_workers.py:22-97 with the 15-state class_args bound in (K: custom diagonal constants).

    Returns [(0, traj, combo, x_final, None, log_det, k), ...]."""
    results = []
    for combo in chunk:
        x = xt.copy()
        P = Pt.copy()
        traj = [(prev_time, *x[:6])]
        s, l = np.linalg.slogdet(P)
        log_det = [s * l]
        cur = prev_time
        for (_, stype, t, sdata) in combo:
            dt = t - cur
            if dt < 0:
                continue
            x, P = step15(x, P, stype, sdata, dt, K)
            traj.append((t, *x[:6]))
            cur = t
            s, l = np.linalg.slogdet(P)
            log_det.append(s * l)
        if cur < target_end_time - 1e-8:  # kf_workers.py:74-82
            dt = target_end_time - cur
            F = F_ref15(dt)
            x = np.dot(F, x)
            P = predict_covariance(P, F, Q_ref15(dt) if K is None else consts_matrices(K, 15)[0](dt))
            traj.append((target_end_time, *x[:6]))
            s, l = np.linalg.slogdet(P)
            log_det.append(s * l)
        results.append((0, traj, combo, x.copy(), None, log_det, len(combo)))
    return results


def run_adaptive_threshold(events, start_idx=0, end_idx=None, R_threshold=-np.inf,
                           initial_pt=None, initial_state=None):
    """kf_workers.py:959-1058: update only when logdet(P_pred) > R_threshold."""
    if end_idx is None or end_idx > len(events):
        end_idx = len(events)
    xt = np.zeros(15)
    times = []
    if initial_pt is not None and initial_state is not None:
        Pt = initial_pt
        xt[0:6] = initial_state[1:7]
        prev = initial_state[0]
        start_off = start_idx
    else:
        Pt = P0_REF15.copy()
        start_off = -1
        prev = None
        for i, (_, stype, t, sdata) in enumerate(events[start_idx:end_idx]):
            if stype == 'GPS':
                xt[0] = sdata['easting']
                xt[1] = sdata['northing']
                xt[2] = sdata['altitude']
                prev = t
                start_off = start_idx + i
                times.append(t)
                break
        if start_off == -1:
            return None
    states = [(prev, *xt[:6])]
    logdets = [np.linalg.slogdet(Pt)[1]]
    for (_, stype, t, sdata) in events[start_off:end_idx]:
        dt = t - prev
        if dt < 0:
            # kf_workers.py:1013-1015 assigns an unused name (prev_time), so the
            # reference keeps previous_time unchanged here; reproduced as-is.
            continue
        F = F_ref15(dt)
        xt = np.dot(F, xt)
        Pt = predict_covariance(Pt, F, Q_ref15(dt))
        sgn, ld = np.linalg.slogdet(Pt)
        if ld * sgn > R_threshold:
            times.append(t)
            if stype == 'GPS':
                H, R = H_gps15(), R_gps15()
                Z = [sdata['easting'], sdata['northing'], sdata['altitude']]
            else:
                Z = imu_pseudo_measurement15(xt, sdata, dt)
                H, R = H_imu15(), R_imu15()
            xt, Pt = update(xt, Pt, H, R, Z)
        states.append((t, *xt[:6]))
        logdets.append(np.linalg.slogdet(Pt)[1])
        prev = t
    return states, logdets, Pt, prev, times


def step8(x, P, stype, sdata, dt, K=None):
    """One event of hw5_2.run_kalman_filter (hw5_2.py:336-366); K: custom diagonal constants."""
    I = np.eye(8)
    F = F_ref8(dt)
    x = np.dot(F, x)
    if K is None:
        Qt, Rg, Ri = Q_ref8(dt), R_gps8(), R_imu8()
    else:
        Qf, Rg, Ri, _ = consts_matrices(K, 8)
        Qt = Qf(dt)
    P = predict_covariance(P, F, Qt)
    if stype == 'GPS':
        H, R = H_gps8(), Rg
        Z = [sdata['easting'], sdata['northing']]
        K = calculate_kalman_gain(P, H, R)
        y = Z - np.dot(H, x)
        x = x + np.dot(K, y)
        P = np.dot(I - np.dot(K, H), P)
    elif stype == 'IMU':
        Z = imu_pseudo_measurement8(x, sdata, dt)
        H, R = H_imu8(), Ri
        K = calculate_kalman_gain(P, H, R)
        y = np.array(Z) - np.dot(H, x)
        x = x + np.dot(K, y)
        P = np.dot(I - np.dot(K, H), P)
    return x, P


def run_kalman_filter_8state(events):
    """hw5_2.py:313-380 (8-state, x0 = 0, starts at the first GPS event)."""
    xt = np.array([0, 0, 0, 0, 0, 0, 0, 0])
    Pt = P0_REF8.astype(np.int64)  # integer literal array as in hw5_2.py:317-326
    states = [(xt[0], xt[1], xt[2])]
    started = False
    prev = None
    for (_, stype, t, sdata) in events:
        if stype == 'GPS' and not started:
            started = True
            prev = t
        if not started:
            continue
        dt = t - prev if prev is not None else 0
        xt, Pt = step8(xt, Pt, stype, sdata, dt)
        states.append((xt[0], xt[1], xt[2]))
        prev = t
    return states, Pt


def run_dead_reckoning_8state(events):
    """hw5_2.py:382-436 (run_dead_reckoning_for_IMU): the 8-state filter over the IMU events
    alone — GPS events neither predict nor move the previous time (:403-404), the first IMU
    event has dt 0 (:401, 407), x0 = 0 and P0 as :385-395, every IMU event predicts and applies
    the H = I8 pseudo-measurement (:410-431), one (x, y, theta) per IMU event and no initial
    record (:399, 433)."""
    xt = np.array([0, 0, 0, 0, 0, 0, 0, 0])
    Pt = P0_REF8.astype(np.int64)
    states = []
    prev = None
    for (_, stype, t, sdata) in events:
        if stype != 'IMU':
            continue
        dt = t - prev if prev is not None else 0
        xt, Pt = step8(xt, Pt, 'IMU', sdata, dt)
        states.append((xt[0], xt[1], xt[2]))
        prev = t
    return states, Pt


# --------------------------------------------------------------------------------------
# Batched constant-velocity filters (the BASELINE configs), reference op order
# --------------------------------------------------------------------------------------

def is_update_step(t, update_every):
    """Step ``t`` (0-based) ends with a GPS update when (t+1) % k == 0: with k=1 every step
    updates (configs 2-4); with k=10 and dt=0.01 s, a 10 Hz GPS update after every tenth
    100 Hz predict (config 5)."""
    return (t + 1) % update_every == 0


def run_filter_loop(model, x0, P0, dt, u, z, update_every=1, mask=None):
    """ONE filter, one event at a time with the reference's per-step NumPy calls
    (kf_workers.py:688-717). This is the 'reference CPU loop' bench.py times.

    x0 [n], P0 [n,n], dt [T], u [T,c], z [U,m] with U = T // update_every.
    Returns traj [T,n], logdet [T], x [n], P [n,n]."""
    T = len(dt)
    x = np.array(x0, dtype=np.float64)
    P = np.array(P0, dtype=np.float64)
    H, R = model.H(), model.R()
    I = np.eye(model.n)
    traj = np.empty((T, model.n))
    logdet = np.empty(T)
    for t in range(T):
        F = model.F(dt[t])
        Qt = model.Q(dt[t])
        x = np.dot(F, x) + np.dot(model.G(dt[t]), u[t])
        P = predict_covariance(P, F, Qt)
        if is_update_step(t, update_every) and (mask is None or mask[t // update_every]):
            K = calculate_kalman_gain(P, H, R)
            y = np.array(z[t // update_every]) - np.dot(H, x)
            x = x + np.dot(K, y)
            P = np.dot(I - np.dot(K, H), P)
        traj[t] = x
        logdet[t] = np.linalg.slogdet(P)[1]
    return traj, logdet, x, P


def run_batch(model, x0, P0, dt, u, z, update_every=1, mask=None):
    """The same recursion as ``run_filter_loop`` vectorised over independent filters.

    x0 [B,n]; P0 [B,n,n] or [n,n]; dt [T]; u [T,c,B]; z [U,m,B] (U = T // update_every);
    mask [U,B] bool or None (False = skip that filter's update, like a dropped fix).
    Returns traj [T,n,B], logdet [T,B], x [B,n], P [B,n,n]."""
    x0 = np.asarray(x0, dtype=np.float64)
    B = x0.shape[0]
    T = len(dt)
    x = x0.copy()
    P = np.broadcast_to(np.asarray(P0, dtype=np.float64), (B, model.n, model.n)).copy()
    H, R = model.H(), model.R()
    I = np.eye(model.n)
    traj = np.empty((T, model.n, B))
    logdet = np.empty((T, B))
    for t in range(T):
        F = model.F(dt[t])
        Qt = model.Q(dt[t])
        G = model.G(dt[t])
        x = x @ F.T + np.asarray(u[t], dtype=np.float64).T @ G.T
        P = np.matmul(np.matmul(F, P), F.T) + Qt
        if is_update_step(t, update_every):
            S = np.matmul(np.matmul(H, P), H.T) + R
            K = np.matmul(np.matmul(P, H.T), np.linalg.inv(S))
            y = np.asarray(z[t // update_every], dtype=np.float64).T - x @ H.T
            xn = x + np.einsum('bij,bj->bi', K, y)
            Pn = np.matmul(I - np.matmul(K, H), P)
            if mask is not None:
                mk = np.asarray(mask[t // update_every], dtype=bool)
                xn = np.where(mk[:, None], xn, x)
                Pn = np.where(mk[:, None, None], Pn, P)
            x, P = xn, Pn
        traj[t] = x.T
        logdet[t] = np.linalg.slogdet(P)[1]
    return traj, logdet, x, P


def tri_pack(P):
    """[B,n,n] -> upper-triangle packed [n(n+1)/2, B] (row-major over i<=j), the engine's
    HBM layout for covariance."""
    n = P.shape[-1]
    iu = np.triu_indices(n)
    return np.ascontiguousarray(P[:, iu[0], iu[1]].T)


def tri_unpack(Ptri, n):
    """[n(n+1)/2, B] -> [B,n,n] symmetric."""
    B = Ptri.shape[1]
    P = np.zeros((B, n, n))
    iu = np.triu_indices(n)
    P[:, iu[0], iu[1]] = Ptri.T
    P[:, iu[1], iu[0]] = Ptri.T
    return P


def parity_errors(traj, logdet, traj_ref, logdet_ref):
    """SURVEY.md §8d parity metric: per filter, per step
    ||x - x_ref||_2 / max(||x_ref||_2, 1) and |dlogdet| / max(|logdet_ref|, 1).
    Arrays [T,n,B] / [T,B]. Returns (max state err, max logdet err)."""
    dx = np.linalg.norm(traj - traj_ref, axis=1)
    nx = np.maximum(np.linalg.norm(traj_ref, axis=1), 1.0)
    dl = np.abs(logdet - logdet_ref) / np.maximum(np.abs(logdet_ref), 1.0)
    return float(np.max(dx / nx)) if dx.size else 0.0, float(np.max(dl)) if dl.size else 0.0


def run_brute_force(events, start_idx, end_idx, R_threshold, initial_pt, initial_state):
    """run_brute_force_kalman_filter_no_sampling_min_usage (kf_workers.py:1218-1392), warm-start
    branch, serially: the first k-subset (smallest k, itertools.combinations order) whose
    max(log_det) < R_threshold (:1349-1371)."""
    from itertools import combinations
    xt = np.zeros(15)
    Pt = np.asarray(initial_pt, dtype=np.float64)
    xt[0:6] = initial_state[1:7]
    prev_time = initial_state[0]
    cand = list(events[start_idx:end_idx])
    target_end = events[end_idx - 1][2]
    for k in range(1, len(cand) + 1):
        for combo in combinations(cand, k):
            res = evaluate_combo_chunk([combo], xt, Pt, prev_time, target_end)
            if res and max(res[0][5]) < R_threshold:
                metric, traj, combo, x_bf, P_bf, log_det, used = res[0]
                return {'selected_sensors': combo, 'final_state': x_bf, 'final_covariance': P_bf,
                        'trajectory': traj, 'accuracy_metric': metric, 'log_determinants': log_det,
                        'num_measurements_used': used}
    return None


# --------------------------------------------------------------------------------------
# Sensor scheduling (kf_workers.py:99-213, 826-957)
# --------------------------------------------------------------------------------------

def scheduler_cov_matrix(S, Sigma_prev, R, H):
    """Scheduler.cov_matrix, device='cpu' branch (kf_workers.py:112-147): posterior covariance
    after updating with the 1-based measurement rows S of (H, R) (all rows if len(S) == m)."""
    k = len(S)
    if k == R.shape[0]:
        R_hat, H_hat = R, H
    else:
        idx = np.array(sorted(S)) - 1
        R_hat, H_hat = R[np.ix_(idx, idx)], H[idx, :]
    Sm = R_hat + np.dot(H_hat, np.dot(Sigma_prev, H_hat.T))
    K = np.dot(np.dot(Sigma_prev, H_hat.T), np.linalg.inv(Sm))
    return Sigma_prev - np.dot(np.dot(K, H_hat), Sigma_prev)


def scheduler_gain(stype, Sigma, K=None):
    """Scheduler.gain (kf_workers.py:174-185): trace of cov_matrix(S=[1]) for the sensor."""
    Rg, Ri = (R_gps15(), R_imu15()) if K is None else consts_matrices(K, 15)[1:3]
    if stype == 'GPS':
        return np.trace(scheduler_cov_matrix([1], Sigma, Rg, H_gps15()))
    return np.trace(scheduler_cov_matrix([1], Sigma, Ri, H_imu15()))


def greedy_schedule(queue, Sigma, K=None):
    """Scheduler.greedy_schedule (kf_workers.py:195-213): first candidate with the largest gain."""
    best, best_i = -np.inf, None
    for i, (_, stype, _, _) in enumerate(queue):
        g = scheduler_gain(stype, Sigma, K)
        if g > best:
            best, best_i = g, i
    return best_i


def run_kalman_filter_scheduled(events, start_idx=None, end_idx=None, initial_pt=None, initial_state=None,
                                selection_method=None, processing_frequency=None, rng_choice=None, K=None):
    """kf_workers.py:826-957: events whose time is within 1/f of the last processed one are
    queued; the next event past the window triggers a selection from the queue (random or
    greedy), then one predict over the accumulated dt and one update on the selection.  The
    triggering event itself is dropped unless the queue was empty (as in the reference).
    rng_choice(n) supplies the random pick (default np.random.choice)."""
    if start_idx is None or start_idx < 0:
        start_idx = 0
    if end_idx is None or end_idx > len(events):
        end_idx = len(events)
    if selection_method not in ('random', 'greedy'):
        return None
    choice = rng_choice or np.random.choice
    xt = np.zeros(15)
    if initial_state is not None:
        Pt = initial_pt
        xt[0:6] = initial_state[1:7]
        start_off = start_idx
        prev = initial_state[0]
    else:
        Pt = P0_REF15.copy() if K is None else consts_matrices(K, 15)[3]
        prev, start_off = None, 0
        for i, (_, stype, t, sdata) in enumerate(events[start_idx:end_idx]):
            if stype == 'GPS':
                xt[0], xt[1], xt[2] = sdata['easting'], sdata['northing'], sdata['altitude']
                prev, start_off = t, start_idx + i
                break
        if prev is None:
            return None, None
    states = [(prev, *xt[:6])]
    logdets = [np.linalg.slogdet(Pt)[1]]
    queue = []
    if end_idx == -1:
        end_idx = len(events)
    for ev in events[start_off + 1:end_idx]:
        (_, stype, t, sdata) = ev
        if t - prev < 1 / processing_frequency:
            queue.append(ev)
            continue
        if not queue:
            queue.append(ev)
        if selection_method == 'random':
            sel = choice(len(queue))
        else:
            sel = greedy_schedule(queue, Pt, K)
        (_, s_type, s_t, s_data) = queue[sel]
        queue = []
        dt = s_t - prev
        xt, Pt = step15(xt, Pt, s_type, s_data, dt, K)
        states.append((s_t, *xt[:6]))
        logdets.append(np.linalg.slogdet(Pt)[1])
        prev = s_t
    return states, logdets, Pt
