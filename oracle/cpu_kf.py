"""ctypes binding of oracle/cpu_kf.c — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this.  The C
restatement runs the reference's dense per-filter step (oracle/cpu_kf.c header) on host cores
with OpenMP; build it with ``make -C oracle`` (__graft_entry__.build() does).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, 'build', 'libcpu_kf.so')
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            raise FileNotFoundError(f'{LIB} not built: make -C oracle')
        L = ctypes.CDLL(LIB)
        vp, i32, i64, f64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_double
        L.cpu_cv_run.argtypes = [i32, i64, i32, f64, vp, i32, vp, vp, vp, vp, f64, f64, f64, vp, vp, vp, vp, vp, i64, i64,
                                 i32]
        L.cpu_cv_run.restype = None
        L.cpu_ref15_events.argtypes = [i64, i32, vp, vp, vp, vp, vp, vp, vp, i64, i64, i32]
        L.cpu_ref15_events.restype = None
        L.cpu_ref15_sched.argtypes = [i64, i32, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, i64, i64, i32]
        L.cpu_ref15_sched.restype = None
        L.cpu_ref8_events.argtypes = [i64, i32, vp, vp, vp, vp, vp, vp, vp, i64, i64, i32]
        L.cpu_ref8_events.restype = None
        L.cpu_ref8_dead_reckoning.argtypes = [i64, vp, vp, vp, vp, vp]
        L.cpu_ref8_dead_reckoning.restype = i64
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype=np.float64):
    return np.ascontiguousarray(a, dtype=dtype)


def threads():
    """The cores this process may use (the GPU box gives each job a 16-core share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, int(os.environ.get('OMP_NUM_THREADS', n))))


def cv_run(d, x0, P0, dt, u, z, update_every=1, q_pos=5.0, q_vel=1.0, r_gps=3.0, filters=None, nthreads=None,
           records=True, R=None):
    """BASELINE 4/2 (d = 2) / 6/3 (d = 3) filters: x0 [n, B], P0 [n, n], u [T, d, B],
    z [T // k, d, B], dt scalar or [T]; R [d, d] (None: r_gps I).  Returns (traj [T, n, B], logdet [T, B], x [n, B],
    P [B, n, n]) for the filter range ``filters`` = (f0, f1) (others left zero)."""
    n = 2 * d
    x0, P0, u, z = _c(x0), _c(P0), _c(u), _c(z)
    dts = None if np.ndim(dt) == 0 else _c(dt)
    T, B = u.shape[0], x0.shape[1]
    f0, f1 = filters or (0, B)
    traj = np.zeros((T, n, B)) if records else None
    ld = np.zeros((T, B)) if records else None
    x = np.zeros((n, B))
    P = np.zeros((B, n, n))
    lib().cpu_cv_run(d, B, T, float(dt) if dts is None else 0.0, _p(dts), int(update_every), _p(u), _p(z), _p(x0),
                     _p(P0), q_pos, q_vel, r_gps, _p(None if R is None else _c(R)),
                     _p(traj), _p(ld), _p(x), _p(P), f0, f1, nthreads or threads())
    return traj, ld, x, P


def ref15_events(etype, dt, payload, x0, P0, filters=None, nthreads=None, records=True):
    """The reference's 15-state events: etype [T, B] u8, dt [T, B], payload [T, 9, B],
    x0 [15, B], P0 15x15.  Returns (traj [T, 6, B], logdet [T, B])."""
    etype, dt, payload, x0, P0 = _c(etype, np.uint8), _c(dt), _c(payload), _c(x0), _c(P0)
    T, B = etype.shape
    f0, f1 = filters or (0, B)
    traj = np.zeros((T, 6, B)) if records else None
    ld = np.zeros((T, B)) if records else None
    lib().cpu_ref15_events(B, T, _p(etype), _p(dt), _p(payload), _p(x0), _p(P0), _p(traj), _p(ld), f0, f1,
                           nthreads or threads())
    return traj, ld


def ref8_events(etype, dt, payload, x0, P0, filters=None, nthreads=None, records=True):
    """hw5_2.py's 8-state model on event streams (cpu_ref8_events): etype [T, B] u8, dt [T, B],
    payload [T, 9, B], x0 [8, B], P0 8x8.  Returns (traj [T, 3, B] (x, y, theta), logdet [T, B])."""
    etype, dt, payload, x0, P0 = _c(etype, np.uint8), _c(dt), _c(payload), _c(x0), _c(P0)
    T, B = etype.shape
    f0, f1 = filters or (0, B)
    traj = np.zeros((T, 3, B)) if records else None
    ld = np.zeros((T, B)) if records else None
    lib().cpu_ref8_events(B, T, _p(etype), _p(dt), _p(payload), _p(x0), _p(P0), _p(traj), _p(ld), f0, f1,
                          nthreads or threads())
    return traj, ld


def ref8_dead_reckoning(etype, t, payload):
    """hw5_2.run_dead_reckoning_for_IMU (cpu_ref8_dead_reckoning) over one merged stream:
    etype [N] u8 (0 GPS, 1 IMU), t [N], payload [N, 9].  Returns (traj [K, 3] (x, y, theta),
    logdet [K]) for the K IMU events."""
    etype, t, payload = _c(etype, np.uint8), _c(t), _c(payload)
    N = etype.shape[0]
    K = int(np.count_nonzero(etype == 1))
    traj, ld = np.zeros((K, 3)), np.zeros(K)
    k = lib().cpu_ref8_dead_reckoning(N, _p(etype), _p(t), _p(payload), _p(traj), _p(ld))
    assert k == K
    return traj, ld


def ref15_sched(t, etype, payload, prev0, freq, P0, x0=None, filters=None, nthreads=None):
    """The greedy scheduled driver (kf_workers.py:826-957, warm start): t [T, B], etype [T, B] u8,
    payload [T, 9, B], prev0 [B], freq [B], P0 15x15, x0 [6, B] or None (zeros).  Returns
    (sel_time [T, B], traj [T, 6, B], logdet [T, B], n_sel [B]); rows j >= n_sel[f] stay zero."""
    t, etype, payload = _c(t), _c(etype, np.uint8), _c(payload)
    prev0, freq, P0 = _c(prev0), _c(freq), _c(P0)
    x0 = None if x0 is None else _c(x0)
    T, B = etype.shape
    f0, f1 = filters or (0, B)
    st, traj, ld = np.zeros((T, B)), np.zeros((T, 6, B)), np.zeros((T, B))
    ns = np.zeros(B, np.int32)
    lib().cpu_ref15_sched(B, T, _p(t), _p(etype), _p(payload), _p(prev0), _p(freq), _p(x0), _p(P0), _p(st),
                          _p(traj), _p(ld), _p(ns), f0, f1, nthreads or threads())
    return st, traj, ld, ns
