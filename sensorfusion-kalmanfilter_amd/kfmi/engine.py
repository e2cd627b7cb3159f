"""BatchedKF — the Python face of libkfmi.so: B independent Kalman filters on one MI355X.

The per-step call shape follows the reference's fusion loop (kf_workers.py:688-717):
``predict(dt, u)`` then ``update(z)`` per event, or the fused ``run(...)`` over T steps
(the hot path, one kernel launch).  Device buffers are torch tensors (torch is only the
allocator / stream provider here); all arithmetic happens in the HIP kernels.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import KFError, check

MODELS = {
    # name: (model id, n, m, c, covariance rows)
    'cv2': (_lib.KF_MODEL_CV2, 4, 2, 2, 10),    # 4-state/2-meas, hw5_2.py:219-304 restricted to [x,y,vx,vy]
    'cv3': (_lib.KF_MODEL_CV3, 6, 3, 3, 21),    # 6-state/3-meas, kf_workers.py:493-614 restricted to pos/vel
    'ref15': (_lib.KF_MODEL_REF15, 15, 3, 0, 27),  # the reference's 15-state model; P block-packed
    'ref8': (_lib.KF_MODEL_REF8, 8, 2, 0, 15),     # hw5_2.py's 8-state model; P block-packed
}
REF_MODELS = ('ref15', 'ref8')
TRAJ_WIDTH = {'ref15': 6, 'ref8': 3}  # kf_workers.py:714 (x, y, z, roll, pitch, yaw); hw5_2.py:369 (x, y, theta)
DTYPES = {'f32': (_lib.KF_F32, torch.float32, np.float32), 'f64': (_lib.KF_F64, torch.float64, np.float64)}


# kf_set_option (include/kf.h): option name -> (id, value names); 0 = the library's choice
OPTIONS = {
    'predict': (_lib.KF_OPT_PREDICT, {'auto': 0, 'deferred': 0, 'eager': 1}),
    'cv_kernel': (_lib.KF_OPT_CV_KERNEL, {'auto': 0, 'general': 1, 'block2': 2, 'block4': 4, 'block8': 8}),
    'blocks_per_cu': (_lib.KF_OPT_BLOCKS_PER_CU, {'auto': 0}),
    'events_kernel': (_lib.KF_OPT_EVENTS_KERNEL, {'auto': 0, 'lane': 1, 'chain': 2, 'lds': 3, 'gated': 4}),
    'stream': (_lib.KF_OPT_STREAM, {'auto': 0, 'off': 1}),
    'stream_chunks': (_lib.KF_OPT_STREAM_CHUNKS, {'auto': 0}),
    'stream_final': (_lib.KF_OPT_STREAM_FINAL, {'auto': 0, 'off': 0, 'on': 1}),
    'start_threads': (_lib.KF_OPT_START_THREADS, {'auto': 0}),
    'search_kernel': (_lib.KF_OPT_SEARCH_KERNEL, {'auto': 0, 'cm': 1, 'pm': 2}),
    'search_pm': (_lib.KF_OPT_SEARCH_PM, {'auto': 0, 'lds': 0, 'regs': 1}),
    'search_head': (_lib.KF_OPT_SEARCH_HEAD, {'auto': 0, 'on': 0, 'off': 1}),
    'search_end': (_lib.KF_OPT_SEARCH_END, {'auto': 0, 'on': 0, 'off': 1}),
    'search_pair': (_lib.KF_OPT_SEARCH_PAIR, {'auto': 0, 'off': 1, 'all': 2, 'cm': 3}),
    'axis_sym': (_lib.KF_OPT_AXIS_SYM, {'auto': 0, 'on': 0, 'off': 1}),
    'sched_kernel': (_lib.KF_OPT_SCHED_KERNEL, {'auto': 0, 'regs': 1, 'fused': 2, 'two_pass': 3, 'one_launch': 4}),
    'sched_group': (_lib.KF_OPT_SCHED_GROUP, {'auto': 0, 'wave': 1, 'block': 4}),
    'sched_order': (_lib.KF_OPT_SCHED_ORDER, {'auto': 0, 'heaviest_first': 0, 'batch': 1}),
    'sched_rec_time': (_lib.KF_OPT_SCHED_REC_TIME, {'auto': 0, 'off': 0, 'on': 1}),
}


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def default_params(model):
    p = _lib.kf_params()
    check(_lib.lib().kf_default_params(MODELS[model][0], ctypes.byref(p)))
    return p


def device_count():
    n = ctypes.c_int(0)
    check(_lib.lib().kf_device_count(ctypes.byref(n)))
    return n.value


class BatchedKF:
    """``batch`` independent filters of ``model`` ('cv2' | 'cv3') in ``dtype`` ('f32' | 'f64').

    State layout in HBM (SoA, filter index fastest): x [n, B], P [n(n+1)/2, B] (upper
    triangle packed row-major), status [B] int32.
    """

    def __init__(self, model='cv3', batch=1, dtype='f64', device=0, params=None, options=None):
        if model not in MODELS:
            raise ValueError(f'unknown model {model!r}; choose from {sorted(MODELS)}')
        if dtype not in DTYPES:
            raise ValueError(f'unknown dtype {dtype!r}; choose from {sorted(DTYPES)}')
        self.model = model
        self.dtype = dtype
        self.batch = int(batch)
        if self.batch < 0:
            raise ValueError('batch must be >= 0')
        self.device = torch.device('cuda', device)
        _, self.n, self.m, self.c, self.ntri = MODELS[model]
        self.torch_dtype = DTYPES[dtype][1]
        L = _lib.lib()
        check(L.kf_init(device))
        torch.cuda.set_device(self.device)
        # reference models: params carries the caller's diagonal constants (kf_params.ref_*,
        # e.g. kfmi.ref15.ModelConsts(...).params()), None = the reference's
        self.params = params if params is not None else (None if model in REF_MODELS else default_params(model))
        h = ctypes.c_void_p()
        check(L.kf_alloc(ctypes.byref(h), MODELS[model][0], self.batch, DTYPES[dtype][0],
                         ctypes.byref(self.params) if self.params is not None else None))
        self._h = h
        for k, v in (options or {}).items():
            self.set_option(k, v)

    # -- lifecycle ---------------------------------------------------------------------
    def close(self):
        if getattr(self, '_h', None):
            _lib.lib().kf_free(self._h)
            self._h = None

    def release_retired(self):
        """Free the workspaces earlier graph captures used and larger eager calls replaced
        (kf_release_retired); only once every graph captured from this handle is destroyed.
        Returns the bytes freed."""
        out = ctypes.c_int64(0)
        check(_lib.lib().kf_release_retired(self.handle, ctypes.byref(out)))
        return out.value

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        if not self._h:
            raise KFError(_lib.KF_EINVAL, 'BatchedKF is closed')
        return self._h

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    # -- options (kf_set_option): per handle, nothing is read from the environment --------
    def set_option(self, name, value):
        """Select a kernel variant for this handle (A/B runs, tests); ``name`` is one of
        OPTIONS, ``value`` an int or one of that option's names (``'auto'`` = 0 everywhere)."""
        opt, names = OPTIONS[name]
        v = names[value] if isinstance(value, str) else int(value)
        check(_lib.lib().kf_set_option(self.handle, opt, v))
        return self

    def get_option(self, name):
        out = ctypes.c_int64(0)
        check(_lib.lib().kf_get_option(self.handle, OPTIONS[name][0], ctypes.byref(out)))
        return out.value

    # -- buffers -------------------------------------------------------------------------
    def empty(self, *shape, dtype=None):
        return torch.empty(shape, dtype=dtype or self.torch_dtype, device=self.device)

    def _dev(self, a, shape, name, dtype=None):
        """Validate (or move) an input stream to a contiguous device tensor of `shape`."""
        dt = dtype or self.torch_dtype
        if isinstance(a, np.ndarray):
            a = torch.from_numpy(np.ascontiguousarray(a))
        if not torch.is_tensor(a):
            raise TypeError(f'{name}: expected a torch tensor or numpy array, got {type(a)}')
        if tuple(a.shape) != tuple(shape):
            raise ValueError(f'{name}: shape {tuple(a.shape)} != expected {tuple(shape)}')
        if a.dtype != dt:
            raise TypeError(f'{name}: dtype {a.dtype} != expected {dt}')
        if a.device != self.device:
            a = a.to(self.device)
        return a.contiguous()

    # -- state ---------------------------------------------------------------------------
    def reset(self, x0=None):
        """x = x0 ([n, B]; None = zeros), P = P0, status = OK (kf_workers.py:651-666)."""
        x0d = self._dev(x0, (self.n, self.batch), 'x0') if x0 is not None else None
        check(_lib.lib().kf_reset(self.handle, _ptr(x0d), self._stream()))

    def set_state(self, x, P):
        xd = self._dev(x, (self.n, self.batch), 'x')
        Pd = self._dev(P, (self.ntri, self.batch), 'P')
        check(_lib.lib().kf_set_state(self.handle, _ptr(xd), _ptr(Pd), 1, self._stream()))

    def state(self):
        """(x [n, B], P_packed [n(n+1)/2, B]) as new device tensors."""
        x = self.empty(self.n, self.batch)
        P = self.empty(self.ntri, self.batch)
        check(_lib.lib().kf_get_state(self.handle, _ptr(x), _ptr(P), 1, self._stream()))
        return x, P

    def status(self):
        s = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        check(_lib.lib().kf_get_status(self.handle, _ptr(s), 1, self._stream()))
        return s

    # -- per-step call shape (kf_workers.py:688-717) ----------------------------------------
    def predict(self, dt, u=None, dt_per_filter=None, logdet=False):
        """x = F(dt) x + G(dt) u, P = F P F^T + Q(dt).  Returns logdet(P_pred) [B] if asked.
        Reference models: one KF_EVENT_PREDICT event per filter (kf_run_events, T = 1)."""
        if self.model in REF_MODELS:
            if u is not None:
                raise ValueError(f'{self.model}: no control input (the IMU enters as a measurement)')
            dts = (dt_per_filter if dt_per_filter is not None else
                   np.full(self.batch, float(dt if dt is not None else 0.0)))
            return self._event(_lib.KF_EVENT_PREDICT, dts, None, None, logdet)
        ud = self._dev(u, (self.c, self.batch), 'u') if u is not None else None
        dtf = (self._dev(dt_per_filter, (self.batch,), 'dt_per_filter', torch.float64)
               if dt_per_filter is not None else None)
        ld = self.empty(self.batch) if logdet else None
        check(_lib.lib().kf_predict(self.handle, float(dt if dt is not None else 0.0), _ptr(dtf),
                                    _ptr(ud), _ptr(ld), self._stream()))
        return ld

    def update(self, z, mask=None, logdet=True, sensor='gps'):
        """GPS update with z [m, B]; mask [B] (0 = skip).  Returns logdet(P) [B] if asked.
        Reference models: a GPS fix event at dt = 0 (the predict is then exactly the identity);
        the IMU pseudo-measurement is built from the predicted state and the event's dt
        (kf_workers.py:698-706), so it is an event: ``step('imu', dt, payload)``."""
        if self.model in REF_MODELS:
            if sensor != 'gps':
                raise ValueError("the IMU update needs the event's dt: use step('imu', dt, payload)")
            zz = z.cpu().numpy() if torch.is_tensor(z) else np.asarray(z)
            if zz.shape != (self.m, self.batch):
                raise ValueError(f'z: shape {zz.shape} != expected {(self.m, self.batch)}')
            pay = np.zeros((9, self.batch))
            pay[:self.m] = zz
            return self._event(_lib.KF_EVENT_GPS, np.zeros(self.batch), pay, mask, logdet)
        zd = self._dev(z, (self.m, self.batch), 'z')
        md = self._dev(mask, (self.batch,), 'mask', torch.uint8) if mask is not None else None
        ld = self.empty(self.batch) if logdet else None
        check(_lib.lib().kf_update(self.handle, _ptr(zd), _ptr(md), _ptr(ld), self._stream()))
        return ld

    def step(self, sensor, dt, payload, mask=None, logdet=True):
        """Reference models: one event of the reference loop for every filter (kf_workers.py:
        688-717): predict over dt (scalar or [B]), then the GPS fix (payload [3, B]: easting,
        northing, altitude) or the IMU pseudo-measurement (payload [9, B]: roll, pitch, yaw,
        wx, wy, wz, ax, ay, az).  mask [B]: 0 = no event for that filter.  Returns logdet [B]."""
        if self.model not in REF_MODELS:
            raise ValueError('step() is the event call of the reference models (ref15 / ref8)')
        et = {'gps': _lib.KF_EVENT_GPS, 'imu': _lib.KF_EVENT_IMU}.get(sensor)
        if et is None:
            raise ValueError(f"sensor must be 'gps' or 'imu', not {sensor!r}")
        pp = payload.cpu().numpy() if torch.is_tensor(payload) else np.asarray(payload)
        rows = 3 if sensor == 'gps' else 9
        if pp.shape != (rows, self.batch):
            raise ValueError(f'payload: shape {pp.shape} != expected {(rows, self.batch)}')
        pay = np.zeros((9, self.batch))
        pay[:rows] = pp
        dts = np.array(np.broadcast_to(np.asarray(dt, dtype=np.float64), (self.batch,)))
        return self._event(et, dts, pay, mask, logdet)

    def logdet(self):
        """log det P of every filter's current covariance [B] (no state change)."""
        if self.model in REF_MODELS:
            return self._event(_lib.KF_EVENT_NONE, np.zeros(self.batch), None, None, True)
        return self.predict(0.0, logdet=True)  # F(0) = I, Q(0) = 0: P is left exactly as it is

    def _event(self, etype, dts, payload, mask, logdet):
        et = np.full((1, self.batch), etype, np.uint8)
        if mask is not None:
            m = mask.cpu().numpy() if torch.is_tensor(mask) else np.asarray(mask)
            et[0, m.reshape(-1) == 0] = _lib.KF_EVENT_NONE
        npd = DTYPES[self.dtype][2]
        pay = np.zeros((1, 9, self.batch), npd) if payload is None else np.asarray(payload, npd)[None]
        _, ld, _, _ = self.run_events(et, np.asarray(dts, np.float64).reshape(1, self.batch), pay, traj=False,
                                      logdet=logdet)
        return ld[0] if logdet else None

    # -- fused hot path -----------------------------------------------------------------
    def run(self, u, z, dt=None, dt_steps=None, update_every=1, mask=None, traj=True, logdet=True,
            out=None):
        """T fused predict(+update) steps in one launch.

        u [T, c, B]; z [T // update_every, m, B]; dt scalar or dt_steps [T] (float64);
        mask [T // update_every, B] uint8 or None.  Returns (traj [T, n, B], logdet [T, B]);
        pass ``out=(traj, logdet)`` to reuse buffers (either may be None to skip it)."""
        T = int(u.shape[0])
        U = T // update_every
        ud = self._dev(u, (T, self.c, self.batch), 'u')
        zd = self._dev(z, (U, self.m, self.batch), 'z') if U > 0 else None
        md = self._dev(mask, (U, self.batch), 'mask', torch.uint8) if mask is not None else None
        dts = self._dev(dt_steps, (T,), 'dt_steps', torch.float64) if dt_steps is not None else None
        if dts is None and dt is None:
            raise ValueError('run: give dt (scalar) or dt_steps [T]')
        if out is not None:
            tr, ld = out
            if tr is not None:
                tr = self._dev(tr, (T, self.n, self.batch), 'traj')
            if ld is not None:
                ld = self._dev(ld, (T, self.batch), 'logdet')
        else:
            tr = self.empty(T, self.n, self.batch) if traj else None
            ld = self.empty(T, self.batch) if logdet else None
        check(_lib.lib().kf_run(self.handle, T, float(dt or 0.0), _ptr(dts), _ptr(ud), _ptr(zd),
                                _ptr(md), int(update_every), _ptr(tr), _ptr(ld), self._stream()))
        return tr, ld

    def run_host(self, u, z, dt, update_every=1, chunks=8, traj=None, logdet=None):
        """``run`` for streams that live in host memory (numpy arrays or CPU tensors, the shapes
        of ``run``): T is cut into ``chunks`` time chunks and the H2D copy of chunk i+1, the
        launch on chunk i and the D2H copy of chunk i-1 overlap on three streams (the filter
        state carries across launches in the handle, so the result is that of one ``run``).
        traj/logdet: pinned CPU tensors to fill (allocated pinned when None).  Returns them
        after the last copy has landed.  DESIGN.md §4 gives the measured rate (1.5x serial)."""
        def host(a, shape, name):
            if isinstance(a, np.ndarray):
                a = torch.from_numpy(np.ascontiguousarray(a))
            if tuple(a.shape) != tuple(shape) or a.dtype != self.torch_dtype or a.device.type != 'cpu':
                raise ValueError(f'{name}: expected a CPU {self.torch_dtype} array of shape {tuple(shape)}')
            return a.contiguous() if a.is_pinned() else a.contiguous().pin_memory()
        T, k = int(u.shape[0]), int(update_every)
        if T % k:
            raise ValueError('run_host: T must be a multiple of update_every')
        while chunks > 1 and T % (chunks * k):
            chunks -= 1
        hu = host(u, (T, self.c, self.batch), 'u')
        hz = host(z, (T // k, self.m, self.batch), 'z')
        ht = traj if traj is not None else torch.empty(T, self.n, self.batch, dtype=self.torch_dtype).pin_memory()
        hl = logdet if logdet is not None else torch.empty(T, self.batch, dtype=self.torch_dtype).pin_memory()
        host(ht, (T, self.n, self.batch), 'traj')
        host(hl, (T, self.batch), 'logdet')
        du, dz = self.empty(T, self.c, self.batch), self.empty(T // k, self.m, self.batch)
        dtr, dld = self.empty(T, self.n, self.batch), self.empty(T, self.batch)
        sh, sc, sd = (torch.cuda.Stream(self.device) for _ in range(3))
        prev = torch.cuda.current_stream(self.device)
        sh.wait_stream(prev)
        tc = T // chunks
        for i in range(chunks):
            a, b = i * tc, (i + 1) * tc
            with torch.cuda.stream(sh):
                du[a:b].copy_(hu[a:b], non_blocking=True)
                dz[a // k:b // k].copy_(hz[a // k:b // k], non_blocking=True)
                ev_in = torch.cuda.Event()
                ev_in.record(sh)
            with torch.cuda.stream(sc):
                sc.wait_event(ev_in)
                self.run(du[a:b], dz[a // k:b // k], dt=dt, update_every=k, out=(dtr[a:b], dld[a:b]))
                ev_run = torch.cuda.Event()
                ev_run.record(sc)
            with torch.cuda.stream(sd):
                sd.wait_event(ev_run)
                ht[a:b].copy_(dtr[a:b], non_blocking=True)
                hl[a:b].copy_(dld[a:b], non_blocking=True)
        sd.synchronize()
        prev.wait_stream(sc)
        return ht, hl

    # -- reference models: per-filter event streams ----------------------------------------
    def run_events(self, etype, dt, payload, traj=True, logdet=True, updated=False, threshold=None, cov=False,
                   sequential=False):
        """KF_MODEL_REF15 / KF_MODEL_REF8: T events per filter in one launch (kf_run_events).

        etype [T, B] uint8 (KF_EVENT_*), dt [T, B] float64, payload [T, 9, B] (GPS: e, n, alt;
        IMU: roll, pitch, yaw, wx, wy, wz, ax, ay, az).  threshold: adaptive-threshold gating
        (update only if logdet(P_pred) > threshold).  sequential=True: never the time-parallel
        route kf_run_events takes by itself for one long filter (kf_run_events_seq).  Returns
        (traj [T, W, B], logdet [T, B], updated [T, B], cov [T, rows, B]) with None for outputs
        not asked for (W = 6 for ref15, 3 for ref8; cov is block-packed)."""
        if self.model not in REF_MODELS:
            raise ValueError('run_events needs a ref15 or ref8 handle')
        T = int(etype.shape[0])
        et = self._dev(etype, (T, self.batch), 'etype', torch.uint8)
        dtd = self._dev(dt, (T, self.batch), 'dt', torch.float64)
        pay = self._dev(payload, (T, 9, self.batch), 'payload')
        tr = self.empty(T, TRAJ_WIDTH[self.model], self.batch) if traj else None
        ld = self.empty(T, self.batch) if logdet else None
        up = torch.empty(T, self.batch, dtype=torch.uint8, device=self.device) if updated else None
        cv = self.empty(T, self.ntri, self.batch) if cov else None
        gate = threshold is not None
        fn = _lib.lib().kf_run_events_seq if sequential else _lib.lib().kf_run_events
        check(fn(self.handle, T, _ptr(et), _ptr(dtd), _ptr(pay), _ptr(tr), _ptr(cv), _ptr(ld), _ptr(up), int(gate),
                 float(threshold) if gate else 0.0, self._stream()))
        return tr, ld, up, cv

    def run_stream(self, etype, dt, payload, traj=True, logdet=True, updated=False, cov=False, chunk=0,
                   warmup=-1):
        """One filter (a handle of batch 1) over a long event stream, parallel over time
        (kf_run_stream): etype [T] uint8, dt [T] float64, payload [T, 9].  Same outputs as
        run_events with B = 1 ([T, W, 1], [T, 1], ...).  chunk <= 0 / warmup < 0: the library's
        defaults.  stream_check() tells whether the chunked records stood or the sequential
        fallback rewrote them."""
        if self.model not in REF_MODELS or self.batch != 1:
            raise ValueError('run_stream needs a ref15 or ref8 handle of one filter')
        T = int(etype.shape[0])
        et = self._dev(etype.reshape(T, 1), (T, 1), 'etype', torch.uint8)
        dtd = self._dev(dt.reshape(T, 1), (T, 1), 'dt', torch.float64)
        pay = self._dev(payload.reshape(T, 9, 1), (T, 9, 1), 'payload')
        tr = self.empty(T, TRAJ_WIDTH[self.model], 1) if traj else None
        ld = self.empty(T, 1) if logdet else None
        up = torch.empty(T, 1, dtype=torch.uint8, device=self.device) if updated else None
        cv = self.empty(T, self.ntri, 1) if cov else None
        check(_lib.lib().kf_run_stream(self.handle, T, _ptr(et), _ptr(dtd), _ptr(pay), _ptr(tr), _ptr(cv), _ptr(ld),
                                       _ptr(up), int(chunk), int(warmup), self._stream()))
        return tr, ld, up, cv

    def stream_check(self):
        """The checks of the last run_stream (kf_stream_check; synchronises the stream)."""
        out = (ctypes.c_double * 8)()
        check(_lib.lib().kf_stream_check(self.handle, out, self._stream()))
        return dict(ok=bool(out[0]), failed_chunk=bool(out[1]), cov_gap=out[2], state_gap=out[3],
                    chunks=int(out[4]), chunk=int(out[5]), warmup=int(out[6]),
                    fallback={0: None, 2: 'chain', 4: 'gated'}[int(out[7])])

    def eval_combos(self, events, init, prev_time, target_end, k, combo_offset=0, logdets=True):
        """KF_MODEL_REF15 brute force (kf_eval_combos): filter f evaluates combination
        combo_offset + f of k out of the n candidate events.  events: host [n, 11] float64
        (t, type, payload[9]); init: host [42] float64 (x[15], block-packed P[27]).
        Returns (max_logdet [B], logdets [k+2, B] or None, n_records [B] int32)."""
        if self.model != 'ref15':
            raise ValueError('eval_combos needs a ref15 handle')
        ev = np.ascontiguousarray(events, dtype=np.float64)
        ini = np.ascontiguousarray(init, dtype=np.float64)
        if ev.ndim != 2 or ev.shape[1] != 11 or ini.shape != (42,):
            raise ValueError('events must be [n, 11] and init [42]')
        mx = self.empty(self.batch)
        ld = self.empty(k + 2, self.batch) if logdets else None
        nr = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        check(_lib.lib().kf_eval_combos(self.handle, ev.shape[0], ev.ctypes.data_as(ctypes.c_void_p),
                                        ini.ctypes.data_as(ctypes.c_void_p), float(prev_time), float(target_end),
                                        int(k), int(combo_offset), _ptr(ld), _ptr(mx), _ptr(nr), self._stream()))
        torch.cuda.current_stream(self.device).synchronize()  # host arrays were staged; keep them alive
        return mx, ld, nr

    def search_combos(self, events, init, prev_time, target_end, threshold, k_max=None, exhaustive=False,
                      subset_max=False, n_fixed=0, fixed_mask=0):
        """KF_MODEL_REF15 brute-force search with shared prefixes (kf_search_combos): sizes
        k = 1 .. k_max of the n candidate events, each subset's filter advanced from its prefix's
        by one event.  Stops after the first size with a subset whose max log-det is below
        threshold unless ``exhaustive``.  ``n_fixed`` / ``fixed_mask`` restrict it to the subsets
        whose intersection with candidates 0 .. n_fixed - 1 is fixed_mask (one shard of the
        search).  Returns (k_found, winner indices tuple or None, accepted count per size
        [k_max + 1], subset_max [2^n] or None).  ``subset_max`` may be a device tensor of 2^n
        entries of the handle's dtype, which receives this search's subsets (untouched
        elsewhere: the classes of one search fill one buffer)."""
        if self.model != 'ref15':
            raise ValueError('search_combos needs a ref15 handle')
        ev = np.ascontiguousarray(events, dtype=np.float64)
        ini = np.ascontiguousarray(init, dtype=np.float64)
        if ev.ndim != 2 or ev.shape[1] != 11 or ini.shape != (42,):
            raise ValueError('events must be [n, 11] and init [42]')
        n = ev.shape[0]
        k_max = n if k_max is None else int(k_max)
        win = ctypes.c_uint64(0)
        kf = ctypes.c_int(0)
        acc = np.zeros(max(k_max, 0) + 1, dtype=np.uint64)
        if isinstance(subset_max, torch.Tensor):
            sm = subset_max
            if (sm.numel() != 1 << n or sm.dtype != self.torch_dtype or sm.device != self.device
                    or not sm.is_contiguous()):
                raise ValueError(f'subset_max must be a contiguous {self.torch_dtype} tensor of 2^{n} entries on '
                                 f'{self.device}')
        else:
            sm = self.empty(1 << n) if subset_max else None
            if sm is not None:
                sm.fill_(float('nan'))
        check(_lib.lib().kf_search_combos(self.handle, n, ev.ctypes.data_as(ctypes.c_void_p),
                                          ini.ctypes.data_as(ctypes.c_void_p), float(prev_time), float(target_end),
                                          float(threshold), k_max, int(bool(exhaustive)), int(n_fixed),
                                          int(fixed_mask), ctypes.byref(win),
                                          ctypes.byref(kf), acc.ctypes.data_as(ctypes.c_void_p), _ptr(sm),
                                          self._stream()))
        combo = tuple(i for i in range(n) if (win.value >> i) & 1) if kf.value else None
        return kf.value, combo, acc, sm

    def search_plan(self, init, n, k_max=None, n_fixed=0, fixed_mask=0):
        """How search_combos would run over n candidates (kf_search_plan, no device work):
        dict(sym, workspace_bytes, widest, max_parents, over_cap)."""
        if self.model != 'ref15':
            raise ValueError('search_plan needs a ref15 handle')
        ini = np.ascontiguousarray(init, dtype=np.float64)
        if ini.shape != (42,):
            raise ValueError('init must be [42]')
        out = np.zeros(5, dtype=np.int64)
        check(_lib.lib().kf_search_plan(self.handle, int(n), ini.ctypes.data_as(ctypes.c_void_p), int(n_fixed),
                                        int(fixed_mask), int(n if k_max is None else k_max),
                                        out.ctypes.data_as(ctypes.c_void_p)))
        return {'sym': bool(out[0]), 'workspace_bytes': int(out[1]), 'widest': int(out[2]),
                'max_parents': int(out[3]), 'over_cap': int(out[4])}

    def search_info(self):
        """How the last search_combos ran (kf_search_info): axis-symmetric or not, the sizes its
        head launch covered, its level launches after the head, the bytes of one level buffer."""
        out = np.zeros(4, dtype=np.int64)
        check(_lib.lib().kf_search_info(self.handle, out.ctypes.data_as(ctypes.c_void_p)))
        return {'sym': bool(out[0]), 'head_sizes': int(out[1]), 'level_launches': int(out[2]),
                'level_bytes': int(out[3])}

    def score_candidates(self, types, full=False, posterior=False):
        """KF_MODEL_REF15 scheduler scoring (kf_score_candidates): [len(types), B] traces of the
        posterior covariance each candidate sensor would give (full=False: the reference's
        Scheduler.gain, first measurement row only).  posterior=True also returns the
        block-packed posterior covariances [len(types), 27, B] (Scheduler.cov_matrix)."""
        if self.model != 'ref15':
            raise ValueError('score_candidates needs a ref15 handle')
        ty = np.ascontiguousarray(types, dtype=np.int32)
        out = self.empty(len(ty), self.batch)
        post = self.empty(len(ty), 27, self.batch) if posterior else None
        check(_lib.lib().kf_score_candidates(self.handle, len(ty), ty.ctypes.data_as(ctypes.c_void_p), int(full),
                                             _ptr(out), _ptr(post), self._stream()))
        return (out, post) if posterior else out

    def score_rows(self, types, row_masks, posterior=False):
        """KF_MODEL_REF15 Scheduler.cov_matrix for any measurement rows (kf_score_rows):
        candidate c is sensor types[c] updated with the rows of row_masks[c] (bit i = 1-based row
        i + 1 of its H).  Returns gain [n, B] (posterior traces) and, with posterior=True, the
        block-packed posteriors [n, 27, B]."""
        if self.model != 'ref15':
            raise ValueError('score_rows needs a ref15 handle')
        ty = np.ascontiguousarray(types, dtype=np.int32)
        mk = np.ascontiguousarray(row_masks, dtype=np.uint32)
        if ty.shape != mk.shape or ty.ndim != 1:
            raise ValueError('score_rows: types and row_masks must be 1-D of one length')
        out = self.empty(len(ty), self.batch)
        post = self.empty(len(ty), 27, self.batch) if posterior else None
        check(_lib.lib().kf_score_rows(self.handle, len(ty), ty.ctypes.data_as(ctypes.c_void_p),
                                       mk.ctypes.data_as(ctypes.c_void_p), _ptr(out), _ptr(post), self._stream()))
        return (out, post) if posterior else out

    def run_scheduled(self, t, etype, payload, prev_time, freq, records=False):
        """KF_MODEL_REF15 rate-decimated greedy filter (kf_run_scheduled).  t [T, B] float64
        absolute times, etype [T, B] uint8, payload [T, 9, B] — or, with records=True, one record
        per event [T, B, rec] (rec >= 9, rec * element size a multiple of 16 B: kf_run_scheduled_rec)
        — prev_time [B] float64, freq scalar or [B] float64 (a sampling sweep in one launch).
        Returns (traj [T, 6, B], logdet [T, B], sel_time [T, B], n_sel [B]) with the first n_sel[f]
        rows of filter f valid."""
        if self.model != 'ref15':
            raise ValueError('run_scheduled needs a ref15 handle')
        T = int(t.shape[0])
        td = self._dev(t, (T, self.batch), 't', torch.float64)
        et = self._dev(etype, (T, self.batch), 'etype', torch.uint8)
        rec = int(payload.shape[2]) if records else 0
        pay = self._dev(payload, (T, self.batch, rec) if records else (T, 9, self.batch), 'payload')
        pv = self._dev(prev_time, (self.batch,), 'prev_time', torch.float64)
        fr = None
        if np.ndim(freq) != 0:
            fr = self._dev(freq, (self.batch,), 'freq', torch.float64)
        tr = self.empty(max(T, 1), 6, self.batch)
        ld = self.empty(max(T, 1), self.batch)
        stt = torch.empty(max(T, 1), self.batch, dtype=torch.float64, device=self.device)
        ns = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        fa = float(freq) if fr is None else 0.0
        if records:
            check(_lib.lib().kf_run_scheduled_rec(self.handle, T, _ptr(td), _ptr(et), _ptr(pay), rec, _ptr(pv),
                                                  _ptr(fr), fa, _ptr(tr), _ptr(ld), _ptr(stt), _ptr(ns),
                                                  self._stream()))
        else:
            check(_lib.lib().kf_run_scheduled(self.handle, T, _ptr(td), _ptr(et), _ptr(pay), _ptr(pv), _ptr(fr),
                                              fa, _ptr(tr), _ptr(ld), _ptr(stt), _ptr(ns), self._stream()))
        return tr, ld, stt, ns

    def run_scheduled_random(self, t, etype, payload, prev_time, freq, words, records=False):
        """KF_MODEL_REF15 random-selection scheduled filter (kf_run_scheduled_random): the
        windows of run_scheduled, each pick np.random.choice(len(queue)) drawn on the device from
        ``words`` [n_words, B] uint32 — column f the raw 32-bit generator outputs filter f
        consumes, in order (see kfmi.ref15.legacy_words).  Returns (traj, logdet, sel_time, n_sel,
        words_used [B] int32: outputs taken, -1 if a column ran out)."""
        if self.model != 'ref15':
            raise ValueError('run_scheduled_random needs a ref15 handle')
        T = int(t.shape[0])
        td = self._dev(t, (T, self.batch), 't', torch.float64)
        et = self._dev(etype, (T, self.batch), 'etype', torch.uint8)
        rec = int(payload.shape[2]) if records else 0
        pay = self._dev(payload, (T, self.batch, rec) if records else (T, 9, self.batch), 'payload')
        pv = self._dev(prev_time, (self.batch,), 'prev_time', torch.float64)
        W = int(words.shape[0])
        if isinstance(words, np.ndarray):
            words = np.ascontiguousarray(words, np.uint32).view(np.int32)
        elif words.dtype == torch.uint32:
            words = words.view(torch.int32)
        wd = self._dev(words, (W, self.batch), 'words', torch.int32)  # the bits of the uint32 outputs
        fr = None
        if np.ndim(freq) != 0:
            fr = self._dev(freq, (self.batch,), 'freq', torch.float64)
        tr = self.empty(max(T, 1), 6, self.batch)
        ld = self.empty(max(T, 1), self.batch)
        stt = torch.empty(max(T, 1), self.batch, dtype=torch.float64, device=self.device)
        ns = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        used = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        check(_lib.lib().kf_run_scheduled_random(self.handle, T, _ptr(td), _ptr(et), _ptr(pay), rec, _ptr(pv), _ptr(fr),
                                                 float(freq) if fr is None else 0.0, _ptr(wd), W, _ptr(used),
                                                 _ptr(tr), _ptr(ld), _ptr(stt), _ptr(ns), self._stream()))
        return tr, ld, stt, ns, used

    def sched_random_picks(self, t, etype, prev_time, freq, words):
        """The random arm's picks alone (kf_sched_random_picks): t [T, B], etype [T, B],
        prev_time [B], freq scalar or [B], words [n_words, B] uint32.  Returns (pick [T, B] int32
        event indices, sel_time [T, B], n_sel [B], words_used [B]); run the picked events with
        run_events."""
        T = int(t.shape[0])
        td = self._dev(t, (T, self.batch), 't', torch.float64)
        et = self._dev(etype, (T, self.batch), 'etype', torch.uint8)
        pv = self._dev(prev_time, (self.batch,), 'prev_time', torch.float64)
        W = int(words.shape[0])
        if isinstance(words, np.ndarray):
            words = np.ascontiguousarray(words, np.uint32).view(np.int32)
        elif words.dtype == torch.uint32:
            words = words.view(torch.int32)
        wd = self._dev(words, (W, self.batch), 'words', torch.int32)
        fr = None
        if np.ndim(freq) != 0:
            fr = self._dev(freq, (self.batch,), 'freq', torch.float64)
        pick = torch.empty(max(T, 1), self.batch, dtype=torch.int32, device=self.device)
        stt = torch.empty(max(T, 1), self.batch, dtype=torch.float64, device=self.device)
        ns = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        used = torch.empty(self.batch, dtype=torch.int32, device=self.device)
        check(_lib.lib().kf_sched_random_picks(self.handle, T, _ptr(td), _ptr(et), _ptr(pv), _ptr(fr),
                                               float(freq) if fr is None else 0.0, _ptr(wd), W, _ptr(used),
                                               _ptr(pick), _ptr(stt), _ptr(ns), self._stream()))
        return pick, stt, ns, used

    # -- synthetic streams -----------------------------------------------
    def synth(self, T, dt, update_every=1, seed=20251015, filter_offset=0):
        """Deterministic synthetic (x0 [n,B], u [T,c,B], z [U,m,B]) generated on the GPU."""
        U = T // update_every
        x0 = self.empty(self.n, self.batch)
        u = self.empty(T, self.c, self.batch)
        z = self.empty(max(U, 0), self.m, self.batch)
        check(_lib.lib().kf_synth(self.handle, int(seed), int(filter_offset), int(T), float(dt),
                                  int(update_every), _ptr(x0), _ptr(u), _ptr(z), self._stream()))
        return x0, u, z
