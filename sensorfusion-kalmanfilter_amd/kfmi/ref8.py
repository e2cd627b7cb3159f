"""The reference's 8-state planar GPS+IMU filter (hw5_2.py) on the engine (KF_MODEL_REF8).

    run_kalman_filter      hw5_2.py:313-380
    run_dead_reckoning     hw5_2.py:382-436 (run_dead_reckoning_for_IMU)

State [x, y, theta, vx, vy, theta_dot, ax, ay] (hw5_2.py:219-231); a GPS fix updates (x, y)
with R = 3 (hw5_2.py:258-284, 341-349), an IMU sample the whole state through the
pseudo-measurement built from the predicted state, with theta = yaw and theta_dot = wz
(hw5_2.py:352-366).  The covariance is exactly block-diagonal over (x, vx, ax), (y, vy, ay) and
(theta, theta_dot), stored as 15 block-packed rows.  Every predict/update runs in the HIP
kernel (kf_run_events); host code only differences time stamps in fp64.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .engine import BatchedKF
from .ref15 import GPS, IMU, _params, _run_streams, event_payload, from_blocks, to_blocks

# hw5_2.py:317-326
P0 = np.diag([1000.0, 1000.0, 100.0, 100.0, 100.0, 100.0, 1000.0, 1000.0])


def run_kalman_filter(events, dtype='f64', device=0, return_covariance=False, consts=None):
    """hw5_2.py:313-380 on the GPU: x0 = 0, events from the first GPS fix on (that fix at
    dt = 0), no dt < 0 guard (a negative dt is predicted over, as the reference does).
    Returns sf_KF_state = [(x, y, theta), ...] with the initial (0, 0, 0) first (and the final
    8x8 covariance with return_covariance=True).  consts: a ModelConsts('ref8', ...) (the
    reference's by default)."""
    stream = []
    prev = None
    for (_, stype, t, sdata) in events:
        if stype == 'GPS' and prev is None:
            prev = t
        if prev is None:
            continue
        stream.append((GPS if stype == 'GPS' else IMU, t - prev, event_payload(stype, sdata)))
        prev = t
    P = consts.P0 if consts is not None else P0
    tr, _, _, _, Pb, _ = _run_streams([stream], np.zeros((1, 8)), to_blocks(P)[None], dtype, device,
                                      model='ref8', consts=consts)
    states = [tuple(tr[i, :, 0]) for i in range(len(stream) + 1)]
    if return_covariance:
        return states, from_blocks(Pb[:, 0])
    return states


def _stream_of(events):
    """The EventStream behind a kfmi.ingest.EventStream or the façades' EventList, else None."""
    from .ingest import EventStream
    if isinstance(events, EventStream):
        return events
    s = getattr(events, 's', None)
    return s if isinstance(s, EventStream) and len(events) == len(s) else None


# the device checks of the last run_dead_reckoning that took the time-parallel route (diagnostics)
dead_reckoning_check = {}


def run_dead_reckoning(events, dtype='f64', device=0, return_covariance=False, consts=None,
                       parallel_min_events=1 << 16):
    """hw5_2.py:382-436 (run_dead_reckoning_for_IMU) on the GPU: the 8-state filter over the IMU
    events alone — a GPS fix neither predicts nor moves the previous time (:403-404), the first
    IMU event has dt 0 (:401, 407), later ones dt = t - the previous IMU time with no dt < 0
    guard, x0 = 0 and P0 as :385-395, and every event predicts then applies the H = I8
    pseudo-measurement (:410-431).  Returns deadreckoned_IMU_estimates = [(x, y, theta), ...],
    one per IMU event and no initial entry (:399, 433) (and the final 8x8 covariance with
    return_covariance=True).

    ``events``: the reference's list, or an EventStream / the façade's EventList over one —
    then the IMU events are compacted on the device (kf_events_select), differenced there
    (kf_events_dt, KF_DT_RAW from no previous time) and run as one filter: kf_run_stream (the
    time-parallel route, checked on the device, ``dead_reckoning_check``) for at least
    ``parallel_min_events`` IMU events, else kf_run_events."""
    P = consts.P0 if consts is not None else P0
    es = _stream_of(events)
    if es is None:
        stream = []
        prev = None
        for (_, stype, t, sdata) in events:
            if stype != 'IMU':
                continue
            stream.append((IMU, t - prev if prev is not None else 0.0, event_payload(stype, sdata)))
            prev = t
        if not stream:
            return ([], np.asarray(P, np.float64).copy()) if return_covariance else []
        tr, _, _, _, Pb, _ = _run_streams([stream], np.zeros((1, 8)), to_blocks(P)[None], dtype, device,
                                          model='ref8', consts=consts)
        states = [tuple(tr[i, :, 0]) for i in range(1, len(stream) + 1)]
        return (states, from_blocks(Pb[:, 0])) if return_covariance else states
    from .ingest import events_dt, select_events
    t, pay, _ = select_events(es, _lib.KF_EVENT_IMU)
    T = int(t.shape[0])
    if T == 0:
        return ([], np.asarray(P, np.float64).copy()) if return_covariance else []
    dt, et = events_dt(t, float('nan'), _lib.KF_DT_RAW)       # etype_in NULL: all IMU
    dev = t.device
    kf = BatchedKF('ref8', 1, dtype, device=dev.index or 0, params=_params(consts))
    npd = torch.float64 if dtype == 'f64' else torch.float32
    try:
        kf.set_state(torch.zeros(8, 1, dtype=npd, device=dev),
                     torch.as_tensor(to_blocks(P)[:, None], dtype=npd, device=dev))
        dead_reckoning_check.clear()
        if T >= parallel_min_events:
            tr, _, _, _ = kf.run_stream(et, dt, pay.to(npd), logdet=False)
            dead_reckoning_check.update(kf.stream_check())
        else:
            tr, _, _, _ = kf.run_events(et[:, None], dt[:, None], pay.to(npd)[:, :, None], logdet=False)
        x, Pb = kf.state()
        torch.cuda.synchronize(dev)
        tr = tr[:, :, 0].double().cpu().numpy()
        Pf = from_blocks(Pb[:, 0].double().cpu().numpy())
    finally:
        kf.close()
    states = [tuple(r) for r in tr]
    return (states, Pf) if return_covariance else states
