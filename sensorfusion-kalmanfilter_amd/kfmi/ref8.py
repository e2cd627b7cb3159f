"""The reference's 8-state planar GPS+IMU filter (hw5_2.py) on the engine (KF_MODEL_REF8).

    run_kalman_filter      hw5_2.py:313-380

State [x, y, theta, vx, vy, theta_dot, ax, ay] (hw5_2.py:219-231); a GPS fix updates (x, y)
with R = 3 (hw5_2.py:258-284, 341-349), an IMU sample the whole state through the
pseudo-measurement built from the predicted state, with theta = yaw and theta_dot = wz
(hw5_2.py:352-366).  The covariance is exactly block-diagonal over (x, vx, ax), (y, vy, ay) and
(theta, theta_dot), stored as 15 block-packed rows.  Every predict/update runs in the HIP
kernel (kf_run_events); host code only differences time stamps in fp64.
"""
from __future__ import annotations

import numpy as np

from .ref15 import GPS, IMU, _run_streams, event_payload, to_blocks

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
        from .ref15 import from_blocks
        return states, from_blocks(Pb[:, 0])
    return states
