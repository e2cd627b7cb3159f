"""Rebuild the reference's event tuples (kf_workers.py:375-385 layout) from a golden .npz."""
import numpy as np


def unpack_events(g):
    events = []
    for k in range(len(g['ev_t'])):
        t = float(g['ev_t'][k])
        if g['ev_type'][k] == 0:
            e, n, a = (float(v) for v in g['ev_gps'][k])
            payload = {'time': t, 'easting': e, 'northing': n, 'zone_number': 19,
                       'zone_letter': 'T', 'altitude': a}
            events.append((k, 'GPS', t, payload))
        else:
            events.append((k, 'IMU', t, [repr(t), *(float(v) for v in g['ev_imu'][k])]))
    return events
