"""Rebuild the reference's event tuples (kf_workers.py:375-385 layout) from a golden .npz."""
import numpy as np


def unpack_events(g, prefix=''):
    events = []
    for k in range(len(g[prefix + 'ev_t'])):
        t = float(g[prefix + 'ev_t'][k])
        if g[prefix + 'ev_type'][k] == 0:
            e, n, a = (float(v) for v in g[prefix + 'ev_gps'][k])
            payload = {'time': t, 'easting': e, 'northing': n, 'zone_number': 19,
                       'zone_letter': 'T', 'altitude': a}
            events.append((k, 'GPS', t, payload))
        else:
            events.append((k, 'IMU', t, [repr(t), *(float(v) for v in g[prefix + 'ev_imu'][k])]))
    return events
