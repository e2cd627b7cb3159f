"""Ingest: GPS/IMU CSV logs -> one merged, time-sorted event stream resident in HBM.

The reference builds its event list with per-row Python (kf_workers.py:290-385):

    load_data_from_csv (290-298)   -> read_csv: native multithreaded parser (kf_csv_read)
    gps_to_modified_utm (304-331)  -> kf_ingest: keep/drop test + UTM projection per fix (HIP)
    compute_imu_biases (333-347)   -> kf_ingest: bias means on the GPU
    unbias_imu_data (349-373),
    quaternion_to_euler (399-425)  -> kf_ingest: fused into the gather of the merged stream
    combine_sensor_data (375-385)  -> kf_ingest: stable radix sort on time, fixes first on ties

``EventStream`` holds the result as SoA device tensors (etype [N], t [N], payload [N, 9]) — the
layout ``kf_run_events`` reads for a single filter — and can rebuild the reference's
``indexed_sensor_data`` list for code that wants the tuples.  The UTM projection restates the
``utm`` package's published algorithm (the reference pins no version, see oracle/ref_ingest.py).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import check

GPS_COLUMNS = ('time', 'latitude', 'longitude', 'altitude')                        # hw5_1.py:28
IMU_COLUMNS = ('time', 'orientation_x', 'orientation_y', 'orientation_z', 'orientation_w',
               'angular_velocity_x', 'angular_velocity_y', 'angular_velocity_z',
               'linear_acceleration_x', 'linear_acceleration_y', 'linear_acceleration_z')  # hw5_1.py:29-31


def _ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def csv_shape(path, has_header=True):
    """(data rows, fields in the first data row) of a CSV file (kf_csv_shape)."""
    rows = ctypes.c_int64()
    cols = ctypes.c_int()
    check(_lib.lib().kf_csv_shape(os.fsencode(path), int(has_header), ctypes.byref(rows), ctypes.byref(cols)))
    return rows.value, cols.value


def read_csv(path, ncols=None, has_header=True):
    """Parse a numeric CSV into a [ncols, rows] float64 array (kf_csv_read).  A field containing
    'nan' in any case becomes NaN, as the reference's 'nan' in s.lower() tests treat it."""
    rows, cols = csv_shape(path, has_header)
    ncols = cols if ncols is None else ncols
    out = np.empty((max(ncols, 1), max(rows, 1)), dtype=np.float64)
    if rows:
        check(_lib.lib().kf_csv_read(os.fsencode(path), int(has_header), ncols,
                                     out.ctypes.data_as(ctypes.c_void_p), out.shape[1], rows))
    return out[:ncols, :rows]


@dataclass
class EventStream:
    """A merged GPS+IMU event stream on the device (kf_ingest)."""
    etype: torch.Tensor            # [N] uint8: KF_EVENT_GPS / KF_EVENT_IMU
    t: torch.Tensor                # [N] float64
    payload: torch.Tensor          # [N, 9] float64
    src: torch.Tensor              # [N] int32: utm_data position (fix) / IMU row
    zone_number: torch.Tensor      # [N] int8 (0 for IMU)
    zone_letter: torch.Tensor      # [N] uint8 (ASCII; 0 for IMU)
    first_valid_index: int         # compute_imu_biases (kf_workers.py:336)
    gyro_bias: np.ndarray          # angular_velocity_bias
    accel_bias: np.ndarray         # linear_acceleration_bias
    utm_origin: np.ndarray         # (easting, northing) of the first kept fix
    n_fixes: int
    n_imu: int
    with_altitude: bool = True
    _host: dict = field(default_factory=dict, repr=False)

    def __len__(self):
        return int(self.t.shape[0])

    def host(self):
        """NumPy copies of the stream (cached)."""
        if not self._host:
            self._host.update(etype=self.etype.cpu().numpy(), t=self.t.cpu().numpy(),
                              payload=self.payload.cpu().numpy(), src=self.src.cpu().numpy(),
                              zone_number=self.zone_number.cpu().numpy(), zone_letter=self.zone_letter.cpu().numpy())
        return self._host

    def utm_data(self):
        """The reference's utm_data list (kf_workers.py:331; hw5_2.py:54 has no altitude)."""
        h = self.host()
        out = []
        for k in np.nonzero(h['etype'] == _lib.KF_EVENT_GPS)[0]:
            p = h['payload'][k]
            d = {'time': float(h['t'][k]), 'easting': float(p[0]), 'northing': float(p[1]),
                 'zone_number': int(h['zone_number'][k]), 'zone_letter': chr(int(h['zone_letter'][k]))}
            if self.with_altitude:
                d['altitude'] = float(p[2])
            out.append(d)
        return out

    def unbias_imu_data(self):
        """The reference's unbias_imu_data list in IMU row order (kf_workers.py:367): [t_str,
        roll, pitch, yaw, wx, wy, wz, ax, ay, az] (t_str = repr of the parsed time)."""
        h = self.host()
        k = np.nonzero(h['etype'] == _lib.KF_EVENT_IMU)[0]
        k = k[np.argsort(h['src'][k], kind='stable')]
        return [[repr(float(h['t'][i])), *(float(v) for v in h['payload'][i])] for i in k]

    def to_indexed_sensor_data(self):
        """The reference's indexed_sensor_data (kf_workers.py:385): [(i, 'GPS'|'IMU', t, payload)]."""
        h = self.host()
        fixes = self.utm_data()
        out = []
        for i in range(len(self)):
            if h['etype'][i] == _lib.KF_EVENT_GPS:
                out.append((i, 'GPS', fixes[int(h['src'][i])]['time'], fixes[int(h['src'][i])]))
            else:
                t = float(h['t'][i])
                out.append((i, 'IMU', t, [repr(t), *(float(v) for v in h['payload'][i])]))
        return out


def ingest_arrays(gps, imu, with_altitude=True, device=0, bias=None):
    """Merged event stream from parsed columns: gps [4, n] (time, latitude, longitude,
    altitude), imu [11, m] (GPS_COLUMNS / IMU_COLUMNS order), NumPy or torch.  bias: optional
    (angular_velocity_bias[3], linear_acceleration_bias[3]) to use instead of the
    compute_imu_biases means."""
    dev = torch.device('cuda', device) if isinstance(device, int) else torch.device(device)
    g = torch.as_tensor(np.ascontiguousarray(gps, dtype=np.float64) if not torch.is_tensor(gps) else gps,
                        dtype=torch.float64).to(dev).contiguous()
    m = torch.as_tensor(np.ascontiguousarray(imu, dtype=np.float64) if not torch.is_tensor(imu) else imu,
                        dtype=torch.float64).to(dev).contiguous()
    if g.ndim != 2 or g.shape[0] < 4 or m.ndim != 2 or m.shape[0] < 11:
        raise ValueError(f'expected gps [4, n] and imu [11, m] columns, got {tuple(g.shape)} and {tuple(m.shape)}')
    ng, ni = int(g.shape[1]), int(m.shape[1])
    cap = max(ng + ni, 1)
    etype = torch.empty(cap, dtype=torch.uint8, device=dev)
    t = torch.empty(cap, dtype=torch.float64, device=dev)
    payload = torch.empty(cap, 9, dtype=torch.float64, device=dev)
    src = torch.empty(cap, dtype=torch.int32, device=dev)
    zn = torch.empty(cap, dtype=torch.int8, device=dev)
    zl = torch.empty(cap, dtype=torch.uint8, device=dev)
    info = _lib.kf_ingest_info()
    flags = _lib.KF_INGEST_GPS_ALTITUDE if with_altitude else 0
    b = None
    if bias is not None:
        b = np.ascontiguousarray(np.concatenate([np.ravel(bias[0]), np.ravel(bias[1])]), dtype=np.float64)
        if b.shape != (6,):
            raise ValueError('bias must be (angular_velocity_bias[3], linear_acceleration_bias[3])')
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    with torch.cuda.device(dev):
        check(_lib.lib().kf_ingest(_ptr(g) if ng else None, ng, ng, _ptr(m) if ni else None, ni, ni, flags,
                                   None if b is None else b.ctypes.data_as(ctypes.c_void_p),
                                   _ptr(etype), _ptr(t), _ptr(payload), _ptr(src), _ptr(zn), _ptr(zl),
                                   ctypes.byref(info), stream))
    n = int(info.n_events)
    return EventStream(etype[:n], t[:n], payload[:n], src[:n], zn[:n], zl[:n], int(info.first_valid_index),
                       np.array(info.gyro_bias[:]), np.array(info.accel_bias[:]), np.array(info.utm_origin[:]),
                       int(info.n_fixes), int(info.n_imu), with_altitude)


def ingest_csv(gps_csv, imu_csv, with_altitude=True, device=0):
    """The reference's ingest sequence (kf_workers.py:2256-2274: load_data, gps_to_modified_utm,
    compute_imu_biases, unbias_imu_data, combine_sensor_data) as parse + one kf_ingest."""
    return ingest_arrays(read_csv(gps_csv, 4), read_csv(imu_csv, 11), with_altitude, device)


def quaternion_to_euler(q, device=0):
    """quaternion_to_euler (kf_workers.py:399-425) on the device for q [4, n] (x, y, z, w);
    returns [3, n] (roll, pitch, yaw)."""
    dev = torch.device('cuda', device) if isinstance(device, int) else torch.device(device)
    qd = torch.as_tensor(np.asarray(q, dtype=np.float64) if not torch.is_tensor(q) else q,
                         dtype=torch.float64).to(dev).reshape(4, -1).contiguous()
    n = int(qd.shape[1])
    out = torch.empty(3, n, dtype=torch.float64, device=dev)
    stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    with torch.cuda.device(dev):
        check(_lib.lib().kf_quat_to_euler(n, _ptr(qd), n, _ptr(out), stream))
    return out


def select_events(stream, etype):
    """The events of one type of an EventStream, in stream order (kf_events_select): returns
    device (t [K], payload [K, 9], src [K] int32 stream positions)."""
    n = len(stream)
    dev = stream.t.device
    t = torch.empty(max(n, 1), dtype=torch.float64, device=dev)
    pay = torch.empty(max(n, 1), 9, dtype=torch.float64, device=dev)
    src = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    k = ctypes.c_int64(0)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    with torch.cuda.device(dev):
        check(_lib.lib().kf_events_select(n, _ptr(stream.etype.contiguous()), _ptr(stream.t.contiguous()),
                                          _ptr(stream.payload.contiguous()), int(etype), _ptr(t), _ptr(pay),
                                          _ptr(src), ctypes.byref(k), st))
    return t[:k.value], pay[:k.value], src[:k.value]


def events_dt(t, prev0, rule, etype=None):
    """Per-event dt of a driver over a stream slice (kf_events_dt); returns (dt, etype_out) with
    skipped events marked KF_EVENT_NONE.  rule: _lib.KF_DT_FULL / KF_DT_MONOTONE / KF_DT_RAW.
    prev0 NaN (FULL / RAW): no previous time yet, the first event gets dt 0."""
    n = int(t.shape[0])
    tc = t.contiguous()
    ec = None if etype is None else etype.contiguous()
    dt = torch.empty(n, dtype=torch.float64, device=t.device)
    eo = torch.empty(n, dtype=torch.uint8, device=t.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)
    with torch.cuda.device(t.device):
        check(_lib.lib().kf_events_dt(n, _ptr(tc), _ptr(ec), float(prev0), int(rule), _ptr(dt), _ptr(eo), stream))
    return dt, eo
