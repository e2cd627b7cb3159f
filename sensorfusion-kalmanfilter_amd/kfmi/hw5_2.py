"""Drop-in for the reference module hw5_2.py: ``from kfmi.hw5_2 import KF_SensorFusion``.

The 8-state planar filter (KF_MODEL_REF8): ingest as hw5_2 does it (gps_to_utm keeps fixes
with a latitude and longitude and stores no altitude, hw5_2.py:29-54) and run_kalman_filter
(hw5_2.py:313-380) on the GPU.  The plotting helpers are out of scope.
"""
from __future__ import annotations

import numpy as np

from . import ingest, ref8
from .kf_workers import CsvTable, EventList, ImuRows, KF_SensorFusion as _KF15

__all__ = ['KF_SensorFusion']


class KF_SensorFusion:
    def __init__(self, gps_csv_file, imu_csv_file, dtype='f64', device=0):
        self.gps_csv_file = gps_csv_file
        self.imu_csv_file = imu_csv_file
        self.gps_data = []
        self.imu_data = []
        self.utm_data = []
        self.dtype = dtype
        self.device = device

    def load_data_from_csv(self, filename, has_header=True):
        return CsvTable(ingest.read_csv(filename, has_header=has_header))

    def load_data(self):
        self.gps_data = CsvTable(ingest.read_csv(self.gps_csv_file, 4))
        self.imu_data = CsvTable(ingest.read_csv(self.imu_csv_file, 11))

    def gps_to_utm(self):
        g = _KF15._cols(self.gps_data, 4)
        if not np.any(~np.isnan(g[1])):
            self.utm_data = []
            return
        self.utm_data = ingest.ingest_arrays(g, np.zeros((11, 0)), False, self.device).utm_data()

    compute_imu_biases = staticmethod(_KF15.compute_imu_biases)

    def unbias_imu_data(self, angular_velocity_bias, linear_acceleration_bias):
        self._stream = ingest.ingest_arrays(_KF15._cols(self.gps_data, 4), _KF15._cols(self.imu_data, 11), False,
                                            self.device, bias=(angular_velocity_bias, linear_acceleration_bias))
        self.unbias_imu_data = ImuRows(self._stream)

    def combine_sensor_data(self):
        self.events = self._stream
        self.indexed_sensor_data = EventList(self._stream)

    def quaternion_to_euler(self, x, y, z, w):
        r = ingest.quaternion_to_euler(np.array([[x], [y], [z], [w]], dtype=np.float64), self.device)
        return tuple(float(v) for v in r[:, 0].cpu().numpy())

    def run_kalman_filter(self):
        """hw5_2.py:313-380: [(x, y, theta), ...]."""
        return ref8.run_kalman_filter(self.indexed_sensor_data, self.dtype, self.device)

    def run_dead_reckoning_for_IMU(self):
        raise NotImplementedError('hw5_2.run_dead_reckoning_for_IMU is a plotting aid, out of scope')
