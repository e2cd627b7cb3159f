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


# The 8-state model (x, y, theta, vx, vy, theta_dot, ax, ay) as hw5_2.py:219-311 defines it, for
# callers that build their own step from the getters (the device kernels never materialise them).
def _F8(dt):
    F = np.eye(8)
    for p, v, a in ((0, 3, 6), (1, 4, 7)):   # x, y: position, velocity, acceleration chains
        F[p, v] = dt
        F[p, a] = 0.5 * dt ** 2
        F[v, a] = dt
    F[2, 5] = dt                              # theta from theta_dot
    return F


def _Q8(dt):
    return np.diag([5 * dt, 5 * dt, 0.05 * dt, 1 * dt, 1 * dt, 0.1 * dt, 2 * dt, 2 * dt])


_H_GPS8 = np.eye(8, dtype=np.int64)[:2]
_H_IMU8 = np.eye(8, dtype=np.int64)
_R_GPS8 = np.diag([3, 3])
_R_IMU8 = np.diag([50, 50, 0.05, 10, 10, 0.1, 100, 100])


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

    def compute_stationary_orientation(self, first_valid_index):
        """hw5_2.py:149-164 without its plot: mean roll, pitch, yaw of the unbiased IMU rows."""
        return _KF15.compute_stationary_orientation(self, first_valid_index)

    euler_to_rotation_matrix = _KF15.euler_to_rotation_matrix  # hw5_2.py:166-184

    # -- model (hw5_2.py:219-311) -----------------------------------------------------------
    def get_state_transition_matrix(self, dt):
        return _F8(dt)

    def get_process_noise_covariance_matrix(self, dt):
        return _Q8(dt)

    def predict_covariance(self, Pt, F, Qt):
        return np.dot(np.dot(F, Pt), F.T) + Qt

    def get_gps_observation_matrix(self):
        return _H_GPS8.copy()

    def get_imu_observation_matrix(self):
        return _H_IMU8.copy()

    def get_gps_measurement_noise_covariance_matrix(self):
        return _R_GPS8.copy()

    def get_imu_measurement_noise_covariance_matrix(self):
        return _R_IMU8.copy()

    def calculate_kalman_gain(self, P_next, H, R):
        return np.dot(np.dot(P_next, H.T), np.linalg.inv(np.dot(np.dot(H, P_next), H.T) + R))

    def run_kalman_filter(self):
        """hw5_2.py:313-380: [(x, y, theta), ...], with the constants of this object's getters
        (a subclass may replace them with diagonal ones) and ``self.P0``."""
        return ref8.run_kalman_filter(self.indexed_sensor_data, self.dtype, self.device, consts=self._consts())

    def _consts(self):
        from .ref15 import ModelConsts
        return ModelConsts.from_matrices('ref8', F=self.get_state_transition_matrix,
                                         Q=self.get_process_noise_covariance_matrix,
                                         H_gps=self.get_gps_observation_matrix(), H_imu=self.get_imu_observation_matrix(),
                                         R_gps=self.get_gps_measurement_noise_covariance_matrix(),
                                         R_imu=self.get_imu_measurement_noise_covariance_matrix(),
                                         P0=getattr(self, 'P0', None))

    def run_dead_reckoning_for_IMU(self):
        """hw5_2.py:382-436: [(x, y, theta), ...] per IMU event of indexed_sensor_data (fixes
        skipped, first dt 0, x0 = 0), the IMU events compacted and filtered on the GPU."""
        return ref8.run_dead_reckoning(self.indexed_sensor_data, self.dtype, self.device, consts=self._consts())
