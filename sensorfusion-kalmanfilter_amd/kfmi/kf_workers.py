"""Drop-in for the reference module kf_workers.py: ``from kfmi.kf_workers import KF_SensorFusion``.

Same class and function names, arguments, return layouts and printed messages for the fusion
path (ingest -> drivers -> scheduler -> brute force); every filter step, the ingest conversion
and merge, the scheduler scoring and the combination search run in the HIP kernels behind
libkfmi.so.  What differs, by design:

* the big lists (``imu_data`` rows, ``unbias_imu_data``, ``indexed_sensor_data``, the per-step
  covariances of ``run_kalman_filter_full``) are lazy sequences over device/host arrays — they
  index and slice like the reference's lists without materialising ~600k Python objects;
* covariances must stay block-diagonal over the axis chains, which every covariance the
  reference's own model produces is (kfmi.ref15);
* the plotting helpers, the experiment logger and the ``__main__`` loop are not part of the
  engine (out of scope).
"""
from __future__ import annotations

import math
from collections.abc import Sequence

import numpy as np
import torch

from . import _lib, ingest, ref15
from .ref15 import from_blocks

__all__ = ['KF_SensorFusion', 'Scheduler', 'evaluate_combo_chunk_worker', 'find_start_idx_for_time_offset']


# ------------------------------------------------------------------------------------------
# lazy list views
# ------------------------------------------------------------------------------------------

class CsvTable(Sequence):
    """The rows load_data_from_csv returns (kf_workers.py:290-298), backed by parsed columns:
    row i is a list of strings ('nan' where the field held a nan)."""

    def __init__(self, cols):
        self.cols = cols  # [ncols, rows] float64

    def __len__(self):
        return int(self.cols.shape[1])

    def _row(self, i):
        return ['nan' if math.isnan(v) else repr(float(v)) for v in self.cols[:, i]]

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._row(k) for k in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        return self._row(i)


class _StreamList(Sequence):
    def __init__(self, stream: ingest.EventStream):
        self.s = stream
        self.h = stream.host()

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self._item(k) for k in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        return self._item(i)


class EventList(_StreamList):
    """indexed_sensor_data (kf_workers.py:385) over an EventStream: (i, 'GPS'|'IMU', t, payload)."""

    def __len__(self):
        return len(self.s)

    def _item(self, i):
        h = self.h
        t = float(h['t'][i])
        p = h['payload'][i]
        if h['etype'][i] == _lib.KF_EVENT_GPS:
            d = {'time': t, 'easting': float(p[0]), 'northing': float(p[1]),
                 'zone_number': int(h['zone_number'][i]), 'zone_letter': chr(int(h['zone_letter'][i]))}
            if self.s.with_altitude:
                d['altitude'] = float(p[2])
            return (i, 'GPS', t, d)
        return (i, 'IMU', t, [repr(t), *(float(v) for v in p)])


class ImuRows(_StreamList):
    """unbias_imu_data (kf_workers.py:367) in IMU row order."""

    def __init__(self, stream):
        super().__init__(stream)
        k = np.nonzero(self.h['etype'] == _lib.KF_EVENT_IMU)[0]
        self.k = k[np.argsort(self.h['src'][k], kind='stable')]

    def __len__(self):
        return len(self.k)

    def _item(self, i):
        j = self.k[i]
        return [repr(float(self.h['t'][j])), *(float(v) for v in self.h['payload'][j])]


class CovList(Sequence):
    """Per-step 15x15 covariances from block-packed records [R, 27]."""

    def __init__(self, blocks):
        self.b = blocks

    def __len__(self):
        return int(self.b.shape[0])

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [from_blocks(self.b[k]) for k in range(*i.indices(len(self)))]
        return from_blocks(self.b[i])


# ------------------------------------------------------------------------------------------
# Scheduler (kf_workers.py:99-233)
# ------------------------------------------------------------------------------------------

def _sensor_of(R, H, consts=None):
    """(sensor, constants) for a sensor's (R, H): H must be the model's GPS or IMU observation
    matrix (the engine's update selects those states), R a diagonal noise of its size — the
    reference's or a caller's (kf_workers.py:112-147 takes any R, H; a coupled R or another H
    raises ValueError).  consts: the ModelConsts to extend (the other sensor's R)."""
    for name, (r, h) in _MODEL_RH.items():
        if np.shape(H) == h.shape and np.array_equal(np.asarray(H, np.float64), h):
            if np.shape(R) != r.shape:
                raise ValueError(f'Scheduler: R is {np.shape(R)}, the {name} sensor has {r.shape[0]} rows')
            base = consts or ref15.ModelConsts('ref15')
            kw = dict(q=base.q, r_imu=base.r_imu, r_gps=base.r_gps, p0=base.p0)
            c = ref15.ModelConsts.from_matrices('ref15', **{'R_gps' if name == 'GPS' else 'R_imu': R})
            kw['r_gps' if name == 'GPS' else 'r_imu'] = c.r_gps if name == 'GPS' else c.r_imu
            return name, ref15.ModelConsts('ref15', **kw)
    raise ValueError('Scheduler: H is not the reference model\'s GPS or IMU observation matrix')


class Scheduler:
    """kf_workers.py:99-233 on kf_score_candidates.  ``device`` is accepted for signature
    compatibility; scoring always runs on the engine's GPU."""

    def cov_matrix(_, S, Sigma_prev, R, H, device='cuda'):
        """Posterior covariance after an update with measurement rows S (1-based) of the sensor
        (R, H) (kf_workers.py:112-172): S = [1] and S = every row as the reference's own callers
        use them, any other subset through kf_score_rows (H_hat = H[S], R_hat = R[S, S])."""
        assert type(S) == list, "S should be a list"
        assert len(S) > 0, "S should not be empty"
        assert type(Sigma_prev) == np.ndarray, "Sigma_prev should be a np.ndarray array"
        assert type(R) == np.ndarray, "R should be a np.ndarray array"
        assert type(H) == np.ndarray, "H should be a np.ndarray array"
        sensor, consts = _sensor_of(R, H)
        rows = sorted(S)
        if not all(1 <= r <= R.shape[0] for r in rows):
            raise IndexError(f'cov_matrix: rows {rows} outside 1..{R.shape[0]}')
        if rows == list(range(1, R.shape[0] + 1)) or rows == [1]:
            _, post = _score(Sigma_prev[None], [sensor], rows != [1], posterior=True, consts=consts)
        else:
            _, post = _score_rows(Sigma_prev[None], [sensor], [sum(1 << (r - 1) for r in set(rows))], consts)
        return from_blocks(post[0, :, 0])

    def gain(self, measurement=None, S_sigma=None, measurement_cov=(tuple), observation_cov=(tuple), device='cuda'):
        """kf_workers.py:174-185."""
        assert type(measurement) != list, "only have one measurement"
        assert S_sigma is not None, "S_sigma should not be None"
        if measurement is None or len(measurement) == 0:
            return 0
        s = measurement[1]
        if s not in ('GPS', 'IMU'):
            return None
        _, consts = _sensor_of(measurement_cov[s], observation_cov[s])
        return float(_score(np.asarray(S_sigma)[None], [s], False, consts=consts)[0][0, 0])

    def random_schedule(self, num_measurements=None):
        """kf_workers.py:188-193 (the global NumPy RNG, as the reference)."""
        assert num_measurements is not None, "measurements should not be None"
        return np.random.choice(num_measurements)

    def greedy_schedule(self, measurements=None, S_sigma=None, measurement_cov=None, observation_cov=None,
                        device='cuda'):
        """kf_workers.py:195-213: index of the first measurement with the largest gain; both sensor
        types are scored in one kernel launch."""
        assert measurements is not None, "measurements should not be None"
        if len(measurements) == 0:
            raise ValueError('None is not in list')  # the reference's measurements.index(None) (:213)
        consts = None
        for s in ('GPS', 'IMU'):
            _, consts = _sensor_of(measurement_cov[s], observation_cov[s], consts)
        g = _score(np.asarray(S_sigma)[None], ['GPS', 'IMU'], False, consts=consts)[0][:, 0]
        best, best_i = -np.inf, None
        for i, m in enumerate(measurements):
            v = g[0] if m[1] == 'GPS' else g[1]
            if v > best:
                best, best_i = v, i
        if best_i is None:
            # an empty queue or no gain above -inf (NaN gains): the reference's
            # measurements.index(None) raises (kf_workers.py:213)
            raise ValueError('None is not in list')
        return best_i

    def randomized_greedy_schedule(self, total_num_sensors, device='cuda'):
        return None  # the reference's is a stub (kf_workers.py:215-216)


def _score(Ps, sensors, full, posterior=False, dtype='f64', device=0, consts=None):
    Ps = np.asarray(Ps, np.float64)
    B = Ps.shape[0]
    kf = ref15.BatchedKF('ref15', B, dtype, device=device, params=ref15._params(consts))
    kf.set_state(np.zeros((15, B)), np.ascontiguousarray(ref15.to_blocks(Ps).T))
    ty = [_lib.KF_EVENT_GPS if s == 'GPS' else _lib.KF_EVENT_IMU for s in sensors]
    r = kf.score_candidates(ty, full=full, posterior=posterior)
    if posterior:
        out = (r[0].double().cpu().numpy(), r[1].double().cpu().numpy())
    else:
        out = (r.double().cpu().numpy(), None)
    kf.close()
    return out


def _score_rows(Ps, sensors, masks, consts=None, dtype='f64', device=0):
    """(gain [n, B], posterior blocks [n, 27, B]) for candidates (sensor, row mask) on covariances
    Ps [B, 15, 15] (kf_score_rows)."""
    Ps = np.asarray(Ps, np.float64)
    B = Ps.shape[0]
    kf = ref15.BatchedKF('ref15', B, dtype, device=device, params=ref15._params(consts))
    kf.set_state(np.zeros((15, B)), np.ascontiguousarray(ref15.to_blocks(Ps).T))
    ty = [_lib.KF_EVENT_GPS if s == 'GPS' else _lib.KF_EVENT_IMU for s in sensors]
    g, post = kf.score_rows(ty, masks, posterior=True)
    out = (g.double().cpu().numpy(), post.double().cpu().numpy())
    kf.close()
    return out


# ------------------------------------------------------------------------------------------
# model matrices (kf_workers.py:493-621) — model definition for class_args callers
# ------------------------------------------------------------------------------------------

def _F(dt):
    F = np.eye(15)
    for i in range(3):
        F[i, 6 + i] = dt
        F[i, 12 + i] = 0.5 * dt ** 2
        F[3 + i, 9 + i] = dt
        F[6 + i, 12 + i] = dt
    return F


def _Q(dt):
    return np.diag([5 * dt] * 3 + [0.05 * dt] * 3 + [1 * dt] * 3 + [0.1 * dt] * 3 + [2 * dt] * 3)


_H_GPS = np.eye(15, dtype=np.int64)[:3]
_H_IMU = np.eye(15, dtype=np.int64)
_R_GPS = np.diag([3, 3, 3])
_R_IMU = np.diag([50] * 3 + [0.05] * 3 + [10] * 3 + [0.1] * 3 + [100] * 3)
_MODEL_RH = {'GPS': (_R_GPS, _H_GPS), 'IMU': (_R_IMU, _H_IMU)}


# ------------------------------------------------------------------------------------------
# KF_SensorFusion (kf_workers.py:277-1428)
# ------------------------------------------------------------------------------------------

_GETTERS = ('get_state_transition_matrix', 'get_process_noise_covariance_matrix', 'predict_covariance',
            'get_gps_observation_matrix', 'get_gps_measurement_noise_covariance_matrix', 'get_imu_observation_matrix',
            'get_imu_measurement_noise_covariance_matrix', 'calculate_kalman_gain')
_REFERENCE_CONSTS = None  # KF_SensorFusion._consts of an object with none of _GETTERS replaced


class KF_SensorFusion:
    def __init__(self, gps_csv_file, imu_csv_file, dtype='f64', device=0):
        self.gps_csv_file = gps_csv_file
        self.imu_csv_file = imu_csv_file
        self.gps_data = []
        self.imu_data = []
        self.utm_data = []
        self.scheduler = Scheduler()
        self.processing_frequency = None
        self.dtype = dtype
        self.device = device
        self.events = None  # the EventStream behind indexed_sensor_data, once combined
        # the drivers' cold-start covariance (the reference's literal, kf_workers.py:651); a
        # diagonal replacement (e.g. the notebook's diag(1000, 100, ..., 1000),
        # KF_SensorFusion.ipynb:814) runs on the engine too
        self.P0 = ref15.P0.copy()

    def set_processing_frequency(self, frequency):
        self.processing_frequency = frequency

    # -- ingest (kf_workers.py:290-385) ------------------------------------------------------
    def load_data_from_csv(self, filename, has_header=True):
        """Rows of a CSV log (native parser; rows are views over the parsed columns)."""
        return CsvTable(ingest.read_csv(filename, has_header=has_header))

    def load_data(self):
        self.gps_data = CsvTable(ingest.read_csv(self.gps_csv_file, 4))
        self.imu_data = CsvTable(ingest.read_csv(self.imu_csv_file, 11))

    @staticmethod
    def _cols(data, n):
        if isinstance(data, CsvTable):
            return data.cols[:n]
        rows = list(data)
        return np.array([[math.nan if 'nan' in str(f).lower() else float(f) for f in r[:n]] for r in rows],
                        dtype=np.float64).reshape(-1, n).T

    def gps_to_modified_utm(self):
        """Fixes with a latitude, longitude and altitude, projected to UTM relative to the first
        (kf_workers.py:304-331), on the GPU."""
        g = self._cols(self.gps_data, 4)
        if not np.any(~np.isnan(g[1])):  # no fix at all: the reference's loop keeps nothing
            self.utm_data = []
            return
        self.utm_data = ingest.ingest_arrays(g, np.zeros((11, 0)), True, self.device).utm_data()

    @staticmethod
    def compute_imu_biases(gps_data, imu_data):
        """kf_workers.py:333-347 (the bias means are computed on the GPU)."""
        g = KF_SensorFusion._cols(gps_data, 4)
        if not np.any(~np.isnan(g[1])):
            print("Warning: No valid GPS data found. Cannot compute IMU biases.")
            return None, None
        s = ingest.ingest_arrays(g, KF_SensorFusion._cols(imu_data, 11), True)
        print(f"First valid GPS entry index: {s.first_valid_index}")
        print(f"Computed Angular Velocity Bias: {s.gyro_bias}")
        print(f"Computed Linear Acceleration Bias: {s.accel_bias}")
        return s.gyro_bias, s.accel_bias, s.first_valid_index

    def unbias_imu_data(self, angular_velocity_bias, linear_acceleration_bias):
        """kf_workers.py:349-373: Euler angles and unbiased rates/accelerations on the GPU; like
        the reference, the result replaces this method on the instance."""
        self._stream = ingest.ingest_arrays(self._cols(self.gps_data, 4), self._cols(self.imu_data, 11), True,
                                            self.device, bias=(angular_velocity_bias, linear_acceleration_bias))
        self.unbias_imu_data = ImuRows(self._stream)

    def combine_sensor_data(self):
        """kf_workers.py:375-385: the merged, time-sorted stream (already built on the GPU)."""
        self.events = self._stream
        self.indexed_sensor_data = EventList(self._stream)

    def quaternion_to_euler(self, x, y, z, w):
        r = ingest.quaternion_to_euler(np.array([[x], [y], [z], [w]], dtype=np.float64), self.device)
        return tuple(float(v) for v in r[:, 0].cpu().numpy())

    def compute_stationary_orientation(self, first_valid_index):
        """kf_workers.py:427-439: mean roll, pitch, yaw of the unbiased IMU rows before
        first_valid_index (the reference slices the IMU rows with that GPS index; kept)."""
        rows = self.unbias_imu_data
        pay = rows.h['payload'][rows.k[:first_valid_index]]
        return tuple(np.mean([float(v) for v in pay[:, c]]) for c in range(3))

    def euler_to_rotation_matrix(self, roll, pitch, yaw):
        """kf_workers.py:441-458: R = Rz(yaw) Ry(pitch) Rx(roll)."""
        cr, sr, cp, sp, cy, sy = np.cos(roll), np.sin(roll), np.cos(pitch), np.sin(pitch), np.cos(yaw), np.sin(yaw)
        rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
        ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
        rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
        return rz @ ry @ rx

    def get_utm_data(self):
        return self.utm_data

    # -- model (kf_workers.py:493-621): definitions for class_args callers ---------------------
    def get_state_transition_matrix(self, dt):
        return _F(dt)

    def get_process_noise_covariance_matrix(self, dt):
        return _Q(dt)

    def predict_covariance(self, Pt, F, Qt):
        return np.dot(np.dot(F, Pt), F.T) + Qt

    def get_gps_observation_matrix(self):
        return _H_GPS.copy()

    def get_imu_observation_matrix(self):
        return _H_IMU.copy()

    def get_gps_measurement_noise_covariance_matrix(self):
        return _R_GPS.copy()

    def get_imu_measurement_noise_covariance_matrix(self):
        return _R_IMU.copy()

    def calculate_kalman_gain(self, P_next, H, R):
        return np.dot(np.dot(P_next, H.T), np.linalg.inv(np.dot(np.dot(H, P_next), H.T) + R))

    # -- drivers ---------------------------------------------------------------------------
    def _consts(self):
        """The model constants the drivers run with, read from this object's getters (which a
        subclass or a class_args caller may replace, kf_workers.py:1242-1251) and P0.  With none
        of them replaced (the class's and the instance's getters are this class's own and P0 is
        the reference's) the reference constants, read once (the getters' probes cost ~0.35 ms a
        driver call)."""
        global _REFERENCE_CONSTS
        own = (not any(g in vars(self) for g in _GETTERS)
               and all(getattr(type(self), g) is getattr(KF_SensorFusion, g) for g in _GETTERS)
               and np.array_equal(np.asarray(self.P0), ref15.P0))
        if own and _REFERENCE_CONSTS is not None:
            return _REFERENCE_CONSTS
        c = _consts_of({'get_state_transition_matrix': self.get_state_transition_matrix,
                           'get_process_noise_covariance_matrix': self.get_process_noise_covariance_matrix,
                           'predict_covariance': self.predict_covariance,
                           'get_gps_observation_matrix': self.get_gps_observation_matrix,
                           'get_gps_measurement_noise_covariance_matrix':
                               self.get_gps_measurement_noise_covariance_matrix,
                           'get_imu_observation_matrix': self.get_imu_observation_matrix,
                           'get_imu_measurement_noise_covariance_matrix':
                               self.get_imu_measurement_noise_covariance_matrix,
                           'calculate_kalman_gain': self.calculate_kalman_gain}, self.P0)
        if own:
            _REFERENCE_CONSTS = c
        return c

    def _ev(self):
        return self.events if self.events is not None else self.indexed_sensor_data

    def run_kalman_filter_full(self, start_idx=None, end_idx=None, initial_pt=None, initial_state=None,
                               print_output=False):
        """kf_workers.py:623-728; also keeps _ground_truth / _ground_truth_cov (:723-724)."""
        ev = self._ev()
        if isinstance(ev, ingest.EventStream):
            r = ref15.run_full_stream(ev, start_idx, end_idx, initial_pt, initial_state, self.dtype, cov=True,
                                      consts=self._consts())
            if r is None:
                return [], [], []
            t, traj, ld, P, prev, covb = r
            states = [(float(t[i]), *traj[i]) for i in range(len(t))]
            logdets = [float(v) for v in ld]
            self._ground_truth_cov = CovList(covb)
            if print_output:
                print(f"Full Kalman Filter (GPU): processed {len(t) - 1} measurements")
        else:
            out = ref15.run_kalman_filter_full(ev, start_idx, end_idx, initial_pt, initial_state, print_output,
                                               self.dtype, self.device, consts=self._consts())
            if len(out) == 3:
                return out
            states, logdets, P, prev = out
            self._ground_truth_cov = None
        self._ground_truth = states
        return states, logdets, P, prev

    def get_GT(self):
        if hasattr(self, '_ground_truth'):
            return self._ground_truth
        print("Ground truth not computed yet. Please run run_kalman_filter_full() first.")
        return None

    def run_kalman_filter(self, start_idx, end_idx):
        return ref15.run_kalman_filter(self.indexed_sensor_data, start_idx, end_idx, self.dtype, self.device,
                                       consts=self._consts())

    def run_kalman_filter_scheduled(self, start_idx=None, end_idx=None, initial_pt=None, initial_state=None,
                                    selection_method=None, print_output=False):
        return ref15.run_kalman_filter_scheduled(self.indexed_sensor_data, start_idx, end_idx, initial_pt,
                                                 initial_state, selection_method, self.processing_frequency,
                                                 print_output, self.dtype, self.device, consts=self._consts())

    def run_adaptive_threshold_kalman_filter(self, start_idx=None, end_idx=None, R_threshold=None, initial_pt=None,
                                             initial_state=None, print_output=False):
        return ref15.run_adaptive_threshold_kalman_filter(self.indexed_sensor_data, start_idx, end_idx, R_threshold,
                                                          initial_pt, initial_state, print_output, self.dtype,
                                                          self.device, consts=self._consts())

    def run_no_update_kalman_filter(self, start_idx=None, end_idx=None, R_threshold=None, initial_pt=None,
                                    initial_state=None, print_output=False):
        return ref15.run_no_update_kalman_filter(self.indexed_sensor_data, start_idx, end_idx, R_threshold,
                                                 initial_pt, initial_state, print_output, self.dtype, self.device,
                                                 consts=self._consts())

    def run_brute_force_kalman_filter_no_sampling_min_usage(self, start_idx=0, end_idx=None, R_threshold=None,
                                                            initial_pt=None, initial_state=None,
                                                            max_combos_in_memory=10000):
        return ref15.run_brute_force_kalman_filter_no_sampling_min_usage(
            self.indexed_sensor_data, start_idx, end_idx, R_threshold, initial_pt, initial_state,
            max_combos_in_memory=max_combos_in_memory, dtype=self.dtype, device=self.device, consts=self._consts())

    def run_dead_reckoning_for_IMU(self):
        return []  # the reference's body is commented out and returns an empty list (kf_workers.py:1394-1425)

    def calculate_accuracy_metrics(self, candidate_trajectory):
        """kf_workers.py:1162-1216: candidate positions against the full filter's trajectory,
        linearly interpolated (and extrapolated) at the candidate's time stamps."""
        from scipy.interpolate import interp1d
        if not candidate_trajectory:
            print("Candidate trajectory is empty. Cannot calculate accuracy.")
            return None
        if not (hasattr(self, "_ground_truth") and self._ground_truth):
            print("Ground truth trajectory is not available. Run run_kalman_filter_full() first.")
            return None
        c0, c1 = candidate_trajectory[0][0], candidate_trajectory[-1][0]
        gt = self._ground_truth
        sec = [s for s in gt if c0 <= s[0] <= c1]
        src = gt if len(sec) < 2 else sec
        gt_t = np.array([s[0] for s in src])
        gt_p = np.array([s[1:4] for s in src])
        ct = np.array([s[0] for s in candidate_trajectory])
        cp = np.array([s[1:4] for s in candidate_trajectory])
        gi = np.stack([interp1d(gt_t, gt_p[:, k], kind='linear', fill_value="extrapolate")(ct) for k in range(3)],
                      axis=1)
        err = cp - gi
        eu = np.linalg.norm(err, axis=1)
        return {'total_position_rmse': np.sqrt(np.mean(eu ** 2)), 'position_errors': err, 'euclidean_errors': eu,
                'candidate_times': ct, 'candidate_positions': cp, 'ground_truth_interp': gi,
                'gt_start_time': c0, 'gt_end_time': c1}


# ------------------------------------------------------------------------------------------
# module-level helpers
# ------------------------------------------------------------------------------------------

def _consts_of(class_args, P0=None):
    """ModelConsts from a class_args dict of the model's callables (kf_workers.py:1242-1251):
    the reference's F and H with any diagonal Q(dt) = diag(q dt), R_gps, R_imu (and P0).
    predict_covariance / calculate_kalman_gain must compute the reference's formulas (checked on
    a probe).  Anything else raises ValueError — the engine's kernels run that model."""
    get = class_args.get
    for name, fn, want in (('predict_covariance', get('predict_covariance'), None),
                           ('calculate_kalman_gain', get('calculate_kalman_gain'), None)):
        if fn is None:
            continue
        rng = np.random.default_rng(7)
        A = rng.normal(size=(15, 15))
        P = A @ A.T + 15 * np.eye(15)
        if name == 'predict_covariance':
            Fm, Qm = _F(0.37), _Q(0.37)
            ok = np.allclose(fn(P, Fm, Qm), np.dot(np.dot(Fm, P), Fm.T) + Qm, rtol=1e-12, atol=1e-9)
        else:
            ok = np.allclose(fn(P, _H_IMU, _R_IMU), np.dot(np.dot(P, _H_IMU.T),
                                                            np.linalg.inv(np.dot(np.dot(_H_IMU, P), _H_IMU.T) + _R_IMU)),
                             rtol=1e-9, atol=1e-12)
        if not ok:
            raise ValueError(f'class_args[{name!r}] is not the reference formula (kf_workers.py:546-549, 616-621)')
    call = lambda k: get(k)() if get(k) is not None else None
    return ref15.ModelConsts.from_matrices(
        'ref15', F=get('get_state_transition_matrix'), Q=get('get_process_noise_covariance_matrix'),
        H_gps=call('get_gps_observation_matrix'), H_imu=call('get_imu_observation_matrix'),
        R_gps=call('get_gps_measurement_noise_covariance_matrix'),
        R_imu=call('get_imu_measurement_noise_covariance_matrix'), P0=P0)


def evaluate_combo_chunk_worker(chunk, xt, Pt, class_args, prev_time, target_end_time):
    """kf_workers.py:22-97 for a whole chunk in one kernel launch, with the model constants
    class_args gives (diagonal Q, R: _consts_of; any other model raises ValueError)."""
    return ref15.evaluate_combo_chunk(chunk, xt, Pt, prev_time, target_end_time, consts=_consts_of(class_args))


def find_start_idx_for_time_offset(sensor_fusion, target_seconds):
    """kf_workers.py:1986-2003 (its fixed first time stamp included)."""
    if not hasattr(sensor_fusion, 'indexed_sensor_data') or not sensor_fusion.indexed_sensor_data:
        print("Sensor data not available. Run combine_sensor_data() first.")
        return None
    first_timestamp = 1697739552.3362827
    target = first_timestamp + target_seconds
    ev = getattr(sensor_fusion, 'events', None)
    if isinstance(ev, ingest.EventStream):
        hits = torch.nonzero(ev.t >= target)  # first index in list order, as the reference's scan
        i = int(hits[0, 0]) if hits.numel() else None
    else:
        i = next((k for k, e in enumerate(sensor_fusion.indexed_sensor_data) if e[2] >= target), None)
    if i is None:
        print(f"Target time {target_seconds}s not found in data")
        return None
    t = float(sensor_fusion.indexed_sensor_data[i][2])
    print(f"Found index {i} at time {t:.3f}s (offset: {t - first_timestamp:.3f}s)")
    return i
