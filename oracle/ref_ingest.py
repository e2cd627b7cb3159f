"""CPU oracle for the ingest path (CSV -> merged event stream) — TEST INFRASTRUCTURE ONLY.

The checker, never the product: only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import it.  The shipped ingest (``kfmi.ingest``: native CSV reader +
HIP conversion/merge kernels) never imports it.

What it restates (citations into the reference, IseanB/SensorFusion-KalmanFilter):

* ``load_data_from_csv`` (``kf_workers.py:290-298``): csv.reader rows as strings, header skipped.
* ``gps_to_modified_utm`` (``kf_workers.py:304-331``): a row whose latitude, longitude or
  altitude string contains 'nan' is dropped; UTM easting/northing relative to the first kept
  fix; ``hw5_2.gps_to_utm`` (``hw5_2.py:29-54``) tests latitude/longitude only and stores no
  altitude.
* ``compute_imu_biases`` (``kf_workers.py:333-347``): the first GPS row whose LATITUDE string has
  no 'nan' gives ``first_valid_index``, and the biases are the means of the first
  ``first_valid_index`` IMU rows (a GPS row index applied to the IMU list, as the reference does).
* ``unbias_imu_data`` (``kf_workers.py:349-373``) with ``quaternion_to_euler`` (``399-425``).
* ``combine_sensor_data`` (``kf_workers.py:375-385``): GPS entries then IMU entries, stable sort
  on time (so GPS first on ties), enumerated.

Third-party arithmetic: the UTM projection is ``utm.from_latlon`` of the PyPI ``utm`` package,
which the reference imports (``kf_workers.py:4``) without pinning a version
(``KF_SensorFusion.ipynb:56`` runs an unpinned ``pip install utm``) and which is absent here.
``utm_from_latlon`` below restates that package's published algorithm (Krueger-series
transverse Mercator, WGS84 with its truncated E = 0.00669438, K0 = 0.9996, the Norway/Svalbard
zone exceptions).  Pinning: the package's README example (51.2, 7.5) ->
(395201.3103811303, 5673135.241182375, 32, 'U') to full precision, its known-value table to
1 m, and the reference's own first fix (zone 19T, ``KF_SensorFusion.ipynb:1331``); see
tests/test_ingest.py.  Everything around the projection is pinned by
``tests/golden/ingest.npz``, produced by running the reference's own ingest methods with this
projection injected as ``utm.from_latlon`` (tests/golden/make_golden.py).
"""
from __future__ import annotations

import csv
import math

import numpy as np

# --------------------------------------------------------------------------------------
# utm.from_latlon (published algorithm of the `utm` package; see the module docstring)
# --------------------------------------------------------------------------------------
K0 = 0.9996
E = 0.00669438
E2 = E * E
E3 = E2 * E
E_P2 = E / (1 - E)
M1 = (1 - E / 4 - 3 * E2 / 64 - 5 * E3 / 256)
M2 = (3 * E / 8 + 3 * E2 / 32 + 45 * E3 / 1024)
M3 = (15 * E2 / 256 + 45 * E3 / 1024)
M4 = (35 * E3 / 3072)
R_EARTH = 6378137
ZONE_LETTERS = "CDEFGHJKLMNPQRSTUVWXX"


def utm_zone_number(lat, lon):
    if 56 <= lat < 64 and 3 <= lon < 12:
        return 32
    if 72 <= lat <= 84 and lon >= 0:
        if lon < 9:
            return 31
        if lon < 21:
            return 33
        if lon < 33:
            return 35
        if lon < 42:
            return 37
    return int((lon + 180) / 6) + 1


def utm_zone_letter(lat):
    return ZONE_LETTERS[int(lat + 80) >> 3] if -80 <= lat <= 84 else None


def utm_from_latlon(lat, lon):
    """(easting, northing, zone_number, zone_letter) for WGS84 latitude/longitude in degrees."""
    lat_rad = math.radians(lat)
    lat_sin = math.sin(lat_rad)
    lat_cos = math.cos(lat_rad)
    lat_tan = lat_sin / lat_cos
    lat_tan2 = lat_tan * lat_tan
    lat_tan4 = lat_tan2 * lat_tan2
    zone_number = utm_zone_number(lat, lon)
    zone_letter = utm_zone_letter(lat)
    lon_rad = math.radians(lon)
    central_lon_rad = math.radians((zone_number - 1) * 6 - 180 + 3)
    n = R_EARTH / math.sqrt(1 - E * lat_sin ** 2)
    c = E_P2 * lat_cos ** 2
    a = lat_cos * (lon_rad - central_lon_rad)
    m = R_EARTH * (M1 * lat_rad - M2 * math.sin(2 * lat_rad) + M3 * math.sin(4 * lat_rad)
                   - M4 * math.sin(6 * lat_rad))
    easting = K0 * n * (a + a ** 3 / 6 * (1 - lat_tan2 + c)
                        + a ** 5 / 120 * (5 - 18 * lat_tan2 + lat_tan4 + 72 * c - 58 * E_P2)) + 500000
    northing = K0 * (m + n * lat_tan * (a ** 2 / 2 + a ** 4 / 24 * (5 - lat_tan2 + 9 * c + 4 * c ** 2)
                                        + a ** 6 / 720 * (61 - 58 * lat_tan2 + lat_tan4 + 600 * c - 330 * E_P2)))
    if lat < 0:
        northing += 10000000
    return easting, northing, zone_number, zone_letter


# --------------------------------------------------------------------------------------
# The reference's ingest steps
# --------------------------------------------------------------------------------------

def load_data_from_csv(filename, has_header=True):
    """kf_workers.py:290-298."""
    with open(filename, newline='') as f:
        reader = csv.reader(f)
        if has_header:
            next(reader)
        return [row for row in reader]


def gps_to_modified_utm(gps_data, with_altitude=True, from_latlon=utm_from_latlon):
    """kf_workers.py:304-331 (with_altitude=True) / hw5_2.py:29-54 (False)."""
    out = []
    e0 = n0 = None
    for entry in gps_data:
        time, lat_str, lon_str, alt_str = entry
        bad = 'nan' in lat_str.lower() or 'nan' in lon_str.lower()
        if with_altitude:
            bad = bad or 'nan' in alt_str.lower()
        if bad:
            continue
        e, n, zn, zl = from_latlon(float(lat_str), float(lon_str))
        if e0 is None or n0 is None:
            e0, n0 = e, n
        d = {'time': float(time), 'easting': e - e0, 'northing': n - n0, 'zone_number': zn, 'zone_letter': zl}
        if with_altitude:
            d['altitude'] = float(alt_str)
        out.append(d)
    return out


def compute_imu_biases(gps_data, imu_data):
    """kf_workers.py:333-347: (angular_velocity_bias, linear_acceleration_bias,
    first_valid_index), or (None, None) without a valid GPS latitude."""
    fvi = next((i for i, entry in enumerate(gps_data) if 'nan' not in entry[1].lower()), None)
    if fvi is None:
        return None, None
    stat = imu_data[:fvi]
    w = [np.array([float(e[5]), float(e[6]), float(e[7])]) for e in stat]
    a = [np.array([float(e[8]), float(e[9]), float(e[10])]) for e in stat]
    return np.mean(w, axis=0), np.mean(a, axis=0), fvi


def quaternion_to_euler(x, y, z, w):
    """kf_workers.py:399-425."""
    sinr_cosp = 2 * (w * x + y * z)
    cosr_cosp = 1 - 2 * (x * x + y * y)
    roll = np.arctan2(sinr_cosp, cosr_cosp)
    sinp = 2 * (w * y - z * x)
    if abs(sinp) >= 1:
        pitch = np.pi / 2 * np.sign(sinp)
    else:
        pitch = np.arcsin(sinp)
    siny_cosp = 2 * (w * z + x * y)
    cosy_cosp = 1 - 2 * (y * y + z * z)
    yaw = np.arctan2(siny_cosp, cosy_cosp)
    return roll, pitch, yaw


def unbias_imu_data(imu_data, angular_velocity_bias, linear_acceleration_bias):
    """kf_workers.py:349-373: [t_str, roll, pitch, yaw, w - bw, a - ba, *extra]."""
    out = []
    for entry in imu_data:
        w = np.array([float(entry[5]), float(entry[6]), float(entry[7])]) - angular_velocity_bias
        a = np.array([float(entry[8]), float(entry[9]), float(entry[10])]) - linear_acceleration_bias
        x, y, z, q = float(entry[1]), float(entry[2]), float(entry[3]), float(entry[4])
        roll, pitch, yaw = quaternion_to_euler(x, y, z, q)
        out.append(entry[:1] + [roll, pitch, yaw] + w.tolist() + a.tolist() + entry[11:])
    return out


def combine_sensor_data(utm_data, unbias_imu):
    """kf_workers.py:375-385."""
    combined = [('GPS', float(g['time']), g) for g in utm_data]
    combined += [('IMU', float(e[0]), e) for e in unbias_imu]
    combined.sort(key=lambda x: x[1])
    return [(i, *d) for i, d in enumerate(combined)]


def ingest(gps_csv, imu_csv, with_altitude=True):
    """The reference's __main__ ingest sequence (kf_workers.py:2256-2274)."""
    gps = load_data_from_csv(gps_csv)
    imu = load_data_from_csv(imu_csv)
    utm_data = gps_to_modified_utm(gps, with_altitude)
    bw, ba, fvi = compute_imu_biases(gps, imu)
    unb = unbias_imu_data(imu, bw, ba)
    return combine_sensor_data(utm_data, unb), (bw, ba, fvi), utm_data
