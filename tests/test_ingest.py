"""Ingest path without a GPU: the oracle (oracle/ref_ingest.py) against the reference's own
outputs (tests/golden/ingest.npz, made by running the reference's ingest methods), the UTM
restatement against the `utm` package's published examples, and the native CSV reader
(kf_csv_shape / kf_csv_read, host-only) against Python's csv + float().
"""
import gzip
import math
import os

import numpy as np
import pytest

from kfmi import KFError, ingest
from oracle import ref_ingest


@pytest.fixture(scope='module')
def csvs(golden_dir, tmp_path_factory):
    d = tmp_path_factory.mktemp('ingest')
    out = []
    for name in ('gps_synth.csv.gz', 'imu_synth.csv.gz'):
        p = d / name[:-3]
        with gzip.open(os.path.join(golden_dir, name), 'rt') as fi:
            p.write_text(fi.read())
        out.append(str(p))
    return out


def test_utm_readme_example():
    # the utm package's README example, full precision
    assert ref_ingest.utm_from_latlon(51.2, 7.5) == (395201.3103811303, 5673135.241182375, 32, 'U')


@pytest.mark.parametrize('latlon,want', [
    ((50.77535, 6.08389), (294409, 5628898, 32, 'U')),       # Aachen
    ((40.71435, -74.00597), (583960, 4507523, 18, 'T')),     # New York
    ((-41.28646, 174.77624), (313784, 5427057, 60, 'G')),    # Wellington
    ((-33.92487, 18.42406), (261878, 6243186, 34, 'H')),     # Cape Town
    ((-32.89018, -68.84405), (514586, 6360877, 19, 'H')),    # Mendoza
    ((64.83778, -147.71639), (466013, 7190568, 6, 'W')),     # Fairbanks
    ((56.79680, -5.00601), (377486, 6296562, 30, 'V')),      # Ben Nevis
    ((84, -5.00601), (476594, 9328501, 30, 'X')),            # latitude 84
])
def test_utm_known_values(latlon, want):
    """The utm package's known-value table (rounded to metres)."""
    e, n, z, l = ref_ingest.utm_from_latlon(*latlon)
    assert abs(e - want[0]) < 1 and abs(n - want[1]) < 1 and (z, l) == want[2:]


def test_utm_zone_exceptions():
    assert ref_ingest.utm_zone_number(60.0, 5.0) == 32           # Norway
    assert ref_ingest.utm_zone_number(78.0, 15.0) == 33          # Svalbard
    assert ref_ingest.utm_zone_letter(-81.0) is None


def test_oracle_ingest_matches_reference(golden_dir, csvs):
    g = np.load(os.path.join(golden_dir, 'ingest.npz'))
    events, (bw, ba, fvi), utm = ref_ingest.ingest(*csvs)
    assert fvi == int(g['first_valid_index'])
    np.testing.assert_array_equal(bw, g['gyro_bias'])
    np.testing.assert_array_equal(ba, g['accel_bias'])
    np.testing.assert_array_equal([u['time'] for u in utm], g['utm_time'])
    np.testing.assert_array_equal([u['easting'] for u in utm], g['utm_easting'])
    np.testing.assert_array_equal([u['northing'] for u in utm], g['utm_northing'])
    np.testing.assert_array_equal([u['altitude'] for u in utm], g['utm_altitude'])
    np.testing.assert_array_equal([u['zone_number'] for u in utm], g['utm_zone_number'])
    np.testing.assert_array_equal([ord(u['zone_letter']) for u in utm], g['utm_zone_letter'])
    np.testing.assert_array_equal([e[1] == 'IMU' for e in events], g['ev_is_imu'])
    np.testing.assert_array_equal([e[2] for e in events], g['ev_time'])
    imu = ref_ingest.unbias_imu_data(ref_ingest.load_data_from_csv(csvs[1]), bw, ba)
    np.testing.assert_array_equal([[float(v) for v in e[1:10]] for e in imu], g['imu_values'])
    hw5 = ref_ingest.gps_to_modified_utm(ref_ingest.load_data_from_csv(csvs[0]), with_altitude=False)
    np.testing.assert_array_equal([u['time'] for u in hw5], g['hw5_utm_time'])
    np.testing.assert_array_equal([u['easting'] for u in hw5], g['hw5_utm_easting'])
    assert not bool(g['hw5_has_altitude']) and all('altitude' not in u for u in hw5)


def test_golden_exercises_edge_cases(golden_dir):
    """The fixture covers ties (GPS first), both gimbal-lock branches and altitude-only drops."""
    g = np.load(os.path.join(golden_dir, 'ingest.npz'))
    t, imu = g['ev_time'], g['ev_is_imu']
    ties = np.nonzero(np.diff(t) == 0)[0]
    assert len(ties) > 10 and all(not imu[i] and imu[i + 1] for i in ties)
    pitch = g['imu_values'][:, 1]
    assert (pitch == math.pi / 2).any() and (pitch == -math.pi / 2).any()
    assert len(g['hw5_utm_time']) > len(g['utm_time'])


def test_csv_reader_matches_python(csvs):
    for path, nc in zip(csvs, (4, 11)):
        cols = ingest.read_csv(path, nc)
        rows = ref_ingest.load_data_from_csv(path)
        assert cols.shape == (nc, len(rows))
        want = np.array([[float('nan') if 'nan' in f.lower() else float(f) for f in r[:nc]] for r in rows]).T
        np.testing.assert_array_equal(cols, want)
    assert ingest.csv_shape(csvs[1]) == (2500, 11)


def test_csv_reader_semantics(tmp_path):
    p = tmp_path / 'a.csv'
    p.write_text('t,a,b\n1.5, -2e3 ,NaN\r\n+7,inf,-nan\n0.1,1e-320,4\n\n\n')
    assert ingest.csv_shape(str(p)) == (3, 3)
    c = ingest.read_csv(str(p))
    assert c[0].tolist() == [1.5, 7.0, 0.1]
    assert c[1, 0] == -2000.0 and c[1, 1] == math.inf and c[1, 2] == float('1e-320')
    assert math.isnan(c[2, 0]) and math.isnan(c[2, 1]) and c[2, 2] == 4.0
    assert ingest.csv_shape(str(p), has_header=False) == (4, 3)
    with pytest.raises(KFError, match='row 0 column 0'):   # the header is not data
        ingest.read_csv(str(p), has_header=False)


@pytest.mark.parametrize('text,msg', [
    ('t,a\n1,2\n3,x\n', 'row 1 column 1'),
    ('t,a\n1,2\n3\n', 'has 1 fields'),
    ('t,a\n1,2\n\n3,4\n', 'not a number'),
    ('t,a\n1,\n', 'not a number'),
])
def test_csv_reader_errors(tmp_path, text, msg):
    p = tmp_path / 'bad.csv'
    p.write_text(text)
    with pytest.raises(KFError, match=msg):
        ingest.read_csv(str(p), 2)


def test_csv_reader_large_multithreaded(tmp_path):
    """Several MiB so the reader splits the file across threads; rows stay in order."""
    rng = np.random.default_rng(5)
    v = rng.normal(size=(120000, 5)) * 10.0 ** rng.integers(-5, 6, size=(120000, 5))
    p = tmp_path / 'big.csv'
    with open(p, 'w') as f:
        f.write('a,b,c,d,e\n')
        for r in v:
            f.write(','.join(repr(float(x)) for x in r) + '\n')
    c = ingest.read_csv(str(p))
    np.testing.assert_array_equal(c, v.T)


def test_real_gps_log_first_fix_kat():
    """On the reference's own gps_data.csv (only where the reference checkout exists; never
    copied into this repository): the first valid index and first fix that
    KF_SensorFusion.ipynb:1331 prints."""
    path = '/root/reference/gps_data.csv'
    if not os.path.exists(path):
        pytest.skip('reference checkout not present')
    cols = ingest.read_csv(path, 4)
    lat_ok = ~np.isnan(cols[1])
    assert int(np.argmax(lat_ok)) == 2735
    rows = ref_ingest.load_data_from_csv(path)
    u = ref_ingest.gps_to_modified_utm(rows)
    assert (u[0]['easting'], u[0]['northing'], u[0]['zone_number'], u[0]['zone_letter'], u[0]['altitude']) == \
        (0.0, 0.0, 19, 'T', -32.6)
    assert u[0]['time'] == 1697739552.3362827
    assert len(u) == 21871


def test_compat_model_matrices_are_the_reference_model():
    """kfmi.kf_workers keeps the reference's model definitions for class_args callers."""
    from kfmi import kf_workers as kfw
    from oracle import ref_kf
    sf = kfw.KF_SensorFusion('g.csv', 'i.csv')
    for dt in (0.0, 0.005, 0.1, 1.3):
        np.testing.assert_array_equal(sf.get_state_transition_matrix(dt), ref_kf.F_ref15(dt))
        np.testing.assert_array_equal(sf.get_process_noise_covariance_matrix(dt), ref_kf.Q_ref15(dt))
    np.testing.assert_array_equal(sf.get_gps_observation_matrix(), ref_kf.H_gps15())
    np.testing.assert_array_equal(sf.get_imu_observation_matrix(), ref_kf.H_imu15())
    np.testing.assert_array_equal(sf.get_gps_measurement_noise_covariance_matrix(), ref_kf.R_gps15())
    np.testing.assert_array_equal(sf.get_imu_measurement_noise_covariance_matrix(), ref_kf.R_imu15())
    t = kfw.CsvTable(np.array([[1.5, 2.0], [np.nan, 3.25]]))
    assert t[0] == ['1.5', 'nan'] and t[-1] == ['2.0', '3.25'] and len(t) == 2 and t[:1] == [t[0]]


def test_csv_reader_out_of_range_like_float(tmp_path):
    """Fields beyond the double range parse as float() parses them (inf, 0.0, subnormals), not
    as errors: from_chars reports them out of range, the reader then rounds them with strtod."""
    vals = ['1e400', '-1e400', '1e-400', '4.9406564584124654e-324', '2.2250738585072011e-308',
            '123456789012345678901234567890e-350', '1.7976931348623159e308', '0.5']
    p = tmp_path / 'r.csv'
    p.write_text('v\n' + '\n'.join(vals) + '\n')
    got = ingest.read_csv(str(p), 1)[0]
    want = np.array([float(v) for v in vals])
    assert (got.view(np.uint64) == want.view(np.uint64)).all(), (got, want)
