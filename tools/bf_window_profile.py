"""Where one brute-force window call's time goes (diagnostic): the façade's
run_brute_force_kalman_filter_no_sampling_min_usage on the synthetic log's 40-event windows
(as tools/bf_window_timing.py), repeated, under cProfile; prints the top functions by
cumulative time.

    python tools/bf_window_profile.py [--start 900] [--reps 20]
"""
import argparse
import cProfile
import gzip
import os
import pstats
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--start', type=int, default=900)
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--r', type=float, default=-10.0)
    args = ap.parse_args()
    from kfmi import kf_workers as kfw
    d = tempfile.mkdtemp()
    paths = []
    for name in ('gps_synth.csv.gz', 'imu_synth.csv.gz'):
        p = os.path.join(d, name[:-3])
        with gzip.open(os.path.join(ROOT, 'tests', 'golden', name), 'rt') as fi, open(p, 'w') as fo:
            fo.write(fi.read())
        paths.append(p)
    sf = kfw.KF_SensorFusion(*paths)
    sf.load_data()
    sf.gps_to_modified_utm()
    bw, ba, _ = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    sf.unbias_imu_data(bw, ba)
    sf.combine_sensor_data()
    s = args.start
    st, _, pt, _, _ = sf.run_adaptive_threshold_kalman_filter(end_idx=s, R_threshold=args.r)

    def call():
        return sf.run_brute_force_kalman_filter_no_sampling_min_usage(start_idx=s, end_idx=s + 40, initial_pt=pt,
                                                                      initial_state=st[-1], R_threshold=args.r)
    call()
    t = time.perf_counter()
    for _ in range(args.reps):
        call()
    print(f'{(time.perf_counter() - t) / args.reps * 1e3:.3f} ms per window call', flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(args.reps):
        call()
    pr.disable()
    pstats.Stats(pr).sort_stats('cumulative').print_stats(30)


if __name__ == '__main__':
    main()
