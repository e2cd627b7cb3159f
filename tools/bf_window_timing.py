"""The reference's visualizing run end to end (kf_workers_visualizing.py:2286-2340) on the
synthetic log (tests/golden/*_synth.csv.gz): the adaptive filter up to each window's start, then
the brute-force search over the next 40 events from its state, through the façade (kfmi.kf_workers),
timed per window beside the oracle's NumPy restatement of the reference's search where that finishes
within its budget (diagnostic).

    python tools/bf_window_timing.py [--r -10] [--starts 600,900,1200,1500] [--numpy-budget 60]
"""
import argparse
import gzip
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--r', type=float, default=-10.0, help="R_threshold (the reference's r_value = -10)")
    ap.add_argument('--starts', default='600,900,1200,1500')
    ap.add_argument('--offset', type=int, default=40, help="start_offset (the reference's 40)")
    ap.add_argument('--numpy-budget', type=float, default=60.0, help='skip the NumPy search past this many seconds')
    args = ap.parse_args()
    import multiprocessing as mp

    from kfmi import kf_workers as kfw
    from oracle import ref_ingest, ref_kf
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
    events, _, _ = ref_ingest.ingest(*paths)
    for s in (int(x) for x in args.starts.split(',')):
        st, _, pt, _, _ = sf.run_adaptive_threshold_kalman_filter(end_idx=s, R_threshold=args.r)
        sf.run_brute_force_kalman_filter_no_sampling_min_usage(start_idx=s, end_idx=s + args.offset, initial_pt=pt,
                                                               initial_state=st[-1], R_threshold=args.r)  # warm
        t = time.perf_counter()
        got = sf.run_brute_force_kalman_filter_no_sampling_min_usage(start_idx=s, end_idx=s + args.offset,
                                                                     initial_pt=pt, initial_state=st[-1],
                                                                     R_threshold=args.r)
        gpu_s = time.perf_counter() - t
        sel = [e[0] for e in got['selected_sensors']] if got else None
        rec = {'start_idx': s, 'window': args.offset, 'R_threshold': args.r, 'gpu_s': round(gpu_s, 4),
               'winner_size': len(sel) if sel else 0, 'winner': sel}
        # the oracle's NumPy search of the same window, in a child process with a time limit
        rst, _, rpt, _, _ = ref_kf.run_adaptive_threshold(events, 0, s, R_threshold=args.r)
        q = mp.get_context('spawn').Queue()
        p = mp.get_context('spawn').Process(target=_numpy_search, args=(q, events, s, s + args.offset, args.r, rpt,
                                                                          tuple(rst[-1])))
        t = time.perf_counter()
        p.start()
        p.join(args.numpy_budget)
        if p.is_alive():
            p.kill()
            p.join()
            rec['numpy_s'] = f'> {args.numpy_budget}'
        else:
            ref_sel = q.get(timeout=10)
            rec['numpy_s'] = round(time.perf_counter() - t, 3)
            rec['numpy_winner_equal'] = ref_sel == sel
        print(json.dumps(rec), flush=True)


def _numpy_search(q, events, s, e, r, P, state):
    from oracle import ref_kf
    ref = ref_kf.run_brute_force(events, s, e, r, P, state)
    q.put([x[0] for x in ref['selected_sensors']] if ref else None)


if __name__ == '__main__':
    main()
