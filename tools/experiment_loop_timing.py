"""The reference's experiment loop (kf_workers.py:2276-2400, its __main__ without the logger) on
the config-1 synthetic drive log, through the kfmi façade and through the oracle's NumPy
restatement, for a sample of its 284 iterations (diagnostic): per iteration the adaptive filter
from the log's start to the iteration's start, the 25-event window's full and adaptive filters,
its brute-force search and its no-update filter, with r_value = lb * choice(0.2 .. 0.8) as the
reference draws it (seeded here).  The NumPy brute force runs in a child process under
--numpy-budget seconds.  Prints one JSON line per iteration and a summary extrapolated to the
loop's 284 iterations.

    python tools/experiment_loop_timing.py [--every 35] [--numpy-budget 60]
"""
import argparse
import json
import multiprocessing as mp
import os
import random
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]


def _numpy_bf(q, events, s, e, r, P, state):
    from oracle import ref_kf
    t = time.perf_counter()
    ref = ref_kf.run_brute_force(events, s, e, r, P, state)
    q.put(([x[0] for x in ref['selected_sensors']] if ref else None, time.perf_counter() - t))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--every', type=int, default=35, help='run iterations 16, 16 + every, ... < 300')
    ap.add_argument('--numpy-budget', type=float, default=60.0)
    args = ap.parse_args()
    import torch
    import bench
    from kfmi import kf_workers as kfw
    from oracle import ref_ingest, ref_kf
    d = tempfile.mkdtemp()
    gp, ip = bench.synth_log(bench.CONFIGS['1'], d)
    sf = kfw.KF_SensorFusion(gp, ip)
    sf.load_data()
    sf.gps_to_modified_utm()
    bw, ba, _ = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    sf.unbias_imu_data(bw, ba)
    sf.combine_sensor_data()
    events, _, _ = ref_ingest.ingest(gp, ip)

    def clock(fn):
        torch.cuda.synchronize()
        t = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        return out, time.perf_counter() - t
    # the loop's bound (kf_workers.py:2285-2289)
    (_, ld_full, _, _), g_pre = clock(lambda: sf.run_kalman_filter_full(start_idx=0, end_idx=100000))
    lb = min(ld_full)
    t = time.perf_counter()
    _, rld_full, _, _ = ref_kf.run_kalman_filter_full(events, 0, 100000)
    c_pre = time.perf_counter() - t
    rng = random.Random(2025)
    rows = []
    for i in range(16, 300):
        frac = rng.choice([0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8])  # the reference draws one per iteration
        if (i - 16) % args.every:
            continue
        s = kfw.find_start_idx_for_time_offset(sf, int(i * (2800 - 25) / 300))
        e = s + 25
        r = lb * frac
        rec = {'iteration': i, 'start_idx': s, 'r_value': r}
        g, c = {}, {}
        (st, _, pt, _, _), g['adaptive_to_start'] = clock(lambda: sf.run_adaptive_threshold_kalman_filter(
            end_idx=s, R_threshold=r))
        (_, fld, _, _), g['full_window'] = clock(lambda: sf.run_kalman_filter_full(
            start_idx=s, end_idx=e, initial_pt=pt, initial_state=st[-1]))
        r2 = (r / lb) * min(fld)
        _, g['adaptive_window'] = clock(lambda: sf.run_adaptive_threshold_kalman_filter(
            start_idx=s, end_idx=e, initial_pt=pt, initial_state=st[-1], R_threshold=r2))
        bf, g['brute_force'] = clock(lambda: sf.run_brute_force_kalman_filter_no_sampling_min_usage(
            start_idx=s, end_idx=e, initial_pt=pt, initial_state=st[-1], R_threshold=r2))
        _, g['no_update'] = clock(lambda: sf.run_no_update_kalman_filter(
            start_idx=s, end_idx=e, initial_pt=pt, initial_state=st[-1], R_threshold=r2))
        t = time.perf_counter()
        rst, _, rpt, _, _ = ref_kf.run_adaptive_threshold(events, 0, s, R_threshold=r)
        c['adaptive_to_start'] = time.perf_counter() - t
        t = time.perf_counter()
        _, rfld, _, _ = ref_kf.run_kalman_filter_full(events, s, e, initial_pt=rpt, initial_state=tuple(rst[-1]))
        c['full_window'] = time.perf_counter() - t
        rr2 = (r / lb) * min(rfld)
        t = time.perf_counter()
        ref_kf.run_adaptive_threshold(events, s, e, R_threshold=rr2, initial_pt=rpt, initial_state=tuple(rst[-1]))
        c['adaptive_window'] = time.perf_counter() - t
        t = time.perf_counter()
        ref_kf.run_no_update(events, s, e, initial_pt=rpt, initial_state=tuple(rst[-1]))
        c['no_update'] = time.perf_counter() - t
        q = mp.get_context('spawn').Queue()
        p = mp.get_context('spawn').Process(target=_numpy_bf, args=(q, events, s, e, rr2, rpt, tuple(rst[-1])))
        p.start()
        p.join(args.numpy_budget)
        win = [x[0] for x in bf['selected_sensors']] if bf else None
        if p.is_alive():
            p.kill()
            p.join()
            c['brute_force'] = None
            rec['brute_force_winner_equal'] = f'numpy search past {args.numpy_budget} s'
        else:
            ref_win, c['brute_force'] = q.get(timeout=10)
            rec['brute_force_winner_equal'] = ref_win == win
        rec['winner_size'] = len(win) if win else 0
        rec['gpu_s'] = {k: round(v, 5) for k, v in g.items()}
        rec['numpy_s'] = {k: (round(v, 4) if v is not None else f'> {args.numpy_budget}') for k, v in c.items()}
        rows.append(rec)
        print(json.dumps(rec), flush=True)
    n = len(rows)
    g_it = sum(sum(r['gpu_s'].values()) for r in rows) / n
    c_fin = [r for r in rows if not isinstance(r['numpy_s']['brute_force'], str)]
    c_it_lo = sum(sum(v if not isinstance(v, str) else args.numpy_budget for v in r['numpy_s'].values())
                  for r in rows) / n
    print(json.dumps({'iterations_sampled': n, 'loop_iterations': 284, 'bound_full_filter_s': {'gpu': round(g_pre, 4),
                      'numpy': round(c_pre, 3)},
                      'gpu_s_per_iteration': round(g_it, 4), 'gpu_s_loop_extrapolated': round(g_pre + 284 * g_it, 2),
                      'numpy_s_per_iteration_at_least': round(c_it_lo, 3),
                      'numpy_s_loop_extrapolated_at_least': round(c_pre + 284 * c_it_lo, 1),
                      'numpy_brute_force_finished': f'{len(c_fin)} of {n}',
                      'winners_equal_where_finished': all(r['brute_force_winner_equal'] is True for r in c_fin)}),
          flush=True)


if __name__ == '__main__':
    main()
