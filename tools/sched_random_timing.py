"""Timing of the scheduled drivers on a whole drive log.

    python tools/sched_random_timing.py [--freq 50] [--reps 3]

The bench's synthetic config-1 log (583k events from the first fix) through the drop-in
KF_SensorFusion façade, run_kalman_filter_scheduled (kf_workers.py:826-957) for the greedy and
the random arm on the device, and — for comparison, same seed, same outputs — the round-3 random
arm, whose windowing and np.random.choice draws were a per-event Python loop on the host
(kfmi/ref15.py before round 4) with only the selected events run on the device.  Prints one JSON
line.  Needs an MI355X.
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from kfmi import kf_workers as kfw, ref15  # noqa: E402


def host_loop_random(events, f):
    """The round-3 random arm: windows and draws in a Python loop over the event tuples, then
    one kf_run_events launch over the selected events."""
    x0, P, prev0, cands = ref15._scheduled_window_events(list(events), None, None, None, None)
    selected, queue, prev = [], [], prev0
    for ev in cands:
        if ev[2] - prev < 1 / f:
            queue.append(ev)
            continue
        if not queue:
            queue.append(ev)
        sel = queue[np.random.choice(len(queue))]
        queue = []
        selected.append((ref15.GPS if sel[1] == 'GPS' else ref15.IMU, sel[2] - prev,
                         ref15.event_payload(sel[1], sel[3]), sel[2]))
        prev = sel[2]
    tr, ld, _, _, _, _ = ref15._run_streams([[s[:3] for s in selected]], x0[None], ref15.to_blocks(P)[None])
    return [(prev0, *tr[0, :, 0])] + [(s[3], *tr[i + 1, :, 0]) for i, s in enumerate(selected)], ld[:len(selected) + 1, 0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--freq', type=float, default=50.0)
    ap.add_argument('--reps', type=int, default=3)
    args = ap.parse_args()
    root = tempfile.mkdtemp(prefix='kfmi_sched_')
    gp, ip = bench.synth_log(bench.CONFIGS['1'], root)
    sf = kfw.KF_SensorFusion(gp, ip)
    sf.load_data()
    sf.gps_to_modified_utm()
    bw, ba, _ = sf.compute_imu_biases(sf.gps_data, sf.imu_data)
    sf.unbias_imu_data(bw, ba)
    sf.combine_sensor_data()
    sf.set_processing_frequency(args.freq)
    n = len(sf.indexed_sensor_data)
    out = {'events': n, 'processing_frequency': args.freq, 'host': bench.host_cpu()}
    for method in ('greedy', 'random'):
        times = []
        for r in range(args.reps + 1):   # the first call loads code objects: not timed
            np.random.seed(5)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            st, ld, _ = sf.run_kalman_filter_scheduled(selection_method=method)
            torch.cuda.synchronize()
            if r:
                times.append(time.perf_counter() - t0)
        out[method] = {'seconds': min(times), 'selected': len(st) - 1,
                       'path': 'kf_run_scheduled' if method == 'greedy' else
                       'kf_sched_random_picks + kf_run_events (time-parallel)'}
        if method == 'random':
            rand = (st, ld)
    # the same picks through the one-launch random kernel (kf_run_scheduled_random: windows, draws
    # and the filter in one lane, the fused kernel for B = 1) instead of picks + the event engine
    x0, P, prev0, cands = ref15._scheduled_window_events(sf.indexed_sensor_data, None, None, None, None)
    t, et, pay, n_cand = ref15._stream_arrays(cands, events=sf.indexed_sensor_data)
    import kfmi
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    np.random.seed(5)  # the draws of the timed random runs above
    words = ref15.legacy_words(2 * n_cand + 64)[:, None]
    td, etd, payd = (torch.as_tensor(v, device=kf.device) for v in (t, et, pay))
    fused = []
    for r in range(args.reps + 1):
        kf.set_state(x0[:, None], ref15.to_blocks(P)[:, None])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out_f = kf.run_scheduled_random(td, etd, payd, np.array([prev0]), args.freq, words)
        torch.cuda.synchronize()
        if r:
            fused.append(time.perf_counter() - t0)
    kf.close()
    out['random_fused_kernel'] = {'seconds': min(fused), 'selected': int(out_f[3][0]),
                                  'same_times': bool(np.array_equal(out_f[2][:int(out_f[3][0]), 0].cpu().numpy(),
                                                                    np.array([s_[0] for s_ in rand[0][1:]])))}
    np.random.seed(5)
    t0 = time.perf_counter()
    hs, hl = host_loop_random(sf.indexed_sensor_data, args.freq)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    same = len(hs) == len(rand[0]) and all(a[0] == b[0] for a, b in zip(hs, rand[0]))
    err = float(np.max(np.abs(np.array(hs, float) - np.array(rand[0], float)) /
                       np.maximum(np.abs(np.array(hs, float)), 1.0))) if same else None
    out['random_round3_host_loop'] = {'seconds': el, 'selected': len(hs) - 1, 'same_picks': same,
                                      'max_rel_state_diff': err}
    out['random_speedup'] = el / out['random']['seconds']
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
