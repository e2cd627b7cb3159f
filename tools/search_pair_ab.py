"""In-process A/B of KF_OPT_SEARCH_PAIR on whole exhaustive searches of the bf rows' candidates
(diagnostic; DESIGN.md §3 "Pairs").  One handle per arm, arms interleaved round by round on one
set of level buffers each, so the per-process HBM placement is shared.

    python tools/search_pair_ab.py [--n 25,28,30,32] [--arms off,all,1048576,4194304] [--rounds 5]

An arm is a KF_OPT_SEARCH_PAIR value: off (1), all (2), auto (0), or a least stored-parent count
(>= 1024) for a paired level.  Prints one JSON line per n: median ms per arm, per-round times.
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', default='25,28,30,32')
    ap.add_argument('--arms', default='off,all,1048576,4194304,16777216')
    ap.add_argument('--rounds', type=int, default=5)
    args = ap.parse_args()
    import torch
    import bench
    import kfmi
    from kfmi import ref15
    for n in (int(x) for x in args.n.split(',')):
        ev, init, _, t0, t_end = bench.bf_events(n)
        arms = args.arms.split(',')
        kfs = {}
        for a in arms:
            v = int(a) if a.isdigit() else a
            kfs[a] = kfmi.BatchedKF('ref15', 1, 'f64', options={'search_pair': v})
            kfs[a].search_combos(ev, init, t0, t_end, -1e30, exhaustive=True)  # sizes the level buffers
        times = {a: [] for a in arms}
        for _ in range(args.rounds):
            for a in arms:
                torch.cuda.synchronize()
                t = time.perf_counter()
                kfs[a].search_combos(ev, init, t0, t_end, -1e30, exhaustive=True)  # returns synchronised
                times[a].append(round((time.perf_counter() - t) * 1e3, 4))
        plans = {a: [k for kind, k in ref15.search_plan(n, sym=True, pair=int(a) if a.isdigit() else a)[0]
                     if kind == 'pair'] for a in arms}
        print(json.dumps({'n': n, 'median_ms': {a: statistics.median(v) for a, v in times.items()},
                          'per_round_ms': times, 'paired_levels': plans}), flush=True)
        for kf in kfs.values():
            kf.close()
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
