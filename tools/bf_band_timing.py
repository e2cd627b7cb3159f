"""Searches past one call's sizes (diagnostic, DESIGN.md §3 "Prefix bands"): for windows of n
candidates (the bf rows' candidate events, target 5 s past the last) at a threshold just below
every score of sizes 1 .. k_search, the time of the driver's steps — the one call, then
ref15.search_past (bands of prefix classes, then the fixed-pattern classes) — against the
fixed-pattern classes alone (search_combos_classed with search_class_width's w, as before the
bands), where those finish within --budget seconds.

    python tools/bf_band_timing.py [--n 40,48,64] [--budget 60]
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--n', default='40,48,64')
    ap.add_argument('--budget', type=float, default=60.0, help='skip the fixed-pattern classes past this estimate')
    args = ap.parse_args()
    import bench
    import kfmi
    from kfmi import ref15
    for n in (int(x) for x in args.n.split(',')):
        ev, init, _, t0, t_end = bench.bf_events(n)
        t_far = t_end + 5.0
        kfe = kfmi.BatchedKF('ref15', 1 << 22, 'f64')
        kfs = kfmi.BatchedKF('ref15', 1, 'f64')
        sym = kfs.search_plan(init, n)['sym']
        k_lo = ref15.search_levels(n, 'f64', 32 << 30, sym)
        w = ref15.search_class_width(n, 'f64', 32 << 30, sym)
        best = float('inf')
        for k in range(1, k_lo + 1):
            for off in range(0, math.comb(n, k), kfe.batch):
                mx, _, _ = kfe.eval_combos(ev, init, t0, t_far, k, combo_offset=off, logdets=False)
                best = min(best, float(mx[:min(kfe.batch, math.comb(n, k) - off)].min()))
        kfe.close()
        thr = best - 1e-9 * abs(best)
        calls = []

        def search_class(nf, c, k_max):
            calls.append(nf)
            k, idx, _, _ = kfs.search_combos(ev, init, t0, t_far, thr, k_max=k_max, n_fixed=nf, fixed_mask=c)
            return k, idx
        kfs.search_combos(ev, init, t0, t_far, thr, k_max=k_lo)   # warm: level buffers, module load
        rec = {'n': n, 'k_search': k_lo, 'class_width': w}
        t = time.perf_counter()
        k0 = kfs.search_combos(ev, init, t0, t_far, thr, k_max=k_lo)[0]
        k, key = ref15.search_past(search_class, n, k_lo, w, 'f64', 32 << 30, sym)
        rec['driver_s'] = round(time.perf_counter() - t, 4)
        rec.update(k_one_call=k0, k_found=k, winner=[i for i in range(n) if (ref15.bitrev64(key) >> i) & 1],
                   prefix_calls=len(calls), subsets_up_to_k=sum(math.comb(n, j) for j in range(1, k + 1)))
        # the fixed-pattern classes alone (the path before the bands): each class call costs at
        # least its launches; skipped where 2^w calls alone exceed the budget
        if (1 << w) * 50e-6 < args.budget:
            calls.clear()
            t = time.perf_counter()
            kc, keyc = ref15.class_search(search_class, n, w, ref15.class_order(w))
            rec['fixed_pattern_s'] = round(time.perf_counter() - t, 4)
            rec['fixed_pattern_calls'] = len(calls)
            rec['same_winner'] = (kc, keyc) == (k, key)
        else:
            rec['fixed_pattern_s'] = f'not run: 2^{w} class calls'
        kfs.close()
        print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
