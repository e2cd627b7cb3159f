"""How many 128-B lines the sched row's record gathers touch, and how many a wave-level line
cache could save — a CPU model of the apply pass's gathers (no GPU).

The bench's sched streams (bench.sched_streams, 64 filters per rate) are windowed on the host
with the pick rule of ref15_pick_kernel (kf_workers.py:870-912: queue while t - prev < 1/f, the
triggering event ends the window, the larger R wins where both classes are queued); the picks
are checked against the C oracle's greedy driver (oracle/cpu_kf.c cpu_ref15_sched) on a sample
of filters.  For 80-B records [T][B][10] it then counts, per wave and pick q, the distinct lines
the wave's 64 gathers touch (what the apply pass fetches: lanes of one instruction on one line
share it), against the distinct lines over the wave's WHOLE run (an unbounded per-wave line
cache: every line fetched once) and the coherent case (all lanes on one row: 0.625 lines).

    python tools/sched_line_sim.py [waves_per_rate]
    python tools/sched_line_sim.py --cache [waves_per_rate]

--cache (round 6) adds the caches: an LRU per CU (L1, 32 KiB = 256 lines) in front of an LRU per
XCD (L2, 4 MiB = 32768 lines), fed the gathers of one XCD's waves — heaviest waves first (the
apply pass's order, KF_OPT_SCHED_ORDER), RESIDENT at a time (8 per CU x 32 CUs), stepping pick by
pick in lock step — for three record layouts:
    rows   [T][B][rec]        today's (kf_run_scheduled_rec): a lane's next pick is B x 80 B away
    filter [B][T][rec]        filter-major: a lane's picks lie along its own 20 KB
    tiled  [B/64][T][64][rec] wave-tiled: one wave's rows adjacent (5 KB each)
and reports, per rate class (on the 5-ms event grid: 10/20/40/50/100 Hz, or off it), the lines
fetched from memory per pick (L2 misses), and the row's traffic over its algorithmic bytes:
(9 B per event + 152 B per pick (the 136 algorithmic + the 4-B pick word written and read + the
record's 8-B time) + the record lines' excess over 80 B) / (9 B per event + 136 B per pick).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]
import bench  # noqa: E402

REC, LINE = 80, 128


def picks_of(tt, et, freq, prev):
    T, B = tt.shape
    period = 1.0 / freq
    prev = prev.copy()
    qlen = np.zeros(B, int)
    qi0 = -np.ones(B, int)
    qi1 = -np.ones(B, int)
    picks = [[] for _ in range(B)]
    for i in range(T):
        gps = et[i] == 0
        window = tt[i] - prev < period
        enq = window | (qlen == 0)
        m = enq & gps & (qi0 < 0)
        qi0[m] = i
        m = enq & ~gps & (qi1 < 0)
        qi1[m] = i
        qlen[enq] += 1
        trig = np.nonzero(~window)[0]
        if trig.size:
            sel = np.where(qi1 >= 0, qi1, qi0)[trig]   # R_imu[0] 50 > R_gps[0] 3: the IMU sample wins
            for f, s in zip(trig, sel):
                picks[f].append(int(s))
            prev[trig] = tt[sel, trig]
            qlen[trig] = 0
            qi0[trig] = -1
            qi1[trig] = -1
    return picks


def main():
    cfg = bench.CONFIGS['sched']
    nw = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    rates = cfg['rates']
    B, T = 64 * len(rates) * nw, cfg['T']
    tt, et, pay, freq, prev = bench.sched_streams(B, T, cfg['dt'], cfg['k'], rates, 64, bench.SEED, torch.device('cpu'))
    tt, et, pay, freq, prev = tt.numpy(), et.numpy(), pay.numpy(), freq.numpy(), prev.numpy()
    picks = picks_of(tt, et, freq, prev)
    # the picks against the oracle's greedy driver, 4 filters of every rate
    from oracle import cpu_kf
    from oracle import ref_kf
    cols = np.concatenate([np.arange(r * 64 * nw, r * 64 * nw + 4) for r in range(len(rates))])
    st, _, _, ns = cpu_kf.ref15_sched(tt[:, cols], et[:, cols], pay[:, :, cols], prev[cols], freq[cols],
                                      ref_kf.P0_REF15)
    for j, f in enumerate(cols):
        assert ns[j] == len(picks[f]) and np.array_equal(st[:ns[j], j], tt[picks[f], f]), f
    print(f'picks checked against oracle/cpu_kf.c cpu_ref15_sched on {len(cols)} filters')
    cur = ideal = npk = 0
    rows = {}
    for w in range(B // 64):
        f0 = w * 64
        S = max(len(picks[f]) for f in range(f0, f0 + 64))
        seen, c = set(), 0
        for q in range(S):
            s = set()
            for lane in range(64):
                p = picks[f0 + lane]
                if q < len(p):
                    a = (p[q] * B + f0 + lane) * REC
                    s.update((a // LINE, (a + REC - 1) // LINE))
            c += len(s)
            seen |= s
        n = sum(len(picks[f]) for f in range(f0, f0 + 64))
        d = rows.setdefault(float(freq[f0]), [0, 0, 0])
        d[0] += c
        d[1] += len(seen)
        d[2] += n
        cur += c
        ideal += len(seen)
        npk += n
    print(f'B = {B} ({nw} waves per rate), T = {T}: {npk / (B * T):.4f} picks per event')
    print(f'lines per pick: per-pick gathers {cur / npk:.3f}, unbounded per-wave line cache {ideal / npk:.3f}, '
          f'coherent {REC / LINE:.3f}')
    for r, (c, i, n) in sorted(rows.items()):
        print(f'  {r:5.0f} Hz: {c / n:.3f} / {i / n:.3f} lines per pick, {n / (64 * nw):.1f} picks per filter')
    print(f'record bytes per pick: {cur / npk * LINE:.1f} now, {ideal / npk * LINE:.1f} with the unbounded cache '
          f'(-{(cur - ideal) / npk * LINE:.1f} B of a pick\'s ~{64 + 72 + 8 + 8 + (cur / npk) * LINE - 72:.0f} B of traffic)')


GRID_RATES = (10.0, 20.0, 40.0, 50.0, 100.0)   # periods on the 5-ms event grid


def layout_line(layout, B, T):
    """128-B line of (event row t, filter f)'s record start, for each layout."""
    if layout == 'rows':
        return lambda t, f: (t * B + f) * REC
    if layout == 'filter':
        return lambda t, f: (f * T + t) * REC
    if layout == 'tiled':
        return lambda t, f: ((f // 64) * T * 64 + t * 64 + (f % 64)) * REC
    raise ValueError(layout)


def cache_sim(picks, freq, B, T, layout, resident=256, per_cu=8, l1_lines=256, l2_lines=32768):
    """L2 misses (lines from memory) per rate of one XCD's apply pass over these waves."""
    from collections import OrderedDict
    addr = layout_line(layout, B, T)
    waves = sorted(range(B // 64), key=lambda w: -max(len(picks[f]) for f in range(w * 64, w * 64 + 64)))
    l2 = OrderedDict()
    miss, npk = {}, {}
    for g0 in range(0, len(waves), resident):
        gen = waves[g0:g0 + resident]
        l1 = [OrderedDict() for _ in range((len(gen) + per_cu - 1) // per_cu)]
        steps = max(len(picks[f]) for w in gen for f in range(w * 64, w * 64 + 64))
        for q in range(steps):
            for i, w in enumerate(gen):
                r = float(freq[w * 64])
                lines = set()
                for f in range(w * 64, w * 64 + 64):
                    p = picks[f]
                    if q < len(p):
                        a = addr(p[q], f)
                        lines.add(a // LINE)
                        lines.add((a + REC - 1) // LINE)
                        npk[r] = npk.get(r, 0) + 1
                c1 = l1[i // per_cu]
                for ln in lines:
                    if ln in c1:
                        c1.move_to_end(ln)
                        continue
                    c1[ln] = None
                    if len(c1) > l1_lines:
                        c1.popitem(last=False)
                    if ln in l2:
                        l2.move_to_end(ln)
                        continue
                    l2[ln] = None
                    if len(l2) > l2_lines:
                        l2.popitem(last=False)
                    miss[r] = miss.get(r, 0) + 1
    return miss, npk


def cache_main(nw):
    cfg = bench.CONFIGS['sched']
    rates = cfg['rates']
    B, T = 64 * len(rates) * nw, cfg['T']
    tt, et, pay, freq, prev = bench.sched_streams(B, T, cfg['dt'], cfg['k'], rates, 64, bench.SEED, torch.device('cpu'))
    tt, et, freq, prev = tt.numpy(), et.numpy(), freq.numpy(), prev.numpy()
    picks = picks_of(tt, et, freq, prev)
    npick = sum(len(p) for p in picks)
    print(f'B = {B} filters ({B // 64} waves: {nw} per rate, one XCD\'s share at {256} resident), T = {T}: '
          f'{npick / (B * T):.4f} picks per event')
    base = B * T * 9 + npick * 136
    for layout in ('rows', 'filter', 'tiled'):
        miss, npk = cache_sim(picks, freq, B, T, layout)
        tot_m = sum(miss.values())
        per = {k: (sum(miss.get(r, 0) for r in rates if (r in GRID_RATES) == k),
                   sum(npk.get(r, 0) for r in rates if (r in GRID_RATES) == k)) for k in (True, False)}
        excess = tot_m * LINE - npick * REC
        ratio = (B * T * 9 + npick * 152 + excess) / base
        print(f'{layout:6s}: {tot_m / npick:.3f} lines from memory per pick (coherent 0.625); on-grid rates '
              f'{per[True][0] / max(per[True][1], 1):.3f}, off-grid {per[False][0] / max(per[False][1], 1):.3f}; '
              f'row traffic / algorithmic {ratio:.3f}')
        for r in rates:
            print(f'    {r:5.0f} Hz: {miss.get(float(r), 0) / max(npk.get(float(r), 1), 1):.3f} lines per pick')
    floor = (B * T * 9 + npick * 152) / base
    print(f'floor at 0.625 lines per pick (every wave coherent): {floor:.3f} (the pick word and the record time)')


if __name__ == '__main__':
    if '--cache' in sys.argv:
        args = [a for a in sys.argv[1:] if a != '--cache']
        cache_main(int(args[0]) if args else 32)
    else:
        main()
