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


if __name__ == '__main__':
    main()
