"""The one-wave look-ahead kernel for one gated filter (KF_OPT_EVENTS_KERNEL = 4,
ref_chain_gated_kernel) against the chain kernel's sequential gated filter (= 2), diagnostic:
one filter over a long stream (tests/test_gpu_timeparallel._stream) per threshold: share of
events updated, the update flags equal or not, the largest relative difference of the records
and final state, and the time of each (medians over rounds, interleaved).

    python tools/gated_kernel_ab.py [--T 70000] [--thr -10,-20,-30,-36.4] [--rounds 5] [--dtype f64]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd'), os.path.join(ROOT, 'tests')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--T', type=int, default=70000)
    ap.add_argument('--thr', default='-10,-20,-30,-36.4')
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--seed', type=int, default=11)
    ap.add_argument('--dtype', default='f64')
    args = ap.parse_args()
    import numpy as np
    import torch
    import kfmi
    from kfmi import ref15
    from test_gpu_timeparallel import _stream
    et, dt, pay, x0 = _stream(args.T, seed=args.seed)
    P0 = ref15.to_blocks(ref15.P0)
    if args.dtype == 'f32':
        x0, P0, pay = x0.astype(np.float32), P0.astype(np.float32), pay.astype(np.float32)

    def run(kernel, thr):
        kf = kfmi.BatchedKF('ref15', 1, args.dtype, options={'events_kernel': kernel})
        kf.set_state(x0[:, None], P0[:, None])
        torch.cuda.synchronize()
        t = time.perf_counter()
        tr, ld, up, cv = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], updated=True, cov=True,
                                       threshold=thr, sequential=True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        x, P = kf.state()
        st = kf.status()
        out = [v.double().cpu().numpy() for v in (tr, ld, cv, x, P)]
        flags = up.cpu().numpy()
        kf.close()
        return out, flags, ms, int(st.sum().item())
    for thr in (float(v) for v in args.thr.split(',')):
        run('gated', thr)
        times = {'gated': [], 'chain': []}
        for _ in range(args.rounds):
            g, fg, ms, sg = run('gated', thr)
            times['gated'].append(ms)
            s, fs, ms, ss = run('chain', thr)
            times['chain'].append(ms)
        rel = max(float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1.0))) for a, b in zip(g, s))
        print(json.dumps({'T': args.T, 'dtype': args.dtype, 'threshold': thr, 'updated_share': float(fs.mean()),
                          'flags_equal': bool(np.array_equal(fg, fs)), 'flag_diffs': int((fg != fs).sum()),
                          'max_rel': rel, 'status': [sg, ss],
                          'median_ms': {k: round(statistics.median(v), 3) for k, v in times.items()}}), flush=True)


if __name__ == '__main__':
    main()
