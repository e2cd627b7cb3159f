"""A/B of the gated sequential filter between a variant build and the in-tree library
(diagnostic): one filter over a long stream (tests/test_gpu_timeparallel._stream) with the
adaptive gate, kf_run_events_seq, per threshold: the time of each arm (medians over rounds,
arms interleaved) and whether every record (trajectory, logdet, update flags, final state) is
bitwise the in-tree library's.

    python tools/gate_ab.py --arm sensorfusion-kalmanfilter_amd/kfmi/libkfmi_X.so [--T 70000] [--rounds 5]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd'), os.path.join(ROOT, 'tests')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--arm', required=True)
    ap.add_argument('--T', type=int, default=70000)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--thr', default='-10,-20,-30')
    args = ap.parse_args()
    import numpy as np
    import torch
    import kfmi
    from kfmi import _lib, ref15
    from test_gpu_timeparallel import _stream
    default = _lib.lib()
    h = ctypes.CDLL(os.path.abspath(args.arm))
    for name, (res, argt) in _lib.SIGNATURES.items():
        if hasattr(h, name):
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, argt
    et, dt, pay, x0 = _stream(args.T, seed=11)
    P0 = ref15.to_blocks(ref15.P0)

    def run(lib, thr):
        _lib._lib = lib
        kf = kfmi.BatchedKF('ref15', 1, 'f64')
        kf.set_state(x0[:, None], P0[:, None])
        torch.cuda.synchronize()
        t = time.perf_counter()
        tr, ld, up, _ = kf.run_events(et[:, None], dt[:, None], pay[:, :, None], updated=True, threshold=thr,
                                      sequential=True)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        x, P = kf.state()
        out = [v.cpu().numpy() for v in (tr, ld, up, x, P)]
        kf.close()
        _lib._lib = default
        return out, ms
    for thr in (float(v) for v in args.thr.split(',')):
        times = {'arm': [], 'default': []}
        ref, _ = run(default, thr)
        run(h, thr)
        same = True
        for _ in range(args.rounds):
            o, ms = run(h, thr)
            times['arm'].append(ms)
            same = same and all(np.array_equal(a, b, equal_nan=True) for a, b in zip(o, ref))
            o, ms = run(default, thr)
            times['default'].append(ms)
        print(json.dumps({'T': args.T, 'threshold': thr, 'updated_share': float(ref[2].mean()),
                          'median_ms': {k: round(statistics.median(v), 3) for k, v in times.items()},
                          'bitwise_equal': bool(same)}), flush=True)


if __name__ == '__main__':
    main()
