"""Every subset's score (subset_max) of an exhaustive search through a variant build of the
library against the in-tree one, on the bf rows' candidates (diagnostic, for kernel-side A/Bs
that change the arithmetic): max relative difference, count of bitwise-different scores.

    python tools/search_scores_ab.py --arm sensorfusion-kalmanfilter_amd/kfmi/libkfmi_X.so [--n 25]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--arm', required=True)
    ap.add_argument('--n', type=int, default=25)
    args = ap.parse_args()
    import numpy as np
    import bench
    import kfmi
    from kfmi import _lib
    default = _lib.lib()
    h = ctypes.CDLL(os.path.abspath(args.arm))
    for name, (res, argt) in _lib.SIGNATURES.items():
        if hasattr(h, name):
            fn = getattr(h, name)
            fn.restype, fn.argtypes = res, argt
    ev, init, _, t0, t_end = bench.bf_events(args.n)
    out = {}
    for tag, lib in (('default', default), ('arm', h)):
        _lib._lib = lib
        kf = kfmi.BatchedKF('ref15', 1, 'f64')
        _, _, _, sm = kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True, subset_max=True)
        out[tag] = sm.double().cpu().numpy()
        kf.close()
    _lib._lib = default
    a, b = out['default'][1:], out['arm'][1:]
    rel = np.abs(a - b) / np.maximum(np.abs(a), 1.0)
    print(json.dumps({'n': args.n, 'subsets': int(a.size), 'finite': bool(np.isfinite(b).all()),
                      'max_rel': float(rel.max()), 'bitwise_different': int((a != b).sum())}))


if __name__ == '__main__':
    main()
