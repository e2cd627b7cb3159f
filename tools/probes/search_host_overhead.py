"""Host turnaround of one kf_search_combos call (the bf row's step), measured on the GPU box:
    python tools/probes/search_host_overhead.py
Prints the wall time per call of the n = 25 exhaustive search beside the device time HIP events
see on its stream, and the floors: a search over 4 candidates (launches of nearly no work), the
same through a raw ctypes call (no Python wrapper), and an idle stream synchronisation."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd'))
import bench  # noqa: E402
import kfmi  # noqa: E402
from kfmi import _lib  # noqa: E402


def per_call(fn, reps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def main():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    kf = kfmi.BatchedKF('ref15', 1, 'f64', device=0)
    st = torch.cuda.current_stream()
    out = {}
    for n in (25, 4):
        ev, init, _, t0, t_end = bench.bf_events(n)
        f = lambda: kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True)  # noqa: E731
        out[f'wall_us_n{n}'] = per_call(f, 200 if n == 4 else 40)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f()
        a.record(st)
        for _ in range(20):
            f()
        b.record(st)
        b.synchronize()
        out[f'stream_span_us_n{n}'] = a.elapsed_time(b) * 1e3 / 20
    # a non-exhaustive search that stops at a middle size: one result peek per level
    ev, init, _, t0, t_end = bench.bf_events(25)
    _, _, _, sm = kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True, subset_max=True)
    sm = sm.cpu().numpy()
    masks = np.arange(1 << 25, dtype=np.uint32)
    sizes = np.zeros(1 << 25, np.uint8)
    for b in range(25):
        sizes += ((masks >> b) & 1).astype(np.uint8)
    mins = [float(np.nanmin(sm[sizes == k])) for k in range(1, 26)]
    for label, thr in (('none', -1e30), ('mid', None)):
        if thr is None:  # just above the lowest score of the largest size <= 16 below every
            # smaller size's lowest: the search stops there
            s_mid = max(s for s in range(1, 17) if all(mins[k - 1] > mins[s - 1] for k in range(1, s)))
            thr = mins[s_mid - 1] + abs(mins[s_mid - 1]) * 1e-12 + 1e-15
        out[f'stops_at_size_{label}'] = kf.search_combos(ev, init, t0, t_end, thr)[0]
        out[f'wall_us_n25_stop_{label}'] = per_call(lambda: kf.search_combos(ev, init, t0, t_end, thr), 20)
    del sm, sizes, masks
    ev, init, _, t0, t_end = bench.bf_events(4)
    ev = np.ascontiguousarray(ev)
    init = np.ascontiguousarray(init)
    win, kf_, acc = ctypes.c_uint64(0), ctypes.c_int(0), np.zeros(5, np.uint64)
    fn = _lib.lib().kf_search_combos
    sp = ctypes.c_void_p(st.cuda_stream)
    args = (kf.handle, 4, ev.ctypes.data_as(ctypes.c_void_p), init.ctypes.data_as(ctypes.c_void_p), float(t0),
            float(t_end), -1e30, 4, 1, 0, 0, ctypes.byref(win), ctypes.byref(kf_), acc.ctypes.data_as(ctypes.c_void_p),
            None, sp)
    out['raw_ctypes_us_n4'] = per_call(lambda: fn(*args), 200)
    out['idle_sync_us'] = per_call(lambda: torch.cuda.synchronize(), 500)
    small = torch.zeros(128, dtype=torch.int64, device=dev)
    out['d2h_1KB_us'] = per_call(lambda: small.cpu(), 200)
    for k, v in out.items():
        print(f'{k:24s} {v:9.1f}')


if __name__ == '__main__':
    main()
