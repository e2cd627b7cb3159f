"""In-process A/B of the config-3 access pattern: stores interleaved with loads every step
(kfprobe_pattern, the bench's pattern ceiling) against stores held in registers for 2 / 4 / 8
steps and issued as one burst per wave (kfprobe_pattern_burst) — VERDICT r4 item 6: does
phase-separating a wave's reads and writes raise the mixed stream's HBM rate?  Rounds
interleave the variants on the same buffers; GB/s of the pattern's bytes, HIP events.

    python tools/probes/burst_ab.py [rounds]
"""
import ctypes
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    lib = ctypes.CDLL(os.path.join(HERE, 'libpattern_probe.so'))
    vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    lib.kfprobe_pattern.argtypes = [i32, i32, vp, vp, vp, vp, i64, i32, i32, vp]
    lib.kfprobe_pattern_burst.argtypes = [i32, i32, vp, vp, vp, vp, i64, i32, i32, i32, vp]
    dev = torch.device('cuda', 0)
    B, T, d = 1 << 20, 256, 3
    g = torch.Generator(device=dev).manual_seed(1)
    u = torch.randn(T, d, B, dtype=torch.float64, device=dev, generator=g)
    z = torch.randn(T, d, B, dtype=torch.float64, device=dev, generator=g)
    traj = torch.empty(T, 2 * d, B, dtype=torch.float64, device=dev)
    ld = torch.empty(T, B, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(st.cuda_stream)
    nbytes = B * T * (d + d + 2 * d + 1) * 8
    variants = {'interleaved (kfprobe_pattern)': lambda: lib.kfprobe_pattern(d, 1, u.data_ptr(), z.data_ptr(),
                                                                             traj.data_ptr(), ld.data_ptr(), B, T, 1, sp)}
    for h in (1, 2, 4, 8):
        variants[f'burst hold {h}'] = (lambda h=h: lib.kfprobe_pattern_burst(d, 1, u.data_ptr(), z.data_ptr(),
                                                                             traj.data_ptr(), ld.data_ptr(), B, T, 1,
                                                                             h, sp))
    for f in variants.values():
        assert f() == 0
    torch.cuda.synchronize(dev)
    times = {k: [] for k in variants}
    for r in range(rounds):
        for k, f in (variants.items() if r % 2 == 0 else reversed(list(variants.items()))):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
            for s, e in ev:
                s.record(st)
                f()
                e.record(st)
            torch.cuda.synchronize(dev)
            times[k].append(float(np.mean([s.elapsed_time(e) for s, e in ev])))
    print(f'config-3 pattern, B = {B}, T = {T}, f64, {nbytes / 1e9:.2f} GB per launch; {rounds} interleaved rounds of 5')
    base = np.median(times['interleaved (kfprobe_pattern)'])
    for k, v in times.items():
        m = float(np.median(v))
        print(f'{k:32s} median {m:.4f} ms  {nbytes / m / 1e6:8.1f} GB/s  vs interleaved {base / m:.3f}x  '
              f'(rounds: {" ".join(f"{x:.3f}" for x in v)})')


if __name__ == '__main__':
    main()
