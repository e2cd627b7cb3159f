"""Where kf_csv_shape / kf_csv_read spend their time on the config-1 synthetic logs (diagnostic,
host only): each call timed separately, three repetitions (the first maps cold pages).
    python tools/csv_timing.py"""
import ctypes
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]
import numpy as np  # noqa: E402

import bench  # noqa: E402
from kfmi import _lib  # noqa: E402

root = tempfile.mkdtemp()
gp, ip = bench.synth_log(bench.CONFIGS['1'], root)
L = _lib.lib()
for path, nc in ((gp, 4), (ip, 11)):
    print(os.path.basename(path), f'{os.path.getsize(path) / 1e6:.1f} MB', f'cpus {os.cpu_count()}')
    for rep in range(3):
        rows, cols = ctypes.c_int64(), ctypes.c_int()
        t0 = time.perf_counter()
        L.kf_csv_shape(os.fsencode(path), 1, ctypes.byref(rows), ctypes.byref(cols))
        t1 = time.perf_counter()
        out = np.empty((nc, rows.value))
        t2 = time.perf_counter()
        out.fill(0.0)
        t3 = time.perf_counter()
        rc = L.kf_csv_read(os.fsencode(path), 1, nc, out.ctypes.data_as(ctypes.c_void_p), rows.value, rows.value)
        t4 = time.perf_counter()
        print(f'  rep {rep}: shape {1e3 * (t1 - t0):.1f} ms, alloc {1e3 * (t2 - t1):.2f}, first touch '
              f'{1e3 * (t3 - t2):.1f}, read {1e3 * (t4 - t3):.1f} ms (rc {rc})')
