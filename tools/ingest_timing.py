"""Where kf_ingest's wall time goes (diagnostic): the config-1 synthetic log parsed once, then
ingest_arrays three times (cold / warm allocator), with the H2D copies, allocations and the
library call timed separately.   python tools/ingest_timing.py"""
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from kfmi import ingest  # noqa: E402

dev = torch.device('cuda', 0)
torch.zeros(1, device=dev)
root = tempfile.mkdtemp()
gp, ip = bench.synth_log(bench.CONFIGS['1'], root)
t0 = time.perf_counter()
g, m = ingest.read_csv(gp, 4), ingest.read_csv(ip, 11)
print(f'read_csv {1e3 * (time.perf_counter() - t0):.1f} ms  gps {g.shape} imu {m.shape}')
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gd = torch.as_tensor(np.ascontiguousarray(g)).to(dev)
    md = torch.as_tensor(np.ascontiguousarray(m)).to(dev)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    s = ingest.ingest_arrays(gd, md, device=0)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f'rep {rep}: H2D {1e3 * (t1 - t0):.1f} ms, ingest_arrays (device columns) {1e3 * (t2 - t1):.1f} ms, '
          f'{len(s)} events')

# the oracle's restatement of the reference's ingest (oracle/ref_ingest.ingest: csv module,
# per-row Python loops as kf_workers.py:290-385) on the same files, 1 core: the CPU baseline
sys.path.insert(0, ROOT)
from oracle import ref_ingest  # noqa: E402
t0 = time.perf_counter()
ev = ref_ingest.ingest(gp, ip)[0]
el = time.perf_counter() - t0
print(f'oracle ingest (Python, 1 core): {1e3 * el:.0f} ms, {len(ev)} events, {len(ev) / el:.3g} events/s')
