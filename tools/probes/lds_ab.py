"""In-process A/B of access patterns for the cv3 fp64 bench stream (B = 2^20, T = 256):
the register-ring pattern of cv_block_kernel (kfprobe_pattern) vs LDS-DMA images of two steps
(kfprobe_pattern_lds) vs one filter per wavefront (kfprobe_pattern_wave).  Interleaved rounds on the same buffers, so both see one HBM placement.
Diagnostic only.   python tools/probes/lds_ab.py [rounds]"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(HERE, 'libpattern_probe.so'))
vp, i64, ci = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int
lib.kfprobe_pattern.argtypes = [ci, ci, vp, vp, vp, vp, i64, ci, ci, vp]
lib.kfprobe_pattern_lds.argtypes = [vp, vp, vp, vp, i64, ci, vp]
lib.kfprobe_pattern_wave.argtypes = [vp, vp, vp, vp, i64, ci, vp]

B, T = 1 << 20, 256
dev = torch.device('cuda', 0)
u = torch.randn(T, 3, B, dtype=torch.float64, device=dev)
z = torch.randn(T, 3, B, dtype=torch.float64, device=dev)
traj = torch.empty(T, 6, B, dtype=torch.float64, device=dev)
ld = torch.empty(T, B, dtype=torch.float64, device=dev)
st = torch.cuda.current_stream(dev)
sp = ctypes.c_void_p(st.cuda_stream)
bytes_per = T * B * (6 + 7) * 8

runs = {
    'ring': lambda: lib.kfprobe_pattern(3, 1, u.data_ptr(), z.data_ptr(), traj.data_ptr(), ld.data_ptr(), B, T, 1, sp),
    'lds2': lambda: lib.kfprobe_pattern_lds(u.data_ptr(), z.data_ptr(), traj.data_ptr(), ld.data_ptr(), B, T, sp),
    # one filter per wavefront (SURVEY.md §7's alternative mapping)
    'wave': lambda: lib.kfprobe_pattern_wave(u.data_ptr(), z.data_ptr(), traj.data_ptr(), ld.data_ptr(), B, T, sp),
}
# same values stored by both: acc of the inputs, so check one against the other once
res = {}
for name, fn in runs.items():
    assert fn() == 0, name
    torch.cuda.synchronize()
    res[name] = ld.clone()
print('outputs equal:', bool(torch.equal(res['ring'], res['lds2'])), bool(torch.equal(res['ring'], res['wave'])), flush=True)

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 6
reps = {'ring': 10, 'lds2': 10, 'wave': 2}
out = {k: [] for k in runs}
for r in range(rounds):
    for name, fn in runs.items():
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(st)
        for _ in range(reps[name]):
            fn()
        ev[1].record(st)
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / reps[name]
        out[name].append(ms)
    print(r, {k: f'{v[-1]:.3f} ms {bytes_per / v[-1] / 1e6:.0f} GB/s' for k, v in out.items()}, flush=True)
print(json.dumps({k: dict(ms=sorted(v)[len(v) // 2], gbs=bytes_per / sorted(v)[len(v) // 2] / 1e6) for k, v in out.items()}))
