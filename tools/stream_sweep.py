"""Config 1's time-parallel run (kf_run_stream) over the synthetic drive log, swept over the
warm-up length and the chunk length: device check verdict, covariance / state seam gaps and
the time per run (HIP events).  Diagnostic tool, not product.

    python tools/stream_sweep.py [--warmup 1024,1536,2048,2560] [--chunk 0,192,285,400]
"""
import argparse
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd'))

import torch  # noqa: E402

import bench  # noqa: E402
import kfmi  # noqa: E402
from kfmi import _lib, ingest  # noqa: E402
from kfmi.engine import _ptr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--warmup', default='-2,-3,-1,1536,2048')
    ap.add_argument('--chunk', default='0')
    ap.add_argument('--reps', type=int, default=5)
    args = ap.parse_args()
    dev = torch.device('cuda', 0)
    cfg = dict(bench.CONFIGS['1'])
    gp, ip = bench.synth_log(cfg, tempfile.mkdtemp(prefix='kfmi_sweep_'))
    stream = ingest.ingest_arrays(ingest.read_csv(gp, 4), ingest.read_csv(ip, 11), device=0)
    first = int(torch.nonzero(stream.etype == _lib.KF_EVENT_GPS)[0, 0])
    t_ev = stream.t[first:].contiguous()
    e_ev = stream.etype[first:].contiguous()
    pay = stream.payload[first:].contiguous()
    T = len(t_ev)
    x0 = torch.zeros(15, 1, dtype=torch.float64, device=dev)
    x0[0:3, 0] = pay[0, 0:3]
    kf = kfmi.BatchedKF('ref15', 1, 'f64')
    dt = torch.empty(T, dtype=torch.float64, device=dev)
    et = torch.empty(T, dtype=torch.uint8, device=dev)
    traj = kf.empty(T, 6, 1)
    logdet = kf.empty(T, 1)
    L = _lib.lib()
    _lib.check(L.kf_events_dt(T, _ptr(t_ev), _ptr(e_ev), float(t_ev[0]), _lib.KF_DT_FULL, _ptr(dt), _ptr(et),
                              kf._stream()))
    for w in (int(v) for v in args.warmup.split(',')):
        for c in (int(v) for v in args.chunk.split(',')):
            def run():
                kf.reset(x0)
                _lib.check(L.kf_run_stream(kf.handle, T, _ptr(et), _ptr(dt), _ptr(pay), _ptr(traj), None,
                                           _ptr(logdet), None, c, w, kf._stream()))
            run()
            chk = kf.stream_check()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            chk['ms'] = e0.elapsed_time(e1) / args.reps
            print(json.dumps(chk), flush=True)


if __name__ == '__main__':
    main()
