"""In-process A/B of kernel variants on one bench workload (diagnostic).

HBM placement differs from process to process, so comparing variants across
processes can rank them by the placement they happened to get.  This builds the workload once
and alternates launches between the arms on the same handle and buffers.

    python tools/ab_inproc.py --config ref15 --arms build/ab/base.so,default [--rounds 6] [--launches 10]

An arm is a library path (loaded side by side; valid while `kf_batch`'s layout is the same in
both builds, i.e. for kernel-side changes), `default` (the in-tree libkfmi.so), or NAME=VALUE
(the in-tree library with that kf_set_option on the workload's handle, kfmi.engine.OPTIONS).
Prints the median kernel time per arm and the per-round times.
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='ref15')
    ap.add_argument('--arms', required=True)
    ap.add_argument('--rounds', type=int, default=6)
    ap.add_argument('--rate-block', type=int, default=64, help='config sched: filters per processing rate')
    ap.add_argument('--launches', type=int, default=10)
    ap.add_argument('--bf-n', type=int, default=None, help='config bf: candidate events (default the row\'s 25)')
    args = ap.parse_args()
    import torch
    import bench
    from kfmi import _lib

    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    default = _lib.lib()
    arms = []
    for a in args.arms.split(','):
        if a == 'default':
            arms.append((a, default, None))
        elif '=' in a and not os.path.exists(a):
            k, v = a.split('=', 1)
            arms.append((a, default, (k, v)))
        else:
            h = ctypes.CDLL(os.path.abspath(a))
            for name, (res, argt) in _lib.SIGNATURES.items():
                if not hasattr(h, name):  # an older build: entry points added since are not called
                    continue
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = argt
            arms.append((a, h, None))
    cfg = dict(bench.CONFIGS[args.config])
    cfg['opts'] = {}
    if args.bf_n:
        cfg['n'] = args.bf_n
    ns = argparse.Namespace(ablate='none', gpus=1, no_cpu_baseline=True, rate_block=args.rate_block)
    if args.config in ('ref15', 'ref15f32'):
        w = bench.ref15_workload(cfg, ns, 0, 1, dev)
    elif args.config in ('bf', 'bf_subsets'):
        w = bench.bf_workload(cfg, ns, 0, 1, dev)
    elif args.config in ('1', '1ref8', '1dr'):
        w = bench.log_workload(cfg, ns, 0, 1, dev)
    elif args.config == 'sched':
        w = bench.sched_workload(cfg, ns, 0, 1, dev)
    else:
        w = bench.cv_workload(args.config, cfg, ns, 0, 1, dev)
    stream = torch.cuda.current_stream(dev)
    opt_names = {a[2][0] for a in arms if a[2]}

    def use(arm):
        name, h, opt = arm
        _lib._lib = h
        for k in opt_names:
            w['kf'].set_option(k, 0)
        if opt:
            v = opt[1]
            w['kf'].set_option(opt[0], int(v) if v.lstrip('-').isdigit() else v)

    times = {a[0]: [] for a in arms}
    for arm in arms:   # warm every arm once (module load, first-launch costs)
        use(arm)
        w['step']()
    torch.cuda.synchronize(dev)
    for r in range(args.rounds):
        order = arms if r % 2 == 0 else arms[::-1]
        for arm in order:
            use(arm)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.launches)]
            for s, e in ev:
                s.record(stream)
                w['step']()
                e.record(stream)
            torch.cuda.synchronize(dev)
            times[arm[0]].append(statistics.median(s.elapsed_time(e) for s, e in ev))
    use(arms[0])
    out = {'config': args.config, 'rounds': args.rounds, 'launches': args.launches,
           'median_ms': {k: round(statistics.median(v), 4) for k, v in times.items()},
           'per_round_ms': {k: [round(x, 4) for x in v] for k, v in times.items()}}
    print(json.dumps(out))


if __name__ == '__main__':
    main()
