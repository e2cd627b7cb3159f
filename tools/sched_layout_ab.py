"""In-process A/B of the sched row's payload layout: [T][9][B] rows (kf_run_scheduled) against
[T][B][N] records (kf_run_scheduled_rec), on one set of streams, alternating launches.

    python tools/sched_layout_ab.py [--arms rows,rec10,rec12,rec12t] [--rounds 6] [--launches 10] [--rate-block 64]

recNt: N-double records whose rec[9] holds the event time, read by the apply pass
(KF_OPT_SCHED_REC_TIME = 1).
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rounds', type=int, default=6)
    ap.add_argument('--launches', type=int, default=10)
    ap.add_argument('--rate-block', type=int, default=64)
    ap.add_argument('--arms', default='rows,rec10', help='rows and/or recN (N doubles per record)')
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    arms = {}
    for lay in args.arms.split(','):
        cfg = dict(bench.CONFIGS['sched'])
        cfg['opts'] = {'sched_rec_time': 1} if lay.endswith('t') else {}
        ns = argparse.Namespace(ablate='none', gpus=1, no_cpu_baseline=True, rate_block=args.rate_block,
                                sched_payload='rows' if lay == 'rows' else 'records',
                                sched_rec=0 if lay == 'rows' else int(lay[3:].rstrip('t')))
        arms[lay] = bench.sched_workload(cfg, ns, 0, 1, dev)
    for lay, w in arms.items():
        w['step']()
    torch.cuda.synchronize(dev)
    stream = torch.cuda.current_stream(dev)
    times = {k: [] for k in arms}
    for r in range(args.rounds):
        for lay in (list(arms) if r % 2 == 0 else list(arms)[::-1]):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(args.launches)]
            for s, e in ev:
                s.record(stream)
                arms[lay]['step']()
                e.record(stream)
            torch.cuda.synchronize(dev)
            times[lay].append(statistics.median(s.elapsed_time(e) for s, e in ev))
    print(json.dumps({'config': 'sched', 'rate_block': args.rate_block,
                      'median_ms': {k: round(statistics.median(v), 4) for k, v in times.items()},
                      'per_round_ms': {k: [round(x, 4) for x in v] for k, v in times.items()}}))


if __name__ == '__main__':
    main()
