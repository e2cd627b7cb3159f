"""Per-launch kernel times of one bench workload over a long run, to tell steady-state clock
behaviour (power/thermal) apart from box-to-box variance.

    python tools/launch_series.py --config 3 --launches 200 [--sleep-ms 0]

Each launch is bracketed by its own HIP events on the workload's stream; prints the series
summary (first/last 10, median, min, max) and the GPU's reported sclk/mclk/power if rocm-smi
answers (read-only).
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def smi():
    try:
        out = subprocess.run(['rocm-smi', '--showclocks', '--showpower', '--showtemp', '--json'],
                             capture_output=True, text=True, timeout=20).stdout
        d = json.loads(out)
        card = d[sorted(d)[0]]
        keys = [k for k in card if any(s in k.lower() for s in ('sclk', 'mclk', 'fclk', 'power', 'temp'))]
        return {k: card[k] for k in keys}
    except Exception as e:  # noqa: BLE001 - diagnostic only
        return {'error': str(e)[:200]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='3')
    ap.add_argument('--launches', type=int, default=200)
    ap.add_argument('--sleep-ms', type=float, default=0.0)
    args = ap.parse_args()
    import torch
    import bench
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    cfg = bench.CONFIGS[args.config]
    ns = argparse.Namespace(ablate=[], gpus=1)
    w = bench.cv_workload(args.config, cfg, ns, 0, 1, dev)
    stream = torch.cuda.current_stream(dev)
    print('before', json.dumps(smi()), flush=True)
    times = []
    for i in range(args.launches):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        w['step']()
        e1.record(stream)
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
        if args.sleep_ms:
            time.sleep(args.sleep_ms / 1e3)
        if i == args.launches // 2:
            print('mid', json.dumps(smi()), flush=True)
    print('after', json.dumps(smi()), flush=True)
    s = sorted(times)
    print(json.dumps({'config': args.config, 'launches': len(times), 'sleep_ms': args.sleep_ms,
                      'first10': [round(t, 3) for t in times[:10]],
                      'last10': [round(t, 3) for t in times[-10:]],
                      'median': round(s[len(s) // 2], 3), 'min': round(s[0], 3), 'max': round(s[-1], 3)}))


if __name__ == '__main__':
    main()
