"""Benchmark of the batched KF hot path (kf_run) on 1..N MI355X, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3]
    torchrun --nproc-per-node N bench.py --gpus N ...        (multi-GPU, RCCL)

One bench *step* = one kf_run launch: every filter of this rank's shard advances T time
steps (fused predict + GPS update, trajectory and logdet written to HBM) — one pass of the
hot path over one batch of synthetic streams.  The streams are generated on the GPU by the
counter-based Philox generator (kf_synth) and are resident in HBM before timing starts;
consecutive bench steps continue the same filters (warm start, like the reference's
windowed runs, kf_workers.py:2316-2323) over the same stream chunk.

Configs (BASELINE.json / SURVEY.md §8d); per GPU (weak scaling: each rank owns B filters):
    2  cv2 (4-state/2-meas)  fp32  B=65,536     T=1024 dt=0.1  update every step
    3  cv3 (6-state/3-meas)  fp64  B=1,048,576  T=256  dt=0.1  update every step   [default]
    4  cv3 (6-state/3-meas)  fp32  B=1,048,576  T=256  dt=0.1  update every step   (x8 GPUs)
    5  cv3 (6-state/3-meas)  fp64  B=1,048,576  T=500  dt=0.01 GPS update every 10th step
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, 'sensorfusion-kalmanfilter_amd')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

CONFIGS = {
    2: dict(model='cv2', dtype='f32', B=65536, T=1024, dt=0.1, k=1),
    3: dict(model='cv3', dtype='f64', B=1048576, T=256, dt=0.1, k=1),
    4: dict(model='cv3', dtype='f32', B=1048576, T=256, dt=0.1, k=1),
    5: dict(model='cv3', dtype='f64', B=1048576, T=500, dt=0.01, k=10),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SEED = 20251015


def algorithmic_bytes(cfg):
    """Bytes one kf_run launch must move: per filter per step c control values
    read, m measurement values read on update steps, n state values + 1 logdet written; per
    filter per launch (x, P) loaded and stored once and status read + written."""
    d = 2 if cfg['model'] == 'cv2' else 3
    n, m, c = 2 * d, d, d
    w = 8 if cfg['dtype'] == 'f64' else 4
    T, k, B = cfg['T'], cfg['k'], cfg['B']
    U = T // k
    per_filter = T * (c + n + 1) * w + U * m * w + 2 * (n + n * (n + 1) // 2) * w + 2 * 4
    return per_filter * B, per_filter / T


def cpu_baseline(cfg, x0, u, z, budget_s=12.0):
    """The reference CPU loop (oracle/ref_kf.run_filter_loop: one filter at a time, NumPy in
    the reference's op order, kf_workers.py:688-717) on this host, 1 core, over as many of
    this workload's filters as fit in ``budget_s``."""
    from oracle import ref_kf
    model = ref_kf.CV2 if cfg['model'] == 'cv2' else ref_kf.CV3
    T, k = cfg['T'], cfg['k']
    dt = np.full(T, cfg['dt'])
    nf = min(4096, cfg['B'])
    idx = torch.linspace(0, cfg['B'] - 1, nf).long().to(u.device)
    xs = x0[:, idx].double().cpu().numpy().T
    us = u[:, :, idx].double().cpu().numpy()
    zs = z[:, :, idx].double().cpu().numpy()
    steps = 0
    done = 0
    t0 = time.perf_counter()
    while done < nf and time.perf_counter() - t0 < budget_s:
        ref_kf.run_filter_loop(model, xs[done], model.P0(), dt, us[:, :, done], zs[:, :, done], k)
        steps += T
        done += 1
    el = time.perf_counter() - t0
    return {'value': steps / el, 'unit': 'KF steps/s', 'cores': 1, 'kind': 'port',
            'sample': f'{done} filters x {T} steps of this workload (same synthetic streams), '
                      f'oracle/ref_kf.run_filter_loop, NumPy {np.__version__}, 1 thread, '
                      f'{platform.processor() or platform.machine()}',
            'seconds': round(el, 2)}


def load_traffic(cfg_id, n_gpus):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py),
    if one exists for this config."""
    path = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    try:
        with open(path) as f:
            data = json.load(f)
        rec = data.get(f'config{cfg_id}')
        return rec['bytes_per_launch'] if rec else None
    except (OSError, ValueError, KeyError):
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--config', type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument('--batch', type=int, default=None, help='override filters per GPU')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--ablate', choices=['none', 'no-traj', 'no-logdet', 'no-traj-no-logdet'], default='none',
                    help='diagnostics only: skip an output stream (the JSON line says so)')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.gpus != world and world > 1:
        raise SystemExit(f'--gpus {args.gpus} but WORLD_SIZE={world}')
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))

    import kfmi
    cfg = dict(CONFIGS[args.config])
    if args.batch:
        cfg['B'] = args.batch
    B, T, k, dt = cfg['B'], cfg['T'], cfg['k'], cfg['dt']
    dev = torch.device('cuda', local)

    from kfmi import dist as kdist
    kf = kfmi.BatchedKF(cfg['model'], B, cfg['dtype'], device=local)
    # weak scaling: world*B filters in total; shard r owns a contiguous slice and regenerates
    # its own streams from the counter-based generator (keyed by the global filter index)
    offset, count = kdist.shard_range(world * B, rank, world)
    assert count == B
    x0, u, z = kf.synth(T=T, dt=dt, update_every=k, seed=SEED, filter_offset=offset)
    kf.reset(x0)
    traj = kf.empty(T, kf.n, B)
    logdet = kf.empty(T, B)
    stream = torch.cuda.current_stream(dev)

    out = (None if 'no-traj' in args.ablate else traj, None if 'no-logdet' in args.ablate else logdet)

    def step():
        kf.run(u, z, dt=dt, update_every=k, out=out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for s, e in ev:
        s.record(stream)
        step()
        e.record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev])) if ev else float('nan')

    bad = int((kf.status() != 0).sum().item())
    gather_ms = None
    if dist:
        elapsed, kern_ms, bad = kdist.max_over_ranks([elapsed, kern_ms, bad], dev)
        bad = int(bad)
        # reassemble the final states + logdets of every shard on every rank (RCCL over xGMI);
        # timed separately from the steps: it is a once-per-job reassembly, not the hot path
        xf, _ = kf.state()
        local_out = torch.cat([xf, logdet[-1:]], dim=0).contiguous()
        torch.cuda.synchronize(dev)
        dist.barrier()
        g0 = time.perf_counter()
        gathered = kdist.gather_shards(local_out, world * B)
        torch.cuda.synchronize(dev)
        assert gathered.shape == (kf.n + 1, world * B)
        gather_ms = (time.perf_counter() - g0) * 1e3

    if rank == 0:
        total_steps = world * B * T * args.steps
        value = total_steps / elapsed
        bytes_launch, bytes_step = algorithmic_bytes(cfg)
        achieved = bytes_launch / (kern_ms * 1e-3) / 1e9
        traffic = load_traffic(args.config, world)
        rec = {
            'metric': 'KF predict+update steps/sec (batched filters)',
            'value': value,
            'unit': 'KF steps/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed / max(args.steps, 1) * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': cfg['dtype'],
            'data': 'synthetic (Philox4x32-10 GPS+IMU streams per SURVEY.md §8d, resident in HBM)',
            'config': {'workload': f"BASELINE config {args.config}: {cfg['model']} "
                                   f"({2 * (2 if cfg['model'] == 'cv2' else 3)}-state), "
                                   f"{cfg['dtype']}, B={B} filters/GPU, T={T}, dt={dt}, "
                                   f"GPS update every {k} step(s)",
                       'filters_per_gpu': B, 'time_steps_per_launch': T, 'update_every': k,
                       'parallelism': f'filter shards x{world} (no data-path collective)'},
            'hbm_gbs': achieved,
            'roofline': {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                         'frac': achieved / HBM_PEAK_GBS,
                         'traffic': traffic,
                         'kernel': 'cv_run_kernel', 'kernel_ms': kern_ms,
                         'algorithmic_bytes_per_launch': bytes_launch,
                         'algorithmic_bytes_per_step': bytes_step},
            'failed_filters': bad,
        }
        if args.ablate != 'none':
            rec['ablation'] = args.ablate + ' (diagnostic run: NOT the benchmark workload)'
        if gather_ms is not None:
            rec['allgather_ms'] = gather_ms
        if world == 1 and not args.no_cpu_baseline:
            rec['cpu_baseline'] = cpu_baseline(cfg, x0, u, z)
        else:
            rec['cpu_baseline'] = None
        print(json.dumps(rec), flush=True)
    kf.close()
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
