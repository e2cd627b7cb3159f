"""Benchmark of the batched KF hot path on 1..N MI355X, one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3]
    torchrun --nproc-per-node N bench.py --gpus N ...        (multi-GPU, RCCL)

`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment) starts the N ranks itself
as child processes (torch.distributed.run, rendezvous on 127.0.0.1) before anything touches the
GPU, and exits with their status; the JSON line records `ranks_seen`, and a rank count other
than --gpus is an error.  For N > 1 the final all-gather reassembles every shard's final state,
last log-det and trajectory decimated every --gather-traj-every steps (`allgather`).

One bench *step* = one launch of the hot path over one batch of synthetic input that is
resident in HBM before timing starts.  Consecutive steps continue the same filters (warm
start, like the reference's windowed runs, kf_workers.py:2316-2323) over the same inputs.

Configs (BASELINE.json / SURVEY.md §8d); per GPU (weak scaling: each rank owns B filters):
    1  the reference's own case: ONE filter over a whole drive log — 15-state model,
       run_kalman_filter_full over ~638k merged GPS+IMU events (synthetic log with the shape of
       gps_data.csv + the 200 Hz IMU log: CSV -> kf_ingest -> kf_events_dt + kf_run_stream)
    1ref8  the same log through hw5_2's 8-state filter (hw5_2.py:313-380; the small-state model
       BASELINE config 1 names), one filter
    2  cv2 (4-state/2-meas)  fp32  B=65,536     T=1024 dt=0.1  update every step
    3  cv3 (6-state/3-meas)  fp64  B=1,048,576  T=256  dt=0.1  update every step   [default]
    4  cv3 (6-state/3-meas)  fp32  B=1,048,576  T=256  dt=0.1  update every step   (x8 GPUs)
    5  cv3 (6-state/3-meas)  fp64  B=1,048,576  T=500  dt=0.01 GPS update every 10th step
SURVEY.md §8f rows on the same engine (not BASELINE lines):
    ref15  the reference's 15-state model, fp64, B=1,048,576 filters, T=256 events of a 200 Hz
           IMU + 10 Hz GPS stream (kf_run_events)
    ref15f32  the same in fp32
    bf     the reference's brute-force search: every k-subset (k = 1..25) of n = 25 candidate
           events (kf_workers.py:2311), 2^25 - 1 subsets, one kf_search_combos call; value in
           subsets/s.  N > 1: ONE search split by subset class over the ranks (strong scaling)
    bf40   the same over the reference's n = 40 window (kf_workers_visualizing.py:2293, 2340),
           2^40 - 1 subsets as 256 class searches (--steps 1 --warmup 1: ~20 s a search)
    sched  the rate-decimated greedy scheduled filter, B=1,048,576, rates 10..120 Hz
           (--rate-block 1: every lane its own rate)
Rank 0 prints ONE JSON line.  --dist-backend gloo (rehearsal only) lets N ranks share one GPU
(tools/dist_rehearsal.sh); the real N>1 run is RCCL, one GPU per rank.  --opt NAME=VALUE sets a
kf_set_option on the workload's handle (A/B runs; the library reads no environment).
"""
from __future__ import annotations

import argparse
import json
import math
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
    '1': dict(model='ref15', dtype='f64', B=1, n_gps=30758, n_gps_nan_lead=2735, n_gps_nan=8887, n_imu=616322,
              parallel=True),
    '1seq': dict(model='ref15', dtype='f64', B=1, n_gps=30758, n_gps_nan_lead=2735, n_gps_nan=8887, n_imu=616322,
                 parallel=False),
    # the same log through hw5_2's 8-state planar filter (hw5_2.py:313-380), the model the BASELINE
    # 4-state config restricts: x0 = 0, the first fix at dt = 0, no dt < 0 guard, 2-D fixes
    '1ref8': dict(model='ref8', dtype='f64', B=1, n_gps=30758, n_gps_nan_lead=2735, n_gps_nan=8887, n_imu=616322,
                  parallel=True),
    # hw5_2's run_dead_reckoning_for_IMU (hw5_2.py:382-436) over the same log: the 8-state filter
    # over the IMU events alone (the fixes compacted away on the device), x0 = 0, first dt 0
    '1dr': dict(model='ref8', dtype='f64', B=1, n_gps=30758, n_gps_nan_lead=2735, n_gps_nan=8887, n_imu=616322,
                parallel=True, dead_reckoning=True),
    '2': dict(model='cv2', dtype='f32', B=65536, T=1024, dt=0.1, k=1),
    '3': dict(model='cv3', dtype='f64', B=1048576, T=256, dt=0.1, k=1),
    '4': dict(model='cv3', dtype='f32', B=1048576, T=256, dt=0.1, k=1),
    '5': dict(model='cv3', dtype='f64', B=1048576, T=500, dt=0.01, k=10),
    # config 3 with the axes coupled: correlated GPS noise R and a coupled initial P (a caller's
    # class_args / warm start), so every filter runs the general kernel (cv_run_kernel)
    '3gen': dict(model='cv3', dtype='f64', B=1048576, T=256, dt=0.1, k=1, coupled=True),
    'ref15': dict(model='ref15', dtype='f64', B=1048576, T=256, dt=0.005, k=20),
    'ref15f32': dict(model='ref15', dtype='f32', B=1048576, T=256, dt=0.005, k=20),
    'bf': dict(model='ref15', dtype='f64', n=25, chunk=1 << 22, search=True),
    # the reference's visualizing window (kf_workers_visualizing.py:2293, 2340): 2^40 - 1 subsets as
    # class searches (ref15.search_class_width); one search takes seconds, hence the step counts
    'bf40': dict(model='ref15', dtype='f64', n=40, chunk=1 << 22, search=True, steps=1, warmup=1),
    'bf_subsets': dict(model='ref15', dtype='f64', n=25, chunk=1 << 22, search=False),
    # payload records of 10 doubles carry the event time at rec[9] (KF_OPT_SCHED_REC_TIME; bench.py
    # fills it): 4.52 vs 4.82 ms in-process with 12-double records (profiles/r04_ab1/ab_sched.log),
    # 4.18 vs 4.53 ms for 10 against 12 doubles (profiles/r04_pmc/sched_diag/ab.log)
    'sched': dict(model='ref15', dtype='f64', B=1048576, T=256, dt=0.005, k=20,
                  rates=(10, 20, 30, 40, 50, 60, 70, 80, 90, 100, 110, 120), opts={'sched_rec_time': 1}),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
SEED = 20251015
# config 3gen's coupling: GPS noise correlated across the axes, and an initial covariance with
# 0.2 correlation between axes and 0.1 between each position and the velocities
R_COUPLED = [[3.0, 1.0, 0.5], [1.0, 3.0, 1.0], [0.5, 1.0, 3.0]]


def coupled_p0(d=3):
    """The reference P0 (kf_workers.py:651) with cross-axis correlation (SPD)."""
    sd = np.sqrt(np.r_[[1e4] * d, [1e3] * d])
    C = np.full((d, d), 0.2) + 0.8 * np.eye(d)
    corr = np.block([[C, 0.1 * np.eye(d)], [0.1 * np.eye(d), C]])
    return corr * np.outer(sd, sd)


def cv_params(cfg):
    """kf_params of the config's handle: the reference constants, or R_COUPLED for 3gen."""
    if not cfg.get('coupled'):
        return None
    from kfmi.engine import default_params
    p = default_params(cfg['model'])
    for i in range(3):
        for j in range(3):
            p.r[i * 3 + j] = R_COUPLED[i][j]
    return p


def block_kernel_in_use(cfg):
    """kf_run takes cv_block_kernel for the bench's handles (diagonal R, P = P0) unless the
    handle's cv_kernel option forces the general kernel or the config couples the axes."""
    return cfg.get('opts', {}).get('cv_kernel', 'auto') not in ('general', 1) and not cfg.get('coupled')


def algorithmic_bytes(cfg, block=None):
    """Bytes one kf_run launch must move: per filter per step c control values
    read, m measurement values read on update steps, n state values + 1 logdet written; per
    filter per launch (x, P) loaded and stored once and status read + written.  The block
    kernel keeps P's 3 d per-axis entries (the rest are exact zeros it never touches)."""
    d = 2 if cfg['model'] == 'cv2' else 3
    n, m, c = 2 * d, d, d
    w = 8 if cfg['dtype'] == 'f64' else 4
    T, k, B = cfg['T'], cfg['k'], cfg['B']
    U = T // k
    block = block_kernel_in_use(cfg) if block is None else block
    p_entries = 3 * d if block else n * (n + 1) // 2
    per_filter = T * (c + n + 1) * w + U * m * w + 2 * (n + p_entries) * w + 2 * 4
    return per_filter * B, per_filter / T


def ref15_algorithmic_bytes(cfg):
    """Bytes one kf_run_events launch must move for the 15-state model: per filter per event
    etype 1 + dt 8 (always f64) + payload 9 w read, traj 6 w + logdet w written (w = 8 in f64, 4
    in f32); per filter per launch the state (15 + 27 block rows) loaded and stored and status
    read + written."""
    T, B = cfg['T'], cfg['B']
    w = 8 if cfg['dtype'] == 'f64' else 4
    per_filter = T * (1 + 8 + 9 * w + 6 * w + w) + 2 * (15 + 27) * w + 8
    return per_filter * B, per_filter / T


def host_cpu():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def load_traffic(cfg_id, algorithmic=None):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (tools/pmc_traffic.py);
    with ``algorithmic``, only if the summary was measured on a launch of those algorithmic bytes
    (the same variant of the workload)."""
    try:
        with open(os.path.join(ROOT, 'profiles', 'pmc_traffic.json')) as f:
            rec = json.load(f).get(f'config{cfg_id}')
        if rec and algorithmic is not None and rec.get('algorithmic_bytes_per_launch') != algorithmic:
            return None
        return rec['bytes_per_launch'] if rec else None
    except (OSError, ValueError, KeyError):
        return None


def load_valu(cfg_id):
    """VALU issue of the dominant kernel from the committed rocprofv3 SQ-counter summary
    (tools/pmc_valu.sh; SURVEY.md §8d asks for the VALU fraction beside the HBM roofline)."""
    try:
        with open(os.path.join(ROOT, 'profiles', 'pmc_valu.json')) as f:
            rec = json.load(f).get(f'config{cfg_id}')
        return None if rec is None else {
            'issue_frac': rec['valu_issue_frac'], 'valu_insts_per_wave_step': rec['valu_per_wave_step'],
            'issue_stall_frac_of_wave_cycles': rec['wave_cycles_issue_stall_frac'],
            'source': 'profiles/pmc_valu.json (SQ_INSTS_VALU x 4 cycles / (kernel time x 2.4 GHz x 1024 SIMDs))'}
    except (OSError, ValueError, KeyError):
        return None


# --------------------------------------------------------------------------------------------
# Workloads: each returns dict(step, units, bytes, kernel, cpu, gather, desc, extra, ...)
# --------------------------------------------------------------------------------------------

def cv_workload(cfg_id, cfg, args, rank, world, dev):
    import kfmi
    from kfmi import dist as kdist
    B, T, k, dt = cfg['B'], cfg['T'], cfg['k'], cfg['dt']
    kf = kfmi.BatchedKF(cfg['model'], B, cfg['dtype'], device=dev.index, params=cv_params(cfg),
                        options=cfg.get('opts'))
    # weak scaling: world*B filters in total; shard r owns a contiguous slice and regenerates
    # its own streams from the counter-based generator (keyed by the global filter index)
    offset, count = kdist.shard_range(world * B, rank, world)
    assert count == B
    x0, u, z = kf.synth(T=T, dt=dt, update_every=k, seed=SEED, filter_offset=offset)
    kf.reset(x0)
    P0 = coupled_p0() if cfg.get('coupled') else None
    if P0 is not None:
        iu = np.triu_indices(P0.shape[0])  # the handle's packed upper triangle, row-major (include/kf.h)
        rows = torch.as_tensor(P0[iu], dtype=kf.torch_dtype, device=dev)
        kf.set_state(x0, rows[:, None].expand(-1, B).contiguous())
    traj = kf.empty(T, kf.n, B)
    logdet = kf.empty(T, B)
    out = (None if 'no-traj' in args.ablate else traj, None if 'no-logdet' in args.ablate else logdet)

    def step():
        kf.run(u, z, dt=dt, update_every=k, out=out)

    def gather_payload():
        xf, _ = kf.state()
        return xf, logdet[-1], (None if out[0] is None else traj)

    def cpu():
        """The reference's per-filter step restated in C (oracle/cpu_kf.c: dense matrices in the
        reference's op order, OpenMP over filters) on this host's allotted cores for ~10 s of
        this workload; plus the NumPy reference loop (oracle/ref_kf.run_filter_loop) on 1 core."""
        from oracle import cpu_kf, numpy_pool
        d = 2 if cfg['model'] == 'cv2' else 3
        nth = cpu_kf.threads()
        P0h = coupled_p0() if cfg.get('coupled') else np.diag([kf.params.p0_pos] * d + [kf.params.p0_vel] * d)
        Rh = np.array(R_COUPLED) if cfg.get('coupled') else None
        nf = min(B, 1 << 17)   # ~10 s on 16 cores; the loop below stops at 10 s regardless
        idx = torch.linspace(0, B - 1, nf).long().to(u.device)
        xs = x0[:, idx].double().cpu().numpy()
        us = u[:, :, idx].double().cpu().numpy()
        zs = z[:, :, idx].double().cpu().numpy()
        done, t0 = 0, time.perf_counter()
        chunk = max(nth * 64, 256)
        while done < nf and time.perf_counter() - t0 < 10.0:
            hi = min(nf, done + chunk)
            cpu_kf.cv_run(d, xs, P0h, dt, us, zs, k, filters=(done, hi), nthreads=nth, R=Rh)
            done = hi
        el = time.perf_counter() - t0
        # the NumPy reference loop on every allotted core (the reference's Pool fan-out), ~3 s:
        # each worker its own slice of the sampled filters
        per = min(nf // nth, -(-130000 * 3 // T))
        shards = [dict(d=d, x0=xs[:, r * per:(r + 1) * per], P0=P0h, R=Rh, dt=dt, k=k, n=per,
                       u=us[:, :, r * per:(r + 1) * per], z=zs[:, :, r * per:(r + 1) * per]) for r in range(nth)]
        npl = numpy_pool.run('cv', shards, seconds=3.0)
        return {'value': done * T / el, 'unit': 'KF steps/s', 'cores': nth, 'kind': 'port',
                'sample': f'{done} filters x {T} steps of this workload (same synthetic streams) through '
                          f'oracle/cpu_kf.c (the reference step, dense, C -O3 OpenMP) on {nth} threads, {host_cpu()}',
                'seconds': round(el, 2),
                'numpy_reference_loop': dict(npl, sample=f"{npl['filters']} filters of this workload, "
                                             f"oracle/ref_kf.run_filter_loop (the reference's per-step NumPy calls) "
                                             f"in a spawn Pool of {npl['cores']} processes, one BLAS thread each, "
                                             f"NumPy {np.__version__}")}

    def pcie(reps=3):
        """PCIe-inclusive rate: the inputs start in pinned host memory and the
        trajectory + log-det come back to pinned host memory; H2D, the launch and D2H are timed
        together on the engine's stream.  Never `value`: `value` is HBM-resident."""
        hu = u.cpu().pin_memory() if u is not None else None
        hz = z.cpu().pin_memory()
        ht, hl = torch.empty(traj.shape, dtype=traj.dtype).pin_memory(), torch.empty(logdet.shape, dtype=logdet.dtype).pin_memory()
        times = []
        for _ in range(reps + 1):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            if u is not None:   # the engine launches on torch's current stream
                u.copy_(hu, non_blocking=True)
            z.copy_(hz, non_blocking=True)
            kf.run(u, z, dt=dt, update_every=k, out=(traj, logdet))
            ht.copy_(traj, non_blocking=True)
            hl.copy_(logdet, non_blocking=True)
            torch.cuda.synchronize(dev)
            times.append(time.perf_counter() - t0)
        el = min(times[1:])
        # the product's host-buffer path: kf.run_host pipelines 8 time chunks on three streams
        # (H2D of chunk i+1 | the launch on chunk i | D2H of chunk i-1)
        nch = 8
        ptimes = []
        for _ in range(reps + 1):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            kf.run_host(hu if hu is not None else u.cpu(), hz, dt=dt, update_every=k, chunks=nch, traj=ht, logdet=hl)
            torch.cuda.synchronize(dev)
            ptimes.append(time.perf_counter() - t0)
        pel = min(ptimes[1:])
        h2d = (hu.numel() * hu.element_size() if hu is not None else 0) + hz.numel() * hz.element_size()
        d2h = ht.numel() * ht.element_size() + hl.numel() * hl.element_size()
        return {'value': B * T / el, 'unit': 'KF steps/s', 'ms_per_launch': el * 1e3,
                'h2d_bytes': h2d, 'd2h_bytes': d2h, 'link_gbs': (h2d + d2h) / el / 1e9,
                'note': 'inputs u,z from pinned host, trajectory+logdet to pinned host, '
                        'serial on one stream (no overlap), best of %d' % reps,
                'pipelined': {'value': B * T / pel, 'ms_per_launch': pel * 1e3, 'chunks': nch,
                              'link_gbs': (h2d + d2h) / pel / 1e9,
                              'note': 'BatchedKF.run_host: time chunks on 3 streams, H2D | launch | D2H overlapped'}}

    def per_step(reps=2):
        """The reference's call shape: T steps of BatchedKF.predict(dt, u[t]) then
        BatchedKF.update(z[t]) (its log-det returned).  By default kf_predict is held back and
        runs fused with the next kf_update (one state round trip per step, plus a copy of u);
        the handle option predict='eager' launches each call on its own (two round trips).
        Against kf_run's fused launch on the same streams.  Never `value`."""
        def loop(mode):
            kf.set_option('predict', mode)
            try:
                kf.reset(x0)
                times = []
                for _ in range(reps + 1):
                    torch.cuda.synchronize(dev)
                    t0 = time.perf_counter()
                    for t in range(T):
                        kf.predict(dt, u=u[t])
                        if (t + 1) % k == 0:
                            kf.update(z[(t + 1) // k - 1])
                    torch.cuda.synchronize(dev)
                    times.append(time.perf_counter() - t0)
                return min(times[1:])
            finally:
                kf.set_option('predict', cfg.get('opts', {}).get('predict', 'auto'))

        el = loop('deferred')
        el_eager = loop('eager')
        if k != 1:
            # the async shape: k predicts per update; a predict that follows a predict runs at
            # once, so only the last predict before each update is fused with it
            return {'value': B * T / el, 'unit': 'KF predict-steps/s', 'ms_per_step': el / T * 1e3,
                    'update_every': k, 'note': 'predict every step, update every %d-th, through BatchedKF; '
                    'best of %d' % (k, reps),
                    'eager': {'value': B * T / el_eager, 'ms_per_step': el_eager / T * 1e3,
                              'note': "option predict='eager': one kernel per call"}}
        # the same steps as T launches of kf_run with T = 1 (predict + update fused, one state
        # round trip per step, trajectory and log-det rows written)
        kf.reset(x0)
        times1 = []
        for _ in range(reps + 1):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for t in range(T):
                kf.run(u[t:t + 1], z[t:t + 1], dt=dt, out=(traj[t:t + 1], logdet[t:t + 1]))
            torch.cuda.synchronize(dev)
            times1.append(time.perf_counter() - t0)
        el1 = min(times1[1:])
        w = 8 if cfg['dtype'] == 'f64' else 4
        # the per-axis blocks of P (block-diagonal handle: the calls move only them)
        nt = 3 * d
        # deferred: u copied (in + out), then state + u + z in, state + log-det out
        nbytes = B * T * w * ((kf.n + nt) * 2 + 4 * d + 1)
        # eager: predict state + u in, state out; update state + z in, state + log-det out
        nbytes_eager = B * T * w * ((kf.n + nt) * 4 + 2 * d + 1)
        return {'value': B * T / el, 'unit': 'KF steps/s', 'ms_per_step': el / T * 1e3,
                'gbs': nbytes / el / 1e9, 'launches': T, 'copies': T,
                'note': 'kf_predict + kf_update per time step through BatchedKF (no trajectory kept), the '
                        'predict held back and fused into the update; best of %d' % reps,
                'eager': {'value': B * T / el_eager, 'ms_per_step': el_eager / T * 1e3,
                          'gbs': nbytes_eager / el_eager / 1e9, 'launches': 2 * T,
                          'note': "option predict='eager': one kernel per call"},
                'run_t1': {'value': B * T / el1, 'ms_per_step': el1 / T * 1e3, 'launches': T,
                           'note': 'BatchedKF.run on one step at a time (kf_run, T = 1: predict + update fused)'}}

    def probe(reps):
        """The access pattern's ceiling on these very buffers (tools/probes/pattern_probe.hip:
        the block kernel's loads and stores through the same ring, the arithmetic reduced to a
        sum): GB/s of its stream bytes, HIP events on the engine's stream.  None without the
        probe library (a diagnostic, built by __graft_entry__.build())."""
        import ctypes
        path = os.path.join(ROOT, 'tools', 'probes', 'libpattern_probe.so')
        if not os.path.exists(path):
            return None
        lib = ctypes.CDLL(path)
        lib.kfprobe_pattern.restype = ctypes.c_int
        lib.kfprobe_pattern.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 4 + \
            [ctypes.c_int64, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        stream = torch.cuda.current_stream(dev)
        run = lambda: lib.kfprobe_pattern(d, int(cfg['dtype'] == 'f64'), u.data_ptr(), z.data_ptr(), traj.data_ptr(),
                                          logdet.data_ptr(), B, T, k, ctypes.c_void_p(stream.cuda_stream))
        for _ in range(3):
            if run() != 0:
                return None
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for s, e in ev:
            s.record(stream)
            run()
            e.record(stream)
        torch.cuda.synchronize(dev)
        ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
        w = 8 if cfg['dtype'] == 'f64' else 4
        nbytes = B * (T * (d + 2 * d + 1) * w + (T // k) * d * w)
        return {'gbs': nbytes / (ms * 1e-3) / 1e9, 'ms': ms, 'bytes': nbytes,
                'desc': 'tools/probes/pattern_probe.hip: the bench kernel\'s loads and stores (same ring, same '
                        'rows, same buffers) with the arithmetic reduced to a sum'}

    d = 2 if cfg['model'] == 'cv2' else 3
    bytes_launch, bytes_step = algorithmic_bytes(cfg)
    kernel = 'cv_block_kernel' if block_kernel_in_use(cfg) else 'cv_run_kernel'
    # the committed PMC summaries hold each row's default kernel (the 3gen row's is the general one)
    pmc = kernel == ('cv_run_kernel' if cfg.get('coupled') else 'cv_block_kernel')
    return dict(step=step, units=B * T, bytes=bytes_launch, bytes_per_unit=bytes_step, kernel=kernel,
                traffic=load_traffic(cfg_id) if pmc else None, cpu=cpu,
                valu=load_valu(cfg_id) if pmc else None,
                gather=gather_payload, kf=kf, pcie=pcie, probe=probe, per_step=per_step, update_every=k,
                desc=f"BASELINE config {cfg_id}: {cfg['model']} ({2 * d}-state/{d}-meas), {cfg['dtype']}, "
                     f"B={B} filters/GPU, T={T}, dt={dt}, GPS update every {k} step(s)",
                extra={'filters_per_gpu': B, 'time_steps_per_launch': T, 'update_every': k})


def ref15_streams(B, T, dt, k, seed, dev, dtype=torch.float64):
    """The ref15 rows' event streams (also the bench-size parity tests'): every k-th event a GPS
    fix, the others 200 Hz IMU samples, dt fixed; torch's Philox draws on the device.  Returns
    etype [T, B] u8, dt [T, B] f64, payload [T, 9, B] in ``dtype`` (fp32: the f64 draws rounded
    once)."""
    g = torch.Generator(device=dev).manual_seed(seed)
    etype = torch.ones(T, B, dtype=torch.uint8, device=dev)
    etype[k - 1::k] = 0
    dts = torch.full((T, B), dt, dtype=torch.float64, device=dev)
    pay = torch.randn(T, 9, B, dtype=torch.float64, device=dev, generator=g)
    pay[:, 0:3] *= 0.05   # roll/pitch/yaw
    pay[:, 3:6] *= 0.01   # angular rates
    pay[:, 6:9] *= 0.3    # accelerations
    gps = (etype == 0)[:, None, :]
    pay[:, 0:3] = torch.where(gps, pay[:, 0:3] * 60.0, pay[:, 0:3])  # GPS fixes within ~3 m
    return etype, dts, pay.to(dtype)


SCHED_T0 = 1697739278.761565


def sched_streams(B, T, dt, k, rates, rate_block, seed, dev):
    """The sched row's streams (also its bench-size parity test's): 200 Hz events with +-0.5 ms
    jitter per filter and event, every k-th a GPS fix; one processing rate per ``rate_block``
    consecutive filters.  Returns t [T, B], etype [T, B], payload [T, 9, B], freq [B], prev [B]."""
    g = torch.Generator(device=dev).manual_seed(seed)
    t0 = SCHED_T0
    etype = torch.ones(T, B, dtype=torch.uint8, device=dev)
    etype[k - 1::k] = 0
    tt = (t0 + dt * torch.arange(1, T + 1, dtype=torch.float64, device=dev)[:, None]
          + 5e-4 * (torch.rand(T, B, dtype=torch.float64, device=dev, generator=g) - 0.5))
    pay = torch.randn(T, 9, B, dtype=torch.float64, device=dev, generator=g)
    pay[:, 0:3] *= 0.05
    pay[:, 3:6] *= 0.01
    pay[:, 6:9] *= 0.3
    gps = (etype == 0)[:, None, :]
    pay[:, 0:3] = torch.where(gps, pay[:, 0:3] * 60.0, pay[:, 0:3])
    rates = torch.tensor(rates, dtype=torch.float64, device=dev)
    freq = rates[(torch.arange(B, device=dev) // max(1, rate_block)) % len(rates)].contiguous()
    prev = torch.full((B,), t0, dtype=torch.float64, device=dev)
    return tt, etype, pay, freq, prev


BF_T0 = 1697739552.3362827


def bf_events(n, seed=SEED):
    """The bf row's n candidate events after a warm start (also its parity test's): 200 Hz IMU
    samples with a GPS fix every 20th, a block-diagonal warm-start covariance of the shape the
    reference's own runs produce.  Returns (ev [n, 11] (t, type, payload), init (x, blocks), Pw,
    t0, t_end)."""
    from kfmi import ref15 as r15
    rng = np.random.default_rng(seed)
    t0 = BF_T0
    ev = np.zeros((n, 11))
    ev[:, 0] = t0 + 0.005 * np.arange(1, n + 1)
    ev[:, 1] = 1
    ev[::20, 1] = 0          # GPS fixes among the IMU samples (10 Hz vs 200 Hz)
    ev[:, 2:5] = rng.normal(0, 0.05, (n, 3))
    ev[:, 5:8] = rng.normal(0, 0.01, (n, 3))
    ev[:, 8:11] = rng.normal(0, 0.3, (n, 3))
    gps = ev[:, 1] == 0
    ev[gps, 2:5] = rng.normal(0, 3, (int(gps.sum()), 3))
    Pw = np.diag([0.9, 0.9, 0.9, 0.02, 0.02, 0.02, 0.5, 0.5, 0.5, 0.05, 0.05, 0.05, 20.0, 20.0, 20.0])
    init = np.concatenate([np.zeros(15), r15.to_blocks(Pw)])
    return ev, init, Pw, t0, t0 + 0.005 * (n + 1)


def ref15_workload(cfg, args, rank, world, dev):
    """The reference's 15-state model on 200 Hz IMU + 10 Hz GPS event streams (every k-th event a
    GPS fix), one stream per filter, synthetic (torch RNG on the device; the reference's
    imu_data.csv is absent)."""
    import kfmi
    from kfmi import _lib
    from kfmi.engine import _ptr
    B, T, dt, k = cfg['B'], cfg['T'], cfg['dt'], cfg['k']
    kf = kfmi.BatchedKF('ref15', B, cfg['dtype'], device=dev.index, options=cfg.get('opts'))
    etype, dts, pay = ref15_streams(B, T, dt, k, SEED + rank, dev, kf.torch_dtype)
    traj = kf.empty(T, 6, B)
    logdet = kf.empty(T, B)

    def step():
        _lib.check(_lib.lib().kf_run_events(kf.handle, T, _ptr(etype), _ptr(dts), _ptr(pay), _ptr(traj),
                                            None, _ptr(logdet), None, 0, 0.0, kf._stream()))

    def gather_payload():
        xf, _ = kf.state()
        return xf, logdet[-1], traj

    def cpu():
        """The reference's dense 15x15 event step restated in C (oracle/cpu_kf.c) on this host's
        allotted cores for ~10 s of these streams; plus the NumPy step (oracle/ref_kf.step15 +
        slogdet, kf_workers.py:688-717) on 1 core."""
        from oracle import cpu_kf, ref_kf
        nth = cpu_kf.threads()
        nf = min(B, 1 << 15)
        et = etype[:, :nf].cpu().numpy()
        dd = dts[:, :nf].cpu().numpy()
        pa = pay[:, :, :nf].double().cpu().numpy()
        x0 = np.zeros((15, nf))
        done, t0 = 0, time.perf_counter()
        chunk = max(nth * 16, 64)
        while done < nf and time.perf_counter() - t0 < 10.0:
            hi = min(nf, done + chunk)
            cpu_kf.ref15_events(et, dd, pa, x0, ref_kf.P0_REF15, filters=(done, hi), nthreads=nth)
            done = hi
        el = time.perf_counter() - t0
        from oracle import numpy_pool
        per = min(nf // nth, -(-60000 * 3 // T))
        shards = [dict(et=et[:, r * per:(r + 1) * per], dt=dd[:, r * per:(r + 1) * per],
                       pay=pa[:, :, r * per:(r + 1) * per], n=per) for r in range(nth)]
        npl = numpy_pool.run('ref15', shards, seconds=3.0)
        return {'value': done * T / el, 'unit': 'KF events/s', 'cores': nth, 'kind': 'port',
                'sample': f'{done} filters x {T} events of these streams through oracle/cpu_kf.c (the reference '
                          f'step, dense 15x15, C -O3 OpenMP) on {nth} threads, {host_cpu()}',
                'seconds': round(el, 2),
                'numpy_reference_loop': dict(npl, sample=f"{npl['filters']} filters of these streams, "
                                             f"oracle/ref_kf.step15 + slogdet (kf_workers.py:688-717) in a spawn Pool "
                                             f"of {npl['cores']} processes, NumPy {np.__version__}")}

    bytes_launch, bytes_event = ref15_algorithmic_bytes(cfg)

    def probe(reps):
        """ref_events_lds_kernel's access pattern on these event streams and output rows
        (tools/probes/pattern_probe.hip: the same LDS-DMA loads, waits and row stores, the event
        arithmetic reduced to a sum; scratch state rows, so the handle is untouched)."""
        import ctypes
        path = os.path.join(ROOT, 'tools', 'probes', 'libpattern_probe.so')
        if not os.path.exists(path) or B % 64:
            return None
        lib = ctypes.CDLL(path)
        if not hasattr(lib, 'kfprobe_ref_pattern'):
            return None
        lib.kfprobe_ref_pattern.restype = ctypes.c_int
        lib.kfprobe_ref_pattern.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 7 + \
            [ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
        xs, Ps = kf.empty(15, B), kf.empty(27, B)
        xs.zero_()
        Ps.zero_()
        stream = torch.cuda.current_stream(dev)
        run = lambda: lib.kfprobe_ref_pattern(int(cfg['dtype'] == 'f64'), etype.data_ptr(), dts.data_ptr(), pay.data_ptr(), xs.data_ptr(),
                                              Ps.data_ptr(), traj.data_ptr(), logdet.data_ptr(), B, T,
                                              ctypes.c_void_p(stream.cuda_stream))
        for _ in range(3):
            if run() != 0:
                return None
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for s_, e_ in ev:
            s_.record(stream)
            run()
            e_.record(stream)
        torch.cuda.synchronize(dev)
        ms = float(np.mean([s_.elapsed_time(e_) for s_, e_ in ev]))
        nbytes = bytes_launch - 8 * B  # the probe has no status row
        del xs, Ps
        return {'gbs': nbytes / (ms * 1e-3) / 1e9, 'ms': ms, 'bytes': nbytes,
                'desc': 'tools/probes/pattern_probe.hip: ref_events_lds_kernel\'s LDS-DMA event loads, waits and '
                        'row stores on the same buffers, the event arithmetic reduced to a sum'}

    return dict(step=step, units=B * T, bytes=bytes_launch, bytes_per_unit=bytes_event, probe=probe,
                kernel='ref_events_lds_kernel',
                traffic=load_traffic('ref15' if cfg['dtype'] == 'f64' else 'ref15f32', bytes_launch),
                valu=load_valu('ref15') if cfg['dtype'] == 'f64' else None, cpu=cpu, gather=gather_payload, kf=kf,
                desc=f'SURVEY 8f row 2: reference 15-state model (kf_workers.py:493-614), {cfg["dtype"]}, B={B} filters/GPU, '
                     f'T={T} events (IMU 200 Hz, GPS fix every {k}th event), dt={dt}',
                extra={'filters_per_gpu': B, 'events_per_launch': T})


def synth_log(cfg, root, seed=SEED):
    """CSV logs with the reference drive's shape (gps_data.csv: 30 758 rows at ~10 Hz, 2 735
    leading and 8 887 total no-fix rows; the IMU log at 200 Hz, 616 322 rows = the 638 193
    merged events of KF_SensorFusion.ipynb:1960 minus the 21 871 fixes).  Columns as hw5_1.py
    writes them.  Synthetic: the reference's own log is location data and its IMU log is absent."""
    rng = np.random.default_rng(seed)
    ng, ni = cfg['n_gps'], cfg['n_imu']
    t0g, t0i = 1697739278.761565, 1697739278.7381794
    tg = t0g + np.cumsum(np.r_[0.0, rng.uniform(0.095, 0.105, ng - 1)])
    ti = t0i + np.cumsum(np.r_[0.0, rng.uniform(0.00499, 0.00501, ni - 1)])
    lat = 40.0 + np.cumsum(rng.normal(3e-6, 3e-7, ng))
    lon = -75.0 + np.cumsum(rng.normal(2e-6, 3e-7, ng))
    alt = 12.5 + np.cumsum(rng.normal(0, 0.05, ng))
    gps = np.stack([tg, lat, lon, alt], 1)
    nan_rows = np.r_[np.arange(cfg['n_gps_nan_lead']),
                     rng.choice(np.arange(cfg['n_gps_nan_lead'], ng), cfg['n_gps_nan'] - cfg['n_gps_nan_lead'],
                                replace=False)]
    gps[nan_rows, 1:] = np.nan
    yaw = np.cumsum(rng.normal(0, 2e-4, ni))
    r, p = rng.normal(0, 0.02, ni), rng.normal(-0.05, 0.01, ni)
    cr, sr, cp, sp, cy, sy = np.cos(r / 2), np.sin(r / 2), np.cos(p / 2), np.sin(p / 2), np.cos(yaw / 2), np.sin(yaw / 2)
    q = np.stack([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy,
                  cr * cp * cy + sr * sp * sy], 1)
    w = rng.normal([-0.0017, -0.0075, -0.036], 0.01, (ni, 3))
    a = rng.normal([-0.52, 0.0086, -9.53], 0.3, (ni, 3))
    imu = np.concatenate([ti[:, None], q, w, a], 1)
    gp, ip = os.path.join(root, 'gps_log.csv'), os.path.join(root, 'imu_log.csv')
    np.savetxt(gp, gps, fmt='%.17g', delimiter=',', header='time,latitude,longitude,altitude', comments='')
    np.savetxt(ip, imu, fmt='%.17g', delimiter=',', comments='',
               header='time,orientation_x,orientation_y,orientation_z,orientation_w,angular_velocity_x,'
                      'angular_velocity_y,angular_velocity_z,linear_acceleration_x,linear_acceleration_y,'
                      'linear_acceleration_z')
    return gp, ip


def log_workload(cfg, args, rank, world, dev):
    """BASELINE config 1: ONE filter over a whole drive log — the reference's own use.  With
    model ref15 it is run_kalman_filter_full (kf_workers.py:623-728: x0 = the first fix, which is
    processed again at dt = 0, dt < 0 events skipped); with ref8 (--config 1ref8) hw5_2's
    run_kalman_filter (hw5_2.py:313-380: x0 = 0, fixes without altitude, no dt < 0 guard).
    Ingest runs once, outside the timed region (reported separately); a step is the device dt
    pass + one kf_run_stream (or kf_run_events_seq) over every event."""
    import tempfile
    import kfmi
    from kfmi import _lib, ingest
    from kfmi.engine import _ptr
    ref8 = cfg['model'] == 'ref8'
    n_state, width = (8, 3) if ref8 else (15, 6)
    root = tempfile.mkdtemp(prefix='kfmi_log_')
    gp, ip = synth_log(cfg, root)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    gcols, icols = ingest.read_csv(gp, 4), ingest.read_csv(ip, 11)
    t1 = time.perf_counter()
    stream = ingest.ingest_arrays(gcols, icols, with_altitude=not ref8, device=dev.index)
    torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    # the first call also loads the library's code objects and warms torch's allocator: the
    # ingest itself is the second call's time (both reported)
    stream = ingest.ingest_arrays(gcols, icols, with_altitude=not ref8, device=dev.index)
    torch.cuda.synchronize(dev)
    t3 = time.perf_counter()
    N = len(stream)
    if cfg.get('dead_reckoning'):
        return dead_reckoning_workload(cfg, args, dev, stream, (t1 - t0, t2 - t1, t3 - t2))
    first = int(torch.nonzero(stream.etype == _lib.KF_EVENT_GPS)[0, 0])
    T = N - first
    t_ev = stream.t[first:].contiguous()
    e_ev = stream.etype[first:].contiguous()
    pay = stream.payload[first:].contiguous()
    x0 = torch.zeros(n_state, 1, dtype=torch.float64, device=dev)
    if not ref8:
        x0[0:3, 0] = pay[0, 0:3]      # kf_workers.py:655-659 (hw5_2 starts from 0, hw5_2.py:316)
    rule = _lib.KF_DT_RAW if ref8 else _lib.KF_DT_FULL
    kf = kfmi.BatchedKF(cfg['model'], 1, 'f64', device=dev.index, options=cfg.get('opts'))
    dt = torch.empty(T, dtype=torch.float64, device=dev)
    et = torch.empty(T, dtype=torch.uint8, device=dev)
    traj = kf.empty(T, width, 1)
    logdet = kf.empty(T, 1)
    prev0 = float(t_ev[0])

    stream_check = {}
    graph = {}

    def launches():
        L = _lib.lib()  # looked up per step: tools/ab_inproc.py swaps libraries between launches
        kf.reset(x0)
        _lib.check(L.kf_events_dt(T, _ptr(t_ev), _ptr(e_ev), prev0, rule, _ptr(dt), _ptr(et), kf._stream()))
        if cfg['parallel']:
            # time-parallel (kf_run_stream): chunks of the log as filters, checked on the device
            _lib.check(L.kf_run_stream(kf.handle, T, _ptr(et), _ptr(dt), _ptr(pay), _ptr(traj), None, _ptr(logdet),
                                       None, 0, -1, kf._stream()))
            if not stream_check:  # first (warm-up) step: record the device checks (synchronises)
                stream_check.update(kf.stream_check())
            return
        # the single filter (kf_run_events would route a one-filter log through kf_run_stream)
        _lib.check(L.kf_run_events_seq(kf.handle, T, _ptr(et), _ptr(dt), _ptr(pay), _ptr(traj), None, _ptr(logdet),
                                       None, 0, 0.0, kf._stream()))

    def step():
        """With --graph the step's launches (reset, dt pass, kf_run_stream's kernels: 9 in all)
        are captured into a hipGraph after the first, eager step and replayed: the C ABI launches
        never synchronise or allocate after their first call, so they capture as they are.
        Measured: 0.252 ms per step replayed vs 0.246 eager (profiles/r02_timeparallel/), so
        eager launches are the default."""
        if not cfg['parallel'] or not getattr(args, 'graph', False) or not stream_check:
            launches()
            return
        if 'g' not in graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                launches()
            graph['g'] = g
        graph['g'].replay()

    def cpu():
        """One filter cannot use more than one core: the reference's dense event step restated in
        C (oracle/cpu_kf.c) over the whole log from the first fix (the driver's dt rule applied
        on the host), 1 thread; plus the NumPy reference loop (oracle/ref_kf.
        run_kalman_filter_full / run_kalman_filter_8state) over the first events, 1 core, ~3 s."""
        from oracle import cpu_kf, ref_kf
        from kfmi.kf_workers import EventList
        h = stream.host()
        t_h, e_h, p_h = h['t'][first:], h['etype'][first:].copy(), h['payload'][first:]
        prev = np.r_[t_h[0], t_h[:-1]]
        d_h = t_h - prev
        if not ref8:
            e_h[d_h < 0] = 255                                # kf_workers.py:683-685
        x0h = x0.cpu().numpy()
        n_c = min(T, 1 << 20)
        port = cpu_kf.ref8_events if ref8 else cpu_kf.ref15_events
        ts = time.perf_counter()
        port(e_h[:n_c, None], d_h[:n_c, None], p_h[:n_c, :, None], x0h, ref_kf.P0_REF8 if ref8 else ref_kf.P0_REF15,
             nthreads=1)
        el = time.perf_counter() - ts
        ev = EventList(stream)
        n = 2000
        while True:
            lst = ev[first:first + n]
            t1 = time.perf_counter()
            if ref8:
                st, _ = ref_kf.run_kalman_filter_8state(lst)
            else:
                st, _, _, _ = ref_kf.run_kalman_filter_full(lst, 0, n)
            el_np = time.perf_counter() - t1
            if el_np > 3.0 or n >= T:
                break
            n = min(T, n * 4)
        driver = 'hw5_2.run_kalman_filter' if ref8 else 'run_kalman_filter_full'
        np_fn = 'run_kalman_filter_8state' if ref8 else 'run_kalman_filter_full'
        return {'value': n_c / el, 'unit': 'KF events/s', 'cores': 1, 'kind': 'port',
                'sample': f'{driver} over {n_c} events of this log (from the first fix) through '
                          f'oracle/cpu_kf.c (the reference step, dense {n_state}x{n_state}, C -O3), 1 thread (one '
                          f'filter), {host_cpu()}', 'seconds': round(el, 2),
                'numpy_reference_loop': {'value': (len(st) - 1) / el_np, 'cores': 1,
                                         'sample': f'{len(st) - 1} events, oracle/ref_kf.{np_fn}, '
                                                   f'NumPy {np.__version__}'}}

    # dt pass (t, etype in; dt, etype out) + filter (etype, dt, payload in; traj, logdet out)
    per_event = 1 + 8 + 8 + 72 + 1 + 8 + 8 * width + 8
    model_desc = (f'hw5_2.run_kalman_filter (hw5_2.py:313-380), the 8-state planar model' if ref8 else
                  'run_kalman_filter_full (kf_workers.py:623-728), the 15-state model')
    desc = (f'BASELINE config 1: ONE filter, {model_desc}, over a whole drive log, {N} merged events '
            f'({stream.n_fixes} fixes + {stream.n_imu} IMU at 200 Hz), f64; ')
    extra = {'events': N, 'events_filtered': T, 'csv_parse_ms': (t1 - t0) * 1e3, 'kf_ingest_ms': (t3 - t2) * 1e3,
             'kf_ingest_first_call_ms': (t2 - t1) * 1e3, 'filters': 1, 'model': cfg['model']}
    if cfg['parallel']:
        return dict(step=step, units=T, bytes=per_event * T, bytes_per_unit=per_event,
                    kernel=f'ref_chain_kernel<f64,{"M8" if ref8 else "M15"},stream> (map pass) + stream_* kernels',
                    traffic=None, cpu=cpu, gather=None, kf=kf,
                    roofline_note='latency / issue-bound: the map pass runs its chunk length of events in '
                                  'sequence (one wave per SIMD), the covariance starts walk their windows of maps; '
                                  'the fraction is not the figure of merit',
                    desc=desc + 'time-parallel (kf_run_stream: chunks of the log as filters, covariance warm-up + '
                                'affine state maps composed on the device, checked, sequential fallback); synthetic '
                                "log with the reference log's shape",
                    extra=dict(extra, stream_check=stream_check,
                               launch='hipGraph replay of the step' if getattr(args, 'graph', False) else 'eager'))
    return dict(step=step, units=T, bytes=per_event * T, bytes_per_unit=per_event, kernel='ref_chain_kernel',
                traffic=None, cpu=cpu, gather=None, kf=kf,
                roofline_note='one filter: one wave whose per-event dependency chain bounds the rate (8 lanes, '
                              'one per axis chain); HBM is idle, so the fraction is not the figure of merit',
                desc=desc + "synthetic log with the reference log's shape", extra=extra)


def dead_reckoning_workload(cfg, args, dev, stream, ingest_s):
    """hw5_2.run_dead_reckoning_for_IMU (hw5_2.py:382-436) over a whole ingested drive log: a step
    is the device compaction of the IMU events (kf_events_select: the driver skips every fix,
    :403-404), their dt (kf_events_dt, KF_DT_RAW from no previous time: the first IMU event at dt
    0, :401, 407) and one kf_run_stream of the 8-state filter from x0 = 0 over them (:410-433),
    the trajectory (x, y, theta) recorded per IMU event."""
    import ctypes
    import kfmi
    from kfmi import _lib
    from kfmi.engine import _ptr
    N = len(stream)
    T = int(stream.n_imu)
    kf = kfmi.BatchedKF('ref8', 1, 'f64', device=dev.index, options=cfg.get('opts'))
    x0 = torch.zeros(8, 1, dtype=torch.float64, device=dev)
    t_sel = torch.empty(N, dtype=torch.float64, device=dev)
    p_sel = torch.empty(N, 9, dtype=torch.float64, device=dev)
    dt = torch.empty(T, dtype=torch.float64, device=dev)
    et = torch.empty(T, dtype=torch.uint8, device=dev)
    traj = kf.empty(T, 3, 1)
    et_in, t_in, p_in = stream.etype.contiguous(), stream.t.contiguous(), stream.payload.contiguous()
    stream_check = {}

    def step():
        L = _lib.lib()
        kf.reset(x0)
        k = ctypes.c_int64(0)
        _lib.check(L.kf_events_select(N, _ptr(et_in), _ptr(t_in), _ptr(p_in), _lib.KF_EVENT_IMU, _ptr(t_sel),
                                      _ptr(p_sel), None, ctypes.byref(k), kf._stream()))
        if k.value != T:
            raise SystemExit(f'kf_events_select kept {k.value} IMU events, the stream holds {T}')
        _lib.check(L.kf_events_dt(T, _ptr(t_sel), None, float('nan'), _lib.KF_DT_RAW, _ptr(dt), _ptr(et),
                                  kf._stream()))
        _lib.check(L.kf_run_stream(kf.handle, T, _ptr(et), _ptr(dt), _ptr(p_sel), _ptr(traj), None, None, None, 0, -1,
                                   kf._stream()))
        if not stream_check:  # first (warm-up) step: record the device checks (synchronises)
            stream_check.update(kf.stream_check())

    def cpu():
        """The dead-reckoning walk restated in C (oracle/cpu_kf.c cpu_ref8_dead_reckoning: the
        dense 8x8 step over the IMU events of the merged stream) over the whole log, 1 thread (one
        filter); plus the NumPy restatement (oracle/ref_kf.run_dead_reckoning_8state) over the
        first events, 1 core, ~3 s."""
        from oracle import cpu_kf, ref_kf
        from kfmi.kf_workers import EventList
        h = stream.host()
        ts = time.perf_counter()
        cpu_kf.ref8_dead_reckoning(h['etype'], h['t'], h['payload'])
        el = time.perf_counter() - ts
        ev = EventList(stream)
        n = 2000
        while True:
            lst = ev[:n]
            t1 = time.perf_counter()
            st, _ = ref_kf.run_dead_reckoning_8state(lst)
            el_np = time.perf_counter() - t1
            if el_np > 3.0 or n >= N:
                break
            n = min(N, n * 4)
        return {'value': T / el, 'unit': 'KF events/s', 'cores': 1, 'kind': 'port',
                'sample': f'hw5_2.run_dead_reckoning_for_IMU over the {T} IMU events of this log through '
                          f'oracle/cpu_kf.c (the reference step, dense 8x8, C -O3), 1 thread (one filter), '
                          f'{host_cpu()}', 'seconds': round(el, 2),
                'numpy_reference_loop': {'value': len(st) / el_np, 'cores': 1,
                                         'sample': f'{len(st)} IMU events, oracle/ref_kf.run_dead_reckoning_8state, '
                                                   f'NumPy {np.__version__}'}}

    # select (etype read by its count and its gather pass; t + payload of the kept events read and
    # written; no positions: src_out is NULL), dt pass (t in; dt, etype out), filter (etype, dt,
    # payload in; trajectory out): bytes per IMU event
    per_event = (2 * N * 1) / T + 2 * (8 + 72) + (8 + 8 + 1) + (1 + 8 + 72 + 8 * 3)
    csv_s, ingest_first_s, ingest_s2 = ingest_s
    return dict(step=step, units=T, bytes=per_event * T, bytes_per_unit=per_event,
                kernel='kf_events_select + kf_events_dt + kf_run_stream (ref_chain_kernel<f64,M8,stream> map pass and '
                       'stream_* kernels)',
                traffic=None, cpu=cpu, gather=None, kf=kf,
                roofline_note='latency / issue-bound like config 1 (the map pass runs its chunk length of events in '
                              'sequence); the compaction\'s count is read back by the host once per step; bytes: '
                              'the select reads etype twice over the stream and reads + writes the kept events\' '
                              't and payload (2 x 80 B), the dt pass 17 B, the filter 105 B per IMU event',
                desc=f'hw5_2.run_dead_reckoning_for_IMU (hw5_2.py:382-436): ONE 8-state filter over the {T} IMU events '
                     f'of a whole drive log ({N} merged events, {stream.n_fixes} fixes skipped), f64; IMU events '
                     f'compacted on the device, time-parallel (kf_run_stream); synthetic log with the reference '
                     f"log's shape",
                extra={'events': N, 'events_filtered': T, 'csv_parse_ms': csv_s * 1e3,
                       'kf_ingest_ms': ingest_s2 * 1e3, 'kf_ingest_first_call_ms': ingest_first_s * 1e3,
                       'filters': 1, 'model': 'ref8', 'driver': 'run_dead_reckoning_for_IMU',
                       'stream_check': stream_check})


def sched_workload(cfg, args, rank, world, dev):
    """the rate-decimated greedy scheduled filter (kf_workers.py:826-957,
    Scheduler.greedy_schedule :195-213) over B event streams, the reference's sampling sweep
    (one filter per processing rate, 10..120 Hz, kf_plot_{10..120}.png) replicated across the
    batch, 64 filters per rate: kf_run_scheduled, one launch.  A unit is one input event examined."""
    import kfmi
    from kfmi import _lib
    from kfmi.engine import _ptr
    B, T, dt, k = cfg['B'], cfg['T'], cfg['dt'], cfg['k']
    kf = kfmi.BatchedKF('ref15', B, 'f64', device=dev.index, options=cfg.get('opts'))
    t0 = SCHED_T0
    # one rate per 64 consecutive filters (a wave): the sweep's filters batched by rate, so the
    # lanes of a wave reach their processing windows together (the jitter aside);
    # --rate-block 1 gives every lane of a wave its own rate (the divergent case)
    rb = max(1, int(getattr(args, 'rate_block', 64) or 64))
    if getattr(args, 'sched_rates', None):
        cfg = dict(cfg, rates=tuple(float(x) for x in args.sched_rates.split(',')))
    tt, etype, pay, freq, prev = sched_streams(B, T, dt, k, cfg['rates'], rb, SEED + rank, dev)
    # the payload as one 80-B record per event, its time at rec[9] (kf_run_scheduled_rec, the
    # default), or as the [T][9][B] rows of kf_run_scheduled (--sched-payload rows): same outputs
    rows = getattr(args, 'sched_payload', 'records') == 'rows'
    rec = int(getattr(args, 'sched_rec', 10) or 10)
    recs = None
    if not rows:
        recs = torch.zeros(T, B, rec, dtype=torch.float64, device=dev)
        recs[:, :, :9] = pay.transpose(1, 2)
        if rec >= 10:
            recs[:, :, 9] = tt  # the event's time (read with --opt sched_rec_time=on)
    traj = kf.empty(T, 6, B)
    logdet = kf.empty(T, B)
    sel_time = torch.empty(T, B, dtype=torch.float64, device=dev)
    n_sel = torch.empty(B, dtype=torch.int32, device=dev)

    def gather_payload():
        """N > 1: each rank's final states, each filter's last selected log-det and the
        per-selection trajectory rows (rows past a filter's n_sel are its own unwritten rows:
        the bitwise check compares a shard with itself)."""
        x, _ = kf.state()
        last = (n_sel.long() - 1).clamp(min=0)
        return x, logdet.gather(0, last[None, :])[0], traj

    def step():
        if rows:
            _lib.check(_lib.lib().kf_run_scheduled(kf.handle, T, _ptr(tt), _ptr(etype), _ptr(pay), _ptr(prev),
                                                    _ptr(freq), 0.0, _ptr(traj), _ptr(logdet), _ptr(sel_time),
                                                    _ptr(n_sel), kf._stream()))
        else:
            _lib.check(_lib.lib().kf_run_scheduled_rec(kf.handle, T, _ptr(tt), _ptr(etype), _ptr(recs), rec,
                                                        _ptr(prev), _ptr(freq), 0.0, _ptr(traj), _ptr(logdet),
                                                        _ptr(sel_time), _ptr(n_sel), kf._stream()))

    step()
    torch.cuda.synchronize(dev)
    n_selected = int(n_sel.long().sum().item())

    def cpu():
        """The oracle's NumPy restatement of the scheduled driver (oracle/ref_kf.
        run_kalman_filter_scheduled, kf_workers.py:826-957: Scheduler.gain per queued candidate
        with np.linalg.inv, step15, slogdet) on 1 core, streams of this workload."""
        from oracle import numpy_pool
        nth = numpy_pool.cores()
        # spread the sample over the rates: worker r takes every nth block of 64 filters
        per = -(-60000 * 4 // T)
        cols = [np.concatenate([np.arange(b * 64, b * 64 + 64) for b in range(r, B // 64, nth)])[:per]
                for r in range(nth)]
        idx = [torch.as_tensor(c, device=dev) for c in cols]
        shards = [dict(et=etype[:, i].cpu().numpy(), t=tt[:, i].cpu().numpy(), pay=pay[:, :, i].cpu().numpy(),
                       freq=freq[i].cpu().numpy(), t0=t0, n=len(c)) for i, c in zip(idx, cols)]
        npl = numpy_pool.run('sched', shards, seconds=4.0)
        return {'value': npl['value'], 'unit': 'KF events/s', 'cores': npl['cores'], 'kind': 'port',
                'seconds': round(npl['seconds'], 2), 'filters': npl['filters'],
                'sample': f"{npl['filters']} filters x {T} events of these streams (their rates, 10..120 Hz) "
                          f"through oracle/ref_kf.run_kalman_filter_scheduled (NumPy {np.__version__}, greedy: "
                          f"Scheduler.gain per queued candidate, kf_workers.py:826-957) in a spawn Pool of "
                          f"{npl['cores']} processes, {host_cpu()}"}

    # per event examined: t 8 + etype 1 read; per selection: payload 72 read, traj 48 + logdet 8 +
    # sel_time 8 written; per filter: state (15 + 27) x 8 loaded and stored, prev / freq read,
    # status read + written, n_sel written
    nbytes = B * T * 9 + n_selected * (72 + 64) + B * (2 * 42 * 8 + 8 + 8 + 8 + 4)
    mode = kf.get_option('sched_kernel')
    # the PMC figures (profiles/pmc_traffic.json, pmc_valu.json) are of the default row: two passes,
    # 10-double records with their time, the config's rates 64 filters per rate
    measured_shape = (mode in (0, 3) and B % 64 == 0 and not rows and rec == 10 and rb == 64
                      and kf.get_option('sched_rec_time') == 1 and not getattr(args, 'sched_rates', None))
    if B % 64:
        kernel = 'ref15_sched_kernel'
    elif mode in (0, 3):  # two passes (kf.h KF_OPT_SCHED_KERNEL)
        kernel = 'ref15_pick_kernel + ref15_apply_kernel (+ ref15_sched_kernel over flagged filters)'
    elif mode == 4:
        kernel = 'ref15_apply_kernel<pick phase> (+ ref15_sched_kernel over flagged filters)'
    else:
        kernel = 'ref15_sched_lds_kernel' if mode == 2 else 'ref15_sched_kernel'
    return dict(step=step, units=B * T, bytes=nbytes, bytes_per_unit=nbytes / (B * T),
                kernel=kernel, traffic=load_traffic('sched') if measured_shape else None,
                valu=load_valu('sched') if measured_shape else None,
                cpu=cpu, gather=gather_payload, kf=kf,
                roofline_note=f'{n_selected / (B * T):.3f} of the examined events are selected and applied (a '
                              f'full 15-state event each, its payload gathered per lane); the two passes move '
                              f'their actual HBM traffic (traffic, PMC: the gathers fetch whole 128-B lines) at '
                              f'the HBM\'s practical rate, so frac understates them by traffic / algorithmic',
                desc=f'SURVEY 8f row 3: rate-decimated greedy scheduled filter (kf_workers.py:826-957), reference '
                     f'15-state model, f64, B={B} filters/GPU, T={T} events at 200 Hz (GPS every {k}th), '
                     f'processing rates {cfg["rates"][0]}..{cfg["rates"][-1]} Hz across the batch (64 filters per rate), '
                     + ('payload [T][9][B] rows (kf_run_scheduled)' if rows else
                        f'payload [T][B][{rec}] records (kf_run_scheduled_rec)'),
                extra={'filters_per_gpu': B, 'events_per_launch': T, 'selected_events': n_selected,
                       'rates_hz': list(cfg['rates']),
                       'payload': 'rows' if rows else f'records of {rec}'})


VALU_PEAK = 1024 * 2.4e9 / 4   # wave64 VALU instructions/s: 1024 SIMDs, 4 cycles each, 2.4 GHz


def bf_plan(n, world, sym, mem_bytes=32 << 30):
    """The class split of the bf rows' search: one call (w = 0) when every size fits, otherwise
    ref15.search_class_width; N > 1 at least 4 classes per rank (kfmi.dist.search_classes)."""
    from kfmi import dist as kdist
    from kfmi import ref15 as r15
    return kdist.search_classes(n, world, 'f64', mem_bytes, sym) if world > 1 else \
        r15.search_class_width(n, 'f64', mem_bytes, sym)


def bf_level_bytes(n, w, sym, pair='auto'):
    """Level-buffer bytes of one class search of n - w free candidates: every stored node (the
    C(m-2, k) subsets of size k whose largest free candidate is <= m - 3) written once and read
    once as a parent; the one-launch head (sizes 1 .. K) stores only its level K, a pair launch
    only its second level (KF_OPT_SEARCH_PAIR), and the end launch (sizes k_end .. m) reads level
    k_end - 1 and stores none (kfmi.ref15.search_plan)."""
    from kfmi.ref15 import search_level_bytes, search_stored_levels
    m = n - w
    return 2 * sum(search_level_bytes(math.comb(m - 2, k), 'f64', sym)
                   for k in search_stored_levels(m, sym=sym, pair=pair))


def bf_workload(cfg, args, rank, world, dev):
    """Exhaustive brute-force search (kf_workers.py:1218-1392 without the early exit: R_threshold
    below every subset's score, the reference's longest search, :1391-1392): every k-subset,
    k = 1..n, of n candidate events after a warm start.  search: the shared-prefix search
    (kf_search_combos), one call or 2^w class calls; N > 1, ONE search split by class over the
    ranks with search_winner's all-reduces in the timed step (strong scaling; replaces the
    reference's Pool(30) fan-out, :1320-1346).  bf_subsets: one filter per subset
    (kf_eval_combos), each rank the whole search.  value = subsets/s; the reference-equivalent
    steps (k events + the final predict per k-subset) are a secondary key."""
    import kfmi
    from kfmi import dist as kdist
    from kfmi import ref15 as r15
    n, chunk = cfg['n'], cfg['chunk']
    ev, init, Pw, t0, t_end = bf_events(n)
    total_combos = 2 ** n - 1
    ref_steps = sum(math.comb(n, k) * (k + 1) for k in range(1, n + 1))
    search = cfg['search']

    def cpu():
        """The reference worker's per-subset filter (kf_workers.py:22-97) restated in C
        (oracle/cpu_kf.c, dense 15x15): the 12-subsets of the candidates as event streams (k
        events + the final predict), OpenMP over subsets on this host's allotted cores, ~10 s;
        plus the worker's NumPy loop (oracle/ref_kf.evaluate_combo_chunk) on 1 core, ~3 s.
        value = the worker's subsets/s at this search's mean subset (ref_steps / 2^n - 1 steps):
        KF steps/s x (2^n - 1) / ref_steps."""
        from itertools import combinations, islice
        from oracle import cpu_kf, ref_kf
        nth = cpu_kf.threads()
        kk = 12
        done, ts = 0, time.perf_counter()
        it = combinations(range(n), kk)
        while time.perf_counter() - ts < 10.0:
            combos = np.array(list(islice(it, 4096)))
            if not len(combos):
                break
            nc = len(combos)
            et = np.full((kk + 1, nc), 2, np.uint8)
            et[:kk] = ev[combos.T, 1].astype(np.uint8)
            tt = ev[combos.T, 0]
            dd = np.empty((kk + 1, nc))
            dd[0] = tt[0] - t0
            dd[1:kk] = np.diff(tt, axis=0)
            dd[kk] = t_end - tt[-1]                            # the worker's final predict (:74-82)
            pp = np.zeros((kk + 1, 9, nc))
            pp[:kk] = np.transpose(ev[combos.T, 2:], (0, 2, 1))
            cpu_kf.ref15_events(et, dd, pp, np.zeros((15, nc)), Pw, nthreads=nth, records=True)
            done += nc
        el = time.perf_counter() - ts
        cand = [(i, 'GPS' if ev[i, 1] == 0 else 'IMU', ev[i, 0],
                 ({'easting': ev[i, 2], 'northing': ev[i, 3], 'altitude': ev[i, 4]} if ev[i, 1] == 0
                  else ['t', *ev[i, 2:]])) for i in range(n)]
        # the worker's NumPy loop over the 12-subsets, each Pool process its own range of them
        # (the reference's Pool fan-out, kf_workers.py:1320-1346)
        from oracle import numpy_pool
        per = 4000
        shards = [dict(cand=cand, k=kk, lo=r * per, n=per, x0=np.zeros(15), P0=Pw, t0=t0, t_end=t_end)
                  for r in range(nth)]
        npl = numpy_pool.run('bf', shards, seconds=3.0)
        steps_s = done * (kk + 1) / el
        per_subset = ref_steps / total_combos
        return {'value': steps_s / per_subset, 'unit': 'subsets/s', 'kf_steps_per_s': steps_s,
                'steps_per_subset': per_subset, 'combinations_per_s': done / el, 'cores': nth,
                'kind': 'port', 'sample': f'{done} {kk}-subsets of the {n} candidates as event streams through '
                                          f'oracle/cpu_kf.c (the reference step, dense 15x15, C -O3 OpenMP) on '
                                          f'{nth} threads, {host_cpu()}; value = its KF steps/s / {per_subset:.2f}, '
                                          f'the reference worker\'s steps per subset of this search',
                'seconds': round(el, 2),
                'numpy_reference_loop': dict(npl, combinations_per_s=npl['value'] / (kk + 1),
                                             subsets_per_s=npl['value'] / per_subset,
                                             sample=f"{npl['filters']} {kk}-subsets, oracle/ref_kf."
                                                    f"evaluate_combo_chunk (kf_workers.py:22-97) in a spawn Pool of "
                                                    f"{npl['cores']} processes, NumPy {np.__version__}")}

    if not search:
        width = min(chunk, max(math.comb(n, k) for k in range(1, n + 1)))
        kf = kfmi.BatchedKF('ref15', width, 'f64', device=dev.index)
        launches = [(k, off) for k in range(1, n + 1) for off in range(0, math.comb(n, k), width)]

        def step():
            for k, off in launches:
                kf.eval_combos(ev, init, t0, t_end, k, combo_offset=off, logdets=False)
        return dict(step=step, units=total_combos, unit='subsets/s', ref_steps=ref_steps, bytes=None,
                    bytes_per_unit=None, kernel='ref15_combo_kernel', traffic=None, cpu=cpu, gather=None, kf=kf,
                    combos=total_combos,
                    desc=f'SURVEY 8f row 1: exhaustive brute-force search, n={n} candidate events (kf_workers.py:2311), '
                         f'all 2^{n}-1 subsets, reference 15-state model, f64, {len(launches)} kf_eval_combos launches '
                         f'(one filter per subset; each rank the whole search)',
                    extra={'candidate_events': n, 'combinations': total_combos, 'launch_width': width})

    kf = kfmi.BatchedKF('ref15', 1, 'f64', device=dev.index, options=cfg.get('opts'))
    sym = kf.search_plan(init, n, k_max=1)['sym']
    w = bf_plan(n, world, sym)
    mine = kdist.rank_classes(w, rank, world) if world > 1 else r15.class_order(w)

    def search_class(nf, c, k_max):
        k, idx, _, _ = kf.search_combos(ev, init, t0, t_end, -1e30, k_max=k_max, exhaustive=True, n_fixed=nf,
                                        fixed_mask=c)
        return k, idx

    def step():
        # R_threshold below every subset's score: every size of every class (no early exit)
        if world > 1:
            kdist.search_winner(search_class, n, w, exhaustive=True)
        elif w == 0:
            kf.search_combos(ev, init, t0, t_end, -1e30, exhaustive=True)
        else:
            r15.class_search(search_class, n, w, mine, exhaustive=True)

    def dist_check():
        """N > 1, after the timed region: the reference's search (not exhaustive: it stops at the
        first accepted size, kf_workers.py:1325-1371) sharded by class across the ranks
        (kfmi.dist.search_winner: MIN of the first accepted size, MAX of the bit-reversed winner
        mask) against rank 0's own one-GPU search of the same candidates, at a threshold that
        accepts no single event (the winner has two or more); n <= 25 also exhaustive, with
        every size's acceptance count summed over the ranks."""
        import torch.distributed as tdist
        thr = torch.tensor([float('-inf')], dtype=torch.float64)
        if rank == 0:
            ones = kf_one.eval_combos(ev, init, t0, t_end, 1, logdets=False)[0][:n]
            L0 = float(np.linalg.slogdet(Pw)[1])
            thr[0] = (L0 + float(ones.min())) / 2
        thr = thr.to(kdist._tdev())
        tdist.all_reduce(thr, op=tdist.ReduceOp.MAX)
        thr = float(thr.item())

        def search_thr(nf, c, k_max, exhaustive=False, acc=None):
            k, idx, a, _ = kf.search_combos(ev, init, t0, t_end, thr, k_max=k_max, exhaustive=exhaustive, n_fixed=nf,
                                            fixed_mask=c)
            if acc is not None:
                acc[:len(a)] += a.astype(np.int64)
            return k, idx
        won = kdist.search_winner(search_thr, n, w)
        out = {'threshold': thr, 'classes': 1 << w, 'k_found': won[0] if won else 0,
               'winner': list(won[1]) if won else None}
        acc_t = None
        if n <= 25:
            acc = np.zeros(n + 1, dtype=np.int64)
            won_x = kdist.search_winner(lambda nf, c, k_max: search_thr(nf, c, k_max, True, acc), n, w,
                                        exhaustive=True)
            acc_t = [int(v) for v in kdist.sum_counts(acc)]
            out['exhaustive'] = {'k_found': won_x[0] if won_x else 0, 'winner': list(won_x[1]) if won_x else None,
                                 'accepted_per_size': acc_t}
        if rank == 0:
            w1 = r15.search_class_width(n, 'f64', 32 << 30, sym)
            k1, idx1, acc1, _ = r15.search_combos_classed(kf, ev, init, t0, t_end, thr, w1)
            out['one_rank'] = {'k_found': k1, 'winner': list(idx1) if idx1 else None, 'classes': 1 << w1}
            ok = out['k_found'] == k1 and out['winner'] == out['one_rank']['winner']
            if acc_t is not None:
                kx, idxx, accx, _ = r15.search_combos_classed(kf, ev, init, t0, t_end, thr, w1, exhaustive=True)
                out['one_rank']['accepted_per_size'] = [int(v) for v in accx]
                ok = ok and acc_t == out['one_rank']['accepted_per_size'] and \
                    out['exhaustive']['winner'] == (list(idxx) if idxx else None)
            out['one_rank_equal'] = ok
            if not ok:
                raise SystemExit(f'the {world}-rank search disagrees with the one-rank search: {out}')
        kf_one.close()
        return out

    kf_one = kfmi.BatchedKF('ref15', 64, 'f64', device=dev.index) if world > 1 else None  # scores of the 1-subsets
    step()  # how the library runs this search (kf_search_info): axis-symmetric, head, launches (last class)
    torch.cuda.synchronize(dev)
    info = kf.search_info()
    K, sym_ran = info['head_sizes'], info['sym']
    assert sym_ran == sym, (sym_ran, sym)
    m = n - w
    launches = info['level_launches'] + (1 if K else 0)
    k_end = r15.search_end_size(m)
    classes_here = len(mine)
    per_class = bf_level_bytes(n, w, sym, pair=cfg.get('opts', {}).get('search_pair', 'auto'))
    lvl_bytes = per_class * classes_here
    subsets_here = total_combos if world == 1 else sum(2 ** m for _ in mine) - (1 if 0 in mine else 0)
    chains = ('axis-symmetric: one pva and one aw chain computed and stored for the three of each, '
              'KF_OPT_AXIS_SYM' if sym else 'every chain')
    cfg_id = 'bf' if n == 25 else f'bf{n}'
    valu = load_valu(cfg_id)
    valu_per_search = None
    try:
        with open(os.path.join(ROOT, 'profiles', 'pmc_valu.json')) as f:
            rec = json.load(f).get(f'config{cfg_id}')
        if rec and rec.get('classes', 1) == 1 << w:
            valu_per_search = rec['counters_per_launch']['SQ_INSTS_VALU']
    except (OSError, ValueError, KeyError):
        pass
    split = (f'{1 << w} classes of {m} free candidates (the subsets split by their intersection with candidates '
             f'0..{w - 1}), {classes_here} on this rank, each a kf_search_combos call' if w else 'one kf_search_combos call')
    par = (f'subset classes x{world}: one search split over the ranks, two all-reduces (MIN size, MAX winner '
           f'key) per search' if world > 1 else
           (f'one GPU, {1 << w} class searches in sequence' if w else 'one GPU, one search call'))
    return dict(step=step, units=total_combos, unit='subsets/s', ref_steps=ref_steps, strong=world > 1, parallelism=par,
                bytes=lvl_bytes, bytes_per_unit=lvl_bytes / subsets_here,
                valu_per_launch=valu_per_search if world == 1 else None,
                kernel=f'ref15_search_head_kernel (sizes 1..{K}) + ref15_search_cm/pm_kernel + '
                       f'ref15_search_end_kernel (sizes {k_end}..{m}) ({launches} launches per class search)',
                traffic=load_traffic(cfg_id, lvl_bytes), valu=valu if world == 1 else None,
                cpu=cpu, gather=None, dist_check=dist_check if world > 1 else None, kf=kf, combos=total_combos,
                roofline_note='fp64 VALU issue: wave64 VALU instructions of one search (rocprofv3 SQ_INSTS_VALU, '
                              'profiles/pmc_valu.json) / its time, against 1024 SIMDs x 2.4 GHz / 4 cycles; the '
                              'level buffers (each stored prefix filter written and read once) are the hbm entry',
                desc=f'SURVEY 8f row 1: exhaustive brute-force search, n={n} candidate events '
                     f'({"kf_workers.py:2311" if n == 25 else "kf_workers_visualizing.py:2293, 2340"}), '
                     f'all 2^{n}-1 subsets, reference 15-state model, f64, shared-prefix search (one event step + '
                     f'final predict per subset, sizes 1..{K} in one launch, then one launch per level or per two '
                     f'parent-major levels, sizes {k_end}..{m} in one: {launches} launches per class search; {chains}); '
                     f'{split}; '
                     f'value = subsets/s of ONE search' + (f' split over {world} ranks' if world > 1 else ''),
                extra={'candidate_events': n, 'combinations': total_combos, 'levels': n, 'search': info,
                       'classes': 1 << w, 'classes_this_rank': classes_here, 'free_candidates_per_class': m})


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch_plan(gpus, env, argv, script=None, port=None):
    """How `python bench.py --gpus N` runs: None = in this process (one rank, or a rank that a
    launcher already started: WORLD_SIZE set); otherwise the command that starts the N ranks as
    fresh child processes (torch.distributed.run, one GPU per rank, rendezvous on 127.0.0.1).
    The parent never touches the GPU: it waits for the launcher and exits with its status (the
    worst rank's).  Replaces the reference's Pool(30) fan-out (kf_workers.py:1320-1346) with one
    process per GPU.  A WORLD_SIZE that disagrees with --gpus is an error, never a silent
    one-rank run."""
    if gpus < 1:
        raise SystemExit(f'--gpus {gpus}: need at least one GPU')
    world = env.get('WORLD_SIZE')
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f'--gpus {gpus} but WORLD_SIZE={world}')
        return None
    if gpus == 1:
        return None
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={gpus}',
            '--master-addr=127.0.0.1', f'--master-port={port or _free_port()}',
            script or os.path.abspath(__file__)] + list(argv)


def launch_check(world, rank):
    """--launch-check: each rank joins a gloo group (no GPU) and rank 0 reports the ranks it
    sees; tests/test_bench_launch.py drives `bench.py --gpus N --launch-check` on the CPU."""
    import torch.distributed as dist
    seen = 1
    if world > 1:
        dist.init_process_group('gloo')
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        assert seen == dist.get_world_size()
    if rank == 0:
        print(json.dumps({'launch_check': True, 'ranks_seen': seen, 'world_size': world}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return seen


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=None, help='timed steps (default 20; bf40: 1)')
    ap.add_argument('--warmup', type=int, default=None, help='untimed steps (default 10; bf40: 1)')
    ap.add_argument('--config', default='3', choices=sorted(CONFIGS))
    ap.add_argument('--batch', type=int, default=None, help='override filters per GPU')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--pcie', action='store_true', help='also report the PCIe-inclusive rate (cv configs, N=1)')
    ap.add_argument('--per-step', action='store_true',
                    help='cv configs, N=1: also time the per-step predict()/update() call shape')
    ap.add_argument('--rate-block', type=int, default=64,
                    help='config sched: consecutive filters sharing a processing rate (1 = per-lane rates)')
    ap.add_argument('--sched-payload', choices=['records', 'rows'], default='records',
                    help='config sched: the payload as [T][B][10] records (kf_run_scheduled_rec) or [T][9][B] rows')
    ap.add_argument('--sched-rec', type=int, default=10,
                    help='config sched, records: doubles per record (>= 10, even; 10 = the payload and the '
                         'event time in 80 B, the fastest measured)')
    ap.add_argument('--sched-rates', default=None,
                    help='config sched, diagnostics: comma-separated processing rates (Hz) instead of the '
                         "config's 10..120 sweep (e.g. only rates whose period is, or is not, a multiple of "
                         "the 5-ms event spacing, where the event-time jitter splits a wave's windows)")
    ap.add_argument('--graph', action='store_true',
                    help='config 1: replay the step as a hipGraph (measured no faster than eager launches)')
    ap.add_argument('--ablate', choices=['none', 'no-traj', 'no-logdet', 'no-traj-no-logdet'], default='none',
                    help='diagnostics only: skip an output stream (the JSON line says so)')
    ap.add_argument('--gather-traj-every', type=int, default=16,
                    help='N>1: the final all-gather also reassembles the trajectory decimated every k steps '
                         '(0 = final states and log-dets only); timed apart as allgather_ms')
    ap.add_argument('--opt', action='append', default=[], metavar='NAME=VALUE',
                    help='a kf_set_option of the workload\'s handle (kfmi.engine.OPTIONS), e.g. cv_kernel=general; '
                         'A/B runs only (the JSON line lists them)')
    ap.add_argument('--dist-backend', choices=['nccl', 'gloo'], default='nccl',
                    help='N>1: nccl = RCCL over xGMI, one GPU per rank; gloo = rehearsal only (N ranks share '
                         'one GPU, tools/dist_rehearsal.sh)')
    ap.add_argument('--launch-check', action='store_true',
                    help='start the ranks and report ranks_seen over gloo, no GPU work (tests)')
    args = ap.parse_args()

    cmd = launch_plan(args.gpus, os.environ, sys.argv[1:])
    if cmd is not None:
        # N ranks requested from a plain `python bench.py --gpus N`: start them as children
        import subprocess
        rc = subprocess.run(cmd).returncode
        if rc:
            print(f'bench.py: {args.gpus}-rank launch exited with status {rc}', file=sys.stderr, flush=True)
        raise SystemExit(rc)

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if args.launch_check:
        seen = launch_check(world, rank)
        raise SystemExit(0 if seen == args.gpus else 3)
    dist = None
    # RCCL ('nccl') over xGMI, one GPU per rank.  --dist-backend gloo is a rehearsal switch
    # only: it lets N ranks share the one GPU of a test box (RCCL refuses two ranks on one
    # device) so the N>1 code path — shards, max-over-ranks timing, the final all-gather — runs
    backend = args.dist_backend
    if world > 1 and backend == 'gloo':
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group('gloo')
    ranks_seen = dist.get_world_size() if dist else 1
    if ranks_seen != args.gpus:
        raise SystemExit(f'--gpus {args.gpus} but {ranks_seen} rank(s) joined')
    dev = torch.device('cuda', local)

    cfg = dict(CONFIGS[args.config])
    args.steps = cfg.get('steps', 20) if args.steps is None else args.steps
    args.warmup = cfg.get('warmup', 10) if args.warmup is None else args.warmup
    if args.batch:
        cfg['B'] = args.batch
    cfg['opts'] = dict(cfg.get('opts', {}))
    for o in args.opt:
        name, _, val = o.partition('=')
        cfg['opts'][name] = int(val) if val.lstrip('-').isdigit() else val
    if args.config in ('1', '1seq', '1ref8', '1dr'):
        w = log_workload(cfg, args, rank, world, dev)
    elif args.config in ('ref15', 'ref15f32'):
        w = ref15_workload(cfg, args, rank, world, dev)
    elif args.config == 'sched':
        w = sched_workload(cfg, args, rank, world, dev)
    elif args.config in ('bf', 'bf40', 'bf_subsets'):
        w = bf_workload(cfg, args, rank, world, dev)
    else:
        w = cv_workload(args.config, cfg, args, rank, world, dev)
    step = w['step']
    stream = torch.cuda.current_stream(dev)

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

    kf = w['kf']
    bad = int((kf.status() != 0).sum().item()) if not args.config.startswith('bf') else 0
    gather_ms = gather_info = dist_info = None
    if dist:
        from kfmi import dist as kdist
        elapsed, kern_ms, bad = kdist.max_over_ranks([elapsed, kern_ms, bad], dev)
        bad = int(bad)
        if w['gather'] is not None:
            # reassemble the final states + logdets (+ the trajectory decimated every
            # --gather-traj-every steps) of every shard on every rank, one all-gather (RCCL over
            # xGMI); timed separately: a once-per-job reassembly, not the hot path
            xl, ldl, trl = w['gather']()
            every = max(0, args.gather_traj_every)
            total = world * kf.batch
            torch.cuda.synchronize(dev)
            dist.barrier()
            g0 = time.perf_counter()
            res = kdist.gather_run_outputs(xl, ldl, trl, every, total)
            torch.cuda.synchronize(dev)
            gather_ms = (time.perf_counter() - g0) * 1e3
            # every rank finds its own shard at its global offset in the reassembled arrays
            off, cnt = kdist.shard_range(total, rank, world)
            same = lambda a, b: torch.equal(a.contiguous().view(torch.uint8), b.contiguous().view(torch.uint8))
            steps = kdist.decimated_steps(trl.shape[0], every) if trl is not None else []
            ok = (res['x'].shape[-1] == total and same(res['x'][:, off:off + cnt], xl)
                  and same(res['logdet'][off:off + cnt], ldl)
                  and (not steps or same(res['traj'][:, :, off:off + cnt], trl[steps])))
            if not ok:
                raise SystemExit(f'rank {rank}: the all-gathered shards do not reassemble')
            gather_info = {'ms': gather_ms, 'traj_every': every, 'traj_steps': len(steps),
                           'rows': res['rows'], 'bytes_per_rank': res['bytes_per_rank'],
                           'bytes_gathered': res['bytes_per_rank'] * world,
                           'checked': 'bitwise: every rank finds its shard at its global offset'}
            del res
        if w.get('dist_check') is not None:
            dist_info = w['dist_check']()

    # weak scaling: each rank its own units (filters); strong (the bf rows at N > 1): the ranks
    # share one search, so the job's units are one search's
    mult = 1 if w.get('strong') else world
    if rank == 0:
        rec = {
            'metric': 'KF predict+update steps/sec (batched filters)',
            'value': mult * w['units'] * args.steps / elapsed,
            'unit': w.get('unit', 'KF steps/s'),
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': elapsed / max(args.steps, 1) * 1e3,
            'higher_is_better': True,
            'scaling': 'strong' if w.get('strong') else 'weak',
            'vs_baseline': None,
            'dtype': cfg['dtype'],
            'data': 'synthetic (GPS+IMU streams per SURVEY.md §8d, generated on the GPU, resident in HBM)',
            'config': dict({'workload': w['desc'],
                            'parallelism': w.get('parallelism', f'filter shards x{world} (no data-path collective)')},
                           **w['extra']),
        }
        if 'valu_per_launch' in w:
            # the search rows: fp64 VALU issue is the roof, the level buffers' HBM
            # bandwidth a secondary entry
            hbm = w['bytes'] / (kern_ms * 1e-3) / 1e9
            vp = w['valu_per_launch']
            va = vp / (kern_ms * 1e-3) if vp else None
            rec['hbm_gbs'] = hbm
            rec['roofline'] = {'bound': 'valu', 'achieved': va, 'peak': VALU_PEAK, 'unit': 'wave-instr/s',
                               'frac': va / VALU_PEAK if va else None, 'traffic': w['traffic'],
                               'kernel': w['kernel'], 'kernel_ms': kern_ms, 'valu_instructions_per_launch': vp,
                               'hbm': {'achieved': hbm, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                                       'frac': hbm / HBM_PEAK_GBS, 'algorithmic_bytes_per_launch': w['bytes'],
                                       'algorithmic_bytes_per_subset': w['bytes_per_unit'],
                                       'traffic': w['traffic']},
                               'note': w['roofline_note'] + ('' if vp else '; no SQ_INSTS_VALU summary for this '
                                                                          'split, achieved unmeasured')}
            if w.get('valu'):
                rec['roofline']['valu'] = w['valu']
        elif w['bytes'] is not None:
            achieved = w['bytes'] / (kern_ms * 1e-3) / 1e9
            rec['hbm_gbs'] = achieved
            rec['roofline'] = {'bound': 'hbm', 'achieved': achieved, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                               'frac': achieved / HBM_PEAK_GBS, 'traffic': w['traffic'], 'kernel': w['kernel'],
                               'kernel_ms': kern_ms, 'algorithmic_bytes_per_launch': w['bytes'],
                               'algorithmic_bytes_per_step': w['bytes_per_unit']}
            if w.get('valu'):
                rec['roofline']['valu'] = w['valu']
            if w.get('roofline_note'):
                rec['roofline']['note'] = w['roofline_note']
            if world == 1 and w.get('probe') and args.ablate == 'none':
                # the same access pattern without the filter arithmetic, on the same buffers, right
                # after the timed region: the ceiling this box's HBM placement gives the pattern
                pr = w['probe'](max(args.steps, 5))
                if pr:
                    rec['roofline']['pattern_ceiling'] = {
                        'achieved': pr['gbs'], 'unit': 'GB/s', 'probe_ms': pr['ms'],
                        'frac': achieved / pr['gbs'], 'probe': pr['desc']}
        else:
            rec['roofline'] = {'bound': 'hbm', 'achieved': None, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s', 'frac': None,
                               'traffic': None, 'kernel': w['kernel'], 'kernel_ms': kern_ms,
                               'note': 'compute-bound search: events in LDS, ~350 B of HBM traffic per subset'}
        if w.get('update_every', 1) > 1:
            # the async config: predict-steps/s (= value) and update-steps/s apart
            rec['predict_steps_per_s'] = rec['value']
            rec['update_steps_per_s'] = world * (w['units'] // w['update_every']) * args.steps / elapsed
        if 'combos' in w:
            rec['combinations_per_s'] = mult * w['combos'] * args.steps / elapsed
        if 'ref_steps' in w:
            # the steps the reference's worker would run for the same subsets (k events + the final
            # predict per k-subset, kf_workers.py:22-97): the search shares prefixes instead
            rec['reference_equivalent_steps_per_s'] = mult * w['ref_steps'] * args.steps / elapsed
        rec['failed_filters'] = bad
        if args.ablate != 'none':
            rec['ablation'] = args.ablate + ' (diagnostic run: NOT the benchmark workload)'
        rec['ranks_seen'] = ranks_seen
        if cfg['opts']:
            rec['options'] = cfg['opts']
        from kfmi import _lib as _kl
        rec['build'] = _kl.build_info()
        if gather_ms is not None:
            rec['allgather_ms'] = gather_ms
            rec['allgather'] = gather_info
        if dist_info is not None:
            rec['dist_search'] = dist_info
        rec['cpu_baseline'] = w['cpu']() if (world == 1 and not args.no_cpu_baseline) else None
        if args.pcie and world == 1 and w.get('pcie'):
            rec['pcie_inclusive'] = w['pcie']()
        if args.per_step and world == 1 and w.get('per_step'):
            rec['per_step_api'] = w['per_step']()
        print(json.dumps(rec), flush=True)
    kf.close()
    if dist:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
