"""The reference CPU loop on every allotted host core — TEST INFRASTRUCTURE / CPU BASELINE ONLY.

Only bench.py's ``cpu_baseline`` leg (and tests) use this.  SURVEY.md §8d(i): the NumPy
per-filter loop in the reference's op order (oracle/ref_kf.py) on ``os.sched_getaffinity``
cores through a ``multiprocessing.Pool``, which is the reference's own parallelism: it fans
combinations out over ``Pool(30)`` workers (kf_workers.py:1320-1346).  Each worker runs its
shard of filters for a fixed wall time, one BLAS thread per process; the rate is the sum of
the workers' rates (they run side by side: the pool is warmed up first).
"""
from __future__ import annotations

import os
import time

import numpy as np

_ONE_THREAD = ('OMP_NUM_THREADS', 'OPENBLAS_NUM_THREADS', 'MKL_NUM_THREADS')


def _worker(job):
    from oracle import ref_kf
    kind, sh, seconds = job
    units, tic = 0, time.perf_counter()
    nf = sh['n']
    f = 0
    while f < nf and time.perf_counter() - tic < seconds:
        if kind == 'cv':
            model = ref_kf.CVModel(sh['d'], r_full=sh.get('R'))
            T = sh['u'].shape[0]
            ref_kf.run_filter_loop(model, sh['x0'][:, f], sh['P0'], np.full(T, sh['dt']), sh['u'][:, :, f],
                                   sh['z'][:, :, f], sh['k'])
            units += T
        elif kind == 'ref15':
            et, dd, pa = sh['et'], sh['dt'], sh['pay']
            x, P = np.zeros(15), ref_kf.P0_REF15.copy()
            for t in range(et.shape[0]):
                if et[t, f] == 0:
                    sd = {'easting': pa[t, 0, f], 'northing': pa[t, 1, f], 'altitude': pa[t, 2, f]}
                    x, P = ref_kf.step15(x, P, 'GPS', sd, dd[t, f])
                else:
                    x, P = ref_kf.step15(x, P, 'IMU', ['t', *pa[t, :, f]], dd[t, f])
                np.linalg.slogdet(P)
                units += 1
        elif kind == 'bf':
            if f == 0:
                from itertools import combinations, islice
                combos = islice(combinations(range(len(sh['cand'])), sh['k']), sh['lo'], sh['lo'] + nf)
            combo = next(combos)
            ref_kf.evaluate_combo_chunk([tuple(sh['cand'][i] for i in combo)], sh['x0'], sh['P0'], sh['t0'],
                                        sh['t_end'])
            units += len(combo) + 1   # k events + the worker's final predict (kf_workers.py:74-82)
        elif kind == 'sched':
            et, ts, pa, t0 = sh['et'], sh['t'], sh['pay'], sh['t0']
            ev = [(0, 'GPS', t0, {'easting': 0.0, 'northing': 0.0, 'altitude': 0.0})]
            for i in range(et.shape[0]):
                if et[i, f] == 0:
                    ev.append((i + 1, 'GPS', ts[i, f], {'easting': pa[i, 0, f], 'northing': pa[i, 1, f],
                                                        'altitude': pa[i, 2, f]}))
                else:
                    ev.append((i + 1, 'IMU', ts[i, f], ['t', *pa[i, :, f]]))
            ref_kf.run_kalman_filter_scheduled(ev, 0, len(ev), ref_kf.P0_REF15.copy(), (t0, 0, 0, 0, 0, 0, 0),
                                               'greedy', float(sh['freq'][f]))
            units += et.shape[0]
        else:
            raise ValueError(kind)
        f += 1
    return units, time.perf_counter() - tic, f


def _warm(_):
    import oracle.ref_kf  # noqa: F401
    return os.getpid()


def cores():
    """The cores this process may use (the GPU box allots 16: OMP_NUM_THREADS)."""
    from oracle import cpu_kf
    return cpu_kf.threads()


def run(kind, shards, seconds=5.0):
    """Run ``shards`` (one dict per worker, see _worker) in a spawn Pool of len(shards) workers
    for ``seconds`` each.  Returns dict(value = units/s summed over workers, cores, units,
    filters)."""
    import multiprocessing as mp
    n = len(shards)
    old = {k: os.environ.get(k) for k in _ONE_THREAD}
    os.environ.update({k: '1' for k in _ONE_THREAD})
    try:
        with mp.get_context('spawn').Pool(n) as pool:
            pool.map(_warm, range(4 * n))           # every worker up and importing done
            res = pool.map(_worker, [(kind, sh, seconds) for sh in shards], chunksize=1)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return {'value': sum(u / el for u, el, _ in res if el > 0), 'cores': n, 'units': sum(u for u, _, _ in res),
            'filters': sum(f for _, _, f in res), 'seconds': max(el for _, el, _ in res)}


def split(n_items, n_parts):
    """Contiguous index ranges of n_items over n_parts workers."""
    base, rem = divmod(n_items, n_parts)
    out, lo = [], 0
    for r in range(n_parts):
        hi = lo + base + (1 if r < rem else 0)
        out.append((lo, hi))
        lo = hi
    return out
