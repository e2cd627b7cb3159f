"""The RCCL ('nccl') branches of kfmi.dist on the box's GPU (world size 1: RCCL refuses two
ranks on one device; the N-rank paths are covered with gloo in test_dist_gloo.py).  Every
collective runs on device tensors through the nccl group and through a gloo group of the same
rank, and the results must be bitwise equal; the brute-force search runs on the GPU through both
and must return the reference's pick (tests/golden/ref15_bruteforce.npz)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

from kfmi import dist as kdist

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.fixture(scope='module')
def groups():
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{_free_port()}', rank=0, world_size=1,
                            device_id=dev)
    gloo = dist.new_group([0], backend='gloo')
    assert dist.get_backend() == 'nccl' and dist.get_backend(gloo) == 'gloo'
    yield None, gloo
    dist.destroy_process_group()


def _bits(t):
    return t.contiguous().view(torch.uint8).cpu()


@pytest.mark.parametrize('dtype', [torch.float64, torch.float32])
def test_gather_shards_nccl_equals_gloo(groups, dtype):
    nccl, gloo = groups
    g = torch.Generator(device='cuda').manual_seed(7)
    local = torch.randn(7, 1000, dtype=dtype, device='cuda', generator=g)
    local[3, 17] = float('nan')
    a = kdist.gather_shards(local, 1000, group=nccl)
    b = kdist.gather_shards(local, 1000, group=gloo)
    assert a.device.type == 'cuda' and b.device.type == 'cuda'
    assert torch.equal(_bits(a), _bits(b)) and torch.equal(_bits(a), _bits(local))


def test_gather_run_outputs_nccl_equals_gloo(groups):
    """The bench's reassembly on a real run: x, last log-det and the decimated trajectory."""
    import kfmi
    nccl, gloo = groups
    B, T = 4099, 40
    kf = kfmi.BatchedKF('cv3', B, 'f64')
    x0, u, z = kf.synth(T=T, dt=0.1, update_every=1, seed=3)
    kf.reset(x0)
    tr, ld = kf.run(u, z, dt=0.1)
    x, _ = kf.state()
    a = kdist.gather_run_outputs(x, ld[-1], tr, 8, B, group=nccl)
    b = kdist.gather_run_outputs(x, ld[-1], tr, 8, B, group=gloo)
    for key in ('x', 'logdet', 'traj'):
        assert torch.equal(_bits(a[key]), _bits(b[key])), key
    assert torch.equal(_bits(a['traj']), _bits(tr[7::8]))
    assert a['rows'] == 6 + 1 + 6 * 5
    kf.close()


def test_max_over_ranks_nccl_equals_gloo(groups):
    nccl, gloo = groups
    vals = [1.5, -2.25, 3e10, float('inf')]
    assert kdist.max_over_ranks(vals, torch.device('cuda', 0), group=nccl) == vals
    assert kdist.max_over_ranks(vals, torch.device('cuda', 0), group=gloo) == vals


@pytest.mark.parametrize('thr', [None, -27.0, -1e9])
def test_brute_force_search_nccl_equals_gloo(groups, golden_dir, thr):
    """kf_search_combos on the GPU, reduced through RCCL (device tensors) and through gloo."""
    sys.path.insert(0, os.path.dirname(__file__))
    from golden_events import unpack_events
    nccl, gloo = groups
    g = np.load(os.path.join(golden_dir, 'ref15_bruteforce.npz'))
    events = unpack_events(g)
    s, e = int(g['start']), int(g['end'])
    t = float(g['threshold']) if thr is None else thr
    kw = dict(R_threshold=t, initial_pt=g['init_P'], initial_state=tuple(g['init_state']))
    ra = kdist.brute_force_search(events, s, e, group=nccl, **kw)
    rb = kdist.brute_force_search(events, s, e, group=gloo, **kw)
    rc = kdist.brute_force_search_ranks(events, s, e, group=nccl, **kw)
    if thr == -1e9:
        assert ra is None and rb is None and rc is None
        return
    cand = events[s:e]
    pick = lambda r: [cand.index(ev) for ev in r['selected_sensors']]
    assert pick(ra) == pick(rb) == pick(rc)
    if thr is None:
        assert pick(ra) == list(g['selected'])
    for key in ('final_state', 'log_determinants'):
        np.testing.assert_array_equal(np.asarray(ra[key]), np.asarray(rb[key]))


def test_brute_force_search_n40_window_nccl(groups):
    """The reference's 40-event window sharded through RCCL (world 1): the one-call sizes first,
    then the class split; the same result dict as the one-GPU driver, at a threshold whose winner
    has two events and at one past the one-call sizes (target far beyond the window, as in
    tests/test_gpu_search_classes.py, through the events' own target: the window's last event)."""
    import bench
    from kfmi import ref15
    nccl, _ = groups
    n = 40
    ev, init, Pw, t0, _ = bench.bf_events(n)
    events = [(i, 'GPS', ev[i, 0], {'easting': ev[i, 2], 'northing': ev[i, 3], 'altitude': ev[i, 4]})
              if ev[i, 1] == 0 else (i, 'IMU', ev[i, 0], ['t', *ev[i, 2:]]) for i in range(n)]
    state0 = (t0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
    import kfmi
    kf1 = kfmi.BatchedKF('ref15', 64, 'f64')
    s1 = np.sort(kf1.eval_combos(ev, init, t0, float(ev[-1, 0]), 1, logdets=False)[0][:n].cpu().numpy())
    kf1.close()
    L0 = float(np.linalg.slogdet(Pw)[1])
    for thr in ((L0 + s1[0]) / 2, L0 - 1.0):   # a pair wins; nothing at all (every size by class)
        kw = dict(R_threshold=thr, initial_pt=Pw, initial_state=state0)
        a = kdist.brute_force_search(events, 0, n, group=nccl, **kw)
        b = ref15.run_brute_force_kalman_filter_no_sampling_min_usage(events, 0, n, **kw)
        if b is None:
            assert a is None
            continue
        assert [e[0] for e in a['selected_sensors']] == [e[0] for e in b['selected_sensors']]
        np.testing.assert_array_equal(np.asarray(a['log_determinants']), np.asarray(b['log_determinants']))
