"""bench.py's rank launch (CPU, gloo): `python bench.py --gpus N` must run N ranks, never a
silent single rank.  --launch-check stops each rank after the process group
forms, before any GPU work, so the real launch path runs here."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_plan_single_rank_runs_in_process():
    assert bench.launch_plan(1, {}, []) is None
    assert bench.launch_plan(4, {'WORLD_SIZE': '4'}, []) is None   # a launcher already started us


def test_plan_starts_n_ranks():
    cmd = bench.launch_plan(8, {}, ['--gpus', '8', '--steps', '5'], script='/x/bench.py', port=29512)
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node=8' in cmd and '--master-addr=127.0.0.1' in cmd and '--master-port=29512' in cmd
    assert cmd[-4:] == ['--gpus', '8', '--steps', '5'] and cmd[-5] == '/x/bench.py'


@pytest.mark.parametrize('gpus,world', [(2, '1'), (8, '4'), (1, '2')])
def test_plan_rejects_world_mismatch(gpus, world):
    with pytest.raises(SystemExit):
        bench.launch_plan(gpus, {'WORLD_SIZE': world}, [])


def test_plan_rejects_zero_gpus():
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {}, [])


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    env.update(env_extra or {})
    env.setdefault('OMP_NUM_THREADS', '1')
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, cwd=ROOT,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize('n', [1, 2, 3])
def test_bench_starts_its_own_ranks(n):
    p = _run(['--gpus', str(n), '--launch-check'])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout            # rank 0 alone prints, once
    assert lines[0]['ranks_seen'] == n and lines[0]['world_size'] == n


def test_bench_world_mismatch_exits_nonzero():
    p = _run(['--gpus', '2', '--launch-check'], {'WORLD_SIZE': '1', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert p.returncode != 0
    assert 'WORLD_SIZE=1' in p.stderr


def _bench_ranks(gpus, config, extra=()):
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', str(gpus), '--dist-backend', 'gloo',
           '--config', config, '--no-cpu-baseline'] + list(extra)
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec['n_gpus'] == rec['ranks_seen'] == gpus
    assert rec['failed_filters'] == 0 and rec['value'] > 0
    return rec


def _check_allgather(rec, gpus):
    ag = rec['allgather']
    assert ag['checked'].startswith('bitwise') and ag['traj_steps'] > 0
    assert ag['bytes_gathered'] == gpus * ag['bytes_per_rank'] > 0
    assert rec['scaling'] == 'weak'


@pytest.mark.gpu
@pytest.mark.parametrize('config', ['3', '4', '2', '5', 'ref15', 'sched', 'bf', 'bf40'])
def test_bench_two_ranks_on_the_gpu(config):
    """`python bench.py --gpus 2` end to end on the GPU box, started as a fresh child process:
    two ranks (gloo: they share the box's one GPU; the 8-GPU node's run is RCCL), each owning
    its shard of filters, max-over-ranks timing, and the final all-gather of the final states,
    last log-dets and the decimated trajectory, which every rank checks bitwise against its own
    shard (bench.py's N > 1 path; replaces the reference's Pool(30) fan-out,
    kf_workers.py:1320-1346).  bf / bf40: ONE search split by subset class across the two ranks,
    timed with its cross-rank reductions (kfmi.dist.search_winner), value = one search's
    subsets / the slowest rank's time (strong scaling); after timing, the sharded search at a
    threshold gives rank 0's one-GPU winner (bf: and, exhaustive, its acceptance counts)."""
    if config.startswith('bf'):
        rec = _bench_ranks(2, config, ['--steps', '1', '--warmup', '0' if config == 'bf40' else '1'])
        assert rec['scaling'] == 'strong' and rec['unit'] == 'subsets/s'
        ds = rec['dist_search']
        assert ds['one_rank_equal'] and ds['k_found'] >= 2 and ds['classes'] >= 2
        assert ds['winner'] == ds['one_rank']['winner']
        assert rec['config']['classes'] == ds['classes'] and rec['config']['classes_this_rank'] == ds['classes'] // 2
        if config == 'bf':
            ex = ds['exhaustive']
            assert ex['accepted_per_size'] == ds['one_rank']['accepted_per_size'] and sum(ex['accepted_per_size']) > 0
        return
    rec = _bench_ranks(2, config, ['--batch', '65536', '--steps', '2', '--warmup', '1'])
    _check_allgather(rec, 2)


@pytest.mark.gpu
def test_bench_eight_ranks_config4_on_the_gpu():
    """BASELINE config 4's own rank count (8 x 2^20 fp32 filters over 8 GPUs, RCCL all-gather):
    the launch shape the driver's 8-GPU run uses, eight ranks started by `bench.py --gpus 8`
    (gloo: here they share the box's one GPU, 65,536 filters each), every rank checking its shard
    in the all-gathered arrays bitwise."""
    rec = _bench_ranks(8, '4', ['--batch', '65536', '--steps', '2', '--warmup', '1'])
    _check_allgather(rec, 8)
    assert rec['config']['filters_per_gpu'] == 65536
