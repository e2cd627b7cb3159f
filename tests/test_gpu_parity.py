"""Parity of the HIP path (through the C ABI) with the CPU oracle — needs an MI355X.

Tolerances (north_star / SURVEY.md §8d): per filter, per step,
    ||x - x_ref||_2 / max(||x_ref||_2, 1)  and  |logdet - logdet_ref| / max(|logdet_ref|, 1)
must be <= 1e-6 for fp64 and <= 1e-3 for fp32.  fp32 runs are compared with the fp64
oracle fed the SAME fp32-rounded inputs.
"""
import os

import numpy as np
import pytest
import torch

import kfmi
from oracle import ref_kf

pytestmark = pytest.mark.gpu

TOL = {'f64': 1e-6, 'f32': 1e-3}
NP = {'f64': np.float64, 'f32': np.float32}
TD = {'f64': torch.float64, 'f32': torch.float32}
MODEL = {'cv2': ref_kf.CV2, 'cv3': ref_kf.CV3}


def random_inputs(model, B, T, k, seed, dt=0.1):
    rng = np.random.default_rng(seed)
    d = model.d
    x0 = np.zeros((B, model.n))
    p0 = rng.uniform(-1000, 1000, (B, d))
    x0[:, :d] = p0 + rng.normal(0, np.sqrt(3), (B, d))
    u = rng.normal(0, 0.3, (T, d, B))
    U = T // k
    drift = np.cumsum(rng.normal(0, dt * k, (U, d, B)), axis=0)
    z = p0.T[None] + drift + rng.normal(0, np.sqrt(3), (U, d, B))
    return x0, u, z


def engine_run(name, dtype, x0, u, z, k, dt=None, dt_steps=None, mask=None):
    B = x0.shape[0]
    kf = kfmi.BatchedKF(name, B, dtype)
    kf.reset(torch.from_numpy(np.ascontiguousarray(x0.T.astype(NP[dtype]))).cuda())
    ut = torch.from_numpy(u.astype(NP[dtype])).cuda()
    zt = torch.from_numpy(z.astype(NP[dtype])).cuda()
    mt = torch.from_numpy(mask.astype(np.uint8)).cuda() if mask is not None else None
    dts = torch.from_numpy(np.asarray(dt_steps, np.float64)).cuda() if dt_steps is not None else None
    tr, ld = kf.run(ut, zt, dt=dt, dt_steps=dts, update_every=k, mask=mt)
    x, P = kf.state()
    st = kf.status()
    torch.cuda.synchronize()
    out = (tr.double().cpu().numpy(), ld.double().cpu().numpy(), x.double().cpu().numpy(),
           P.double().cpu().numpy(), st.cpu().numpy())
    kf.close()
    return out


def rounded(a, dtype):
    return np.asarray(a).astype(NP[dtype]).astype(np.float64)


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
@pytest.mark.parametrize('d', [2, 3])
@pytest.mark.parametrize('k', [1, 5])
def test_golden_reference_vectors(golden_dir, dtype, d, k):
    """The fixtures stepped by the reference's own predict_covariance / calculate_kalman_gain."""
    g = np.load(os.path.join(golden_dir, 'cv_batch.npz'))
    key = f'cv{d}_k{k}'
    dt, u, z, x0 = (g[f'{key}_{s}'] for s in ('dt', 'u', 'z', 'x0'))
    tr, ld, x, P, st = engine_run(f'cv{d}', dtype, x0, u, z, k, dt_steps=dt)
    assert (st == 0).all()
    if dtype == 'f64':
        ref_tr, ref_ld, ref_P = g[f'{key}_traj'], g[f'{key}_logdet'], g[f'{key}_Pfinal']
    else:
        ref_tr, ref_ld, _, ref_P = ref_kf.run_batch(MODEL[f'cv{d}'], rounded(x0, dtype), MODEL[f'cv{d}'].P0(),
                                                    dt, rounded(u, dtype), rounded(z, dtype), k)
    ex, el = ref_kf.parity_errors(tr, ld, ref_tr, ref_ld)
    assert ex <= TOL[dtype], ex
    assert el <= TOL[dtype], el
    Pf = ref_kf.tri_unpack(P, 2 * d)
    assert np.max(np.abs(Pf - ref_P) / np.maximum(np.abs(ref_P), 1.0)) <= 10 * TOL[dtype]


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
@pytest.mark.parametrize('name', ['cv2', 'cv3'])
@pytest.mark.parametrize('B,T,k,dt', [(1000, 64, 1, 0.1), (333, 100, 10, 0.01), (1, 8, 1, 0.1)])
def test_random_batches_vs_oracle(dtype, name, B, T, k, dt):
    model = MODEL[name]
    x0, u, z = random_inputs(model, B, T, k, seed=B + T + k)
    tr, ld, x, P, st = engine_run(name, dtype, x0, u, z, k, dt=dt)
    assert (st == 0).all()
    ref_tr, ref_ld, ref_x, _ = ref_kf.run_batch(model, rounded(x0, dtype), model.P0(), np.full(T, dt),
                                                rounded(u, dtype), rounded(z, dtype), k)
    ex, el = ref_kf.parity_errors(tr, ld, ref_tr, ref_ld)
    assert ex <= TOL[dtype], ex
    assert el <= TOL[dtype], el
    np.testing.assert_array_equal(tr[-1], x)  # the handle's final state is the last step


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_mask_skips_updates(dtype):
    model = ref_kf.CV3
    B, T = 256, 40
    x0, u, z = random_inputs(model, B, T, 1, seed=5)
    mask = np.random.default_rng(6).random((T, B)) > 0.3
    mask[:, 7] = False  # one filter never updates (pure prediction)
    tr, ld, _, _, st = engine_run('cv3', dtype, x0, u, z, 1, dt=0.1, mask=mask)
    ref_tr, ref_ld, _, _ = ref_kf.run_batch(model, rounded(x0, dtype), model.P0(), np.full(T, 0.1),
                                            rounded(u, dtype), rounded(z, dtype), 1, mask=mask)
    ex, el = ref_kf.parity_errors(tr, ld, ref_tr, ref_ld)
    assert ex <= TOL[dtype] and el <= TOL[dtype], (ex, el)


def test_per_step_api_matches_fused_run():
    """predict()/update() per event (the reference's call shape) == the fused kf_run."""
    model = ref_kf.CV3
    B, T = 300, 12
    x0, u, z = random_inputs(model, B, T, 1, seed=9)
    tr, ld, xf, Pf, _ = engine_run('cv3', 'f64', x0, u, z, 1, dt=0.1)
    kf = kfmi.BatchedKF('cv3', B, 'f64')
    kf.reset(torch.from_numpy(np.ascontiguousarray(x0.T)).cuda())
    for t in range(T):
        kf.predict(0.1, torch.from_numpy(np.ascontiguousarray(u[t])).cuda())
        l = kf.update(torch.from_numpy(np.ascontiguousarray(z[t])).cuda())
        x, _ = kf.state()
        np.testing.assert_allclose(x.cpu().numpy(), tr[t], rtol=1e-13, atol=1e-9)
        np.testing.assert_allclose(l.cpu().numpy(), ld[t], rtol=1e-12, atol=1e-12)
    x, P = kf.state()
    np.testing.assert_allclose(P.cpu().numpy(), Pf, rtol=1e-12, atol=1e-12)


def test_predict_logdet_and_per_filter_dt():
    model = ref_kf.CV3
    B = 128
    rng = np.random.default_rng(3)
    dtf = rng.uniform(0.0, 0.5, B)
    kf = kfmi.BatchedKF('cv3', B, 'f64')
    ld = kf.predict(None, dt_per_filter=torch.from_numpy(dtf).cuda(), logdet=True).cpu().numpy()
    x, P = kf.state()
    P = ref_kf.tri_unpack(P.cpu().numpy(), 6)
    for b in (0, 17, B - 1):
        F = model.F(dtf[b])
        Pr = ref_kf.predict_covariance(model.P0(), F, model.Q(dtf[b]))
        np.testing.assert_allclose(P[b], Pr, rtol=1e-14)
        assert abs(ld[b] - np.linalg.slogdet(Pr)[1]) < 1e-10


def test_chunked_runs_resume_bit_exactly():
    """(x, P) stay in HBM between launches: T=48 in one launch == 3 launches of 16."""
    model = ref_kf.CV3
    B, T = 513, 48
    x0, u, z = random_inputs(model, B, T, 1, seed=11)
    tr, ld, xf, Pf, _ = engine_run('cv3', 'f64', x0, u, z, 1, dt=0.1)
    kf = kfmi.BatchedKF('cv3', B, 'f64')
    kf.reset(torch.from_numpy(np.ascontiguousarray(x0.T)).cuda())
    parts = []
    for s in range(0, T, 16):
        t_, l_ = kf.run(torch.from_numpy(u[s:s + 16].copy()).cuda(), torch.from_numpy(z[s:s + 16].copy()).cuda(),
                        dt=0.1)
        parts.append((t_.cpu().numpy(), l_.cpu().numpy()))
    np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), tr)
    np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]), ld)
    x, P = kf.state()
    np.testing.assert_array_equal(P.cpu().numpy(), Pf)


@pytest.mark.parametrize('dtype,k,chunks', [('f64', 1, 8), ('f32', 2, 4), ('f64', 4, 5)])
def test_run_host_pipeline_matches_one_run(dtype, k, chunks):
    """run_host (host streams, H2D | launch | D2H overlapped over time chunks) == one run on
    device-resident streams, bit for bit; chunks=5 with T=64, k=4 falls back to 4 chunks."""
    model = ref_kf.CV3
    B, T = 1031, 64
    x0, u, z = random_inputs(model, B, T, k, seed=23)
    tr, ld, xf, Pf, _ = engine_run('cv3', dtype, x0, u, z, k, dt=0.1)
    kf = kfmi.BatchedKF('cv3', B, dtype)
    kf.reset(torch.from_numpy(np.ascontiguousarray(x0.T.astype(NP[dtype]))).cuda())
    ht, hl = kf.run_host(u.astype(NP[dtype]), z.astype(NP[dtype]), dt=0.1, update_every=k, chunks=chunks)
    assert ht.device.type == 'cpu' and ht.is_pinned()
    np.testing.assert_array_equal(ht.double().numpy(), tr)
    np.testing.assert_array_equal(hl.double().numpy(), ld)
    x, P = kf.state()
    np.testing.assert_array_equal(P.double().cpu().numpy(), Pf)
    kf.close()


def test_deterministic_repeat():
    model = ref_kf.CV2
    x0, u, z = random_inputs(model, 2048, 32, 1, seed=2)
    a = engine_run('cv2', 'f32', x0, u, z, 1, dt=0.1)
    b = engine_run('cv2', 'f32', x0, u, z, 1, dt=0.1)
    for p, q in zip(a, b):
        np.testing.assert_array_equal(p, q)


def test_not_spd_flags_only_bad_filters():
    """A filter whose covariance is not PD gets status KF_ENOTSPD and NaN outputs; the others
    are untouched (the reference skips a failing combo, kf_workers.py:88-91)."""
    B, T = 200, 6
    model = ref_kf.CV3
    x0, u, z = random_inputs(model, B, T, 1, seed=4)
    P = np.broadcast_to(model.P0(), (B, 6, 6)).copy()
    bad = [3, 64, 199]
    for b in bad:
        P[b, 1, 1] = -1e5   # S = P[0:3,0:3] + R has a negative pivot
    kf = kfmi.BatchedKF('cv3', B, 'f64')
    kf.set_state(torch.from_numpy(np.ascontiguousarray(x0.T)).cuda(),
                 torch.from_numpy(ref_kf.tri_pack(P)).cuda())
    tr, ld = kf.run(torch.from_numpy(u).cuda(), torch.from_numpy(z).cuda(), dt=0.1)
    st = kf.status().cpu().numpy()
    tr = tr.cpu().numpy()
    assert set(np.nonzero(st)[0]) == set(bad)
    assert (st[bad] == kfmi.KF_ENOTSPD).all()
    assert np.isnan(tr[:, :, bad]).all()
    good = np.setdiff1d(np.arange(B), bad)
    ref_tr, ref_ld, _, _ = ref_kf.run_batch(model, x0[good], model.P0(), np.full(T, 0.1), u[:, :, good],
                                            z[:, :, good], 1)
    ex, el = ref_kf.parity_errors(tr[:, :, good], ld.cpu().numpy()[:, good], ref_tr, ref_ld)
    assert ex <= 1e-6 and el <= 1e-6


def test_empty_batch_and_zero_steps():
    kf = kfmi.BatchedKF('cv3', 0, 'f64')
    tr, ld = kf.run(torch.empty(5, 3, 0, dtype=torch.float64, device='cuda'),
                    torch.empty(5, 3, 0, dtype=torch.float64, device='cuda'), dt=0.1)
    assert tr.shape == (5, 6, 0)
    kf2 = kfmi.BatchedKF('cv3', 10, 'f64')
    tr, ld = kf2.run(torch.empty(0, 3, 10, dtype=torch.float64, device='cuda'),
                     torch.empty(0, 3, 10, dtype=torch.float64, device='cuda'), dt=0.1)
    assert tr.shape == (0, 6, 10)
    x, P = kf2.state()
    np.testing.assert_array_equal(P[0].cpu().numpy(), 1e4)


def test_shape_errors_raise_before_launch():
    kf = kfmi.BatchedKF('cv3', 16, 'f64')
    with pytest.raises(ValueError):
        kf.run(torch.zeros(4, 2, 16, dtype=torch.float64, device='cuda'),
               torch.zeros(4, 3, 16, dtype=torch.float64, device='cuda'), dt=0.1)
    with pytest.raises(TypeError):
        kf.run(torch.zeros(4, 3, 16, dtype=torch.float32, device='cuda'),
               torch.zeros(4, 3, 16, dtype=torch.float64, device='cuda'), dt=0.1)
    with pytest.raises(kfmi.KFError):
        kf.run(torch.zeros(4, 3, 16, dtype=torch.float64, device='cuda'),
               torch.zeros(4, 3, 16, dtype=torch.float64, device='cuda'), dt=-1.0)


def test_synth_is_sharding_consistent():
    """Counter-based generation: shard [500, 1000) regenerates exactly the same streams."""
    full = kfmi.BatchedKF('cv3', 1000, 'f64')
    x0, u, z = full.synth(T=20, dt=0.1, update_every=2, seed=7)
    half = kfmi.BatchedKF('cv3', 500, 'f64')
    x0h, uh, zh = half.synth(T=20, dt=0.1, update_every=2, seed=7, filter_offset=500)
    torch.testing.assert_close(x0[:, 500:], x0h, rtol=0, atol=0)
    torch.testing.assert_close(u[:, :, 500:], uh, rtol=0, atol=0)
    torch.testing.assert_close(z[:, :, 500:], zh, rtol=0, atol=0)
    other = kfmi.BatchedKF('cv3', 1000, 'f64').synth(T=20, dt=0.1, update_every=2, seed=8)
    assert not torch.equal(other[1], u)


def test_synth_statistics():
    kf = kfmi.BatchedKF('cv3', 1 << 16, 'f64')
    x0, u, z = kf.synth(T=8, dt=0.1, update_every=1, seed=1)
    pos = x0[:3].flatten()
    assert -1010 < pos.min().item() < -990 and 990 < pos.max().item() < 1010
    assert abs(u.std().item() - np.sqrt(0.3 ** 2 + 0.1 ** 2)) < 0.01
    assert (x0[3:] == 0).all()
    # first fix vs truth one step later: |z - x0| ~ velocity*dt + noise
    assert torch.isfinite(z).all()


FULL_SIZE = {
    # BASELINE.json configs at the sizes bench.py times: name, dtype, B, T, dt, k
    'config2': ('cv2', 'f32', 1 << 16, 1024, 0.1, 1),
    'config3': ('cv3', 'f64', 1 << 20, 256, 0.1, 1),
    'config4': ('cv3', 'f32', 1 << 20, 256, 0.1, 1),   # config 4's per-GPU shard
    'config5': ('cv3', 'f64', 1 << 20, 500, 0.01, 10),  # 100 Hz predict, 10 Hz GPS update
}


@pytest.mark.parametrize('config', sorted(FULL_SIZE))
def test_full_size_config_sampled(config):
    """Every BASELINE GPU config at its bench size, on synthetic streams: the oracle (the
    reference step, kf_workers.py:688-717, fed the same — for fp32 fp32-rounded — inputs) on
    >= 4096 sampled filters spread over the batch plus the wave and batch edges, per step
    (every predict-only step of config 5 and every update step's log-det), and size-independent
    properties on all filters.  Config 2's fp32 drift over 1024 steps is the case the 1e-3 gate
    could bite."""
    name, dtype, B, T, dt, k = FULL_SIZE[config]
    model = MODEL[name]
    kf = kfmi.BatchedKF(name, B, dtype)
    x0, u, z = kf.synth(T=T, dt=dt, update_every=k, seed=20251015)
    kf.reset(x0)
    tr, ld = kf.run(u, z, dt=dt, update_every=k)
    st = kf.status()
    assert int((st != 0).sum()) == 0
    assert bool(torch.isfinite(ld).all()) and bool(torch.isfinite(tr).all())
    edges = [0, 1, 62, 63, 64, 65, 127, 128, 255, 256, B // 2 - 1, B // 2, B - 129, B - 65, B - 64, B - 2, B - 1]
    idx = np.unique(np.concatenate([np.linspace(0, B - 1, 4096).astype(np.int64), edges]))
    assert len(idx) >= 4096
    it = torch.from_numpy(idx).cuda()
    xs = x0[:, it].double().cpu().numpy().T
    us = u[:, :, it].double().cpu().numpy()
    zs = z[:, :, it].double().cpu().numpy()
    ref_tr, ref_ld, _, _ = ref_kf.run_batch(model, xs, model.P0(), np.full(T, dt), us, zs, k)
    got_tr, got_ld = tr[:, :, it].double().cpu().numpy(), ld[:, it].double().cpu().numpy()
    ex, el = ref_kf.parity_errors(got_tr, got_ld, ref_tr, ref_ld)
    assert ex <= TOL[dtype], ex
    assert el <= TOL[dtype], el
    if k > 1:  # the update steps on their own (10 Hz GPS): logdet drops there
        up = np.arange(k - 1, T, k)
        _, el_up = ref_kf.parity_errors(got_tr[up], got_ld[up], ref_tr[up], ref_ld[up])
        assert el_up <= TOL[dtype], el_up
        assert (np.diff(ref_ld, axis=0)[up - 1] < 0).all()
    # logdet is identical across filters that share dt/P0 when no filter fails (P does not
    # depend on the data in a linear KF): a checksum across the whole batch
    spread = (ld.max(dim=1).values - ld.min(dim=1).values).abs().max().item()
    assert spread <= (1e-9 if dtype == 'f64' else 1e-3)
    # the handle's final state is the last trajectory row, for every filter
    x, _ = kf.state()
    assert torch.equal(x, tr[-1])
    kf.close()


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
@pytest.mark.parametrize('name', ['cv2', 'cv3'])
@pytest.mark.parametrize('wide', [False, True])
def test_logdet_kernel_on_random_spd(dtype, name, wide):
    """logdet from the in-lane LDL^T (+ reduced-range log) vs numpy slogdet on random SPD
    covariances (predict with dt = 0 leaves P as is).  spread = log10 of the eigenvalue range:
    0.3 isolates the log (strict bound); the wide case checks the factorisation at condition
    number ~1e8 (fp64) / ~1e4 (fp32), where any two backward-stable methods may differ by
    ~kappa * eps."""
    spread = (8.0 if dtype == 'f64' else 4.0) if wide else 0.3
    n = 4 if name == 'cv2' else 6
    B = 4096
    rng = np.random.default_rng(21)
    Qm, _ = np.linalg.qr(rng.normal(size=(B, n, n)))
    ev = 10.0 ** rng.uniform(-spread / 2, spread / 2, (B, n)) * 10.0 ** rng.uniform(-2, 3, (B, 1))
    P = np.einsum('bij,bj,bkj->bik', Qm, ev, Qm)
    P = 0.5 * (P + P.transpose(0, 2, 1))
    Pt = ref_kf.tri_pack(P).astype(NP[dtype])
    kf = kfmi.BatchedKF(name, B, dtype)
    kf.set_state(torch.zeros(n, B, dtype=TD[dtype], device='cuda'), torch.from_numpy(Pt).cuda())
    ld = kf.predict(0.0, logdet=True).double().cpu().numpy()
    Pd = ref_kf.tri_unpack(Pt.astype(np.float64), n)
    ref = np.linalg.slogdet(Pd)[1]
    kappa = np.linalg.cond(Pd)
    eps = np.finfo(NP[dtype]).eps
    err = np.abs(ld - ref) / np.maximum(np.abs(ref), 1.0)
    bound = np.maximum(50 * kappa * eps, 1e-13 if dtype == 'f64' else 2e-6)
    assert (err <= bound).all(), float((err / bound).max())
    assert (kf.status().cpu().numpy() == 0).all()


def _run_with_kernel(kernel, name, dtype, x0, u, z, k, dt, P=None):
    B = x0.shape[0]
    kf = kfmi.BatchedKF(name, B, dtype, options={'cv_kernel': kernel})
    kf.reset(torch.from_numpy(np.ascontiguousarray(x0.T.astype(NP[dtype]))).cuda())
    if P is not None:
        kf.set_state(np.ascontiguousarray(x0.T.astype(NP[dtype])), np.ascontiguousarray(P.astype(NP[dtype])))
    tr, ld = kf.run(torch.from_numpy(u.astype(NP[dtype])).cuda(), torch.from_numpy(z.astype(NP[dtype])).cuda(),
                    dt=dt, update_every=k)
    x, Pp = kf.state()
    out = [v.cpu().numpy() for v in (tr, ld, x, Pp, kf.status())]
    kf.close()
    return out


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
@pytest.mark.parametrize('name', ['cv2', 'cv3'])
@pytest.mark.parametrize('k', [1, 10])
@pytest.mark.parametrize('variant', ['block2', 'block4', 'block8'])
def test_block_kernel_equals_general_kernel(dtype, name, k, variant):
    """With the reference's diagonal R and P0, P stays block-diagonal over the axes and
    kf_run uses cv_block_kernel (prefetch depth 2, or 4 for few filters); it evaluates the general
    kernel's expressions for the non-zero entries in the same order, so all produce the same
    numbers."""
    model = MODEL[name]
    x0, u, z = random_inputs(model, 777, 60, k, seed=11 + k)
    blk = _run_with_kernel(variant, name, dtype, x0, u, z, k, 0.1 if k == 1 else 0.01)
    gen = _run_with_kernel('general', name, dtype, x0, u, z, k, 0.1 if k == 1 else 0.01)
    for a, b in zip(blk, gen):
        np.testing.assert_array_equal(a, b)


def test_block_check_falls_back_for_coupled_covariance():
    """set_state with a P that couples the axes must take the general kernel (the block check
    on the device); a block-diagonal P keeps the block kernel; both match the oracle."""
    model = MODEL['cv3']
    B, T = 64, 30
    x0, u, z = random_inputs(model, B, T, 1, seed=5)
    rng = np.random.default_rng(6)
    A = rng.normal(size=(B, 6, 6))
    Pfull = np.einsum('bij,bkj->bik', A, A) + 50 * np.eye(6)
    Pblock = Pfull.copy()
    for i in range(6):
        for j in range(6):
            if i % 3 != j % 3:
                Pblock[:, i, j] = 0.0
    for P in (Pfull, Pblock):
        packed = ref_kf.tri_pack(P)                        # [21, B]
        tr, ld, _, _, st = _run_with_kernel('auto', 'cv3', 'f64', x0, u, z, 1, 0.1, P=packed)
        gen = _run_with_kernel('general', 'cv3', 'f64', x0, u, z, 1, 0.1, P=packed)
        np.testing.assert_array_equal(tr, gen[0])
        rt, rl, _, _ = ref_kf.run_batch(model, x0, P, np.full(T, 0.1), u, z, 1)
        ex, el = ref_kf.parity_errors(tr, ld, rt, rl)
        assert ex <= 1e-6 and el <= 1e-6 and (st == 0).all()


@pytest.mark.parametrize('name,dtype', [('cv3', 'f64'), ('cv2', 'f32'), ('cv3', 'f32')])
@pytest.mark.parametrize('coupled', [False, True])
def test_per_step_calls_block_and_coupled(name, dtype, coupled):
    """predict()/update() per step from a set_state P: block-diagonal (the calls move only the
    per-axis blocks) or coupling the axes (the calls move all of P), against the oracle loop."""
    model = MODEL[name]
    n, d = model.n, model.d
    B, T = 96, 20
    x0, u, z = random_inputs(model, B, T, 1, seed=11)
    rng = np.random.default_rng(12)
    A = rng.normal(size=(B, n, n))
    P = np.einsum('bij,bkj->bik', A, A) + 50 * np.eye(n)
    if not coupled:
        for i in range(n):
            for j in range(n):
                if i % d != j % d:
                    P[:, i, j] = 0.0
    if dtype == 'f32':
        x0, u, z, P = (rounded(v, 'f32') for v in (x0, u, z, P))
    kf = kfmi.BatchedKF(name, B, dtype)
    kf.set_state(torch.from_numpy(np.ascontiguousarray(x0.T.astype(NP[dtype]))).cuda(),
                 torch.from_numpy(ref_kf.tri_pack(P).astype(NP[dtype])).cuda())
    xs, lds = [], []
    for t in range(T):
        kf.predict(0.1, torch.from_numpy(np.ascontiguousarray(u[t].astype(NP[dtype]))).cuda())
        lds.append(kf.update(torch.from_numpy(np.ascontiguousarray(z[t].astype(NP[dtype]))).cuda())
                   .double().cpu().numpy())
        xs.append(kf.state()[0].double().cpu().numpy())
    kf.close()
    rt, rl, _, _ = ref_kf.run_batch(model, x0, P, np.full(T, 0.1), u, z, 1)
    ex, el = ref_kf.parity_errors(np.array(xs), np.array(lds), rt, rl)
    assert ex <= TOL[dtype] and el <= TOL[dtype], (ex, el)
