"""kf_predict held back and fused into the next kf_update (the reference's per-step call shape,
kf_workers.py:688-711, run as one kernel step): the same results as eager predict + update
kernels (option predict='eager'), whatever the caller does between the two calls — needs an MI355X.

Tolerance: the fused step is the kf_run kernel's step and the eager pair the per-op kernels;
they evaluate the same expressions, compared at 1e-12 (fp64) / 1e-5 (fp32) relative.
"""
import ctypes

import numpy as np
import pytest
import torch

import kfmi
from kfmi import _lib

pytestmark = pytest.mark.gpu

RTOL = {'f64': 1e-12, 'f32': 1e-5}
NP = {'f64': np.float64, 'f32': np.float32}


def inputs(name, dtype, B, T, seed):
    d = 3 if name == 'cv3' else 2
    rng = np.random.default_rng(seed)
    x0 = np.zeros((2 * d, B))
    x0[:d] = rng.uniform(-1000, 1000, (d, B))
    u = rng.normal(0, 0.3, (T, d, B)).astype(NP[dtype])
    z = (x0[:d][None] + rng.normal(0, 3, (T, d, B))).astype(NP[dtype])
    cuda = lambda a: torch.from_numpy(np.ascontiguousarray(a.astype(NP[dtype]))).cuda()
    return cuda(x0), [cuda(u[t]) for t in range(T)], [cuda(z[t]) for t in range(T)]


def close(a, b, dtype):
    a, b = a.double().cpu().numpy(), b.double().cpu().numpy()
    np.testing.assert_allclose(a, b, rtol=RTOL[dtype], atol=RTOL[dtype])


def run_script(name, dtype, x0, script):
    """script(kf) -> list of tensors to compare; run once deferred, once eager."""
    outs = []
    for mode in ('deferred', 'eager'):
        kf = kfmi.BatchedKF(name, x0.shape[1], dtype, options={'predict': mode})
        kf.reset(x0)
        res = [r.clone() for r in script(kf)]
        x, P = kf.state()
        res += [x, P, kf.status()]
        torch.cuda.synchronize()
        kf.close()
        outs.append(res)
    return outs


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
@pytest.mark.parametrize('name', ['cv2', 'cv3'])
def test_per_step_loop_deferred_equals_eager(name, dtype):
    """predict(dt, u) + update(z) per step, with a mask, no-control predicts, and an async
    stretch (three predicts before an update: the first two run as plain predicts)."""
    B, T = 1000, 16
    x0, u, z = inputs(name, dtype, B, T, seed=3)
    mask = torch.from_numpy((np.random.default_rng(4).random(B) > 0.3).astype(np.uint8)).cuda()

    def script(kf):
        out = []
        for t in range(T):
            if t % 5 == 4:
                kf.predict(0.05, u[t])
                kf.predict(0.05)
            kf.predict(0.1, u[t] if t % 3 else None)
            out.append(kf.update(z[t], mask=mask if t % 2 else None))
        return out

    got, ref = run_script(name, dtype, x0, script)
    for a, b in zip(got, ref):
        close(a, b, dtype)
    assert int((got[-1] != 0).sum()) == 0


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_control_buffer_reused_after_predict(dtype):
    """The caller may overwrite its u buffer right after kf_predict: the control was copied."""
    B = 512
    x0, u, z = inputs('cv3', dtype, B, 2, seed=5)

    def script(kf):
        buf = u[0].clone()
        kf.predict(0.1, buf)
        buf.fill_(1e6)          # same stream, after the call
        return [kf.update(z[0])]

    def reference(kf):
        kf.predict(0.1, u[0])
        return [kf.update(z[0])]

    got, _ = run_script('cv3', dtype, x0, script)
    ref, _ = run_script('cv3', dtype, x0, reference)
    for a, b in zip(got, ref):
        close(a, b, dtype)


@pytest.mark.parametrize('dtype', ['f64', 'f32'])
def test_state_queries_flush_the_predict(dtype):
    """state(), status(), logdet() and kf_run after a held-back predict see the predicted state."""
    B = 640
    x0, u, z = inputs('cv3', dtype, B, 4, seed=6)

    def script(kf):
        kf.predict(0.1, u[0])
        x1, P1 = kf.state()
        kf.predict(0.2, u[1])
        st = kf.status().to(torch.float64)
        kf.predict(0.3, u[2])
        ld = kf.logdet()
        kf.predict(0.1, u[3])
        ut = torch.stack([u[0], u[1]])
        zt = torch.stack([z[0], z[1]])
        tr, ld2 = kf.run(ut, zt, dt=0.1)
        return [x1, P1, st, ld, tr, ld2]

    got, ref = run_script('cv3', dtype, x0, script)
    for a, b in zip(got, ref):
        close(a, b, dtype)


def test_reset_and_set_state_after_predict():
    """reset / a full set_state overwrite a held-back predict; setting x alone keeps P's predict."""
    B = 320
    x0, u, z = inputs('cv3', 'f64', B, 2, seed=7)
    x_new = x0 * 0.5
    lib = _lib.lib()

    def script(kf):
        kf.predict(0.1, u[0])
        kf.reset(x0)
        a = kf.update(z[0])
        kf.predict(0.1, u[1])
        xs, Ps = kf.state()
        kf.predict(0.4, u[0])
        kf.set_state(xs, Ps)           # both: the predict has no effect
        b = kf.update(z[1])
        kf.predict(0.1, u[1])          # x alone: P keeps this predict
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        _lib.check(lib.kf_set_state(kf.handle, ctypes.c_void_p(x_new.data_ptr()), None, 1, st))
        c = kf.update(z[0])
        return [a, b, c]

    got, ref = run_script('cv3', 'f64', x0, script)
    for a, b in zip(got, ref):
        close(a, b, 'f64')


def test_predict_and_update_on_two_streams():
    """predict on stream A, update on stream B after B waits for A (and the control copy)."""
    B = 2048
    x0, u, z = inputs('cv3', 'f64', B, 6, seed=8)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def script(kf):
        out = []
        torch.cuda.current_stream().synchronize()
        for t in range(6):
            with torch.cuda.stream(sa):
                sa.wait_stream(sb)
                kf.predict(0.1, u[t])
            with torch.cuda.stream(sb):
                sb.wait_stream(sa)
                out.append(kf.update(z[t]).clone())
        torch.cuda.current_stream().wait_stream(sb)
        return out

    got, ref = run_script('cv3', 'f64', x0, script)
    for a, b in zip(got, ref):
        close(a, b, 'f64')


def test_graph_capture_of_the_per_step_loop():
    """A captured predict/update loop replays the control copies and fused steps (the handle
    allocates its control buffer up front, so nothing allocates or synchronises in the loop)."""
    B, T = 1024, 4
    x0, u, z = inputs('cv3', 'f64', B, T, seed=9)
    kf = kfmi.BatchedKF('cv3', B, 'f64')
    ld = [kf.empty(B) for _ in range(T)]
    lib = _lib.lib()

    def loop():
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for t in range(T):
            _lib.check(lib.kf_predict(kf.handle, 0.1, None, ctypes.c_void_p(u[t].data_ptr()), None, st))
            _lib.check(lib.kf_update(kf.handle, ctypes.c_void_p(z[t].data_ptr()), None,
                                     ctypes.c_void_p(ld[t].data_ptr()), st))

    # no warm-up: the C ABI needs none, and a first loop on another stream would make the
    # capture wait on that stream's event (not capturable)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loop()
    kf.reset(x0)
    g.replay()
    torch.cuda.synchronize()
    got = [l.clone() for l in ld] + list(kf.state())
    kf.close()

    kf = kfmi.BatchedKF('cv3', B, 'f64', options={'predict': 'eager'})
    kf.reset(x0)
    ref = []
    for t in range(T):
        kf.predict(0.1, u[t])
        ref.append(kf.update(z[t]))
    ref += list(kf.state())
    torch.cuda.synchronize()
    kf.close()
    for a, b in zip(got, ref):
        close(a, b, 'f64')


def test_warmup_on_one_stream_then_capture_on_another():
    """The torch.cuda.graph pattern: run the per-step loop eagerly on the default
    stream, then capture it (torch captures on a side stream).  The first captured predict's
    control copy would have to wait for the eager loop's last fused step, recorded outside the
    capture: it runs eagerly instead, and the replayed graph gives the eager results."""
    B, T = 1024, 4
    x0, u, z = inputs('cv3', 'f64', B, T, seed=19)
    kf = kfmi.BatchedKF('cv3', B, 'f64')
    ld = [kf.empty(B) for _ in range(T)]
    lib = _lib.lib()

    def loop():
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for t in range(T):
            _lib.check(lib.kf_predict(kf.handle, 0.1, None, ctypes.c_void_p(u[t].data_ptr()), None, st))
            _lib.check(lib.kf_update(kf.handle, ctypes.c_void_p(z[t].data_ptr()), None,
                                     ctypes.c_void_p(ld[t].data_ptr()), st))

    kf.reset(x0)
    loop()                       # warm-up on the default stream: its fused steps read pend_u
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):    # capture on torch's side stream
        loop()
    kf.reset(x0)
    g.replay()
    torch.cuda.synchronize()
    got = [l.clone() for l in ld] + list(kf.state())
    kf.close()

    kf = kfmi.BatchedKF('cv3', B, 'f64', options={'predict': 'eager'})
    kf.reset(x0)
    ref = []
    for t in range(T):
        kf.predict(0.1, u[t])
        ref.append(kf.update(z[t]))
    ref += list(kf.state())
    torch.cuda.synchronize()
    kf.close()
    for a, b in zip(got, ref):
        close(a, b, 'f64')


def test_reader_stream_destroyed_before_next_predict():
    """A fused step on a side stream that the caller then destroys: the next deferred predict
    on the default stream waits on the event recorded right after that read, never on the
    destroyed stream."""
    B, T = 512, 3
    x0, u, z = inputs('cv3', 'f64', B, T, seed=21)
    kf = kfmi.BatchedKF('cv3', B, 'f64')
    kf.reset(x0)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        kf.predict(0.1, u[0])
        l0 = kf.update(z[0])
    torch.cuda.current_stream().wait_stream(s)
    del s
    torch.cuda.synchronize()
    out = [l0]
    for t in range(1, T):
        kf.predict(0.1, u[t])
        out.append(kf.update(z[t]))
    out += list(kf.state())
    torch.cuda.synchronize()
    kf.close()
    kf = kfmi.BatchedKF('cv3', B, 'f64', options={'predict': 'eager'})
    kf.reset(x0)
    ref = []
    for t in range(T):
        kf.predict(0.1, u[t])
        ref.append(kf.update(z[t]))
    ref += list(kf.state())
    torch.cuda.synchronize()
    kf.close()
    for a, b in zip(out, ref):
        close(a, b, 'f64')
