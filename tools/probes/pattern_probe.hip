// The access-pattern ceiling of the bench kernel, measured beside it: cv_block_kernel's memory
// instructions — the same raw buffer loads of u and z (z only on update steps) through the same
// 8-deep register ring, the same trajectory and log-det row stores — with the filter arithmetic
// reduced to a running sum.  bench.py runs it on the bench's own buffers (same physical pages,
// DESIGN.md §4) right after its timed region, so kernel GB/s / probe GB/s says how close the
// filter kernel is to what this access pattern can move on this box.  Not product code: the
// library never loads it.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/probes/libpattern_probe.so tools/probes/pattern_probe.hip
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../sensorfusion-kalmanfilter_amd/csrc/kf_common.h"

namespace {
using namespace kfmi::dev;

template <int D, typename T>
struct ProbeIn {
    T u[D], z[D];
};

template <int D, typename T, int DEPTH>
__global__ __launch_bounds__(256) void pattern_kernel(const void* u, const void* z, void* traj, void* logdet, int64_t B,
                                                      int T_, int k_upd) {
    constexpr int N = 2 * D;
    const int64_t f = int64_t(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(B) * uint32_t(sizeof(T));
    const int U = T_ / k_upd;
    int ld_upd_step = k_upd - 1;
    int ld_s = 0;
    const uint32_t rb_z = U > 0 ? rb : 0u;
    auto load_in = [&](int t, ProbeIn<D, T>& in) {
        const int tc = t < T_ ? t : T_ - 1;
        if (tc > ld_upd_step) {
            ld_upd_step += k_upd;
            ++ld_s;
        }
#pragma unroll
        for (int i = 0; i < D; ++i) in.u[i] = ldb_stream(u, int64_t(tc) * D + i, rb, off, T(0));
        int s = ld_s < U ? ld_s : U - 1;
        s = s > 0 ? s : 0;
        const uint32_t rbz = tc == ld_upd_step ? rb_z : 0u;  // z only on update steps
#pragma unroll
        for (int i = 0; i < D; ++i) in.z[i] = ldb_stream(z, int64_t(s) * D + i, rbz, off, T(0));
    };
    T acc = T(0);
    auto step = [&](int t, const ProbeIn<D, T>& in) {
#pragma unroll
        for (int i = 0; i < D; ++i) acc += in.u[i] + in.z[i];
#pragma unroll
        for (int i = 0; i < N; ++i) stb(traj, int64_t(t) * N + i, rb, off, acc + T(i));
        stb(logdet, t, rb, off, acc);
    };
    ProbeIn<D, T> buf[DEPTH];
#pragma unroll
    for (int j = 0; j < DEPTH - 1; ++j) load_in(j, buf[j]);
    __builtin_amdgcn_s_waitcnt(0);
    int t = 0;
    for (; t + DEPTH <= T_; t += DEPTH) {
#pragma unroll
        for (int j = 0; j < DEPTH; ++j) {
            load_in(t + j + DEPTH - 1, buf[(j + DEPTH - 1) % DEPTH]);
            step(t + j, buf[j]);
        }
    }
#pragma unroll
    for (int j = 0; j < DEPTH - 1; ++j)
        if (t + j < T_) step(t + j, buf[j]);
}

template <int D, typename T>
hipError_t launch(const void* u, const void* z, void* traj, void* logdet, int64_t B, int T_, int k, hipStream_t st) {
    pattern_kernel<D, T, 8><<<dim3(unsigned((B + 255) / 256)), 256, 0, st>>>(u, z, traj, logdet, B, T_, k);
    return hipGetLastError();
}
}  // namespace

// u [T][axes][B], z [T / update_every][axes][B], traj [T][2 axes][B], logdet [T][B] (device,
// element type f64 ? double : float).  0 on success, else the hipError_t.
extern "C" int kfprobe_pattern(int axes, int f64, const void* u, const void* z, void* traj, void* logdet, int64_t B,
                               int T, int update_every, void* stream) {
    if ((axes != 2 && axes != 3) || B <= 0 || T <= 0 || update_every < 1 || B * 8 >= (int64_t(1) << 31))
        return int(hipErrorInvalidValue);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (axes == 3) e = f64 ? launch<3, double>(u, z, traj, logdet, B, T, update_every, st)
                           : launch<3, float>(u, z, traj, logdet, B, T, update_every, st);
    else e = f64 ? launch<2, double>(u, z, traj, logdet, B, T, update_every, st)
                 : launch<2, float>(u, z, traj, logdet, B, T, update_every, st);
    return int(e);
}
