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
        for (int i = 0; i < N; ++i) stb_rec(traj, int64_t(t) * N + i, rb, off, acc + T(i));
        stb_rec(logdet, t, rb, off, acc);
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

// Round 5 candidate: pattern_kernel with its stores phase-separated from its
// loads per wave — each step's six trajectory values and log-det are held in registers for HOLD
// steps and stored as one burst of HOLD * 7 row stores, so a wave alternates runs of loads with
// runs of stores instead of interleaving them every step.  Same loads, same rows, same bytes.
template <int D, typename T, int DEPTH, int HOLD>
__global__ __launch_bounds__(256) void pattern_burst_kernel(const void* u, const void* z, void* traj, void* logdet,
                                                            int64_t B, int T_, int k_upd) {
    constexpr int N = 2 * D;
    static_assert(DEPTH % HOLD == 0, "bursts end at ring boundaries");
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
        const uint32_t rbz = tc == ld_upd_step ? rb_z : 0u;
#pragma unroll
        for (int i = 0; i < D; ++i) in.z[i] = ldb_stream(z, int64_t(s) * D + i, rbz, off, T(0));
    };
    T acc = T(0);
    T held[HOLD][N + 1];
    auto step = [&](int j, const ProbeIn<D, T>& in) {
#pragma unroll
        for (int i = 0; i < D; ++i) acc += in.u[i] + in.z[i];
#pragma unroll
        for (int i = 0; i < N; ++i) held[j % HOLD][i] = acc + T(i);
        held[j % HOLD][N] = acc;
    };
    auto burst = [&](int t0, int n) {
#pragma unroll
        for (int h = 0; h < HOLD; ++h) {
            if (h >= n) break;
#pragma unroll
            for (int i = 0; i < N; ++i) stb_rec(traj, int64_t(t0 + h) * N + i, rb, off, held[h][i]);
            stb_rec(logdet, t0 + h, rb, off, held[h][N]);
        }
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
            step(j, buf[j]);
            if (j % HOLD == HOLD - 1) burst(t + j - (HOLD - 1), HOLD);
        }
    }
    int h = 0;
#pragma unroll
    for (int j = 0; j < DEPTH - 1; ++j)
        if (t + j < T_) {
            step(j, buf[j]);
            ++h;
            if (h == HOLD) {
                burst(t + j - (HOLD - 1), HOLD);
                h = 0;
            }
        }
    if (h) burst(T_ - h, h);
}

// ref_events_lds_kernel's memory instructions (kf_ref.hip): the state rows loaded once and
// stored once, each event's payload / dt / type moved HBM -> LDS by buffer_load ... lds into
// one of two per-wave images while the previous event is consumed, the same counted waits, and
// per event the six trajectory rows, the log-det row and the (zero-length) updated row stored.
// The 15-state event arithmetic is reduced to a sum of the event's inputs.
constexpr int vmcnt_imm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

template <typename T>
__global__ __launch_bounds__(256) void ref_pattern_kernel(const uint8_t* etype, const double* dtp, const void* payload,
                                                          void* x, void* P, void* traj, void* logdet, int64_t B,
                                                          int T_) {
    constexpr int W = int(sizeof(T));
    constexpr int PAY = 9 * 64 * W;
    constexpr int NIP = (PAY + 1023) / 1024;
    constexpr int LPR = 4 * W;
    constexpr int DT_OFF = NIP * 1024, ET_OFF = DT_OFF + 1024, IMG = ET_OFF + 64;
    constexpr int NDMA = NIP + 2;
    constexpr int NST = 6 + 2;  // traj, logdet, updated
    __shared__ __attribute__((aligned(16))) unsigned char lds[4 * 2 * IMG];
    const int lane = int(threadIdx.x & 63);
    const int wave = wave_uniform(int(threadIdx.x >> 6));
    const int64_t f0 = int64_t(blockIdx.x) * 256 + int64_t(wave) * 64;
    if (f0 >= B) return;
    unsigned char* const img0 = lds + wave * 2 * IMG;
    const uint32_t off = uint32_t(f0 + lane) * uint32_t(W);
    const uint32_t rb = uint32_t(B) * uint32_t(W);
    T st[42];
#pragma unroll
    for (int i = 0; i < 15; ++i) st[i] = ldb<T>(x, i, rb, off);
#pragma unroll
    for (int i = 0; i < 27; ++i) st[15 + i] = ldb<T>(P, i, rb, off);
    waitcnt<vmcnt_imm(0)>();
    const uint32_t voff_pay = uint32_t(lane / LPR) * rb + uint32_t(lane % LPR) * 16u;
    auto issue = [&](int t, unsigned char* img) {
        const char* pb = reinterpret_cast<const char*>(payload) + int64_t(t) * 9 * int64_t(rb) + f0 * W;
        const __amdgpu_buffer_rsrc_t rp = bytes_rsrc(pb, 9u * rb - uint32_t(f0) * W);
#pragma unroll
        for (int k = 0; k < NIP; ++k)
            if (k + 1 < NIP || k * 1024 + lane * 16 < PAY) lds_dma16(rp, img + k * 1024, voff_pay, k * (16 / W) * int(rb));
        const char* db = reinterpret_cast<const char*>(dtp) + int64_t(t) * B * 8 + f0 * 8;
        if (lane < 32) lds_dma16(bytes_rsrc(db, uint32_t(B - f0) * 8u), img + DT_OFF, uint32_t(lane) * 16u, 0);
        const char* eb = reinterpret_cast<const char*>(etype) + int64_t(t) * B + f0;
        if (lane < 4) lds_dma16(bytes_rsrc(eb, uint32_t(B - f0)), img + ET_OFF, uint32_t(lane) * 16u, 0);
    };
    issue(0, img0);
    waitcnt<vmcnt_imm(0)>();
    T acc = T(0);
    for (int t = 0; t < T_; ++t) {
        unsigned char* const img = img0 + (t & 1) * IMG;
        if (t + 1 < T_) {
            issue(t + 1, img0 + ((t + 1) & 1) * IMG);
            waitcnt<vmcnt_imm(NST + NDMA)>();
        } else {
            waitcnt<vmcnt_imm(NST)>();
        }
        const int type = img[ET_OFF + lane];
        acc += T(reinterpret_cast<const double*>(img + DT_OFF)[lane]) + T(type);
        const T* pay = reinterpret_cast<const T*>(img) + lane;
#pragma unroll
        for (int i = 0; i < 9; ++i) acc += pay[i * 64];
#pragma unroll
        for (int i = 0; i < 6; ++i) stb(traj, int64_t(t) * 6 + i, rb, off, acc + T(i));
        stb(logdet, t, rb, off, acc);
        stb_u8(nullptr, t, 0u, uint32_t(f0 + lane), uint8_t(type != 255));
    }
#pragma unroll
    for (int i = 0; i < 15; ++i) stb(x, i, rb, off, st[i] + acc);
#pragma unroll
    for (int i = 0; i < 27; ++i) stb(P, i, rb, off, st[15 + i] + acc);
}

// Candidate pattern for the cv kernels (round 2 A/B): the same u, z row loads moved HBM -> LDS by
// buffer_load_dwordx4 ... lds (16 B per lane, 1 KiB per instruction: two 512-B rows) into
// per-wave images of PAIR steps, double-buffered, instead of 8 B per lane into an 8-deep
// register ring.  fp64, update every step.  Per image: u rows 3 PAIR consecutive rows of the
// [T*3][B] array, z likewise; row r of the image at img + r * 512.
template <int PAIR>
__global__ __launch_bounds__(256) void pattern_lds_kernel(const void* u, const void* z, void* traj, void* logdet,
                                                          int64_t B, int T_) {
    constexpr int D = 3, N = 6, W = 8;
    constexpr int ROWS = D * PAIR;              // u rows (and z rows) per image
    constexpr int NI = (ROWS + 1) / 2;          // DMA instructions per array per image
    constexpr int IMG = 2 * NI * 1024;          // u part then z part
    constexpr int NDMA = 2 * NI, NST = PAIR * (N + 1);
    static_assert(ROWS % 2 == 0, "whole 1-KiB DMA instructions only");
    __shared__ __attribute__((aligned(16))) unsigned char lds[4 * 2 * IMG];
    const int lane = int(threadIdx.x & 63);
    const int wave = wave_uniform(int(threadIdx.x >> 6));
    const int64_t f0 = int64_t(blockIdx.x) * 256 + int64_t(wave) * 64;
    if (f0 >= B) return;
    unsigned char* const img0 = lds + wave * 2 * IMG;
    const uint32_t off = uint32_t(f0 + lane) * uint32_t(W);
    const uint32_t rb = uint32_t(B) * uint32_t(W);
    const uint32_t voff = uint32_t(lane >> 5) * rb + uint32_t(lane & 31) * 16u;
    const int NP = T_ / PAIR;
    auto issue = [&](int p, unsigned char* img) {
        const int64_t r0 = int64_t(p) * ROWS;
        const uint32_t len = uint32_t(ROWS) * rb - uint32_t(f0) * W;
        const __amdgpu_buffer_rsrc_t ru =
            bytes_rsrc(reinterpret_cast<const char*>(u) + r0 * int64_t(rb) + f0 * W, len);
        const __amdgpu_buffer_rsrc_t rz =
            bytes_rsrc(reinterpret_cast<const char*>(z) + r0 * int64_t(rb) + f0 * W, len);
#pragma unroll
        for (int k = 0; k < NI; ++k) lds_dma16(ru, img + k * 1024, voff, 2 * k * int(rb));
#pragma unroll
        for (int k = 0; k < NI; ++k) lds_dma16(rz, img + (NI + k) * 1024, voff, 2 * k * int(rb));
    };
    issue(0, img0);
    waitcnt<vmcnt_imm(0)>();
    double acc = 0.0;
    for (int p = 0; p < NP; ++p) {
        unsigned char* const img = img0 + (p & 1) * IMG;
        if (p + 1 < NP) {
            issue(p + 1, img0 + ((p + 1) & 1) * IMG);
            waitcnt<vmcnt_imm(NST + NDMA)>();
        } else {
            waitcnt<vmcnt_imm(NST)>();
        }
        const double* iu = reinterpret_cast<const double*>(img) + lane;
        const double* iz = reinterpret_cast<const double*>(img + NI * 1024) + lane;
#pragma unroll
        for (int s = 0; s < PAIR; ++s) {
            const int t = p * PAIR + s;
#pragma unroll
            for (int i = 0; i < D; ++i) acc += iu[(s * D + i) * 64] + iz[(s * D + i) * 64];
#pragma unroll
            for (int i = 0; i < N; ++i) stb(traj, int64_t(t) * N + i, rb, off, acc + double(i));
            stb(logdet, t, rb, off, acc);
        }
    }
}

// SURVEY.md §7's alternative mapping, one filter per wavefront (the north_star's wording), as an
// arithmetic-free pattern on the same [T][c][B] streams: wave w owns filter w; per step lanes
// 0-2 load u, lanes 3-5 load z (8 B each from rows B * 8 bytes apart), the six values meet in
// an LDS tile (the filter's shared state), and lanes 0-5 store the trajectory, lane 6 the
// log-det.  fp64, cv3, update every step.  Compared with the lane-per-filter ring above it says
// what the layout alone allows this mapping.
__global__ __launch_bounds__(256) void pattern_wave_kernel(const double* __restrict__ u, const double* __restrict__ z,
                                                           double* __restrict__ traj, double* __restrict__ logdet,
                                                           int64_t B, int T_) {
    __shared__ double tile[4][8];
    const int lane = int(threadIdx.x & 63);
    const int wave = int(threadIdx.x >> 6);
    const int64_t f = int64_t(blockIdx.x) * 4 + wave;
    if (f >= B) return;
    double acc = 0.0;
    for (int t = 0; t < T_; ++t) {
        double v = 0.0;
        if (lane < 3) v = u[(int64_t(t) * 3 + lane) * B + f];
        else if (lane < 6) v = z[(int64_t(t) * 3 + lane - 3) * B + f];
        if (lane < 6) tile[wave][lane] = v;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        double s = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) s += tile[wave][i];
        acc += s;
        if (lane < 6) traj[(int64_t(t) * 6 + lane) * B + f] = acc + double(lane);
        else if (lane == 6) logdet[int64_t(t) * B + f] = acc;
        __builtin_amdgcn_wave_barrier();
    }
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

// pattern_burst_kernel (cv3 / cv2 buffers as kfprobe_pattern; hold = 1, 2, 4 or 8 steps per
// store burst; hold 1 is pattern_kernel's interleaving).
extern "C" int kfprobe_pattern_burst(int axes, int f64, const void* u, const void* z, void* traj, void* logdet,
                                     int64_t B, int T, int update_every, int hold, void* stream) {
    if ((axes != 2 && axes != 3) || B <= 0 || T <= 0 || update_every < 1 || B * 8 >= (int64_t(1) << 31))
        return int(hipErrorInvalidValue);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 g(unsigned((B + 255) / 256));
#define KF_BURST(H)                                                                                            \
    if (hold == H) {                                                                                           \
        if (axes == 3 && f64) pattern_burst_kernel<3, double, 8, H><<<g, 256, 0, st>>>(u, z, traj, logdet, B, T, update_every); \
        else if (axes == 3) pattern_burst_kernel<3, float, 8, H><<<g, 256, 0, st>>>(u, z, traj, logdet, B, T, update_every);   \
        else if (f64) pattern_burst_kernel<2, double, 8, H><<<g, 256, 0, st>>>(u, z, traj, logdet, B, T, update_every);        \
        else pattern_burst_kernel<2, float, 8, H><<<g, 256, 0, st>>>(u, z, traj, logdet, B, T, update_every);                  \
        return int(hipGetLastError());                                                                         \
    }
    KF_BURST(1)
    KF_BURST(2)
    KF_BURST(4)
    KF_BURST(8)
#undef KF_BURST
    return int(hipErrorInvalidValue);
}

// etype [T][B] u8, dt [T][B] f64, payload [T][9][B], x [15][B], P [27][B], traj [T][6][B],
// logdet [T][B] (device; element type f64 ? double : float).  B % 64 == 0.
extern "C" int kfprobe_ref_pattern(int f64, const void* etype, const void* dt, const void* payload, void* x, void* P,
                                   void* traj, void* logdet, int64_t B, int T, void* stream) {
    if (B <= 0 || B % 64 != 0 || T <= 0 || 9 * B * 8 >= (int64_t(1) << 32)) return int(hipErrorInvalidValue);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    const dim3 grid(unsigned((B + 255) / 256));
    const uint8_t* et = static_cast<const uint8_t*>(etype);
    const double* d = static_cast<const double*>(dt);
    if (f64) ref_pattern_kernel<double><<<grid, 256, 0, st>>>(et, d, payload, x, P, traj, logdet, B, T);
    else ref_pattern_kernel<float><<<grid, 256, 0, st>>>(et, d, payload, x, P, traj, logdet, B, T);
    return int(hipGetLastError());
}

// pattern_lds_kernel<2> on cv3 f64 buffers, update every step (u, z [T][3][B], traj [T][6][B],
// logdet [T][B]); B % 64 == 0, T even.
extern "C" int kfprobe_pattern_lds(const void* u, const void* z, void* traj, void* logdet, int64_t B, int T,
                                   void* stream) {
    if (B <= 0 || B % 64 != 0 || T <= 0 || T % 2 != 0 || 6 * B * 8 >= (int64_t(1) << 32))
        return int(hipErrorInvalidValue);
    pattern_lds_kernel<2><<<dim3(unsigned((B + 255) / 256)), 256, 0, static_cast<hipStream_t>(stream)>>>(
        u, z, traj, logdet, B, T);
    return int(hipGetLastError());
}

// pattern_wave_kernel on cv3 f64 buffers (as kfprobe_pattern_lds).
extern "C" int kfprobe_pattern_wave(const void* u, const void* z, void* traj, void* logdet, int64_t B, int T,
                                    void* stream) {
    if (B <= 0 || T <= 0) return int(hipErrorInvalidValue);
    pattern_wave_kernel<<<dim3(unsigned((B + 3) / 4)), 256, 0, static_cast<hipStream_t>(stream)>>>(
        static_cast<const double*>(u), static_cast<const double*>(z), static_cast<double*>(traj),
        static_cast<double*>(logdet), B, T);
    return int(hipGetLastError());
}
