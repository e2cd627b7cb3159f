// gfx950 kernels for batched constant-velocity Kalman filters (KF_MODEL_CV2 / KF_MODEL_CV3).
//
// Mapping: ONE FILTER PER LANE.  A filter's state x[n] and packed covariance P[n(n+1)/2]
// live in VGPRs for the whole launch; 64 filters advance in lockstep per wave64.  The
// per-filter contractions are at most 6x6 (no MFMA: nothing here has an inner dimension
// >= 16), so the work is VALU arithmetic fed by fully coalesced SoA streams:
// lane f reads u[t][i][f], z[s][i][f] and writes traj[t][i][f], logdet[t][f] — every wave
// instruction touches one contiguous 256 B (fp32) / 512 B (fp64) segment.
//
// Per step (reference: kf_workers.py:688-717, op semantics):
//   predict  x = F x + G u,  P = F P F^T + Q       F = [[I, dt I],[0, I]] exploited in closed
//                                                  form — F is never materialised
//   update   S = P[0:m,0:m] + R (H = [I 0] is a row selection, no multiply)
//            LDL^T(S) in-lane; K = P H^T S^-1 by forward/back substitution per row
//            x += K (z - x[0:m])
//            Joseph: P = (I-KH) P (I-KH)^T + K R K^T evaluated as Y + E K^T with
//            Y = (I-KH) P and E = K R - Y H^T (the same polynomial in K, so the same
//            first-order insensitivity to gain error; only the upper triangle is formed)
//   logdet   LDL^T(P): log of the pivot product (no sqrt, one log per step)
// A non-positive pivot of S turns its reciprocal into NaN, which poisons K, x and P of that
// filter without a branch (status KF_ENOTSPD); the other lanes are unaffected.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <stdint.h>
#include <stdlib.h>

#include "kf_common.h"
#include "kf_internal.h"

namespace kfmi {
namespace {

using namespace dev;



template <int D, typename T>
struct Cv {
    static constexpr int N = 2 * D;            // state
    static constexpr int M = D;                // GPS measurement
    static constexpr int NT = N * (N + 1) / 2; // packed covariance
    static constexpr int MT = M * (M + 1) / 2;

    // x = F x + G u ; P = F P F^T + Q   (kf_workers.py:493-549, 690-691 restricted to pos/vel)
    __device__ static __forceinline__ void predict(T (&x)[N], T (&P)[NT], T dt, const T (&u)[D],
                                                   T qp_dt, T qv_dt) {
        const T hdt2 = T(0.5) * dt * dt;
#pragma unroll
        for (int i = 0; i < D; ++i) {
            x[i] = fmaT(hdt2, u[i], fmaT(dt, x[D + i], x[i]));
            x[D + i] = fmaT(dt, u[i], x[D + i]);
        }
        // With P = [[A, Bm], [Bm^T, C]]:  Bm' = Bm + dt C,  A' = A + dt (Bm' + Bm^T),  C' = C.
        T Bn[D][D];
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int j = 0; j < D; ++j)
                Bn[i][j] = fmaT(dt, P[tri<N>(D + i, D + j)], P[tri<N>(i, D + j)]);
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int j = i; j < D; ++j)
                P[tri<N>(i, j)] = fmaT(dt, Bn[i][j] + P[tri<N>(j, D + i)], P[tri<N>(i, j)]);
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int j = 0; j < D; ++j) P[tri<N>(i, D + j)] = Bn[i][j];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            P[tri<N>(i, i)] += qp_dt;
            P[tri<N>(D + i, D + i)] += qv_dt;
        }
    }

    // GPS update with H = [I 0] (kf_workers.py:551-558, 616-621, 708-711; Joseph form).
    template <bool DIAG_R>
    __device__ static __forceinline__ bool update(T (&x)[N], T (&P)[NT], const T (&z)[M],
                                                  const T (&R)[MT]) {
        return sel_update<N, M, DIAG_R, T>(x, P, z, R);
    }
};


template <int D, typename T>
__device__ __forceinline__ void load_state(const CvArgs& a, uint32_t rb, uint32_t off, T (&x)[2 * D],
                                           T (&P)[D * (2 * D + 1)]) {
#pragma unroll
    for (int i = 0; i < 2 * D; ++i) x[i] = ldb<T>(a.x, i, rb, off);
#pragma unroll
    for (int k = 0; k < D * (2 * D + 1); ++k) P[k] = ldb<T>(a.P, k, rb, off);
}

template <int D, typename T>
__device__ __forceinline__ void store_state(const CvArgs& a, uint32_t rb, uint32_t off, const T (&x)[2 * D],
                                            const T (&P)[D * (2 * D + 1)]) {
#pragma unroll
    for (int i = 0; i < 2 * D; ++i) stb(a.x, i, rb, off, x[i]);
#pragma unroll
    for (int k = 0; k < D * (2 * D + 1); ++k) stb(a.P, k, rb, off, P[k]);
}

// BLOCK: P is block-diagonal over the axes (CvArgs::block_p: the handle's P started so and a
// diagonal R keeps it so), so only the same-axis entries are read and written; the others are
// compile-time zeros, which also removes their arithmetic.
template <int D, typename T, bool BLOCK>
__device__ __forceinline__ void load_state_b(const CvArgs& a, uint32_t rb, uint32_t off, T (&x)[2 * D],
                                             T (&P)[D * (2 * D + 1)]) {
    constexpr int N = 2 * D;
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = ldb<T>(a.x, i, rb, off);
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = i; j < N; ++j)
            P[tri<N>(i, j)] = (!BLOCK || i % D == j % D) ? ldb<T>(a.P, tri<N>(i, j), rb, off) : T(0);
}

template <int D, typename T, bool BLOCK>
__device__ __forceinline__ void store_state_b(const CvArgs& a, uint32_t rb, uint32_t off, const T (&x)[2 * D],
                                              const T (&P)[D * (2 * D + 1)]) {
    constexpr int N = 2 * D;
#pragma unroll
    for (int i = 0; i < N; ++i) stb(a.x, i, rb, off, x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = i; j < N; ++j)
            if (!BLOCK || i % D == j % D) stb(a.P, tri<N>(i, j), rb, off, P[tri<N>(i, j)]);
}

template <int D, typename T>
__device__ __forceinline__ void load_R(const CvArgs& a, T (&R)[D * (D + 1) / 2]) {
#pragma unroll
    for (int k = 0; k < D * (D + 1) / 2; ++k) R[k] = T(a.r[k]);
}

// Inputs of one time step, double-buffered in registers by the run kernel.
template <int D, typename T>
struct StepIn {
    T u[D];
    T z[D];
    uint8_t use;
};

// ------------------------------------------------------------------------------------
// The fused hot path: T predict(+update) steps in one launch.
// GENERAL = false: scalar dt, control present, no mask, trajectory and logdet written (the
// bench / fusion configuration) with no runtime checks; GENERAL = true: every optional
// stream decided at run time by a wave-uniform branch.
// The time loop is unrolled by two with statically named input buffers A and B: step t+1's
// inputs are loaded before step t computes, and no loop-carried register copy forces the
// wave to wait for its own trajectory stores (s_waitcnt counts loads and stores together).
// z is read only for the steps that update: on the others its row descriptor has length 0 (the
// step index is wave-uniform), so the load instruction issues but the range check returns 0
// without touching memory — no branch, and no re-reads of the same fix between updates.
// ------------------------------------------------------------------------------------
// Minimum waves per SIMD requested from the register allocator for the run kernel (1 = let
// the compiler choose).  Overridable at build time for occupancy experiments.
#ifndef KF_OCC_CV3_F64
#define KF_OCC_CV3_F64 1
#endif
#ifndef KF_OCC_CV3_F32
#define KF_OCC_CV3_F32 1
#endif
#ifndef KF_OCC_CV2_F64
#define KF_OCC_CV2_F64 1
#endif
#ifndef KF_OCC_CV2_F32
#define KF_OCC_CV2_F32 1
#endif
template <int D, typename T>
struct RunOcc {
    static constexpr int value = D == 3 ? (sizeof(T) == 8 ? KF_OCC_CV3_F64 : KF_OCC_CV3_F32)
                                        : (sizeof(T) == 8 ? KF_OCC_CV2_F64 : KF_OCC_CV2_F32);
};

template <int D, typename T, bool GENERAL, bool DIAG_R>
__global__ __launch_bounds__(kBlock, (RunOcc<D, T>::value)) void cv_run_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    constexpr int N = K::N, M = K::M;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const int64_t B = a.B;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    const bool has_dts = GENERAL && a.dt_steps != nullptr;
    const bool has_u = !GENERAL || a.u != nullptr;
    const bool has_mask = GENERAL && a.mask != nullptr;
    const bool has_traj = !GENERAL || a.traj != nullptr;
    const bool has_ld = !GENERAL || a.logdet != nullptr;

    T x[N], P[K::NT];
    load_state<D, T>(a, rb, off, x, P);
    int32_t st = a.status[f];
    T R[K::MT];
    load_R<D, T>(a, R);

    const int T_ = a.T;
    const int k_upd = a.update_every;
    const int U = T_ / k_upd;

    // z index for the inputs of step t: the update at or after t (ceil((t+1)/k) - 1),
    // tracked incrementally (load_in is called with t = 0, 1, 2, ...), clamped to U - 1.
    int ld_upd_step = k_upd - 1;
    int ld_s = 0;
    // Optional streams cost no branch: a zero-length row descriptor makes the hardware range
    // check return 0 for every load (no control / no update) without touching memory.
    const uint32_t rb_u = has_u ? rb : 0u;
    const uint32_t rb_z = U > 0 ? rb : 0u;
    const uint32_t rb_tr = has_traj ? rb : 0u;  // no trajectory: stores dropped by the range check
    auto load_in = [&](int t, StepIn<D, T>& in) {
        const int tc = t < T_ ? t : T_ - 1;
        if (tc > ld_upd_step) {
            ld_upd_step += k_upd;
            ++ld_s;
        }
#pragma unroll
        for (int i = 0; i < D; ++i) in.u[i] = ldb_stream(a.u, int64_t(tc) * D + i, rb_u, off, T(0));
        int s = ld_s < U ? ld_s : U - 1;
        s = s > 0 ? s : 0;
        const bool upd = tc == ld_upd_step;  // wave-uniform
        const uint32_t rbz = upd ? rb_z : 0u;
#pragma unroll
        for (int i = 0; i < M; ++i) in.z[i] = ldb_stream(a.z, int64_t(s) * M + i, rbz, off, T(0));
        in.use = (has_mask && U > 0 && upd) ? a.mask[int64_t(s) * B + f] : uint8_t(1);
    };

    int until_upd = k_upd;
    auto step = [&](int t, const StepIn<D, T>& in) {
        const double dtd = has_dts ? a.dt_steps[t] : a.dt;
        K::predict(x, P, T(dtd), in.u, T(a.q_pos * dtd), T(a.q_vel * dtd));
        if (--until_upd == 0) {  // wave-uniform
            until_upd = k_upd;
            if (!has_mask) {
                const bool ok = K::template update<DIAG_R>(x, P, in.z, R);
                st = ok ? st : kNotSpd;
            } else if (in.use) {
                const bool ok = K::template update<DIAG_R>(x, P, in.z, R);
                st = ok ? st : kNotSpd;
            }
        }
#pragma unroll
        for (int i = 0; i < N; ++i) stb_rec(a.traj, int64_t(t) * N + i, rb_tr, off, x[i]);
        if (has_ld) {
            const T ld = logdet_ldl<N, T>(P);
            st = (ld == ld) ? st : kNotSpd;
            stb_rec(a.logdet, t, rb, off, ld);
        }
    };

    StepIn<D, T> A, Bf;
    load_in(0, A);
    // Drain the prologue loads (state + first inputs) once, so the compiler's wait analysis
    // does not carry them into the loop header and stall every iteration on them.
    __builtin_amdgcn_s_waitcnt(0);
    int t = 0;
    for (; t + 1 < T_; t += 2) {
        load_in(t + 1, Bf);
        step(t, A);
        load_in(t + 2, A);
        step(t + 1, Bf);
    }
    if (t < T_) step(t, A);

    store_state<D, T>(a, rb, off, x, P);
    a.status[f] = st;
}

// ------------------------------------------------------------------------------------
// Block variant of the fused run for a block-diagonal P and diagonal R (the reference's
// constants: Q, R, P0 diagonal; F and H couple only pos_i with vel_i).  P then stays exactly
// block-diagonal — D independent 2-state (pos_i, vel_i) chains — and the general kernel spends
// most of its VALU on entries that are exact zeros.  This kernel keeps, per axis, x = (p, v)
// and P_i = (pp, pv, vv) and evaluates the general kernel's expressions for those entries in
// the same order (the dropped terms are exact zeros), so its results equal the general
// kernel's; the logdet multiplies the LDL pivots in the general kernel's order (positions,
// renormalise, velocities, renormalise).  The host selects it only when the handle's P is
// known to be block-diagonal (kf_alloc / kf_reset, or checked on the device in kf_set_state).
// ------------------------------------------------------------------------------------
template <int D, typename T, int DEPTH>
__global__ __launch_bounds__(kBlock) void cv_block_kernel(const CvArgs a) {
    constexpr int N = 2 * D;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    T xp[D], xv[D], pp[D], pv[D], vv[D], r[D];
#pragma unroll
    for (int i = 0; i < D; ++i) {
        xp[i] = ldb<T>(a.x, i, rb, off);
        xv[i] = ldb<T>(a.x, D + i, rb, off);
        pp[i] = ldb<T>(a.P, tri<N>(i, i), rb, off);
        pv[i] = ldb<T>(a.P, tri<N>(i, D + i), rb, off);
        vv[i] = ldb<T>(a.P, tri<N>(D + i, D + i), rb, off);
        r[i] = T(a.r[tri<D>(i, i)]);
    }
    int32_t st = a.status[f];
    const int T_ = a.T;
    const int k_upd = a.update_every;
    const int U = T_ / k_upd;
    int ld_upd_step = k_upd - 1;
    int ld_s = 0;
    const uint32_t rb_z = U > 0 ? rb : 0u;
    const T dt = T(a.dt);
    const T hdt2 = T(0.5) * dt * dt;
    const T qp = T(a.q_pos * a.dt), qv = T(a.q_vel * a.dt);
    auto load_in = [&](int t, StepIn<D, T>& in) {
        const int tc = t < T_ ? t : T_ - 1;
        if (tc > ld_upd_step) {
            ld_upd_step += k_upd;
            ++ld_s;
        }
#pragma unroll
        for (int i = 0; i < D; ++i) in.u[i] = ldb_stream(a.u, int64_t(tc) * D + i, rb, off, T(0));
        int s = ld_s < U ? ld_s : U - 1;
        s = s > 0 ? s : 0;
        const uint32_t rbz = tc == ld_upd_step ? rb_z : 0u;  // z only on update steps
#pragma unroll
        for (int i = 0; i < D; ++i) in.z[i] = ldb_stream(a.z, int64_t(s) * D + i, rbz, off, T(0));
    };
    int until_upd = k_upd;
    auto step = [&](int t, const StepIn<D, T>& in) {
        // predict (Cv::predict per axis): Bm' = Bm + dt C, A' = A + dt (Bm' + Bm^T), + Q
#pragma unroll
        for (int i = 0; i < D; ++i) {
            xp[i] = fmaT(hdt2, in.u[i], fmaT(dt, xv[i], xp[i]));
            xv[i] = fmaT(dt, in.u[i], xv[i]);
            const T bn = fmaT(dt, vv[i], pv[i]);
            pp[i] = fmaT(dt, bn + pv[i], pp[i]);
            pv[i] = bn;
            pp[i] += qp;
            vv[i] += qv;
        }
        if (--until_upd == 0) {  // wave-uniform
            until_upd = k_upd;
            bool ok = true;
#pragma unroll
            for (int i = 0; i < D; ++i) {
                // sel_update with a diagonal S: one scalar pivot per axis, Joseph form
                const T S = pp[i] + r[i];
                ok = ok && (S > T(0));
                const T dinv = rcp_pos<2>(S);
                const T k0 = pp[i] * dinv, k1 = pv[i] * dinv;
                const T y = in.z[i] - xp[i];
                xp[i] = fmaT(k0, y, xp[i]);
                xv[i] = fmaT(k1, y, xv[i]);
                const T e0 = fmaT(k0, S, -pp[i]);
                const T e1 = fmaT(k1, S, -pv[i]);
                const T npp = fmaT(e0, k0, fmaT(-k0, pp[i], pp[i]));
                const T npv = fmaT(e0, k1, fmaT(-k0, pv[i], pv[i]));
                const T nvv = fmaT(e1, k1, fmaT(-k1, pv[i], vv[i]));
                pp[i] = npp;
                pv[i] = npv;
                vv[i] = nvv;
            }
            // a bad pivot poisons the whole filter, as in the general kernel (where its NaN
            // reaches every row through the LDL factors)
            const T poison = ok ? T(0) : quiet_nan<T>();
#pragma unroll
            for (int i = 0; i < D; ++i) {
                xp[i] += poison;
                xv[i] += poison;
                pp[i] += poison;
                pv[i] += poison;
                vv[i] += poison;
            }
            st = ok ? st : kNotSpd;
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {
            stb_rec(a.traj, int64_t(t) * N + i, rb, off, xp[i]);
            stb_rec(a.traj, int64_t(t) * N + D + i, rb, off, xv[i]);
        }
        // logdet: LDL pivots in the general 6x6 order (positions, then velocities)
        T prod = T(1);
        int ex = 0, e;
        bool pd = true;
        T dv[D];
#pragma unroll
        for (int i = 0; i < D; ++i) {
            pd = pd && (pp[i] > T(0));
            prod *= pp[i];
            const T l = pv[i] * rcp_nr<1>(pp[i]);
            const T v = l * pp[i];
            dv[i] = fmaT(-l, v, vv[i]);
        }
        prod = frexp(prod, &e);
        ex += e;
#pragma unroll
        for (int i = 0; i < D; ++i) {
            pd = pd && (dv[i] > T(0));
            prod *= dv[i];
        }
        prod = frexp(prod, &e);
        ex += e;
        const T ld = pd ? log_mant(prod, ex) : quiet_nan<T>();
        st = (ld == ld) ? st : kNotSpd;
        stb_rec(a.logdet, t, rb, off, ld);
    };
    // Inputs are prefetched DEPTH - 1 steps ahead through a ring of DEPTH named buffers (the
    // ring is fully unrolled, so every buffer index is static and nothing is copied): with few
    // filters a SIMD has one or two waves, and the bytes in flight — not the arithmetic — bound
    // the step rate.
    StepIn<D, T> buf[DEPTH];
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
#pragma unroll
    for (int i = 0; i < D; ++i) {
        stb(a.x, i, rb, off, xp[i]);
        stb(a.x, D + i, rb, off, xv[i]);
        stb(a.P, tri<N>(i, i), rb, off, pp[i]);
        stb(a.P, tri<N>(i, D + i), rb, off, pv[i]);
        stb(a.P, tri<N>(D + i, D + i), rb, off, vv[i]);
    }
    a.status[f] = st;
}

// 1 in *flag if any filter's packed P has a non-zero entry coupling different axes.
template <int D, typename T>
__global__ __launch_bounds__(kBlock) void cv_offblock_kernel(const CvArgs a, int* flag) {
    constexpr int N = 2 * D;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    bool any = false;
#pragma unroll
    for (int i = 0; i < N; ++i)
#pragma unroll
        for (int j = i; j < N; ++j)
            if ((i % D) != (j % D)) any = any || (ldb<T>(a.P, tri<N>(i, j), rb, off) != T(0));
    if (any) atomicOr(flag, 1);
}

// Single predict step (kf_predict): optional per-filter dt and logdet of the prediction.
template <int D, typename T, bool BLOCK>
__global__ __launch_bounds__(kBlock) void cv_predict_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    T x[K::N], P[K::NT];
    load_state_b<D, T, BLOCK>(a, rb, off, x, P);
    T u[D];
#pragma unroll
    for (int i = 0; i < D; ++i) u[i] = a.u ? ldb<T>(a.u, i, rb, off) : T(0);
    const double dtd = a.dt_filter ? a.dt_filter[f] : a.dt;
    K::predict(x, P, T(dtd), u, T(a.q_pos * dtd), T(a.q_vel * dtd));
    store_state_b<D, T, BLOCK>(a, rb, off, x, P);
    if (a.logdet) {
        const T ld = logdet_ldl<K::N, T>(P);
        stb(a.logdet, 0, rb, off, ld);
        if (!(ld == ld)) a.status[f] = kNotSpd;
    }
}

// Single GPS update (kf_update).
template <int D, typename T, bool BLOCK>
__global__ __launch_bounds__(kBlock) void cv_update_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    T x[K::N], P[K::NT];
    load_state_b<D, T, BLOCK>(a, rb, off, x, P);
    T R[K::MT];
    load_R<D, T>(a, R);
    T z[K::M];
#pragma unroll
    for (int i = 0; i < K::M; ++i) z[i] = ldb<T>(a.z, i, rb, off);
    int32_t st = a.status[f];
    if (!a.mask || a.mask[f] != 0) {
        if (!K::template update<BLOCK>(x, P, z, R)) st = kNotSpd;
    }
    store_state_b<D, T, BLOCK>(a, rb, off, x, P);
    if (a.logdet) {
        const T ld = logdet_ldl<K::N, T>(P);
        if (!(ld == ld)) st = kNotSpd;
        stb(a.logdet, 0, rb, off, ld);
    }
    a.status[f] = st;
}

// kf_predict held back and fused with the next kf_update (kf_capi.cpp): the two kernels above
// in one, so the state crosses HBM once per step.  u is the control copied at kf_predict time.
template <int D, typename T, bool BLOCK>
__global__ __launch_bounds__(kBlock) void cv_step_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    T x[K::N], P[K::NT];
    load_state_b<D, T, BLOCK>(a, rb, off, x, P);
    T u[D];
#pragma unroll
    for (int i = 0; i < D; ++i) u[i] = a.u ? ldb<T>(a.u, i, rb, off) : T(0);
    T R[K::MT];
    load_R<D, T>(a, R);
    T z[K::M];
#pragma unroll
    for (int i = 0; i < K::M; ++i) z[i] = ldb<T>(a.z, i, rb, off);
    int32_t st = a.status[f];
    const double dtd = a.dt;
    K::predict(x, P, T(dtd), u, T(a.q_pos * dtd), T(a.q_vel * dtd));
    if (!a.mask || a.mask[f] != 0) {
        if (!K::template update<BLOCK>(x, P, z, R)) st = kNotSpd;
    }
    store_state_b<D, T, BLOCK>(a, rb, off, x, P);
    if (a.logdet) {
        const T ld = logdet_ldl<K::N, T>(P);
        if (!(ld == ld)) st = kNotSpd;
        stb(a.logdet, 0, rb, off, ld);
    }
    a.status[f] = st;
}

// Device copy with the shader (kf_predict's control snapshot): hipMemcpyAsync of device memory
// goes to an SDMA engine, several times slower than a kernel for tens of MB.
template <typename W>
__global__ __launch_bounds__(kBlock) void copy_kernel(W* __restrict__ dst, const W* __restrict__ src, int64_t n) {
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * kBlock)
        dst[i] = src[i];
}

// x = x0 (or 0), P = diag(p0_pos I, p0_vel I), status = OK.
template <int D, typename T>
__global__ __launch_bounds__(kBlock) void cv_reset_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    T x[K::N], P[K::NT];
#pragma unroll
    for (int i = 0; i < K::N; ++i) x[i] = a.x0 ? ldb<T>(a.x0, i, rb, off) : T(0);
#pragma unroll
    for (int k = 0; k < K::NT; ++k) P[k] = T(0);
#pragma unroll
    for (int i = 0; i < D; ++i) {
        P[tri<K::N>(i, i)] = T(a.p0_pos);
        P[tri<K::N>(D + i, D + i)] = T(a.p0_vel);
    }
    store_state<D, T>(a, rb, off, x, P);
    a.status[f] = 0;
}


template <int D, typename T>
__global__ __launch_bounds__(kBlock) void cv_synth_kernel(const SynthArgs a) {
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    const uint64_t g = uint64_t(a.filter_offset + f);
    const uint32_t g0 = uint32_t(g), g1 = uint32_t(g >> 32);
    const uint32_t k0 = uint32_t(a.seed), k1 = uint32_t(a.seed >> 32);
    const double sd_gps = 1.7320508075688772;  // sqrt(3): R_gps variance (kf_workers.py:583)
    double p[D], v[D];
    // initial truth and first fix: counter t = 0xFFFFFFFF
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const U4 ru = philox4x32_10(0xFFFFFFFFu, uint32_t(i), g0, g1, k0, k1);
        p[i] = -1000.0 + 2000.0 * u53(ru.v[0], ru.v[1]);
        const U4 rn = philox4x32_10(0xFFFFFFFFu, uint32_t(8 + i), g0, g1, k0, k1);
        double n0, n1;
        normal2(rn, n0, n1);
        v[i] = 10.0 * n0;
        stb(a.x0, i, rb, off, T(p[i] + sd_gps * n1));  // position = first GPS fix
        stb(a.x0, D + i, rb, off, T(0));               // other states 0 (kf_workers.py:655-659)
    }
    int until = a.update_every;
    int s = 0;
    for (int t = 0; t < a.T; ++t) {
        const double dt = a.dt;
        double n[2 * D + 2 * ((D + 1) / 2)];
#pragma unroll
        for (int q = 0; q < D; ++q) {
            const U4 r = philox4x32_10(uint32_t(t), uint32_t(q), g0, g1, k0, k1);
            normal2(r, n[2 * q], n[2 * q + 1]);
        }
#pragma unroll
        for (int i = 0; i < D; ++i) {
            const double acc = 0.3 * n[2 * i];
            const double imu = 0.1 * n[2 * i + 1];
            p[i] += v[i] * dt + 0.5 * acc * dt * dt;
            v[i] += acc * dt;
            stb(a.u, int64_t(t) * D + i, rb, off, T(acc + imu));
        }
        if (--until == 0) {
            until = a.update_every;
#pragma unroll
            for (int q = 0; q < (D + 1) / 2; ++q) {
                const U4 r = philox4x32_10(uint32_t(t), uint32_t(16 + q), g0, g1, k0, k1);
                normal2(r, n[2 * D + 2 * q], n[2 * D + 2 * q + 1]);
            }
#pragma unroll
            for (int i = 0; i < D; ++i)
                stb(a.z, int64_t(s) * D + i, rb, off, T(p[i] + sd_gps * n[2 * D + i]));
            ++s;
        }
    }
}

// Optional cap on resident workgroups per CU for the run kernel (experiments / tail tuning):
// KF_OPT_BLOCKS_PER_CU = k reserves 160 KiB / (k + 0.5) of (unused) LDS per workgroup so at most
// k workgroups (k waves per SIMD) fit on a CU.  0 = no cap.
size_t lds_cap_bytes(int k) {
    if (k < 2 || k > 8) return size_t(0);
    return (size_t(160 * 1024) * 2 / (2 * k + 1) + 15) / 16 * 16;
}

template <int D, typename T>
hipError_t launch_run(const CvArgs& a, dim3 grid, hipStream_t st) {
    const size_t lds = lds_cap_bytes(a.blocks_per_cu);
    const bool fast = a.dt_steps == nullptr && a.u != nullptr && a.mask == nullptr &&
                      a.traj != nullptr && a.logdet != nullptr;
    bool diag = true;
    {
        int k = 0;
        for (int i = 0; i < D; ++i)
            for (int j = i; j < D; ++j, ++k)
                if (i != j && a.r[k] != 0.0) diag = false;
    }
    if (fast && diag && a.block_p && a.prefetch_depth == 8)
        cv_block_kernel<D, T, 8><<<grid, kBlock, 0, st>>>(a);
    else if (fast && diag && a.block_p && a.prefetch_depth == 4)
        cv_block_kernel<D, T, 4><<<grid, kBlock, 0, st>>>(a);
    else if (fast && diag && a.block_p)
        cv_block_kernel<D, T, 2><<<grid, kBlock, 0, st>>>(a);
    else if (fast && diag)
        cv_run_kernel<D, T, false, true><<<grid, kBlock, lds, st>>>(a);
    else if (fast)
        cv_run_kernel<D, T, false, false><<<grid, kBlock, lds, st>>>(a);
    else if (diag)
        cv_run_kernel<D, T, true, true><<<grid, kBlock, lds, st>>>(a);
    else
        cv_run_kernel<D, T, true, false><<<grid, kBlock, lds, st>>>(a);
    return hipGetLastError();
}

template <int D, typename T>
hipError_t launch_cv_t(Op op, const CvArgs& a, hipStream_t st) {
    const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
    switch (op) {
        case Op::Run: return launch_run<D, T>(a, grid, st);
        case Op::Predict:
            if (a.block_p) cv_predict_kernel<D, T, true><<<grid, kBlock, 0, st>>>(a);
            else cv_predict_kernel<D, T, false><<<grid, kBlock, 0, st>>>(a);
            break;
        case Op::Update:
            if (a.block_p) cv_update_kernel<D, T, true><<<grid, kBlock, 0, st>>>(a);
            else cv_update_kernel<D, T, false><<<grid, kBlock, 0, st>>>(a);
            break;
        case Op::Step:
            if (a.block_p) cv_step_kernel<D, T, true><<<grid, kBlock, 0, st>>>(a);
            else cv_step_kernel<D, T, false><<<grid, kBlock, 0, st>>>(a);
            break;
        case Op::Reset: cv_reset_kernel<D, T><<<grid, kBlock, 0, st>>>(a); break;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_cv(int axes, bool f64, Op op, const CvArgs& a, hipStream_t stream) {
    if (axes == 2) return f64 ? launch_cv_t<2, double>(op, a, stream) : launch_cv_t<2, float>(op, a, stream);
    return f64 ? launch_cv_t<3, double>(op, a, stream) : launch_cv_t<3, float>(op, a, stream);
}

hipError_t launch_cv_offblock(int axes, bool f64, const CvArgs& a, int* flag, hipStream_t stream) {
    const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
    if (axes == 2) {
        if (f64) cv_offblock_kernel<2, double><<<grid, kBlock, 0, stream>>>(a, flag);
        else cv_offblock_kernel<2, float><<<grid, kBlock, 0, stream>>>(a, flag);
    } else {
        if (f64) cv_offblock_kernel<3, double><<<grid, kBlock, 0, stream>>>(a, flag);
        else cv_offblock_kernel<3, float><<<grid, kBlock, 0, stream>>>(a, flag);
    }
    return hipGetLastError();
}

hipError_t launch_copy(void* dst, const void* src, size_t bytes, hipStream_t stream) {
    if (!bytes) return hipSuccess;
    const bool wide = (reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src) | bytes) % 16 == 0;
    const int64_t n = static_cast<int64_t>(wide ? bytes / 16 : bytes / 4);
    // one chunk per lane: a small copy (65,536 filters: 48 K chunks) is a single HBM round trip
    // per lane instead of a grid-stride chain of them
    const int64_t blocks = std::min<int64_t>((n + kBlock - 1) / kBlock, int64_t(1) << 20);
    if (wide)
        copy_kernel<uint4><<<dim3(unsigned(blocks)), kBlock, 0, stream>>>(
            static_cast<uint4*>(dst), static_cast<const uint4*>(src), n);
    else
        copy_kernel<uint32_t><<<dim3(unsigned(blocks)), kBlock, 0, stream>>>(
            static_cast<uint32_t*>(dst), static_cast<const uint32_t*>(src), n);
    return hipGetLastError();
}

hipError_t launch_synth(int axes, bool f64, const SynthArgs& a, hipStream_t stream) {
    const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
    if (axes == 2) {
        if (f64) cv_synth_kernel<2, double><<<grid, kBlock, 0, stream>>>(a);
        else cv_synth_kernel<2, float><<<grid, kBlock, 0, stream>>>(a);
    } else {
        if (f64) cv_synth_kernel<3, double><<<grid, kBlock, 0, stream>>>(a);
        else cv_synth_kernel<3, float><<<grid, kBlock, 0, stream>>>(a);
    }
    return hipGetLastError();
}

}  // namespace kfmi
