// gfx950 kernels for the reference's chain-structured GPS+IMU models on per-filter event
// streams — KF_MODEL_REF15 (kf_workers.py:493-614) and KF_MODEL_REF8 (hw5_2.py:219-311) — and
// the brute-force combination search and sensor scheduling built on the 15-state one
// (kf_workers.py:22-213, 826-957, 1218-1392).
//
// Structure exploited (exact, not an approximation): F(dt) (kf_workers.py:500-516,
// hw5_2.py:221-230) couples a state only within its axis chain (pos_i, vel_i, acc_i) or
// (att_i, rate_i); Q, R_gps, R_imu and the reference's P0 are diagonal; H_gps selects pos_i and
// H_imu = I.  So every covariance reachable from a diagonal P0 is block-diagonal — 3x3
// (pos, vel, acc) blocks and 2x2 (att, rate) blocks — and the reference's own dense arithmetic
// keeps the off-block entries at exactly 0.0 (checked on its outputs, tests/golden/ref15_*.npz).
// A lane therefore runs small chain filters: REF15 = 3 pva + 3 aw chains (27 covariance entries
// instead of 120), REF8 = 2 pva (x, y) + 1 aw (theta) chain (15 instead of 36); same numbers.
//
// Block-packed covariance rows ([NBLK][B] in HBM):
//   rows 6c .. 6c+5 : pva chain c upper triangle (pp pv pa vv va aa), c = 0..NP-1
//   rows 6NP+3c .. 6NP+3c+2 : aw chain c upper triangle (tt tw ww), c = 0..NA-1
// State x [N][B] in the reference's order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <cstdlib>
#include <cstring>

#include "kf_common.h"
#include "kf_internal.h"

namespace kfmi {
namespace {

// Read-only device tables (the handle's custom constants, a search's events and binomials) read
// through the constant address space: a wave-uniform entry then becomes a scalar load.  Through a
// generic pointer the compiler cannot prove that a kernel's own stores leave them alone, so it
// loads them with vector loads, whose vmcnt wait also waits for every store issued before them
// (on gfx950 vmcnt counts loads and stores, in order).  Every such table is written by the host
// before the launch and never by a kernel.
template <typename T>
__device__ __forceinline__ __attribute__((address_space(4))) const T* ro(const T* p) {
    return (__attribute__((address_space(4))) const T*)p;
}
typedef __attribute__((address_space(4))) const double ro_double;
typedef __attribute__((address_space(4))) const uint64_t ro_u64;

using namespace dev;

constexpr int kGps = 0, kImu = 1;  // KF_EVENT_GPS / KF_EVENT_IMU; 2 = predict only, 255 = none
// Newton steps on the update's pivot reciprocals (see sel_update)
constexpr int kRefNewton = 1;
// Covariance update of the reference models.  fp64 takes the reference's own form
// P = (I - K H) P (kf_workers.py:711, hw5_2.py:358, 376) over the packed upper triangle; fp32 keeps
// Joseph's, which the fp32 parity gate needs (the simple form drifts there).
// KF_REF_JOSEPH_F64=1 builds fp64 with Joseph too (the A/B arm).
#ifndef KF_REF_JOSEPH_F64
#define KF_REF_JOSEPH_F64 0
#endif
template <typename T>
constexpr bool kRefJoseph = sizeof(T) == 4 || KF_REF_JOSEPH_F64 != 0;
// The IMU pseudo-measurement's H = I chain updates take P = K R (sel_update_nv's GAIN_R: the
// same value as (I - K)P, without its cancellation), in both precisions; KF_REF_GAIN_R=0 builds
// the A/B arm without it.
#ifndef KF_REF_GAIN_R
#define KF_REF_GAIN_R 1
#endif
constexpr bool kRefGainR = KF_REF_GAIN_R != 0;


// Noise constants shared by both reference models (kf_workers.py:519-544, 581-614;
// hw5_2.py:233-251, 280-304).
constexpr double kQPos = 5.0, kQAtt = 0.05, kQVel = 1.0, kQRate = 0.1, kQAcc = 2.0;
constexpr double kRGps = 3.0;
constexpr double kRPos = 50.0, kRAtt = 0.05, kRVel = 10.0, kRRate = 0.1, kRAcc = 100.0;

// KF_MODEL_REF15: x = (pos xyz, att rpy, vel xyz, rate xyz, acc xyz) (kf_workers.py:493-517).
struct M15 {
    static constexpr int N = 15, NP = 3, NA = 3, NTRAJ = 6, NBLK = 27;
    __device__ static constexpr int pva(int c, int k) { return c + 6 * k; }          // (i, 6+i, 12+i)
    __device__ static constexpr int aw(int c, int k) { return 3 + c + 6 * k; }       // (3+i, 9+i)
    __device__ static constexpr int imu_acc(int c) { return 6 + c; }                 // ax, ay, az
    __device__ static constexpr int imu_att(int c) { return c; }                     // roll, pitch, yaw
    __device__ static constexpr int imu_rate(int c) { return 3 + c; }                // wx, wy, wz
    static constexpr double P0Pos = 10000.0, P0Att = 1000.0, P0Vel = 1000.0, P0Rate = 1000.0,
                            P0Acc = 10000.0;  // kf_workers.py:651
};

// KF_MODEL_REF8: x = (x, y, theta, vx, vy, theta_dot, ax, ay) (hw5_2.py:219-231); the IMU
// pseudo-measurement takes yaw as theta and wz as theta_dot (hw5_2.py:355-362).
struct M8 {
    static constexpr int N = 8, NP = 2, NA = 1, NTRAJ = 3, NBLK = 15;
    __device__ static constexpr int pva(int c, int k) { return c + 3 * k; }          // (i, 3+i, 6+i)
    __device__ static constexpr int aw(int, int k) { return 2 + 3 * k; }             // (2, 5)
    __device__ static constexpr int imu_acc(int c) { return 6 + c; }                 // ax, ay
    __device__ static constexpr int imu_att(int) { return 2; }                       // yaw
    __device__ static constexpr int imu_rate(int) { return 5; }                      // wz
    static constexpr double P0Pos = 1000.0, P0Att = 100.0, P0Vel = 100.0, P0Rate = 100.0,
                            P0Acc = 1000.0;  // hw5_2.py:317-326
};

// Noise constants of a chain.  CUSTOM = false: the reference's, compile-time literals (the
// default, and the code every bench row runs); CUSTOM = true: a caller's diagonal Q rates, R_imu,
// R_gps and P0 per state (kf_params -> RefConsts, the handle's device copy at kc), read by
// wave-uniform scalar loads.  Both give Chains the same operations in the same order.
template <bool CUSTOM, class M, typename T>
__device__ __forceinline__ void pva_noise(const RefConsts* kc, int c, T (&q)[3], T (&r)[6], T& rg) {
    if constexpr (CUSTOM) {
#pragma unroll
        for (int k = 0; k < 3; ++k) q[k] = T(ro(kc)->q[M::pva(c, k)]);
        r[0] = T(ro(kc)->r_imu[M::pva(c, 0)]);
        r[3] = T(ro(kc)->r_imu[M::pva(c, 1)]);
        r[5] = T(ro(kc)->r_imu[M::pva(c, 2)]);
        rg = T(ro(kc)->r_gps[c]);
    } else {
        q[0] = T(kQPos);
        q[1] = T(kQVel);
        q[2] = T(kQAcc);
        r[0] = T(kRPos);
        r[3] = T(kRVel);
        r[5] = T(kRAcc);
        rg = T(kRGps);
    }
    r[1] = r[2] = r[4] = T(0);
}
template <bool CUSTOM, class M, typename T>
__device__ __forceinline__ void aw_noise(const RefConsts* kc, int c, T (&q)[2], T (&r)[3]) {
    if constexpr (CUSTOM) {
        q[0] = T(ro(kc)->q[M::aw(c, 0)]);
        q[1] = T(ro(kc)->q[M::aw(c, 1)]);
        r[0] = T(ro(kc)->r_imu[M::aw(c, 0)]);
        r[2] = T(ro(kc)->r_imu[M::aw(c, 1)]);
    } else {
        q[0] = T(kQAtt);
        q[1] = T(kQRate);
        r[0] = T(kRAtt);
        r[2] = T(kRRate);
    }
    r[1] = T(0);
}

template <typename T, class M, bool CUSTOM = false>
struct Chains {
    T x[M::N];
    T pva[M::NP][6];  // per chain: (pos, vel, acc) packed upper 3x3
    T aw[M::NA][3];   // per chain: (att, rate) packed upper 2x2
    const RefConsts* kc = nullptr;  // CUSTOM: the noise constants (kf_params)
    // Chain predict x = F x, P = F P F^T + Q for a block whose F row i is
    // e_i + dt e_{i+1} + dt^2/2 e_{i+2} (kf_workers.py:500-516).
    template <int NB>
    __device__ static __forceinline__ void chain_predict(T (&xb)[NB], T (&Pb)[NB * (NB + 1) / 2], T dt,
                                                         const T (&q)[NB]) {
        const T c[3] = {T(1), dt, T(0.5) * dt * dt};
        // the d / e loops run a constant 2 trips with a compile-time guard: a trip count of
        // min(NB - i, 3) - 1 was left as a runtime loop with indexed register reads (s_set_gpr_idx)
        T xn[NB];
#pragma unroll
        for (int i = 0; i < NB; ++i) {
            T s = xb[i];
#pragma unroll
            for (int d = 1; d < 3; ++d)
                if (i + d < NB) s = fmaT(c[d], xb[i + d], s);
            xn[i] = s;
        }
        T FP[NB][NB];
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j) {
                T s = Pb[tri<NB>(i, j)];
#pragma unroll
                for (int d = 1; d < 3; ++d)
                    if (i + d < NB) s = fmaT(c[d], Pb[tri<NB>(i + d, j)], s);
                FP[i][j] = s;
            }
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
            for (int j = i; j < NB; ++j) {
                T s = FP[i][j];
#pragma unroll
                for (int e = 1; e < 3; ++e)
                    if (j + e < NB) s = fmaT(FP[i][j + e], c[e], s);
                Pb[tri<NB>(i, j)] = (i == j) ? s + q[i] * dt : s;
            }
#pragma unroll
        for (int i = 0; i < NB; ++i) xb[i] = xn[i];
    }

    __device__ __forceinline__ void predict(T dt) {
#pragma unroll
        for (int c = 0; c < M::NP; ++c) {
            T qpva[3], r[6], rg;
            pva_noise<CUSTOM, M>(kc, c, qpva, r, rg);
            T xb[3];
            get_pva(c, xb);
            chain_predict<3>(xb, pva[c], dt, qpva);
            put_pva(c, xb);
        }
#pragma unroll
        for (int c = 0; c < M::NA; ++c) {
            T qaw[2], r[3];
            aw_noise<CUSTOM, M>(kc, c, qaw, r);
            T xa[2];
            get_aw(c, xa);
            chain_predict<2>(xa, aw[c], dt, qaw);
            put_aw(c, xa);
        }
    }

    __device__ __forceinline__ void get_pva(int c, T (&xb)[3]) const {
#pragma unroll
        for (int k = 0; k < 3; ++k) xb[k] = x[M::pva(c, k)];
    }
    __device__ __forceinline__ void put_pva(int c, const T (&xb)[3]) {
#pragma unroll
        for (int k = 0; k < 3; ++k) x[M::pva(c, k)] = xb[k];
    }
    __device__ __forceinline__ void get_aw(int c, T (&xa)[2]) const {
#pragma unroll
        for (int k = 0; k < 2; ++k) xa[k] = x[M::aw(c, k)];
    }
    __device__ __forceinline__ void put_aw(int c, const T (&xa)[2]) {
#pragma unroll
        for (int k = 0; k < 2; ++k) x[M::aw(c, k)] = xa[k];
    }

    // GPS fix (kf_workers.py:694-697, hw5_2.py:341-349): H selects pos_c in each (pos, vel,
    // acc) chain, R = 3; z = (easting, northing[, altitude]).
    template <bool POISON = true>
    __device__ __forceinline__ bool update_gps(const T (&z)[3]) {
        bool ok = true;
#pragma unroll
        for (int c = 0; c < M::NP; ++c) {
            T q[3], r[6], rg;
            pva_noise<CUSTOM, M>(kc, c, q, r, rg);
            const T R[1] = {rg};
            T xb[3];
            get_pva(c, xb);
            const T zb[1] = {z[c]};
            ok = sel_update<3, 1, true, T, kRefNewton, POISON, kRefJoseph<T>, kRefGainR>(xb, pva[c], zb, R) && ok;
            put_pva(c, xb);
        }
        return ok;
    }

    // IMU pseudo-measurement (kf_workers.py:698-706, hw5_2.py:352-366): Z from the PREDICTED
    // state and the raw sample, H = I, R = diag(50, 0.05, 10, 0.1, 100 per group).  imu = (roll,
    // pitch, yaw, wx, wy, wz, ax, ay, az).
    // `imu` is any indexable payload: a register array, or an LDS image (ref_events_lds_kernel)
    template <bool POISON = true, class Pay>
    __device__ __forceinline__ bool update_imu(const Pay& imu, T dt) {
        bool ok = true;
#pragma unroll
        for (int c = 0; c < M::NP; ++c) {
            T q[3], Rp[6], rg;
            pva_noise<CUSTOM, M>(kc, c, q, Rp, rg);
            T xb[3];
            get_pva(c, xb);
            const T a = imu[M::imu_acc(c)];
            const T V = fmaT(a, dt, xb[1]);   // V = x_v + a dt
            const T X = fmaT(V, dt, xb[0]);   // X = x_p + V dt
            const T zb[3] = {X, V, a};
            ok = sel_update<3, 3, true, T, kRefNewton, POISON, kRefJoseph<T>, kRefGainR>(xb, pva[c], zb, Rp) && ok;
            put_pva(c, xb);
        }
#pragma unroll
        for (int c = 0; c < M::NA; ++c) {
            T q[2], Ra[3];
            aw_noise<CUSTOM, M>(kc, c, q, Ra);
            T xa[2];
            get_aw(c, xa);
            const T za[2] = {imu[M::imu_att(c)], imu[M::imu_rate(c)]};
            ok = sel_update<2, 2, true, T, kRefNewton, POISON, kRefJoseph<T>, kRefGainR>(xa, aw[c], za, Ra) && ok;
            put_aw(c, xa);
        }
        return ok;
    }

    // slogdet of the full P = sum over the chain blocks (kf_workers.py:716-717): the product of
    // the blocks' determinants, division-free per block (det3_scaled / det2) and one reciprocal
    // for the pva pivots; fp32 renormalises after every block (three pva blocks reach 1e48).
    __device__ __forceinline__ T logdet() const {
        int ex;
        const T prod = det_mant(ex);
        const T ld = log_mant(prod, ex);
        return prod == prod ? ld : quiet_nan<T>();
    }
    // the same determinant before its log: mantissa in [0.5, 1) (NaN unless positive definite)
    // times 2^ex
    __device__ __forceinline__ T det_mant(int& ex) const {
        constexpr bool kNarrow = sizeof(T) == 4;
        T num = T(1), den = T(1);
        ex = 0;
        bool ok = true;
#pragma unroll
        for (int c = 0; c < M::NP; ++c) {
            det3_scaled<T>(pva[c], num, den, ok);
            if (kNarrow || c == M::NP - 1) renorm(num, ex);
        }
#pragma unroll
        for (int c = 0; c < M::NA; ++c) {
            det2<T>(aw[c], num, ok);
            if (kNarrow) renorm(num, ex);
        }
        T prod = num * rcp_nr<kRefNewton>(den);
        renorm(prod, ex);
        return ok ? prod : quiet_nan<T>();
    }

    __device__ __forceinline__ void reset_cov() {
        const T p[6] = {T(M::P0Pos), T(0), T(0), T(M::P0Vel), T(0), T(M::P0Acc)};
        const T w[3] = {T(M::P0Att), T(0), T(M::P0Rate)};
#pragma unroll
        for (int c = 0; c < M::NP; ++c)
#pragma unroll
            for (int k = 0; k < 6; ++k) pva[c][k] = p[k];
#pragma unroll
        for (int c = 0; c < M::NA; ++c)
#pragma unroll
            for (int k = 0; k < 3; ++k) aw[c][k] = w[k];
        if constexpr (CUSTOM) {  // P0 = diag(p0) in the model's state order
#pragma unroll
            for (int c = 0; c < M::NP; ++c) {
                pva[c][0] = T(ro(kc)->p0[M::pva(c, 0)]);
                pva[c][3] = T(ro(kc)->p0[M::pva(c, 1)]);
                pva[c][5] = T(ro(kc)->p0[M::pva(c, 2)]);
            }
#pragma unroll
            for (int c = 0; c < M::NA; ++c) {
                aw[c][0] = T(ro(kc)->p0[M::aw(c, 0)]);
                aw[c][2] = T(ro(kc)->p0[M::aw(c, 1)]);
            }
        }
    }

    // block-packed covariance row r (see the file comment)
    __device__ __forceinline__ T& blk(int r) { return r < 6 * M::NP ? pva[r / 6][r % 6] : aw[(r - 6 * M::NP) / 3][(r - 6 * M::NP) % 3]; }
    __device__ __forceinline__ T blk(int r) const { return r < 6 * M::NP ? pva[r / 6][r % 6] : aw[(r - 6 * M::NP) / 3][(r - 6 * M::NP) % 3]; }

    __device__ __forceinline__ void load(const void* xbase, const void* Pbase, uint32_t rb, uint32_t off) {
#pragma unroll
        for (int i = 0; i < M::N; ++i) x[i] = ldb<T>(xbase, i, rb, off);
#pragma unroll
        for (int r = 0; r < M::NBLK; ++r) blk(r) = ldb<T>(Pbase, r, rb, off);
    }

    __device__ __forceinline__ void store(void* xbase, void* Pbase, uint32_t rb, uint32_t off) const {
#pragma unroll
        for (int i = 0; i < M::N; ++i) stb(xbase, i, rb, off, x[i]);
        store_cov(Pbase, 0, rb, off);
    }

    // covariance rows at row offset r0 of a [.][B] array (r0 = t * NBLK for a per-step record)
    __device__ __forceinline__ void store_cov(void* Pbase, int64_t r0, uint32_t rb, uint32_t off) const {
#pragma unroll
        for (int r = 0; r < M::NBLK; ++r) stb(Pbase, r0 + r, rb, off, blk(r));
    }

    __device__ __forceinline__ void fill_nan() {
#pragma unroll
        for (int i = 0; i < M::N; ++i) x[i] = quiet_nan<T>();
#pragma unroll
        for (int r = 0; r < M::NBLK; ++r) blk(r) = quiet_nan<T>();
    }

    // One event of the reference loop (kf_workers.py:682-717): predict over dt, then the GPS or
    // IMU update; with `gate`, the update only when logdet(P_pred) > threshold
    // (run_adaptive_threshold_kalman_filter, kf_workers.py:1023-1025).  Returns whether the
    // update was applied; `ok` turns false on a non-positive-definite S.
    // POISON = false for callers that fill the filter with NaN when `ok` turns false
    template <bool POISON = true, class Pay>
    __device__ __forceinline__ bool event(int type, T dt, const Pay& pay, bool gate, T threshold, bool& ok) {
        predict(dt);
        bool apply = (type == kGps || type == kImu);
        if (gate && apply) apply = logdet() > threshold;
        if (apply) {
            if (type == kGps) {
                const T z[3] = {pay[0], pay[1], pay[2]};  // (easting, northing, altitude)
                ok = update_gps<POISON>(z) && ok;
            } else {
                ok = update_imu<POISON>(pay, dt) && ok;
            }
        }
        return apply;
    }
};

// ------------------------------------------------------------------------------------
// Per-filter event streams (kf_run_events).
// ------------------------------------------------------------------------------------
template <typename T, class M, bool CUSTOM>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void ref_events_kernel(const RefArgs a) {
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    const uint32_t rb8 = uint32_t(a.B) * 8u;
    const uint32_t off8 = uint32_t(f) * 8u;
    Chains<T, M, CUSTOM> s;
    s.kc = a.kc;
    s.load(a.x, a.P, rb, off);
    int32_t st = a.status[f];
    const uint32_t rb_tr = a.traj ? rb : 0u, rb_ld = a.logdet ? rb : 0u, rb_cv = a.cov ? rb : 0u;
    struct In {
        int type;
        double dt;
        T pay[9];
    };
    auto load = [&](int t, In& in) {
        in.type = int(ldb<uint8_t>(a.etype, t, uint32_t(a.B), uint32_t(f)));
        in.dt = ldb<double>(a.dt, t, rb8, off8);
#pragma unroll
        for (int i = 0; i < 9; ++i) in.pay[i] = ldb<T>(a.payload, int64_t(t) * 9 + i, rb, off);
    };
    auto step = [&](int t, const In& in) {
        bool applied = false;
        if (in.type != 255) {
            bool ok = true;
            applied = s.template event<false>(in.type, T(in.dt), in.pay, a.gate != 0, T(a.threshold), ok);
            if (!ok) {
                st = kNotSpd;
                s.fill_nan();
            }
        }
#pragma unroll
        for (int i = 0; i < M::NTRAJ; ++i) stb(a.traj, int64_t(t) * M::NTRAJ + i, rb_tr, off, s.x[i]);
        if (a.cov) s.store_cov(a.cov, int64_t(t) * M::NBLK, rb_cv, off);
        if (a.logdet) {
            const T ld = s.logdet();
            st = (ld == ld) ? st : kNotSpd;
            stb(a.logdet, t, rb_ld, off, ld);
        }
        if (a.updated) a.updated[int64_t(t) * a.B + f] = applied ? 1 : 0;
    };
    // no prefetch: at 3 waves/SIMD this kernel is instruction-bound, and a second input buffer
    // (A/B-measured: 8.93 vs 9.00 ms at B = 2^20, T = 256) costs a wave of occupancy
    for (int t = 0; t < a.T; ++t) {
        In in;
        load(t, in);
        step(t, in);
    }
    s.store(a.x, a.P, rb, off);
    a.status[f] = st;
}

// ------------------------------------------------------------------------------------
// ref_events_kernel with its inputs staged through LDS by the DMA engine (buffer_load ... lds):
// event t+1's payload, dt and type travel HBM -> LDS while event t computes, without VGPRs
// (a register prefetch of the same inputs costs this fp64 kernel its third wave per SIMD).
// Each wave owns one LDS image of an event's inputs:
//   [0, 9*64*W)              payload rows 0..8, 64 filters each (row-major, lane-linear)
//   [DT_OFF, DT_OFF + 512)   dt, 64 doubles
//   [ET_OFF, ET_OFF + 64)    event type, 64 bytes
// Every DMA instruction moves 64 lanes x 16 B of ONE input (a wave-uniform row-span descriptor,
// the lane's chunk in voffset; the range check drops what lies beyond the span).  Order per
// event: wait for the image (counted vmcnt: only the previous event's NST stores are younger),
// read it into registers, drain those reads (lgkmcnt), issue the next event's DMA into the same
// image, compute, store.  The per-event store count NST is fixed (absent records go to
// zero-length descriptors) so the wait can be counted.  Requires B % 16 == 0 (no 16-B chunk
// straddles B) and 9 * B * W < 2^32; the host falls back to ref_events_kernel otherwise.
// ------------------------------------------------------------------------------------
constexpr int vmcnt_imm(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }
constexpr int lgkmcnt0_imm = 15 | (7 << 4) | (0 << 8) | (3 << 14);  // LDS reads drained, vmcnt untouched

// payload element i of this lane, read from the wave's LDS image where the update uses it
template <typename T>
struct LdsPayload {
    const T* img;  // image base + lane
    __device__ __forceinline__ T operator[](int i) const { return img[i * 64]; }
};

template <typename T, class M, bool COV, bool CUSTOM>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3))) void ref_events_lds_kernel(
    const RefArgs a) {
    constexpr int W = int(sizeof(T));
    constexpr int PAY = 9 * 64 * W;
    constexpr int NIP = (PAY + 1023) / 1024;    // payload DMA instructions
    constexpr int LPR = 4 * W;                  // lanes per 64-filter row (16 B each)
    constexpr int DT_OFF = NIP * 1024, ET_OFF = DT_OFF + 1024, IMG = ET_OFF + 64;
    constexpr int NDMA = NIP + 2;
    constexpr int NST = M::NTRAJ + 2 + (COV ? M::NBLK : 0);  // traj, logdet, updated (+ cov)
    static_assert(NST + NDMA <= 63, "vmcnt range");
    __shared__ __attribute__((aligned(16))) unsigned char lds[(kBlock / 64) * 2 * IMG];
    const int lane = int(threadIdx.x & 63);
    const int wave = wave_uniform(int(threadIdx.x >> 6));
    const int64_t f0 = int64_t(blockIdx.x) * kBlock + int64_t(wave) * 64;
    if (f0 >= a.B) return;  // whole wave; partial waves keep their dead lanes for the DMA
    const int64_t f = f0 + lane;
    unsigned char* const img0 = lds + wave * 2 * IMG;
    const uint32_t off = uint32_t(f) * uint32_t(W);  // dead lanes: beyond every row
    const uint32_t rb = uint32_t(a.B) * uint32_t(W);
    Chains<T, M, CUSTOM> s;
    s.kc = a.kc;
    s.load(a.x, a.P, rb, off);
    int32_t st = f < a.B ? a.status[f] : 0;
    const uint32_t rb_tr = a.traj ? rb : 0u, rb_ld = a.logdet ? rb : 0u, rb_cv = a.cov ? rb : 0u;
    const uint32_t rb_up = a.updated ? uint32_t(a.B) : 0u;
    // drain the state loads once: left pending into the loop, the waitcnt pass puts a wait for
    // them at each first use in every iteration, and those waits would drain the DMA prefetch
    waitcnt<vmcnt_imm(0)>();
    // payload DMA instruction k moves rows 16/W*k + lane / LPR, 16-B chunk lane % LPR of each;
    // the row step k * (16/W) * rb goes into soffset
    const uint32_t voff_pay = uint32_t(lane / LPR) * rb + uint32_t(lane % LPR) * 16u;
    auto issue = [&](int t, unsigned char* img) {
        const char* pb = reinterpret_cast<const char*>(a.payload) + int64_t(t) * 9 * int64_t(rb) + f0 * W;
        const __amdgpu_buffer_rsrc_t rp = bytes_rsrc(pb, 9u * rb - uint32_t(f0) * W);
#pragma unroll
        for (int k = 0; k < NIP; ++k)
            if (k + 1 < NIP || k * 1024 + lane * 16 < PAY)
                lds_dma16(rp, img + k * 1024, voff_pay, k * (16 / W) * int(rb));
        const char* db = reinterpret_cast<const char*>(a.dt) + int64_t(t) * int64_t(a.B) * 8 + f0 * 8;
        if (lane < 32) lds_dma16(bytes_rsrc(db, uint32_t(a.B - f0) * 8u), img + DT_OFF, uint32_t(lane) * 16u, 0);
        const char* eb = reinterpret_cast<const char*>(a.etype) + int64_t(t) * int64_t(a.B) + f0;
        if (lane < 4) lds_dma16(bytes_rsrc(eb, uint32_t(a.B - f0)), img + ET_OFF, uint32_t(lane) * 16u, 0);
    };
    issue(0, img0);
    // the in-loop count assumes a previous event's NST stores are younger than this image's
    // DMA; event 0 has none, so its image is waited for here
    waitcnt<vmcnt_imm(0)>();
    for (int t = 0; t < a.T; ++t) {
        unsigned char* const img = img0 + (t & 1) * IMG;
        // the other image was last read by event t - 1, whose reads have completed
        if (t + 1 < a.T) {
            issue(t + 1, img0 + ((t + 1) & 1) * IMG);
            // event t's image: its DMA is older than event t-1's NST stores and this NDMA
            waitcnt<vmcnt_imm(NST + NDMA)>();
        } else {
            waitcnt<vmcnt_imm(NST)>();
        }
        const int type = img[ET_OFF + lane];
        const T dt = T(reinterpret_cast<const double*>(img + DT_OFF)[lane]);
        const LdsPayload<T> pay{reinterpret_cast<const T*>(img) + lane};
        bool applied = false;
        if (type != 255) {
            bool ok = true;
            applied = s.template event<false>(type, dt, pay, a.gate != 0, T(a.threshold), ok);
            if (!ok) {
                st = kNotSpd;
                s.fill_nan();
            }
        }
#pragma unroll
        for (int i = 0; i < M::NTRAJ; ++i) stb(a.traj, int64_t(t) * M::NTRAJ + i, rb_tr, off, s.x[i]);
        if constexpr (COV) s.store_cov(a.cov, int64_t(t) * M::NBLK, rb_cv, off);
        const T ld = a.logdet ? s.logdet() : T(0);
        st = (ld == ld) ? st : kNotSpd;
        stb(a.logdet, t, rb_ld, off, ld);
        stb_u8(a.updated, t, rb_up, uint32_t(f), applied ? uint8_t(1) : uint8_t(0));
    }
    s.store(a.x, a.P, rb, off);
    if (f < a.B) a.status[f] = st;
}

template <typename T, class M, bool CUSTOM>
__global__ __launch_bounds__(kBlock) void ref_reset_kernel(const RefArgs a) {
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    Chains<T, M, CUSTOM> s;
    s.kc = a.kc;
#pragma unroll
    for (int i = 0; i < M::N; ++i) s.x[i] = a.x0 ? ldb<T>(a.x0, i, rb, off) : T(0);
    s.reset_cov();
    s.store(a.x, a.P, rb, off);
    a.status[f] = 0;
}

// ------------------------------------------------------------------------------------
// Chain-parallel variant of ref_events_kernel for few filters (a single drive log): one lane
// per axis chain, kGroup lanes per filter.  Without the adaptive gate the chains are
// independent filters sharing an event stream, so a filter's per-event instruction stream
// shrinks to one chain's; the log-determinant (and the gate) is the sum of the chains' logs
// over the lane group (xor shuffles).  Every lane runs a 3-state chain: an (att, rate) chain
// carries an inert third state (F couples nothing to it, Q = 0; its IMU row measures z = 0
// with R = 1 and is reset after each update), so pva and aw lanes execute the same code.
// The arithmetic per chain is the lane kernel's, operation for operation (the extra terms are
// exact zeros); only the logdet is summed per chain instead of multiplied then logged.
// ------------------------------------------------------------------------------------
constexpr int kGroup = 8;
#ifndef KF_CHAIN_DEPTH
#define KF_CHAIN_DEPTH 2
#endif
constexpr int kChainDepth = KF_CHAIN_DEPTH;  // input ring of ref_chain_kernel
#ifndef KF_STREAM_DEPTH
#define KF_STREAM_DEPTH 8
#endif
constexpr int kStreamDepth = KF_STREAM_DEPTH;  // its input ring in stream mode (kf_run_stream)
#ifndef KF_STREAM_VAR_DEPTH
#define KF_STREAM_VAR_DEPTH 4
#endif
// the map pass's ring (4 state variants per lane): shallower, so the lane fits 2 waves per SIMD
constexpr int kStreamVarDepth = KF_STREAM_VAR_DEPTH;
#ifndef KF_STREAM_LD_BATCH
#define KF_STREAM_LD_BATCH 1
#endif
// the map pass's log-det records: the group's determinant product per event, kept by lane
// (event mod 8) and logged every 8 events (one log per lane-8-events instead of per lane-event;
// the pass is bound by its instruction issue).  0: every lane logs its chain every event and the
// group sums the logs (the NV = 1 chain kernel's form)
constexpr bool kStreamLdBatch = KF_STREAM_LD_BATCH != 0;
#ifndef KF_STREAM_RECORD_PAIRS
#define KF_STREAM_RECORD_PAIRS 1
#endif
// the records from the map pass two entries per thread (stream_records2_kernel; 0: one each)
constexpr bool kStreamRecordPairs = KF_STREAM_RECORD_PAIRS != 0;
#ifndef KF_STREAM_VAR_SPLIT
#define KF_STREAM_VAR_SPLIT 0
#endif
// the map pass's four state variants as two per lane over two 8-lane groups per chunk (variants
// 0, 1 and 2, 3): twice the waves, each lane's event a little shorter (the covariance work
// repeated in both groups).  Measured slower on config 1, 0.2196 vs 0.2045 ms per log in-process
// (profiles/r04_pmc/cfg1_diag/ab_split_sym_halves.log), so off; kept for A/B builds
constexpr bool kStreamVarSplit = KF_STREAM_VAR_SPLIT != 0;
// lanes per filter of ref_chain_kernel
template <int NV>
__host__ __device__ constexpr int chain_lanes() {
    return NV == 4 && kStreamVarSplit ? 2 * 8 : 8;
}

// Sums / ORs over the 8-lane group with DPP (a VALU-latency lane exchange, no LDS round trip):
// quad_perm [1,0,3,2] (xor 1), quad_perm [2,3,0,1] (xor 2), then row_half_mirror (lane i <-> 7-i
// within each 8 lanes), which pairs the two quads.  Every lane of the group ends with the total.
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141;
constexpr int kDppRowRor8 = 0x128;  // row_ror:8: lane l of a 16-lane row reads lane l +- 8

template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    const v2u u = __builtin_bit_cast(v2u, v);
    v2u r;
    r.x = __builtin_amdgcn_mov_dpp(int(u.x), CTRL, 0xF, 0xF, false);
    r.y = __builtin_amdgcn_mov_dpp(int(u.y), CTRL, 0xF, 0xF, false);
    return __builtin_bit_cast(double, r);
}
template <int CTRL>
__device__ __forceinline__ float dpp_d(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

template <typename T>
__device__ __forceinline__ T group_sum(T v) {
    v += dpp_d<kDppXor1>(v);
    v += dpp_d<kDppXor2>(v);
    v += dpp_d<kDppHalfMirror>(v);
    return v;
}

__device__ __forceinline__ bool group_any(bool b) {
    int v = b ? 1 : 0;
    v |= __builtin_amdgcn_mov_dpp(v, kDppXor1, 0xF, 0xF, false);
    v |= __builtin_amdgcn_mov_dpp(v, kDppXor2, 0xF, 0xF, false);
    v |= __builtin_amdgcn_mov_dpp(v, kDppHalfMirror, 0xF, 0xF, false);
    return v != 0;
}

template <typename T>
__device__ __forceinline__ T chain_log_det(const T (&P)[6]) {
    // one 3-state chain's log det (an aw chain's inert third state has variance 1, no coupling)
    T num = T(1), den = T(1);
    int ex = 0;
    bool ok = true;
    det3_scaled<T>(P, num, den, ok);
    T prod = num * rcp_nr<kRefNewton>(den);
    renorm(prod, ex);
    const T ld = log_mant(prod, ex);
    return ok ? ld : quiet_nan<T>();
}

// chain_log_det before its log: the determinant as a mantissa in [0.5, 1) (NaN unless the
// block is positive definite) and a binary exponent
template <typename T>
__device__ __forceinline__ void chain_det_mant(const T (&P)[6], T& m, int& ex) {
    T num = T(1), den = T(1);
    bool ok = true;
    det3_scaled<T>(P, num, den, ok);
    m = num * rcp_nr<kRefNewton>(den);
    ex = 0;
    renorm(m, ex);
    m = ok ? m : quiet_nan<T>();
}

// (mantissa, exponent) product over the 8-lane group, the same DPP pattern as group_sum: every
// lane ends with the same bits (each step multiplies a pair in both orders, and x * y == y * x)
template <typename T>
__device__ __forceinline__ void group_prod(T& m, int& ex) {
    m *= dpp_d<kDppXor1>(m);
    ex += __builtin_amdgcn_mov_dpp(ex, kDppXor1, 0xF, 0xF, false);
    m *= dpp_d<kDppXor2>(m);
    ex += __builtin_amdgcn_mov_dpp(ex, kDppXor2, 0xF, 0xF, false);
    m *= dpp_d<kDppHalfMirror>(m);
    ex += __builtin_amdgcn_mov_dpp(ex, kDppHalfMirror, 0xF, 0xF, false);
}

// non-negative doubles (and +NaN) order as their bit patterns: atomic max via uint64
__device__ __forceinline__ void atomic_max_pos(double* p, double v) {
    if (!(v >= 0.0)) v = __builtin_nan("");
    atomicMax(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v));
}

// The adaptive gate logdet(P_pred) > threshold (kf_workers.py:1023-1025) of the chain kernel,
// decided on the group's determinant product (mantissa, binary exponent) against
// exp(threshold) (1 -+ eps); only inside that band are the logs taken, as
// group_sum(chain_log_det) > threshold, so every decision is the logs' (eps far above the logs'
// and the products' rounding: 1e-10 in f64, 1e-4 in f32).  The log is the longest part of a
// gated event's dependent chain, and a gated filter with few updates runs little else.
// Non-finite or huge thresholds take the logs every event.
template <typename T>
struct GateBand {
    T lo_m = T(0), hi_m = T(0);
    int lo_e = 0, hi_e = 0;
    bool banded = false;
    __device__ __forceinline__ void init(double thr) {
        banded = thr == thr && thr > -1e6 && thr < 1e6;
        if (!banded) return;
        const double eps = sizeof(T) == 8 ? 1e-10 : 1e-4;
        const double k = floor(thr * 1.4426950408889634);  // exp(thr) = 2^k exp(r), r in [0, ln 2)
        const double r = thr - k * 0.6931471805599453;
        int e1, e2;
        const double lo = frexp(exp(r) * (1.0 - eps), &e1), hi = frexp(exp(r) * (1.0 + eps), &e2);
        lo_m = T(lo);
        hi_m = T(hi);
        lo_e = int(k) + e1;
        hi_e = int(k) + e2;
    }
    // the gate for this lane's chain covariance P (live: a chain lane of the group)
    __device__ __forceinline__ bool open(const T (&P)[6], bool live, T thr) const {
        if (banded) {
            T m;
            int ex;
            chain_det_mant(P, m, ex);
            m = live ? m : T(1);
            ex = live ? ex : 0;
            group_prod(m, ex);
            int e;
            m = frexp(m, &e);
            ex += e;
            if (!(m > T(0))) return false;                           // NaN (a failed block) or 0: log -inf
            if (ex < lo_e || (ex == lo_e && m < lo_m)) return false;  // the logs' sum below thr
            if (ex > hi_e || (ex == hi_e && m > hi_m)) return true;   // above
        }
        return group_sum(live ? chain_log_det(P) : T(0)) > thr;
    }
};

// Inputs of one event for one lane.
template <typename T>
struct ChainIn {
    int type;
    double dt;
    T va, vb;
};

// NV > 1 (stream mode only): NV variants of each filter that differ only in their start state
// (kf_run_stream's map pass: a chunk from its guess and from the guess + delta on each chain
// component) share one lane.  The covariance recursion does not read the state, so P, S and K
// are computed once per event and every variant's state is updated with them (sel_update_nv);
// each variant's arithmetic is the single-state lane's, term for term.  Variant v's state is
// column v * B + f of a state bank of NV * B columns (the covariance: column f), and its
// trajectory records go to rows v * s_vstride.
template <typename T, class M, bool STREAM, bool CUSTOM, int NV = 1>
__global__ __launch_bounds__(kBlock) void ref_chain_kernel(const RefArgs a) {
    static_assert(NV == 1 || STREAM, "state variants are a stream-mode feature");
    if (a.skip && *a.skip) return;  // the sequential fallback of a stream run that passed its checks
    constexpr int LPF = chain_lanes<NV>();         // lanes per filter
    constexpr int NL = LPF == 2 * kGroup ? 2 : NV;  // variants this lane holds
    const int64_t g = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    const int64_t f = g / LPF;
    if (f >= a.B) return;  // whole groups leave together (LPF divides the wave)
    const int c = static_cast<int>(g % kGroup);
    const int vb = NL < NV ? int((g % LPF) / kGroup) * NL : 0;  // this lane's first variant
    const bool pva = c < M::NP;
    const bool live = c < M::NP + M::NA;
    const int ca = pva ? c : (live ? c - M::NP : 0);
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    const uint32_t rbank = uint32_t(NV) * rb;  // row stride of the state / covariance bank
    const uint32_t rb8 = uint32_t(a.B) * 8u;
    const uint32_t off8 = uint32_t(f) * 8u;
    // this lane's state indices and block rows (-1: none), as voffsets into row spans
    int xi[3], pr[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) xi[k] = !live ? -1 : pva ? M::pva(ca, k) : (k < 2 ? M::aw(ca, k) : -1);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int aw_row = k == 0 ? 0 : k == 1 ? 1 : k == 3 ? 2 : -1;  // (tt tw ww) of the 3x3 packing
        pr[k] = !live ? -1 : pva ? 6 * ca + k : (aw_row < 0 ? -1 : 6 * M::NP + 3 * ca + aw_row);
    }
    uint32_t vx[3], vp[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) vx[k] = xi[k] >= 0 ? uint32_t(xi[k]) * rbank + off : kDropOffset;
#pragma unroll
    for (int k = 0; k < 6; ++k) vp[k] = pr[k] >= 0 ? uint32_t(pr[k]) * rbank + off : kDropOffset;
    const uint32_t v_tr = (xi[0] >= 0 && xi[0] < M::NTRAJ) ? uint32_t(xi[0]) * rb + off : kDropOffset;
    const uint32_t v_ld = c == 0 ? off : kDropOffset;
    const int ia = pva ? ca : M::imu_att(ca);              // GPS position / IMU attitude column
    const int ib = pva ? M::imu_acc(ca) : M::imu_rate(ca);  // IMU acceleration / rate column
    const uint32_t v_a = uint32_t(ia) * rb + off, v_b = uint32_t(ib) * rb + off;
    T q[3] = {T(pva ? kQPos : kQAtt), T(pva ? kQVel : kQRate), T(pva ? kQAcc : 0.0)};
    T Rimu[6] = {T(pva ? kRPos : kRAtt), T(0), T(0), T(pva ? kRVel : kRRate), T(0), T(pva ? kRAcc : 1.0)};
    T Rgps = T(kRGps);
    if constexpr (CUSTOM) {  // this lane's chain states (the inert third state of an aw lane keeps 0 / 1)
        const RefConsts* kc = a.kc;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (xi[k] >= 0) {
                q[k] = T(ro(kc)->q[xi[k]]);
                Rimu[k == 0 ? 0 : k == 1 ? 3 : 5] = T(ro(kc)->r_imu[xi[k]]);
            }
        if (pva) Rgps = T(ro(kc)->r_gps[ca]);
    }

    T x[NL][3], P[6];
    T xs0[3];  // variant 0's start (the map pass's guess)
    {
        const auto rx = span_rsrc(a.x, 0, rbank, M::N), rp = span_rsrc(a.P, 0, rbank, M::NBLK);
#pragma unroll
        for (int v = 0; v < NL; ++v)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                x[v][k] = ldv(rx, vx[k] == kDropOffset ? kDropOffset : vx[k] + uint32_t(vb + v) * rb, T(0));
#pragma unroll
        for (int k = 0; k < 6; ++k) P[k] = pr[k] >= 0 ? ldv(rp, vp[k], T(0)) : T(k == 0 || k == 3 || k == 5 ? 1 : 0);
        if constexpr (NL < NV) {
#pragma unroll
            for (int k = 0; k < 3; ++k) xs0[k] = ldv(rx, vx[k], T(0));
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) xs0[k] = x[0][k];
        }
    }
    // the map pass's seam check reads the next chunk's start covariance: loaded here, before
    // any of this lane's stores (a later load would wait for all of them, vmcnt being in order)
    double wnx[6] = {0, 0, 0, 0, 0, 0};
    if constexpr (NV == 4) {
        if (live && a.s_maps && a.s_check && f + 1 < a.B) {
            const T* wn = static_cast<const T*>(a.s_wnext);
#pragma unroll
            for (int k = 0; k < 6; ++k)
                if (pr[k] >= 0) wnx[k] = double(wn[int64_t(pr[k]) * a.B + f + 1]);
        }
    }
    int32_t st = a.status[f];
    const bool need_ld = a.logdet != nullptr;
    GateBand<T> gate;
    if (a.gate) gate.init(a.threshold);
    constexpr bool kLdBatch = STREAM && NV == 4 && kStreamLdBatch;
    T bm = T(1);  // kLdBatch: the group's determinant product of event (t - t mod 8 + c)
    int bex = 0;

    // stream mode: this filter's event t is stream event e0 + t; one descriptor per stream
    // (events outside [0, S) are skipped: dropped loads, NONE type, dropped records)
    const int64_t e0 = STREAM ? (f % a.s_nchunks) * a.s_chunk + a.s_shift : 0;
    const uint32_t S = STREAM ? uint32_t(a.s_len) : 0u;
    const auto r_et = bytes_rsrc(a.etype, S), r_dt = bytes_rsrc(a.dt, S * 8u);
    const auto r_pay = bytes_rsrc(a.payload, S * 9u * uint32_t(sizeof(T)));
    // filter f is variant f / s_nchunks of its chunk (NV = 1) or carries variants 0 .. NV - 1:
    // with s_nvar > 1, variant q's trajectory records go to rows [q * s_vstride, q * s_vstride +
    // S) (s_vstride >= S + chunk, so a padded chunk's rows past S stay inside its own variant),
    // and only variant 0 writes the others
    const int var = STREAM ? int(f / a.s_nchunks) + vb : 0;
    const uint32_t trows = STREAM ? (a.s_nvar > 1 ? uint32_t(a.s_nvar) * uint32_t(a.s_vstride) : S) : 0u;
    const auto r_str = bytes_rsrc(a.traj, trows * uint32_t(M::NTRAJ * sizeof(T)));
    const auto r_scv = bytes_rsrc(a.cov, S * uint32_t(M::NBLK * sizeof(T)));
    const auto r_sld = bytes_rsrc(a.logdet, S * uint32_t(sizeof(T)));
    const auto r_sup = bytes_rsrc(a.updated, S);
    // Stream offsets are plain 32-bit products of ue = uint32(e): an event before the stream
    // start wraps far past every descriptor's length and one past its end lands beyond it, so
    // loads return 0 and stores drop without a select on the address (a select there was turned
    // into branches around the loads, whose joins drained the prefetch ring with vmcnt(0)).
    // Lanes without a record OR in bit 31 (kf_run_stream keeps (S + W) * rows * w < 2^31).
    const uint32_t m_tr = v_tr != kDropOffset ? 0u : kDropOffset;
    const uint32_t col_tr = v_tr != kDropOffset ? (uint32_t(var) * uint32_t(a.s_vstride) * M::NTRAJ + uint32_t(xi[0])) *
                                                      uint32_t(sizeof(T))
                                                : 0u;
    const uint32_t vstep_tr = uint32_t(a.s_vstride) * uint32_t(M::NTRAJ * sizeof(T));  // next variant's rows
    const uint32_t m_ld = c == 0 && var == 0 ? 0u : kDropOffset;  // variant 0's group only
    uint32_t col_cv[6];
#pragma unroll
    for (int k = 0; k < 6; ++k)
        col_cv[k] = pr[k] >= 0 && var == 0 ? uint32_t(pr[k]) * uint32_t(sizeof(T)) : kDropOffset;
    auto load = [&](int t, ChainIn<T>& in) {
        if constexpr (STREAM) {
            const uint32_t ue = uint32_t(e0 + t);
            const int ty = int(__builtin_amdgcn_raw_buffer_load_b8(r_et, ue, 0, 0));
            in.type = ue < S ? ty : 255;
            in.dt = ldv(r_dt, ue * 8u, 0.0);
            in.va = ldv(r_pay, (ue * 9u + uint32_t(ia)) * uint32_t(sizeof(T)), T(0));
            in.vb = ldv(r_pay, (ue * 9u + uint32_t(ib)) * uint32_t(sizeof(T)), T(0));
        } else {
            in.type = int(ldb<uint8_t>(a.etype, t, uint32_t(a.B), uint32_t(f)));
            in.dt = ldb<double>(a.dt, t, rb8, off8);
            const auto rpay = span_rsrc(a.payload, int64_t(t) * 9, rb, 9);
            in.va = ldv(rpay, v_a, T(0));
            in.vb = ldv(rpay, v_b, T(0));
        }
    };
    auto step = [&](int t, const ChainIn<T>& in) {
        const int type = in.type;
        const T dt = T(in.dt);
        const T va = in.va, vb = in.vb;
        bool applied = false;
        if (type != 255) {
            // predict: F = [[1, dt, c02], [0, 1, c12], [0, 0, 1]] (c02 = c12 = 0 on an aw lane)
            const T c02 = pva ? T(0.5) * dt * dt : T(0);
            const T c12 = pva ? dt : T(0);
#pragma unroll
            for (int v = 0; v < NL; ++v) {
                const T xn0 = fmaT(c02, x[v][2], fmaT(dt, x[v][1], x[v][0]));
                const T xn1 = fmaT(c12, x[v][2], x[v][1]);
                x[v][0] = xn0;
                x[v][1] = xn1;
            }
            T FP[3][3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                FP[0][j] = fmaT(c02, P[tri<3>(2, j)], fmaT(dt, P[tri<3>(1, j)], P[tri<3>(0, j)]));
                FP[1][j] = fmaT(c12, P[tri<3>(2, j)], P[tri<3>(1, j)]);
                FP[2][j] = P[tri<3>(2, j)];
            }
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = i; j < 3; ++j) {
                    T s = FP[i][j];
                    if (j == 0) s = fmaT(FP[i][2], c02, fmaT(FP[i][1], dt, s));
                    if (j == 1) s = fmaT(FP[i][2], c12, s);
                    P[tri<3>(i, j)] = (i == j) ? s + q[i] * dt : s;
                }
            applied = (type == kGps || type == kImu);
            if (a.gate && applied) applied = gate.open(P, live, T(a.threshold));
            bool ok = true;
            if (applied) {
                if (type == kGps) {
                    if (pva) {
                        T zb[NL][1];
#pragma unroll
                        for (int v = 0; v < NL; ++v) zb[v][0] = va;
                        const T R[1] = {Rgps};
                        ok = sel_update_nv<3, 1, true, T, kRefNewton, true, NL, kRefJoseph<T>, kRefGainR>(x, P, zb, R);
                    }
                } else {
                    T zb[NL][3];
#pragma unroll
                    for (int v = 0; v < NL; ++v) {
                        const T V = fmaT(vb, dt, x[v][1]);
                        const T X = fmaT(V, dt, x[v][0]);
                        zb[v][0] = pva ? X : va;
                        zb[v][1] = pva ? V : vb;
                        zb[v][2] = pva ? vb : T(0);
                    }
                    ok = sel_update_nv<3, 3, true, T, kRefNewton, true, NL, kRefJoseph<T>, kRefGainR>(x, P, zb, Rimu);
                    if (!pva) {  // reset the inert state
#pragma unroll
                        for (int v = 0; v < NL; ++v) x[v][2] = T(0);
                        P[5] = T(1);
                    }
                }
            }
            if (group_any(!ok)) {
                st = kNotSpd;
#pragma unroll
                for (int v = 0; v < NL; ++v)
#pragma unroll
                    for (int k = 0; k < 3; ++k) x[v][k] = quiet_nan<T>();
#pragma unroll
                for (int k = 0; k < 6; ++k) P[k] = quiet_nan<T>();
            }
        }
        if constexpr (STREAM) {
            const uint32_t ue = uint32_t(e0 + t);
#pragma unroll
            for (int v = 0; v < NL; ++v)
                stv(r_str, (ue * uint32_t(M::NTRAJ * sizeof(T)) + col_tr + uint32_t(v) * vstep_tr) | m_tr, x[v][0]);
            // absent records: skipped by a wave-uniform branch (a store to a zero-length
            // descriptor is dropped, but it is still issued)
            if (a.cov) {
#pragma unroll
                for (int k = 0; k < 6; ++k)
                    stv(r_scv, (ue * uint32_t(M::NBLK * sizeof(T)) + col_cv[k]) | (col_cv[k] & kDropOffset), P[k]);
            }
            if (need_ld) {
                if constexpr (kLdBatch) {
                    T m;
                    int ex;
                    chain_det_mant(P, m, ex);
                    m = live ? m : T(1);
                    ex = live ? ex : 0;
                    group_prod(m, ex);
                    const int slot = t & (kGroup - 1);
                    if (c == slot) {
                        bm = m;
                        bex = ex;
                    }
                    if (slot == kGroup - 1 || t == a.T - 1) {  // wave-uniform: lane j logs event t - slot + j
                        int e;
                        const T ld = log_mant(frexp(bm, &e), bex + e);
                        const bool mine = c <= slot;
                        if (group_any(mine && !(ld == ld))) st = kNotSpd;
                        const uint32_t uj = uint32_t(e0 + t - slot + c);
                        stv(r_sld, (uj * uint32_t(sizeof(T))) | (mine && var == 0 ? 0u : kDropOffset), ld);
                    }
                } else {
                    const T ld = group_sum(live ? chain_log_det(P) : T(0));
                    st = (ld == ld) ? st : kNotSpd;
                    stv(r_sld, (ue * uint32_t(sizeof(T))) | m_ld, ld);
                }
            }
            if (a.updated) __builtin_amdgcn_raw_buffer_store_b8(applied ? uint8_t(1) : uint8_t(0), r_sup, ue | m_ld, 0, 0);
        } else {
            stv(span_rsrc(a.traj, int64_t(t) * M::NTRAJ, rb, M::NTRAJ), v_tr, x[0][0]);
            {
                const auto rc = span_rsrc(a.cov, int64_t(t) * M::NBLK, rb, M::NBLK);
#pragma unroll
                for (int k = 0; k < 6; ++k) stv(rc, vp[k], P[k]);
            }
            if (need_ld) {
                const T ld = group_sum(live ? chain_log_det(P) : T(0));
                st = (ld == ld) ? st : kNotSpd;
                stv(span_rsrc(a.logdet, t, rb, 1), v_ld, ld);
            }
            if (a.updated && c == 0) a.updated[int64_t(t) * a.B + f] = applied ? 1 : 0;
        }
    };

    // Inputs are prefetched kChainDepth - 1 events ahead through a fully unrolled ring of named
    // buffers (static indices, no loop-carried copies); loads past the end re-read the last
    // event, and the prologue's loads are drained once so no in-loop wait targets them.  Depths
    // 2, 3, 4 and 8 were A/B-measured on config 1 (one filter) without a resolvable difference:
    // a single wave's launch time varies +-10% from launch to launch
    // (profiles/r01_ab/chain_depth_inproc.json), and each depth adds a copy of the event body
    // (48 KB of code at 8), so the default stays at 2.
    // stream mode gathers each filter's events from its own part of the stream (a cache line
    // per 1.8 events, lines differ per filter), so its loads see HBM latency: a deeper ring
    constexpr int D = STREAM ? (NV > 1 ? kStreamVarDepth : kStreamDepth) : kChainDepth;
    const int T_ = a.T;
    auto load_c = [&](int t, ChainIn<T>& in) { load(t < T_ ? t : T_ - 1, in); };
    if (T_ > 0) {
        ChainIn<T> buf[D];
#pragma unroll
        for (int j = 0; j < D - 1; ++j) load_c(j, buf[j]);
        __builtin_amdgcn_s_waitcnt(0);
        int t = 0;
        for (; t + D <= T_; t += D) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                load_c(t + j + D - 1, buf[(j + D - 1) % D]);
                step(t + j, buf[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < D - 1; ++j)
            if (t + j < T_) step(t + j, buf[j]);
    }
    {
        const auto rx = span_rsrc(a.x, 0, rbank, M::N), rp = span_rsrc(a.P, 0, rbank, M::NBLK);
#pragma unroll
        for (int v = 0; v < NL; ++v)
#pragma unroll
            for (int k = 0; k < 3; ++k)
                stv(rx, vx[k] == kDropOffset ? kDropOffset : vx[k] + uint32_t(vb + v) * rb, x[v][k]);
        if (vb == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) stv(rp, vp[k], P[k]);
        }
    }
    if (c == 0 && vb == 0) a.status[f] = st;
    if constexpr (NV == 4) {
        // the map pass's epilogue (kf_run_stream): this chunk's affine map per chain, x_end =
        // A x_start + b (fp64), A by differences of the variants (variant q + 1 started at the
        // guess + delta on component q), b = x_end(guess) - A guess; then the covariance seam:
        // this chunk's end covariance against the next chunk's start covariance, relative to
        // the end covariance's largest entry in the chain (one atomic per wave)
        constexpr int NCH = M::NP + M::NA;
        const int ns = pva ? 3 : 2;
        double crel = 0.0;
        // every variant's end state: with the split, variants 2, 3 come from the other group of
        // 16 (DPP row_ror:8 pairs lane l with l + 8 within the row), every lane exchanging
        double xe[4][3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
#pragma unroll
            for (int v = 0; v < NL; ++v) xe[v][k] = double(x[v][k]);
            if constexpr (NL < 4) {
#pragma unroll
                for (int v = 0; v < NL; ++v) xe[NL + v][k] = dpp_d<kDppRowRor8>(xe[v][k]);
            }
        }
        if (live && a.s_maps && vb == 0) {
            double A[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}, b[3] = {0, 0, 0};
            const double rdelta = 1.0 / a.s_delta;  // delta is a power of two: exact
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                if (k >= ns) continue;
                const double e0v = xe[0][k];
                double sacc = e0v;
#pragma unroll
                for (int qq = 0; qq < 3; ++qq) {
                    if (qq >= ns) continue;
                    A[k][qq] = (xe[qq + 1][k] - e0v) * rdelta;
                    sacc = __builtin_fma(-A[k][qq], double(xs0[qq]), sacc);
                }
                b[k] = sacc;
            }
            double* mo = a.s_maps + (f * NCH + c) * 12;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
#pragma unroll
                for (int qq = 0; qq < 3; ++qq) mo[k * 3 + qq] = A[k][qq];
                mo[9 + k] = b[k];
            }
            if (a.s_check && f + 1 < a.B) {
                double scale = 0.0, gap = 0.0;
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    if (pr[k] < 0) continue;
                    const double pe = double(P[k]);
                    scale = fmax(scale, fabs(pe));
                    gap = fmax(gap, fabs(pe - wnx[k]));
                }
                const double rel = gap / fmax(scale, 1e-300);
                crel = rel == rel ? rel : __builtin_inf();
            }
        }
        if (a.s_check) {
            // the wave's max over its chunks (DPP inside a group; lanes of finished groups hold
            // 0), one atomic per wave: every chunk's lanes finish together, and one atomic per
            // chunk on the same address queued up behind each other at the end of the pass
            crel = fmax(crel, dpp_d<kDppXor1>(crel));
            crel = fmax(crel, dpp_d<kDppXor2>(crel));
            crel = fmax(crel, dpp_d<kDppHalfMirror>(crel));
            // a wave whose chunks all exist has every lane here (a partial last wave lost its
            // dead groups at the top, so it keeps one atomic per chunk)
            const bool full = (g & ~int64_t(63)) / LPF + 64 / LPF <= a.B;  // wave-uniform
            if (full) {
#pragma unroll
                for (int sh = kGroup; sh < 64; sh <<= 1) crel = fmax(crel, __shfl_xor(crel, sh, 64));
                const bool lane0 = (threadIdx.x & 63) == 0;
                if (lane0 && crel != 0.0) atomic_max_pos(&a.s_check->cov_gap, crel);
                const bool any_bad = __builtin_amdgcn_ballot_w64(c == 0 && st != 0) != 0;
                if (lane0 && any_bad) atomicOr(&a.s_check->bad, kStreamBadFilter);
            } else {
                if (c == 0 && vb == 0 && crel != 0.0) atomic_max_pos(&a.s_check->cov_gap, crel);
                if (c == 0 && vb == 0 && st != 0) atomicOr(&a.s_check->bad, kStreamBadFilter);
            }
        }
    }
}

// ------------------------------------------------------------------------------------
// ONE gated filter (B = 1, the adaptive threshold, kf_workers.py:959-1058) whose gate blocks
// most updates, on one wave: lane c + 8 j is chain c (the chain kernel's lane layout) of event
// slot j.  Every event that applies an update runs as the chain kernel's event (its arithmetic,
// term for term).  After an event that did not, the wave looks ahead over the next 8 events at
// once: between two updates the filter only predicts, and with the model's additive F (F(a) F(b)
// = F(a + b)) and diagonal Q(dt) a run of predicts has a closed form,
//   P_m = F(tau_m) (P + S_m) F(tau_m)^T,  S_m = sum_{i <= m} F(-tau_i) Q(dt_i) F(-tau_i)^T,
// tau the time since the last event run (prefix sums over the slots), x_m = F(tau_m) x.  Slot j
// takes event t + j; the first slot whose event would open the gate (GateBand on its closed-form
// P_pred, a ballot over the slots) ends the run: the slots before it write their records at
// once and hand their state on, and that event runs next as a chain-kernel event.  The closed
// form rounds differently from one predict after another (records within 1.8e-12 relative of the
// chain kernel's over 70,000 events, every flag equal); a gate decision could only differ within
// that distance of the threshold (in f32 it does: f64 only).  KF_OPT_EVENTS_KERNEL = 4 runs it,
// and kf_run_events' gated one-filter route when the chunked run falls back after updating at
// most 1 event in 8 (launch_stream_choose).
// ------------------------------------------------------------------------------------
template <typename T, class M, bool CUSTOM>
__global__ __launch_bounds__(64) void ref_chain_gated_kernel(const RefArgs a) {
    if (a.skip && *a.skip) return;
    const int lane = int(threadIdx.x);
    const int c = lane & (kGroup - 1);  // chain
    const int slot = lane / kGroup;     // event slot of the look-ahead
    const bool pva = c < M::NP;
    const bool live = c < M::NP + M::NA;
    const int ca = pva ? c : (live ? c - M::NP : 0);
    int xi[3], pr[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) xi[k] = !live ? -1 : pva ? M::pva(ca, k) : (k < 2 ? M::aw(ca, k) : -1);
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const int aw_row = k == 0 ? 0 : k == 1 ? 1 : k == 3 ? 2 : -1;
        pr[k] = !live ? -1 : pva ? 6 * ca + k : (aw_row < 0 ? -1 : 6 * M::NP + 3 * ca + aw_row);
    }
    const int ia = pva ? ca : M::imu_att(ca);
    const int ib = pva ? M::imu_acc(ca) : M::imu_rate(ca);
    T q[3] = {T(pva ? kQPos : kQAtt), T(pva ? kQVel : kQRate), T(pva ? kQAcc : 0.0)};
    T Rimu[6] = {T(pva ? kRPos : kRAtt), T(0), T(0), T(pva ? kRVel : kRRate), T(0), T(pva ? kRAcc : 1.0)};
    T Rgps = T(kRGps);
    if constexpr (CUSTOM) {
        const RefConsts* kc = a.kc;
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (xi[k] >= 0) {
                q[k] = T(ro(kc)->q[xi[k]]);
                Rimu[k == 0 ? 0 : k == 1 ? 3 : 5] = T(ro(kc)->r_imu[xi[k]]);
            }
        if (pva) Rgps = T(ro(kc)->r_gps[ca]);
    }
    const T* hx = static_cast<const T*>(a.x);
    const T* hP = static_cast<const T*>(a.P);
    T x[1][3], P[6];
#pragma unroll
    for (int k = 0; k < 3; ++k) x[0][k] = xi[k] >= 0 ? hx[xi[k]] : T(0);
#pragma unroll
    for (int k = 0; k < 6; ++k) P[k] = pr[k] >= 0 ? hP[pr[k]] : T(k == 0 || k == 3 || k == 5 ? 1 : 0);
    int32_t st = a.status[0];
    GateBand<T> gate;
    gate.init(a.threshold);
    const T thr = T(a.threshold);
    const T* pay = static_cast<const T*>(a.payload);
    const bool cov = a.cov != nullptr, ldo = a.logdet != nullptr;
    const int T_ = a.T;
    // an event step's records (t wave-uniform): slot 0's lanes write, through buffer stores whose
    // offsets drop the other slots' and the absent rows' stores (the chain kernel's form)
    constexpr uint32_t rb = uint32_t(sizeof(T));
    const uint32_t v_tr0 = slot == 0 && xi[0] >= 0 && xi[0] < M::NTRAJ ? uint32_t(xi[0]) * rb : kDropOffset;
    uint32_t vp0[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) vp0[k] = slot == 0 && pr[k] >= 0 ? uint32_t(pr[k]) * rb : kDropOffset;
    const uint32_t v_ld0 = slot == 0 && c == 0 ? 0u : kDropOffset;
    auto record_step = [&](int t, bool applied) {
        stv(span_rsrc(a.traj, int64_t(t) * M::NTRAJ, rb, M::NTRAJ), v_tr0, x[0][0]);
        if (cov) {
            const auto rc = span_rsrc(a.cov, int64_t(t) * M::NBLK, rb, M::NBLK);
#pragma unroll
            for (int k = 0; k < 6; ++k) stv(rc, vp0[k], P[k]);
        }
        if (ldo) {
            const T ld = group_sum(live ? chain_log_det(P) : T(0));
            st = (ld == ld) ? st : kNotSpd;
            stv(span_rsrc(a.logdet, t, rb, 1), v_ld0, ld);
        }
        if (slot == 0 && c == 0 && a.updated) a.updated[t] = applied ? 1 : 0;
    };
    // a look-ahead run's records (events t0 + slot for the slots < n; t0 wave-uniform): one
    // descriptor over the run's rows, each slot's lanes at their row, the other stores dropped
    const uint32_t v_trr = xi[0] >= 0 && xi[0] < M::NTRAJ ? uint32_t(slot * M::NTRAJ + xi[0]) * rb : kDropOffset;
    uint32_t vpr[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) vpr[k] = pr[k] >= 0 ? uint32_t(slot * M::NBLK + pr[k]) * rb : kDropOffset;
    const uint32_t v_ldr = c == 0 ? uint32_t(slot) * rb : kDropOffset;
    auto record_run = [&](int t0, int n, const T (&xr)[3], const T (&Pr)[6]) {
        const uint32_t wm = slot < n ? 0u : kDropOffset;
        const uint32_t rows = uint32_t(T_ - t0 < 8 ? T_ - t0 : 8);
        stv(span_rsrc(a.traj, int64_t(t0) * M::NTRAJ, rb, rows * M::NTRAJ), v_trr | wm, xr[0]);
        if (cov) {
            const auto rc = span_rsrc(a.cov, int64_t(t0) * M::NBLK, rb, rows * M::NBLK);
#pragma unroll
            for (int k = 0; k < 6; ++k) stv(rc, vpr[k] | wm, Pr[k]);
        }
        if (ldo) {
            const T ld = group_sum(live ? chain_log_det(Pr) : T(0));
            st = (ld == ld || slot >= n) ? st : kNotSpd;
            stv(span_rsrc(a.logdet, t0, rb, rows), v_ldr | wm, ld);
        }
        if (slot < n && c == 0 && a.updated) a.updated[t0 + slot] = 0;
    };
    int t = 0;
    // a look-ahead after an event that did not update, unless the last one found its run over at
    // once (then only after `cool` more such events: a regime of frequent updates stays on the
    // chain kernel's event step)
    int cool = 0, backoff = 0;
    // event t's inputs, loaded one event ahead (t + 1 while t runs; a look-ahead that moves t
    // reloads)
    int nt = 0;
    int ntype = T_ > 0 ? int(a.etype[0]) : 255;
    double ndt = T_ > 0 ? a.dt[0] : 0.0;
    T nva = T_ > 0 ? pay[ia] : T(0), nvb = T_ > 0 ? pay[ib] : T(0);
    while (t < T_) {  // wave-uniform
        // ---- event t as the chain kernel runs it (every slot the same arithmetic) ----
        if (nt != t) {
            ntype = int(a.etype[t]);
            ndt = a.dt[t];
            nva = pay[int64_t(t) * 9 + ia];
            nvb = pay[int64_t(t) * 9 + ib];
        }
        const int type = ntype;
        const T dt = T(ndt);
        const T va = nva, vb = nvb;
        nt = t + 1;
        if (nt < T_) {
            ntype = int(a.etype[nt]);
            ndt = a.dt[nt];
            nva = pay[int64_t(nt) * 9 + ia];
            nvb = pay[int64_t(nt) * 9 + ib];
        }
        bool applied = false;
        if (type != 255) {
            const T c02 = pva ? T(0.5) * dt * dt : T(0);
            const T c12 = pva ? dt : T(0);
            {
                const T xn0 = fmaT(c02, x[0][2], fmaT(dt, x[0][1], x[0][0]));
                const T xn1 = fmaT(c12, x[0][2], x[0][1]);
                x[0][0] = xn0;
                x[0][1] = xn1;
            }
            T FP[3][3];
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                FP[0][j] = fmaT(c02, P[tri<3>(2, j)], fmaT(dt, P[tri<3>(1, j)], P[tri<3>(0, j)]));
                FP[1][j] = fmaT(c12, P[tri<3>(2, j)], P[tri<3>(1, j)]);
                FP[2][j] = P[tri<3>(2, j)];
            }
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = i; j < 3; ++j) {
                    T s = FP[i][j];
                    if (j == 0) s = fmaT(FP[i][2], c02, fmaT(FP[i][1], dt, s));
                    if (j == 1) s = fmaT(FP[i][2], c12, s);
                    P[tri<3>(i, j)] = (i == j) ? s + q[i] * dt : s;
                }
            applied = (type == kGps || type == kImu);
            if (applied) applied = gate.open(P, live, thr);
            bool ok = true;
            if (applied) {
                if (type == kGps) {
                    if (pva) {
                        T zb[1][1] = {{va}};
                        const T R[1] = {Rgps};
                        ok = sel_update_nv<3, 1, true, T, kRefNewton, true, 1, kRefJoseph<T>, kRefGainR>(x, P, zb, R);
                    }
                } else {
                    const T V = fmaT(vb, dt, x[0][1]);
                    const T X = fmaT(V, dt, x[0][0]);
                    T zb[1][3] = {{pva ? X : va, pva ? V : vb, pva ? vb : T(0)}};
                    ok = sel_update_nv<3, 3, true, T, kRefNewton, true, 1, kRefJoseph<T>, kRefGainR>(x, P, zb, Rimu);
                    if (!pva) {
                        x[0][2] = T(0);
                        P[5] = T(1);
                    }
                }
            }
            if (group_any(!ok)) {
                st = kNotSpd;
#pragma unroll
                for (int k = 0; k < 3; ++k) x[0][k] = quiet_nan<T>();
#pragma unroll
                for (int k = 0; k < 6; ++k) P[k] = quiet_nan<T>();
            }
        }
        record_step(t, applied);
        ++t;
        // every lane holds the same decision (the gate's group ops, every slot the same event), but
        // the compiler cannot know it: taken from lane 0, so that t and the loop stay scalar (a
        // per-lane `continue` made t divergent, and with it every event's type branches)
        if (__builtin_amdgcn_readfirstlane(int(applied)) || t >= T_) continue;
        if (cool > 0) {
            --cool;
            continue;
        }
        for (;;) {  // look-aheads until a run ends (or the stream does)
        // ---- look-ahead: slot j predicts to event t + j in closed form ----
        const int e = t + slot;
        const bool valid = e < T_;
        const int ty = valid ? int(a.etype[e]) : 255;
        const bool pred = valid && ty != 255;
        const T dte = pred ? T(a.dt[e]) : T(0);
        // tau: time since event t - 1 up to and including slot j's event (prefix over slots)
        T tau = dte;
#pragma unroll
        for (int o = 1; o < 8; o *= 2) {
            const T u = __shfl_up(tau, o * kGroup, 64);
            tau += slot >= o ? u : T(0);
        }
        // this slot's term F(-tau) Q(dt) F(-tau)^T (G = F(-tau): rows (1, -tau, h'), (0, 1, g'), (0, 0, 1))
        const T hm = pva ? T(0.5) * tau * tau : T(0), gm = pva ? -tau : T(0);
        const T d0 = q[0] * dte, d1 = q[1] * dte, d2 = q[2] * dte;
        T Sx[6];
        Sx[0] = fmaT(hm * hm, d2, fmaT(tau * tau, d1, d0));
        Sx[1] = fmaT(hm * gm, d2, -tau * d1);
        Sx[2] = hm * d2;
        Sx[3] = fmaT(gm * gm, d2, d1);
        Sx[4] = gm * d2;
        Sx[5] = d2;
#pragma unroll
        for (int o = 1; o < 8; o *= 2)
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const T u = __shfl_up(Sx[k], o * kGroup, 64);
                Sx[k] += slot >= o ? u : T(0);
            }
        // P_pred = F(tau) (P + S) F(tau)^T, F = [[1, tau, h], [0, 1, g], [0, 0, 1]]
        const T h = pva ? T(0.5) * tau * tau : T(0), g = pva ? tau : T(0);
        T A[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) A[k] = P[k] + Sx[k];
        T B[3][3];  // F A
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            B[0][j] = fmaT(h, A[tri<3>(2, j)], fmaT(tau, A[tri<3>(1, j)], A[tri<3>(0, j)]));
            B[1][j] = fmaT(g, A[tri<3>(2, j)], A[tri<3>(1, j)]);
            B[2][j] = A[tri<3>(2, j)];
        }
        T Pp[6];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = i; j < 3; ++j) {
                T s = B[i][j];
                if (j == 0) s = fmaT(B[i][2], h, fmaT(B[i][1], tau, s));
                if (j == 1) s = fmaT(B[i][2], g, s);
                Pp[tri<3>(i, j)] = s;
            }
        if (!pva) Pp[5] = P[5];  // the inert state of an aw lane
        T xp[3] = {fmaT(h, x[0][2], fmaT(tau, x[0][1], x[0][0])), fmaT(g, x[0][2], x[0][1]), x[0][2]};
        const bool opens = valid && (ty == kGps || ty == kImu) && gate.open(Pp, live, thr);
        const uint64_t om = __builtin_amdgcn_ballot_w64(opens && c == 0);
        const int nvalid = T_ - t < 8 ? T_ - t : 8;
        const int n = om ? int(__builtin_ctzll(om)) / kGroup : nvalid;  // events of the predict run
        record_run(t, n, xp, Pp);
        st = __builtin_amdgcn_ballot_w64(st == kNotSpd) ? kNotSpd : st;  // a failed record in any slot
        if (n > 0) {
            const int src = (n - 1) * kGroup + c;
#pragma unroll
            for (int k = 0; k < 3; ++k) x[0][k] = __shfl(xp[k], src, 64);
#pragma unroll
            for (int k = 0; k < 6; ++k) P[k] = __shfl(Pp[k], src, 64);
            t += n;
        }
        if (n < 4 && om) {  // a short run: look-aheads do not pay here, back off
            backoff = backoff ? (backoff < 32 ? 2 * backoff : 32) : 1;
            cool = backoff;
        } else if (n >= 4) {
            backoff = 0;
        }
        if (om || n < 8 || t >= T_) break;  // the run ended (its opening event runs next) or the stream did
        }
    }
    if (slot == 0) {
        T* ox = static_cast<T*>(a.x);
        T* oP = static_cast<T*>(a.P);
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (xi[k] >= 0) ox[xi[k]] = x[0][k];
#pragma unroll
        for (int k = 0; k < 6; ++k)
            if (pr[k] >= 0) oP[pr[k]] = P[k];
        if (c == 0) a.status[0] = st;
    }
}

// ------------------------------------------------------------------------------------
// Time-parallel run of ONE filter over a long event stream (kf_run_stream; the reference's own
// use of run_kalman_filter_full, kf_workers.py:623-728, is one filter over a whole drive log).
// The stream is cut into C chunks of L events that run as filters of the chain kernel:
//  * the covariance recursion does not depend on the measurements and forgets its start, so
//    chunk c's start covariance is the handle's P carried over the chunks before it by their
//    linear-fractional covariance maps (phases 6-7; or an event warm-up over the W events before
//    it, the warm-up bank);
//  * given the gains, the state recursion is affine (the IMU pseudo-measurement is built from
//    the predicted state, kf_workers.py:698-706, which keeps it affine), and block-diagonal
//    over the axis chains: the map pass runs each chunk from a guess and from three perturbed
//    guesses (one per chain component; the four variants share one lane and one covariance),
//    its epilogue giving x_end = A x_start + b per chunk and chain;
//  * the maps are composed from the handle's state by a parallel scan (phases 2-4) into every
//    chunk's true start; the records are the map pass's, the trajectory evaluated at the true
//    starts (phase 8), or a final pass runs the chunks from them (KF_OPT_STREAM_FINAL = 1);
//  * checks: each chunk's start covariance equals the previous chunk's end covariance, the
//    starts and the end state are finite (a final pass: each chunk's end state is its
//    successor's start), no chunk filter failed.  Only then does the handle take the end
//    state; otherwise the sequential chain kernel, launched after these with skip = &check.ok,
//    runs the stream as one filter and rewrites every record.
// ------------------------------------------------------------------------------------
template <class M>
__device__ __forceinline__ int chain_state(int a, int q) {  // chain a (pva chains first), component q; -1: none
    return a < M::NP ? M::pva(a, q) : (q < 2 ? M::aw(a - M::NP, q) : -1);
}
template <class M>
__device__ __forceinline__ int chain_row0(int a) {  // first block-packed covariance row of chain a
    return a < M::NP ? 6 * a : 6 * M::NP + 3 * (a - M::NP);
}
template <class M>
__device__ __forceinline__ int state_component(int i) {  // component of state i within its chain
    int comp = 0;
#pragma unroll
    for (int a = 0; a < M::NP + M::NA; ++a)
#pragma unroll
        for (int q = 0; q < 3; ++q)
            if (chain_state<M>(a, q) == i) comp = q;
    return comp;
}

// phase 0: every chunk of the warm-up bank starts from the handle's state; check zeroed
template <typename T, class M>
__global__ __launch_bounds__(kBlock) void stream_init_kernel(const StreamArgs a) {
    const int64_t c = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (c == 0) {
        a.check->ok = 0;
        a.check->bad = 0;
        a.check->cov_gap = 0.0;
        a.check->state_gap = 0.0;
        a.check->done = 0;
        a.check->skip_chain = 0;
    }
    if (c >= a.C) return;
    const T* hx = static_cast<const T*>(a.hx);
    const T* hP = static_cast<const T*>(a.hP);
#pragma unroll
    for (int i = 0; i < M::N; ++i) static_cast<T*>(a.wx)[i * a.C + c] = hx[i];
#pragma unroll
    for (int r = 0; r < M::NBLK; ++r) static_cast<T*>(a.wP)[r * a.C + c] = hP[r];
    a.wst[c] = a.hstatus[0];
}

// phase 1: map bank filter q * C + c = chunk c from its warm-up state, + delta on component q - 1
// of every chain (q = 0: the guess itself)
template <typename T, class M>
__global__ __launch_bounds__(kBlock) void stream_perturb_kernel(const StreamArgs a) {
    const int64_t f = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    const int64_t B = 4 * a.C;
    if (f >= B) return;
    const int q = int(f / a.C);
    const int64_t c = f % a.C;
#pragma unroll
    for (int i = 0; i < M::N; ++i) {
        const T g = static_cast<const T*>(a.wx)[i * a.C + c];
        static_cast<T*>(a.mx)[i * B + f] = (q > 0 && state_component<M>(i) == q - 1) ? g + T(a.delta) : g;
    }
#pragma unroll
    for (int r = 0; r < M::NBLK; ++r) static_cast<T*>(a.mP)[r * B + f] = static_cast<const T*>(a.wP)[r * a.C + c];
    a.mst[f] = a.wst[c];
}

template <class M>
__device__ __forceinline__ void compose_into(double (&A)[3][3], double (&b)[3], const double* m) {
    // (A, b) <- m o (A, b): A = Am A, b = Am b + bm
    double An[3][3], bn[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double t = m[9 + k];
#pragma unroll
        for (int q = 0; q < 3; ++q) t = __builtin_fma(m[k * 3 + q], b[q], t);
        bn[k] = t;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double u = 0.0;
#pragma unroll
            for (int q = 0; q < 3; ++q) u = __builtin_fma(m[k * 3 + q], A[q][j], u);
            An[k][j] = u;
        }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        b[k] = bn[k];
#pragma unroll
        for (int j = 0; j < 3; ++j) A[k][j] = An[k][j];
    }
}
__device__ __forceinline__ void apply_map(double (&x)[3], const double* m) {
    double xn[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double t = m[9 + k];
#pragma unroll
        for (int q = 0; q < 3; ++q) t = __builtin_fma(m[k * 3 + q], x[q], t);
        xn[k] = t;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) x[k] = xn[k];
}

// phases 2-4: the chunk maps (written by the map pass's epilogue) composed into every chunk's
// true start, as a three-kernel parallel scan per chain (a dependent walk over the maps waits
// ~1 us per map load):
//   2  tiles of kScanTile chunks: thread c loads chunk c's map, a Kogge-Stone scan in LDS gives
//      its exclusive in-tile prefix E_c (stored) and the tile's product (stored);
//   3  one block per chain: the same scan over the tile products (rounds of kScanTile tiles with a
//      carry) applied to the handle's state gives every tile's start, and the stream's end state;
//   4  thread per (chunk, chain): start = E_c(tile start), stored (before a final pass also the
//      final bank's state, covariance and status) and checked finite.  The last block to finish
//      (a counter; release / acquire fences) gives the verdict when the records come from the map
//      pass (a.xend): no failed chunk filter, finite starts and end state, covariance seams within
//      tolerance; a passed run leaves the end state and the last chunk's end covariance in the
//      handle.  No state seam is measured there (the starts are the maps' values, not runs from
//      them; KF_OPT_STREAM_FINAL = 1 runs them and checks the seams in phase 5).
constexpr int kScanTile = 256;
__device__ __forceinline__ void affine_compose(double (&o)[12], const double (&l)[12], const double (&e)[12]) {
    // o = l o e: A = A_l A_e, b = A_l b_e + b_l
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double t = l[9 + k];
#pragma unroll
        for (int q = 0; q < 3; ++q) t = __builtin_fma(l[k * 3 + q], e[9 + q], t);
        o[9 + k] = t;
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double u = 0.0;
#pragma unroll
            for (int q = 0; q < 3; ++q) u = __builtin_fma(l[k * 3 + q], e[q * 3 + j], u);
            o[k * 3 + j] = u;
        }
    }
}

__device__ __forceinline__ void affine_identity(double (&m)[12]) {
#pragma unroll
    for (int e = 0; e < 12; ++e) m[e] = (e == 0 || e == 4 || e == 8) ? 1.0 : 0.0;
}

// Inclusive Kogge-Stone scan of one affine map per thread over the block (LDS, struct of
// arrays): v <- v_t o ... o v_0.  The caller syncs before reusing `pre`.
__device__ __forceinline__ void block_scan_affine(double (&v)[12], double (*pre)[kScanTile], int tid) {
#pragma unroll
    for (int e = 0; e < 12; ++e) pre[e][tid] = v[e];
    __syncthreads();
    for (int d = 1; d < kScanTile; d <<= 1) {
        double earlier[12];
        const bool has = tid >= d;
        if (has) {
#pragma unroll
            for (int e = 0; e < 12; ++e) earlier[e] = pre[e][tid - d];
        }
        __syncthreads();
        if (has) {
            double o[12];
            affine_compose(o, v, earlier);
#pragma unroll
            for (int e = 0; e < 12; ++e) {
                v[e] = o[e];
                pre[e][tid] = o[e];
            }
        }
        __syncthreads();
    }
}

// phase 2: grid (tiles, chains)
template <typename T, class M>
__global__ __launch_bounds__(kScanTile) void stream_scan_tiles_kernel(const StreamArgs a) {
    constexpr int NCH = M::NP + M::NA;
    __shared__ double pre[12][kScanTile];
    const int tid = int(threadIdx.x);
    const int ch = int(blockIdx.y);
    const int64_t tile = blockIdx.x, c = tile * kScanTile + tid;
    double v[12];
    if (c < a.C) {
#pragma unroll
        for (int e = 0; e < 12; ++e) v[e] = a.maps[(c * NCH + ch) * 12 + e];
    } else {
        affine_identity(v);
    }
    block_scan_affine(v, pre, tid);
    if (c < a.C) {
        double* o = a.pref + (c * NCH + ch) * 12;
        if (tid == 0) {
            double id[12];
            affine_identity(id);
#pragma unroll
            for (int e = 0; e < 12; ++e) o[e] = id[e];
        } else {
#pragma unroll
            for (int e = 0; e < 12; ++e) o[e] = pre[e][tid - 1];
        }
    }
    if (tid == kScanTile - 1) {
        double* o = a.tiles + (tile * NCH + ch) * 12;
#pragma unroll
        for (int e = 0; e < 12; ++e) o[e] = v[e];
    }
}

// phase 3 (only when there are more tiles than one scan round holds): grid (1, chains).  The
// scan's top phase as a launch of its own: rounds of kScanTile tile products, each scanned and
// applied to the carried state, give every tile's start state in a.tstart.  Below that size
// the starts kernel composes its own prefix (one round per block, no launch).
template <typename T, class M>
__global__ __launch_bounds__(kScanTile) void stream_top_kernel(const StreamArgs a) {
    constexpr int NCH = M::NP + M::NA;
    __shared__ double pre[12][kScanTile];
    __shared__ double carry[3];
    const int tid = int(threadIdx.x);
    const int ch = int(blockIdx.y);
    const int ns = ch < M::NP ? 3 : 2;
    const int64_t ntiles = (a.C + kScanTile - 1) / kScanTile;
    if (tid < 3) carry[tid] = tid < ns ? double(static_cast<const T*>(a.hx)[chain_state<M>(ch, tid)]) : 0.0;
    for (int64_t r0 = 0; r0 < ntiles; r0 += kScanTile) {
        const int64_t t = r0 + tid;
        double v[12];
        if (t < ntiles) {
#pragma unroll
            for (int e = 0; e < 12; ++e) v[e] = a.tiles[(t * NCH + ch) * 12 + e];
        } else {
            affine_identity(v);
        }
        __syncthreads();  // carry written (the previous round / the init), pre free
        block_scan_affine(v, pre, tid);
        if (t < ntiles) {  // tile t's start: the round's carry through the tiles before t
            double x[3] = {carry[0], carry[1], carry[2]};
            if (tid > 0) {
                double e1[12];
#pragma unroll
                for (int e = 0; e < 12; ++e) e1[e] = pre[e][tid - 1];
                apply_map(x, e1);
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) a.tstart[(t * NCH + ch) * 3 + k] = x[k];
        }
        __syncthreads();  // every thread has read carry and pre
        if (tid == kScanTile - 1) {  // the round's product (identity maps past the last tile)
            double xe[3] = {carry[0], carry[1], carry[2]};
            apply_map(xe, v);
#pragma unroll
            for (int k = 0; k < 3; ++k) carry[k] = xe[k];
        }
    }
}

// phase 4: grid (tiles, chains).  Each block first composes the products of the tiles before
// its own into its tile start — at most one round of kScanTile tiles; with more tiles the top
// kernel (phase 3) has written every tile start to a.tstart, since redoing the prefix per block
// would cost O(ntiles^2) — and the block of the last tile also runs through its own
// product: the stream's end state.
template <typename T, class M>
__global__ __launch_bounds__(kScanTile) void stream_starts_kernel(const StreamArgs a) {
    constexpr int NCH = M::NP + M::NA;
    __shared__ double pre[12][kScanTile];
    __shared__ double carry[3];
    const int tid = int(threadIdx.x);
    const int ch = int(blockIdx.y);
    const int ns = ch < M::NP ? 3 : 2;
    const int64_t tile = blockIdx.x, c = tile * kScanTile + tid;
    const int64_t ntiles = gridDim.x;
    if (a.tstart) {
        if (tid < 3) carry[tid] = tid < ns ? a.tstart[(tile * NCH + ch) * 3 + tid] : 0.0;
    } else if (tid < 3) {
        carry[tid] = tid < ns ? double(static_cast<const T*>(a.hx)[chain_state<M>(ch, tid)]) : 0.0;
    }
    for (int64_t r0 = 0; !a.tstart && r0 < tile; r0 += kScanTile) {
        const int64_t t = r0 + tid;
        double v[12];
        if (t < tile) {
#pragma unroll
            for (int e = 0; e < 12; ++e) v[e] = a.tiles[(t * NCH + ch) * 12 + e];
        } else {
            affine_identity(v);
        }
        __syncthreads();  // carry written (the previous round / the init), pre free
        block_scan_affine(v, pre, tid);
        if (tid == kScanTile - 1) {  // the round's product (identity maps past `tile`)
            double xe[3] = {carry[0], carry[1], carry[2]};
            apply_map(xe, v);
#pragma unroll
            for (int k = 0; k < 3; ++k) carry[k] = xe[k];
        }
    }
    __syncthreads();
    bool fin = true;
    if (a.xend && tile == ntiles - 1 && tid == 0) {  // the stream's end state
        double xe[3] = {carry[0], carry[1], carry[2]}, tp[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) tp[e] = a.tiles[(tile * NCH + ch) * 12 + e];
        apply_map(xe, tp);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k >= ns) continue;
            // read by the verdict's block (maybe on another XCD): a device-scope atomic
            atomicExch(reinterpret_cast<unsigned long long*>(&a.xend[chain_state<M>(ch, k)]),
                       static_cast<unsigned long long>(__double_as_longlong(xe[k])));
            fin = fin && (xe[k] - xe[k] == 0.0);
        }
    }
    if (c < a.C) {
        double x[3] = {carry[0], carry[1], carry[2]}, e1[12];
#pragma unroll
        for (int e = 0; e < 12; ++e) e1[e] = a.pref[(c * NCH + ch) * 12 + e];
        apply_map(x, e1);
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            if (k >= ns) continue;
            const int i = chain_state<M>(ch, k);
            a.starts[i * a.C + c] = x[k];
            // the records' offsets, start - guess, in the records kernel's own arithmetic
            if (a.dtab) a.dtab[(c * NCH + ch) * 4 + k] = x[k] - double(static_cast<const T*>(a.wx)[i * a.C + c]);
            fin = fin && (x[k] - x[k] == 0.0);  // NaN or inf fails
            if (!a.xend) static_cast<T*>(a.fx)[i * a.C + c] = T(x[k]);
        }
        if (!a.xend) {  // the final bank: the warm-up covariance, status 0
            const int r0 = chain_row0<M>(ch), nr = ns == 3 ? 6 : 3;
            for (int r = r0; r < r0 + nr; ++r)
                static_cast<T*>(a.fP)[r * a.C + c] = static_cast<const T*>(a.wP)[r * a.C + c];
            if (ch == 0) a.fst[c] = 0;
        }
    }
    const bool all_fin = __syncthreads_and(fin ? 1 : 0) != 0;
    if (tid != 0) return;
    StreamCheck* k = a.check;
    if (!all_fin) atomicOr(&k->bad, kStreamBadStart);
    if (!a.xend) return;  // a final pass follows: phase 5 decides
    // Everything the verdict reads from this launch travels by device-scope atomics (bad here,
    // cov_gap and bad from the map pass and the end state from earlier launches), so no fence:
    // the wave only drains its own atomic before it counts itself (an agent-scope release per
    // block wrote its XCD's L2 back and cost more than the kernel's work).  The empty asm with a
    // memory clobber keeps the compiler from moving the bad update past the count (s_waitcnt
    // alone is not a compiler barrier); the wait then drains it in the hardware.
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0);
    const int blocks = int(gridDim.x * gridDim.y);
    if (atomicAdd(&k->done, 1) != blocks - 1) return;
    asm volatile("" ::: "memory");  // the verdict's reads stay after the count
    const int bad = atomicOr(&k->bad, 0);
    const double cov_gap = __longlong_as_double(atomicOr(reinterpret_cast<unsigned long long*>(&k->cov_gap), 0ull));
    const bool ok = bad == 0 && cov_gap <= a.tol_cov;
    // every read issued before the first store: a read after a store that may alias it waits
    // for the store, which made the 42 reads below round trips one after another
    const int64_t col = a.C - 1, B4 = 4 * a.C;  // the last chunk's end covariance
    double xv[M::N];
    T pv[M::NBLK];
    if (ok) {
#pragma unroll
        for (int i = 0; i < M::N; ++i)  // written by the last tile's block (a device-scope atomic)
            xv[i] = __longlong_as_double(
                static_cast<long long>(atomicOr(reinterpret_cast<unsigned long long*>(&a.xend[i]), 0ull)));
#pragma unroll
        for (int r = 0; r < M::NBLK; ++r) pv[r] = static_cast<const T*>(a.mP)[r * B4 + col];
    }
    k->state_gap = bad & kStreamBadStart ? __builtin_inf() : __builtin_nan("");
    k->ok = ok ? 1 : 0;
    if (ok) {
#pragma unroll
        for (int i = 0; i < M::N; ++i) static_cast<T*>(a.hx)[i] = T(xv[i]);
#pragma unroll
        for (int r = 0; r < M::NBLK; ++r) static_cast<T*>(a.hP)[r] = pv[r];
        a.hstatus[0] = 0;
    }
}

// phase 8 (records from the map pass): thread per (event, trajectory entry i); entry i (the
// first component of its chain) = variant 0's + sum_q A_q (start - guess)_q with A_q =
// (variant q+1 - variant 0) / delta, as the chunk maps
template <typename T, class M>
__global__ __launch_bounds__(kBlock) void stream_records_kernel(const StreamArgs a) {
    constexpr int NCH = M::NP + M::NA;
    const int64_t g = int64_t(blockIdx.x) * kBlock + threadIdx.x;  // e * NTRAJ + i: coalesced rows
    if (g >= a.S * M::NTRAJ) return;
    // 32-bit divisions (S * NTRAJ < 2^31: kf_run_stream's offsets are 32-bit)
    const uint32_t e = uint32_t(g) / uint32_t(M::NTRAJ);
    const int i = int(uint32_t(g) - e * uint32_t(M::NTRAJ));
    const int64_t c = e / uint32_t(a.L);
    const T* t4 = static_cast<const T*>(a.traj4);
    const T* wx = static_cast<const T*>(a.wx);
    int ch = 0;  // the chain whose first component is state i (the trajectory holds those)
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc)
        if (chain_state<M>(cc, 0) == i) ch = cc;
    const int ns = ch < M::NP ? 3 : 2;
    const double x0 = double(t4[g]);
    double acc = x0;
    // start - guess of the chain's components: the starts kernel's table (two loads shared by
    // the chunk's threads), or the starts and guess rows themselves
    double d[3];
    if (a.dtab) {
        const double* dt = a.dtab + (c * NCH + ch) * 4;
        const double2 d01 = *reinterpret_cast<const double2*>(dt);
        d[0] = d01.x;
        d[1] = d01.y;
        d[2] = ns == 3 ? dt[2] : 0.0;
    } else {
#pragma unroll
        for (int qq = 0; qq < 3; ++qq) {
            const int idx = chain_state<M>(ch, qq);
            d[qq] = qq < ns ? a.starts[idx * a.C + c] - double(wx[idx * a.C + c]) : 0.0;
        }
    }
#pragma unroll
    for (int qq = 0; qq < 3; ++qq) {
        if (qq >= ns) continue;
        const double xq = double(t4[(qq + 1) * a.vstride * M::NTRAJ + g]);
        acc = __builtin_fma((xq - x0) * a.rdelta, d[qq], acc);  // delta is a power of two: exact
    }
    static_cast<T*>(a.traj)[g] = T(acc);
}

// The same records two entries per thread (an even NTRAJ: entries 2j, 2j + 1 of one event):
// one 2-wide load per variant row and one 2-wide store instead of two each, the start offsets
// from the starts kernel's table.  Each entry's arithmetic is stream_records_kernel's.
template <typename T, class M>
__global__ __launch_bounds__(kBlock) void stream_records2_kernel(const StreamArgs a) {
    static_assert(M::NTRAJ % 2 == 0, "pairs of one event's entries");
    typedef T T2 __attribute__((ext_vector_type(2)));
    constexpr int NCH = M::NP + M::NA;
    const int64_t p = int64_t(blockIdx.x) * kBlock + threadIdx.x;  // pair: entries 2p, 2p + 1
    if (p >= a.S * (M::NTRAJ / 2)) return;
    const uint32_t e = uint32_t(p) / uint32_t(M::NTRAJ / 2);
    const int i0 = 2 * int(uint32_t(p) - e * uint32_t(M::NTRAJ / 2));
    const int64_t c = e / uint32_t(a.L);
    const T2* t4 = static_cast<const T2*>(a.traj4);
    int ch[2] = {0, 0};
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
        if (chain_state<M>(cc, 0) == i0) ch[0] = cc;
        if (chain_state<M>(cc, 0) == i0 + 1) ch[1] = cc;
    }
    double d[2][3];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const double* dt = a.dtab + (c * NCH + ch[h]) * 4;
        const double2 d01 = *reinterpret_cast<const double2*>(dt);
        d[h][0] = d01.x;
        d[h][1] = d01.y;
        d[h][2] = ch[h] < M::NP ? dt[2] : 0.0;
    }
    const T2 v0 = t4[p];
    const double x0[2] = {double(v0.x), double(v0.y)};
    double acc[2] = {x0[0], x0[1]};
    const bool any3 = ch[0] < M::NP || ch[1] < M::NP;  // a third variant row is needed
#pragma unroll
    for (int qq = 0; qq < 3; ++qq) {
        if (qq == 2 && !any3) continue;
        const T2 vq = t4[(qq + 1) * a.vstride * (M::NTRAJ / 2) + p];
        const double xq[2] = {double(vq.x), double(vq.y)};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ns = ch[h] < M::NP ? 3 : 2;
            if (qq < ns) acc[h] = __builtin_fma((xq[h] - x0[h]) * a.rdelta, d[h][qq], acc[h]);
        }
    }
    T2 out;
    out.x = T(acc[0]);
    out.y = T(acc[1]);
    static_cast<T2*>(a.traj)[p] = out;
}

// ------------------------------------------------------------------------------------
// Covariance warm-up by linear-fractional maps (kf_run_stream's default).  Per axis chain the
// covariance recursion is P <- (A P + B)(C P + D)^-1 with, per event,
//   predict  [[F, Q F^-T], [0, F^-T]]      (F P F^T + Q with P = X Y^-1)
//   update   [[I, 0], [H^T R^-1 H, I]]     ((P^-1 + H^T R^-1 H)^-1, the Joseph form's value)
// so a chunk's covariance map is the 6x6 product of its events' matrices (an (att, rate)
// chain carries the chain kernel's inert third state as an identity row and column).  The
// chunk starts are then the fixed point of P(c) = map_(c-1)(P(c-1)) from P(0) = the handle's
// P, reached by parallel iterations: the recursion forgets its start (each chunk of the
// reference's 200 Hz IMU stream contracts an error by ~1e-3), so a few iterations over all
// chunks at once replace the W-event warm-up; the device seam check still decides.
// ------------------------------------------------------------------------------------
template <class M, bool CUSTOM>
__device__ __forceinline__ void chain_noise(int ch, double (&q)[3], double (&si_imu)[3], double& si_gps,
                                            const RefConsts* kc) {
    const bool pva = ch < M::NP;
    if constexpr (CUSTOM) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const int i = chain_state<M>(ch, k);
            q[k] = i >= 0 ? ro(kc)->q[i] : 0.0;
            si_imu[k] = i >= 0 ? 1.0 / ro(kc)->r_imu[i] : 0.0;
        }
        si_gps = pva ? 1.0 / ro(kc)->r_gps[ch] : 0.0;
        return;
    }
    q[0] = pva ? kQPos : kQAtt;
    q[1] = pva ? kQVel : kQRate;
    q[2] = pva ? kQAcc : 0.0;
    si_imu[0] = 1.0 / (pva ? kRPos : kRAtt);
    si_imu[1] = 1.0 / (pva ? kRVel : kRRate);
    si_imu[2] = pva ? 1.0 / kRAcc : 0.0;
    si_gps = pva ? 1.0 / kRGps : 0.0;
}

// phase 6: the product of each chunk piece's event matrices per chain, one lane per (piece,
// chain) holding the 6x6 product (an event acts on its columns independently).  Rescaled by a
// power of two (the product's max) every 16 events, which a linear-fractional map ignores.
// Event types and dt are loaded 8 events at a time, one batch ahead.
template <class M>
__device__ __forceinline__ void lft_event(double (&v)[6], int type, double dt, bool pva, const double (&q)[3],
                                          const double (&si)[3], double sg) {
    if (type == 255) return;
    const double c02 = pva ? 0.5 * dt * dt : 0.0, c12 = pva ? dt : 0.0;
    const double g20 = dt * c12 - c02;
    // bottom <- F^-T bottom; top <- F top + Q dt (new bottom)
    const double b0 = v[3], b1 = __builtin_fma(-dt, v[3], v[4]);
    const double b2 = __builtin_fma(g20, v[3], __builtin_fma(-c12, v[4], v[5]));
    const double t0 = __builtin_fma(c02, v[2], __builtin_fma(dt, v[1], v[0]));
    const double t1 = __builtin_fma(c12, v[2], v[1]);
    v[0] = __builtin_fma(q[0] * dt, b0, t0);
    v[1] = __builtin_fma(q[1] * dt, b1, t1);
    v[2] = __builtin_fma(q[2] * dt, b2, v[2]);
    v[3] = b0;
    v[4] = b1;
    v[5] = b2;
    if (type == kGps || type == kImu) {  // bottom += H^T R^-1 H top
        const bool gps = type == kGps;
        v[3] = __builtin_fma(gps ? sg : si[0], v[0], v[3]);
        v[4] = __builtin_fma(gps ? 0.0 : si[1], v[1], v[4]);
        v[5] = __builtin_fma(gps ? 0.0 : si[2], v[2], v[5]);
    }
}

// kLftHalves lanes per (chunk piece, chain), each carrying 6 / kLftHalves columns of the 6x6
// product: the columns are independent, so the split multiplies the waves of this latency-bound
// pass (0.75 wave per SIMD at 8192 chunks with all six columns in one lane) at the cost of
// paying an event's type / dt handling in every lane.  Config 1 in-process, with the axis-
// symmetric maps: 1 / 2 / 3 / 6 lanes 0.208 / 0.200 / 0.195 / 0.196 ms per log
// (profiles/r04_pmc/cfg1_diag/ab_halves.log)
#ifndef KF_LFT_HALVES
#define KF_LFT_HALVES 3
#endif
constexpr int kLftHalves = KF_LFT_HALVES;
static_assert(6 % kLftHalves == 0, "columns per lane");
// lanes per product: a power of two for the max exchange (3 / 6 column lanes: one / two lanes
// duplicate the last column and store nothing)
constexpr int kLftStride = kLftHalves == 3 ? 4 : kLftHalves == 6 ? 8 : kLftHalves;
// a.sym: the maps of chains 0 (pva) and NP (aw) only, which stand for every chain
template <class M>
__host__ __device__ constexpr int lft_map_chains(bool sym) {
    return sym ? 1 + (M::NA > 0 ? 1 : 0) : M::NP + M::NA;
}
template <class M>
__device__ __forceinline__ int lft_map_chain(bool sym, int ch) {  // whose maps chain ch uses
    return sym ? (ch < M::NP ? 0 : M::NP) : ch;
}
template <typename T, class M, bool CUSTOM>
__global__ __launch_bounds__(kBlock) void stream_lft_maps_kernel(const StreamArgs a) {
    constexpr int NCH = M::NP + M::NA;
    constexpr int NJ = 6 / kLftHalves;  // columns per lane
    const int nmc = lft_map_chains<M>(a.sym != 0);
    const int64_t gl = int64_t(blockIdx.x) * kBlock + threadIdx.x;
    if (gl >= a.C * a.np * nmc * kLftStride) return;  // whole products (kLftStride divides the wave)
    const int64_t gm = gl / kLftStride;  // (chunk * np + piece) * nmc + map chain
    const int li = int(gl % kLftStride);
    const bool own = li < kLftHalves;
    const int j0 = (own ? li : kLftHalves - 1) * NJ;
    const int64_t cp = gm / nmc;  // chunk * np + piece
    const int cm = int(gm % nmc);
    const int ch = a.sym ? (cm == 0 ? 0 : M::NP) : cm;
    const int64_t grp = cp * NCH + ch;  // the map's slot
    const bool pva = ch < M::NP;
    double q[3], si[3], sg;
    chain_noise<M, CUSTOM>(ch, q, si, sg, a.kc);
    double v[NJ][6];  // v[j] = column j0 + j
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 6; ++i) v[j][i] = i == j0 + j ? 1.0 : 0.0;
    const int64_t c = cp / a.np, piece = cp % a.np;
    const int64_t cend = (c + 1) * a.L < a.S ? (c + 1) * a.L : a.S;
    const int64_t e0 = c * a.L + piece * a.lp, e1 = e0 + a.lp < cend ? e0 + a.lp : cend;
    // events in batches of 8, the next batch's type and dt loaded while this one computes.  The
    // loads are unconditional buffer loads (past the stream they return 0) and the batch's range
    // test is applied where the values are used: loads under a per-lane condition were branched
    // around, and the branches' join waited for every load in flight (vmcnt 0), the batch just
    // issued included
    constexpr int kB = 8;
    const auto r_et = bytes_rsrc(a.etype, uint32_t(a.S));
    const auto r_dt = bytes_rsrc(a.dt, uint32_t(a.S) * 8u);
    uint32_t tyn[kB];
    double dvn[kB];
    auto fetch = [&](int64_t e) {
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const uint32_t ue = uint32_t(e + k);
            tyn[k] = __builtin_amdgcn_raw_buffer_load_b8(r_et, ue, 0, 0);
            dvn[k] = ldv(r_dt, ue * 8u, 0.0);
        }
    };
    fetch(e0);
    for (int64_t e = e0; e < e1; e += kB) {
        uint32_t ty[kB];
        double dv[kB];
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            ty[k] = tyn[k];
            dv[k] = dvn[k];
        }
        fetch(e + kB);
#pragma unroll
        for (int k = 0; k < kB; ++k) {
            const bool in = e + k < e1;
            const int tk = in ? int(ty[k]) : 255;
            const double dk = in ? dv[k] : 0.0;
#pragma unroll
            for (int j = 0; j < NJ; ++j) lft_event<M>(v[j], tk, dk, pva, q, si, sg);
        }
        if (((e - e0) & 15) == kB) {  // every 16 events: rescale by a power of two (the max)
            // of all six columns: the lanes of one product exchange their maxima (adjacent lanes)
            double mx = 0.0;
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int i = 0; i < 6; ++i) mx = fmax(mx, fabs(v[j][i]));
#pragma unroll
            for (int sh = 1; sh < kLftStride; sh <<= 1) mx = fmax(mx, __shfl_xor(mx, sh, 64));
            int ex;
            (void)frexp(mx, &ex);
            const double sc = ldexp(1.0, -ex);
#pragma unroll
            for (int j = 0; j < NJ; ++j)
#pragma unroll
                for (int i = 0; i < 6; ++i) v[j][i] *= sc;
        }
    }
    if (!own) return;
    double* o = a.phi + grp * 36;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) o[i * 6 + j0 + j] = v[j][i];
}

// a chain's block of the block-packed covariance as a full 3x3 (the inert state: variance 1)
template <typename T, class M>
__device__ __forceinline__ void chain_block_full(const T* P, int64_t stride, int64_t col, int ch, double (&p)[3][3]) {
    const int r0 = chain_row0<M>(ch);
    if (ch < M::NP) {
        const double v[6] = {double(P[(r0 + 0) * stride + col]), double(P[(r0 + 1) * stride + col]),
                             double(P[(r0 + 2) * stride + col]), double(P[(r0 + 3) * stride + col]),
                             double(P[(r0 + 4) * stride + col]), double(P[(r0 + 5) * stride + col])};
        p[0][0] = v[0], p[0][1] = p[1][0] = v[1], p[0][2] = p[2][0] = v[2];
        p[1][1] = v[3], p[1][2] = p[2][1] = v[4], p[2][2] = v[5];
    } else {
        const double v[3] = {double(P[(r0 + 0) * stride + col]), double(P[(r0 + 1) * stride + col]),
                             double(P[(r0 + 2) * stride + col])};
        p[0][0] = v[0], p[0][1] = p[1][0] = v[1], p[1][1] = v[2];
        p[0][2] = p[2][0] = p[1][2] = p[2][1] = 0.0;
        p[2][2] = 1.0;
    }
}

// one piece map applied to a chain covariance p (3x3, in place): P' = X Y^-1 with
// [X; Y] = [[A, B], [C, D]] [P; I], via the adjugate of Y, then symmetrised
__device__ __forceinline__ void lft_apply(double (&p)[3][3], const double (&m)[36]) {
    double X[3][3], Y[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double x = m[i * 6 + 3 + j], y = m[(i + 3) * 6 + 3 + j];
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                x = __builtin_fma(m[i * 6 + k], p[k][j], x);
                y = __builtin_fma(m[(i + 3) * 6 + k], p[k][j], y);
            }
            X[i][j] = x;
            Y[i][j] = y;
        }
    const double a00 = Y[1][1] * Y[2][2] - Y[1][2] * Y[2][1], a01 = Y[0][2] * Y[2][1] - Y[0][1] * Y[2][2],
                 a02 = Y[0][1] * Y[1][2] - Y[0][2] * Y[1][1];
    const double a10 = Y[1][2] * Y[2][0] - Y[1][0] * Y[2][2], a11 = Y[0][0] * Y[2][2] - Y[0][2] * Y[2][0],
                 a12 = Y[0][2] * Y[1][0] - Y[0][0] * Y[1][2];
    const double a20 = Y[1][0] * Y[2][1] - Y[1][1] * Y[2][0], a21 = Y[0][1] * Y[2][0] - Y[0][0] * Y[2][1],
                 a22 = Y[0][0] * Y[1][1] - Y[0][1] * Y[1][0];
    const double det = Y[0][0] * a00 + Y[0][1] * a10 + Y[0][2] * a20;
    const double inv[3][3] = {{a00, a01, a02}, {a10, a11, a12}, {a20, a21, a22}};
    const double rd = rcp_nr<2>(det);  // Newton-refined reciprocal: an IEEE division is ~10 dependent ops
    double pn[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 3; ++k) s = __builtin_fma(X[i][k], inv[k][j], s);
            pn[i][j] = s * rd;
        }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = i + 1; j < 3; ++j) pn[i][j] = pn[j][i] = 0.5 * (pn[i][j] + pn[j][i]);
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) p[i][j] = pn[i][j];
}

// phase 7: every chunk's start covariance from the maps, in ONE launch: chunk c starts from the
// handle's P advanced by the piece maps of at least the `iters` chunks before it (every chunk
// from the stream start when c < iters: exact), which covers the recursion's forgetting.  Block
// (x, chain) owns chunks [b0, b0 + a.G) of one chain, a.g consecutive chunks per thread: its
// threads first stage every piece map the windows need, [max(0, b0 - iters), b0 + G - 1) x np,
// into LDS (struct of arrays) with coalesced loads (a dependent walk over global memory waited
// ~2 us per map), then thread t walks from max(0, c_t - iters) through its g chunks, recording
// each start: (iters + g - 1) maps for g chunks.  a.g = 0: no LDS (windows too long for it), one
// chunk per thread, maps read from global memory.  For every chunk it also writes the warm-up
// bank (the handle's state as the guess, its status) and, without event warm-up (a.kp == 0),
// the map bank itself: every variant's covariance column (the map pass reads column c) and the
// guesses, variant q + 1 with + delta on component q of every chain.  Thread 0 of block 0
// zeroes the check.
constexpr int kStartMaxG = 4;  // chunks per thread of the start kernel (their starts stay in registers)
// NU: the LDS maps' row pitch fixed at compile time (where the block's window maps fit it): a
// walk's 36 reads of a map are then immediate offsets from one address, where a runtime pitch
// cost an address add per element and the products of each chunk's rows (~120 of the ~290
// instructions of a map application)
constexpr int kStartNu = 192;
template <typename T, class M, bool LDS, bool NU = false>
__global__ __launch_bounds__(kBlock) void stream_lft_start_kernel(const StreamArgs a) {
    extern __shared__ double lmap[];  // [36][nu]: element e of the block's nu = (G + iters) * np window maps
    constexpr int NCH = M::NP + M::NA;
    const int tid = int(threadIdx.x);
    const int ch = int(blockIdx.y);
    if (blockIdx.x == 0 && ch == 0 && tid == 0) {
        a.check->ok = 0;
        a.check->bad = 0;
        a.check->cov_gap = 0.0;
        a.check->state_gap = 0.0;
        a.check->done = 0;
        a.check->skip_chain = 0;
    }
    const int64_t gt = LDS ? a.g : 1;                  // chunks per thread
    const int64_t BC = LDS ? a.G : int64_t(blockDim.x);  // chunks per block
    const int64_t b0 = int64_t(blockIdx.x) * BC;
    const int64_t ws = b0 - a.iters > 0 ? b0 - a.iters : 0;  // first chunk whose maps the block reads
    // struct of arrays: at each step of the walks, consecutive threads read maps g apart
    const uint32_t nu = NU ? uint32_t(kStartNu) : uint32_t((BC + a.iters) * a.np);
    if constexpr (LDS) {
        const int64_t we = (b0 + BC < a.C ? b0 + BC : a.C) - 1;  // maps of chunks [ws, we)
        // 32-bit indices (a 64-bit division is a ~100-instruction sequence per element), 16 loads
        // in flight per thread (a load-store loop waited one memory latency per element)
        const uint32_t n = uint32_t(we > ws ? we - ws : 0) * uint32_t(a.np) * 36u;
        const double* src = a.phi + (ws * a.np * NCH + lft_map_chain<M>(a.sym != 0, ch)) * 36;
        constexpr int kU = 16;
        const uint32_t nt = blockDim.x;
        for (uint32_t e0 = uint32_t(tid); e0 < n; e0 += kU * nt) {
            double v[kU];
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const uint32_t e = e0 + uint32_t(j) * nt;
                const uint32_t u = e / 36u, k = e - u * 36u;
                v[j] = e < n ? src[u * uint32_t(NCH * 36) + k] : 0.0;
            }
#pragma unroll
            for (int j = 0; j < kU; ++j) {
                const uint32_t e = e0 + uint32_t(j) * nt;
                const uint32_t u = e / 36u, k = e - u * 36u;
                if (e < n) lmap[k * nu + u] = v[j];
            }
        }
        __syncthreads();
    }
    const int64_t ct = b0 + tid * gt;  // this thread's first chunk
    if (ct >= a.C || ct >= b0 + BC) return;
    const int64_t ce = ct + gt < a.C ? ct + gt : a.C;
    const int ns = ch < M::NP ? 3 : 2;
    // every global read before the first store (a load after a store to a pointer that may
    // alias it waits for the store)
    double ph[3][3];
    chain_block_full<T, M>(static_cast<const T*>(a.hP), 1, 0, ch, ph);
    T gx[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) gx[k] = k < ns ? static_cast<const T*>(a.hx)[chain_state<M>(ch, k)] : T(0);
    const int32_t hst = a.hstatus[0];
    double p[3][3], ps[kStartMaxG][3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) p[i][j] = ph[i][j];
    const int64_t cs = ct - a.iters > 0 ? ct - a.iters : 0;
    for (int64_t c = cs; c < ce; ++c) {
        if (c >= ct) {
            const int r = int(c - ct);
#pragma unroll
            for (int rr = 0; rr < kStartMaxG; ++rr)
                if (rr == r)
#pragma unroll
                    for (int i = 0; i < 3; ++i)
#pragma unroll
                        for (int j = 0; j < 3; ++j) ps[rr][i][j] = p[i][j];
        }
        if (c + 1 >= ce) break;
        // chunk c's piece maps in order (each piece short enough for its map to be well
        // conditioned; the LFT error grows with the events one product spans)
        for (int64_t u = c * a.np; u < (c + 1) * a.np; ++u) {
            double m[36];
            if constexpr (LDS) {
                const double* src = lmap + uint32_t(u - ws * a.np);
#pragma unroll
                for (int e = 0; e < 36; ++e) m[e] = src[uint32_t(e) * nu];
            } else {
                const double* src = a.phi + (u * NCH + lft_map_chain<M>(a.sym != 0, ch)) * 36;
#pragma unroll
                for (int e = 0; e < 36; ++e) m[e] = src[e];
            }
            lft_apply(p, m);
        }
    }
    // the starts and the banks; with polish chunks, the warm-up bank runs chunk c + kp from c's
    const int r0 = chain_row0<M>(ch);
    const int64_t B4 = 4 * a.C;
    auto put = [&](T* P, int64_t stride, int64_t col, const double (&q)[3][3]) {
        if (ch < M::NP) {
            P[(r0 + 0) * stride + col] = T(q[0][0]);
            P[(r0 + 1) * stride + col] = T(q[0][1]);
            P[(r0 + 2) * stride + col] = T(q[0][2]);
            P[(r0 + 3) * stride + col] = T(q[1][1]);
            P[(r0 + 4) * stride + col] = T(q[1][2]);
            P[(r0 + 5) * stride + col] = T(q[2][2]);
        } else {
            P[(r0 + 0) * stride + col] = T(q[0][0]);
            P[(r0 + 1) * stride + col] = T(q[0][1]);
            P[(r0 + 2) * stride + col] = T(q[1][1]);
        }
    };
#pragma unroll
    for (int r = 0; r < kStartMaxG; ++r) {
        const int64_t c = ct + r;
        if (c >= ce) break;
        if (c + a.kp < a.C) put(static_cast<T*>(a.wP), a.C, c + a.kp, ps[r]);
        if (c < a.kp) put(static_cast<T*>(a.wP), a.C, c, ph);
#pragma unroll
        for (int k = 0; k < 3; ++k)
            if (k < ns) static_cast<T*>(a.wx)[chain_state<M>(ch, k) * a.C + c] = gx[k];
        if (ch == 0) a.wst[c] = hst;
        if (a.kp == 0) {
            put(static_cast<T*>(a.mP), B4, c, ps[r]);
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int k = 0; k < 3; ++k)
                    if (k < ns)
                        static_cast<T*>(a.mx)[chain_state<M>(ch, k) * B4 + q * a.C + c] =
                            (q > 0 && k == q - 1) ? gx[k] + T(a.delta) : gx[k];
            if (ch == 0) a.mst[c] = hst;
        }
    }
}

// phase 4 (one block): the state seams and the verdict; a passed run leaves the last chunk's
// end state in the handle
template <typename T, class M>
__global__ __launch_bounds__(1024) void stream_finish_kernel(const StreamArgs a) {
    __shared__ double red[1024];
    __shared__ int redb[1024];
    const int tid = int(threadIdx.x);
    const T* fx = static_cast<const T*>(a.fx);
    double gap = 0.0;
    int bad = 0;
    for (int64_t c = tid; c < a.C; c += blockDim.x) {
        bad |= a.fst[c];
        if (c + 1 < a.C) {
#pragma unroll
            for (int i = 0; i < M::N; ++i) {
                const double st = a.starts[i * a.C + c + 1];
                const double d = fabs(double(fx[i * a.C + c]) - st) / fmax(fabs(st), 1.0);
                gap = (d == d) ? fmax(gap, d) : __builtin_inf();
            }
        }
    }
    red[tid] = gap;
    redb[tid] = bad;
    __syncthreads();
    for (int w = blockDim.x / 2; w > 0; w >>= 1) {
        if (tid < w) {
            red[tid] = fmax(red[tid], red[tid + w]);
            redb[tid] |= redb[tid + w];
        }
        __syncthreads();
    }
    if (tid == 0) {
        StreamCheck* k = a.check;
        k->state_gap = red[0];
        k->bad |= redb[0];
        const bool ok = k->bad == 0 && k->cov_gap <= a.tol_cov && red[0] <= a.tol_state;
        k->ok = ok ? 1 : 0;
        if (ok) {
            const int64_t c = a.C - 1;
            for (int i = 0; i < M::N; ++i) static_cast<T*>(a.hx)[i] = fx[i * a.C + c];
            for (int r = 0; r < M::NBLK; ++r) static_cast<T*>(a.hP)[r] = static_cast<const T*>(a.fP)[r * a.C + c];
            a.hstatus[0] = 0;
        }
    }
}

// ------------------------------------------------------------------------------------
// Brute-force combination search (kf_eval_combos).  The n candidate events and the binomial
// table sit in LDS; lane f unranks combination combo_offset + f (lexicographic =
// itertools.combinations order) one index at a time while it runs the filter, so no per-lane
// index list is stored.
// ------------------------------------------------------------------------------------
constexpr int kMaxEvents = 64;

template <typename T, bool CUSTOM = false>
using Ref15 = Chains<T, M15, CUSTOM>;

#ifndef KF_COMBO_WAVES
#define KF_COMBO_WAVES 3  // waves per SIMD the one-filter-per-subset kernel is compiled for
#endif
template <typename T, bool CUSTOM>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KF_COMBO_WAVES))) void ref15_combo_kernel(
    const Ref15ComboArgs a) {
    __shared__ double s_ev[kMaxEvents * 11];
    __shared__ uint64_t s_binom[(kMaxEvents + 1) * (kMaxEvents + 1)];
    const int n = a.n_events;
    for (int i = threadIdx.x; i < n * 11; i += kBlock) s_ev[i] = a.ev[i];
    for (int i = threadIdx.x; i < (n + 1) * (kMaxEvents + 1); i += kBlock) s_binom[i] = a.binom[i];
    __syncthreads();

    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    const uint64_t rank0 = a.combo_offset + uint64_t(f);
    const bool live = rank0 < a.n_combos;
    // records land at a per-lane row (a skipped event shifts them): one span over the k+2 rows
    const auto r_ld = span_rsrc(a.logdets, 0, rb, uint32_t(a.k + 2));

    Ref15<T, CUSTOM> s;
    s.kc = a.kc;
#pragma unroll
    for (int i = 0; i < 15; ++i) s.x[i] = T(a.init[i]);
#pragma unroll
    for (int r = 0; r < 27; ++r) s.blk(r) = T(a.init[15 + r]);

    // record 0: logdet of the initial covariance (kf_workers.py:32)
    T ld = s.logdet();
    T ld_max = ld;
    int rec = 0;
    stv(r_ld, uint32_t(rec) * rb + off, ld);
    ++rec;
    bool ok = true;
    double cur = a.prev_time;
    uint64_t r = live ? rank0 : 0;
    int cand = 0;
    const T no_gate = T(0);
    for (int j = 0; j < a.k; ++j) {
        // unrank the j-th element: skip candidates whose sub-tree is entirely below r
        const int left = a.k - j - 1;
        while (cand < n) {
            const uint64_t cnt = s_binom[(n - cand - 1) * (kMaxEvents + 1) + left];
            if (r < cnt) break;
            r -= cnt;
            ++cand;
        }
        const int e = cand < n ? cand : n - 1;
        ++cand;
        const double te = s_ev[e * 11];
        const double dtd = te - cur;
        if (dtd < 0.0) continue;  // kf_workers.py:38-40: skip, prev time unchanged
        T pay[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) pay[i] = T(s_ev[e * 11 + 2 + i]);
        s.event(int(s_ev[e * 11 + 1]), T(dtd), pay, false, no_gate, ok);
        cur = te;
        ld = s.logdet();
        ld_max = ld > ld_max ? ld : ld_max;
        stv(r_ld, uint32_t(rec) * rb + off, ld);
        ++rec;
    }
    // always propagate to the common end time (kf_workers.py:74-82)
    if (cur < a.target_end - 1e-8) {
        s.predict(T(a.target_end - cur));
        ld = s.logdet();
        ld_max = ld > ld_max ? ld : ld_max;
        stv(r_ld, uint32_t(rec) * rb + off, ld);
        ++rec;
    }
    for (int q = rec; q < a.k + 2; ++q) stv(r_ld, uint32_t(q) * rb + off, quiet_nan<T>());
    int32_t st = ok ? 0 : kNotSpd;
    if (!live) {
        st = 1;
        ld_max = quiet_nan<T>();
    } else if (!ok || !(ld_max == ld_max)) {
        st = kNotSpd;
        s.fill_nan();
        ld_max = quiet_nan<T>();
    }
    if (a.max_logdet) stb(a.max_logdet, 0, rb, off, ld_max);
    if (a.n_records) a.n_records[f] = rec;
    s.store(a.x, a.P, rb, off);
    a.status[f] = st;
}

// ------------------------------------------------------------------------------------
// Brute-force search with shared prefixes (kf_search_combos).  The worker runs every subset's
// filter from the common start (kf_workers.py:29-71), so a k-subset repeats all of the work of
// its (k-1)-prefix: over all subsets of n events that is ~n/2 + 1 event steps per subset.  Here
// the filter of subset S = P + {j} (j > max P) is P's stored filter advanced by event j — the
// same operations in the same order as the per-combination kernel, so the same numbers — and
// each subset costs one event step plus the worker's final predict (:74-82).
//
// One lane per parent P (level k - 1, colex order).  Its children j = max P + 1 .. n - 1 are
// visited in a wave-uniform loop: parents of a wave share max P except at run boundaries, so
// event j is the same for every active lane (scalar loads, uniform GPS/IMU branch), and for a
// fixed j the children of consecutive parents are consecutive ranks (coalesced stores).
// ------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
        const uint64_t o = __shfl_xor(v, s, 64);
        v = o > v ? o : v;
    }
    return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) v += __shfl_xor(v, s, 64);
    return v;
}

// Level buffers in node blocks of 64 (kf_internal.h): a wave's parents are one contiguous block.
template <typename T, bool SYM = false>
__device__ __forceinline__ char* level_block(const void* base, uint64_t c) {
    return static_cast<char*>(const_cast<void*>(base)) + (c >> 6) * search_block_bytes(sizeof(T), SYM);
}
template <typename T>
__device__ __forceinline__ T* level_row(char* blk, uint32_t lane, int r) {
    return reinterpret_cast<T*>(blk + r * 64 * int(sizeof(T))) + lane;
}
// the running max's binary exponent (int32 per node, after the T rows)
template <typename T, bool SYM = false>
__device__ __forceinline__ int32_t* level_exp(char* blk, uint32_t lane) {
    return reinterpret_cast<int32_t*>(blk + search_rows(SYM) * 64 * int(sizeof(T))) + lane;
}
template <typename T, bool SYM = false>
__device__ __forceinline__ double* level_tail(char* blk, uint32_t lane, int q) {
    return reinterpret_cast<double*>(blk + search_rows(SYM) * 64 * int(sizeof(T)) + 256 + q * 512) + lane;
}

// A positive determinant as (mantissa in [0.5, 1), binary exponent); a failed filter's has a NaN
// mantissa.  The search carries each subset's running max this way and compares determinants,
// not their logs (log is monotone): one log per scored subset where its max log-det is an
// output (subset_max), none where only the acceptance test reads it (DetBand), instead of a log
// per record and per final predict.
// A NaN determinant carries the exponent that makes the comparisons below treat it as the log
// domain's `ld > run ? ld : run` treats a NaN: kNanLoses on a failed record or final predict
// (it never wins a max), kNanWins on a failed running max (nothing beats it: it stays NaN).
constexpr int kNanLoses = -2147483647 - 1, kNanWins = 2147483647;
template <typename T>
struct DetV {
    T m;
    int e;
    __device__ __forceinline__ bool valid() const { return m == m; }
    // this > o (by exponent, then mantissa: both normalised)
    __device__ __forceinline__ bool gt(const DetV& o) const { return e > o.e || (e == o.e && m > o.m); }
    __device__ __forceinline__ T log() const { return valid() ? log_mant(m, e) : quiet_nan<T>(); }
    __device__ __forceinline__ void fail() {
        m = quiet_nan<T>();
        e = kNanWins;
    }
};

// `d.gt(r) ? d : r`, the exponent blended with a mask (a select of two loaded members is folded
// into a load from a select of their addresses, which keeps the search node in scratch memory)
template <typename T>
__device__ __forceinline__ DetV<T> dmax(const DetV<T>& d, const DetV<T>& r) {
    const bool g = d.gt(r);
    const int mk = -int(g);
    return DetV<T>{g ? d.m : r.m, (d.e & mk) | (r.e & ~mk)};
}

// The acceptance test max(log_det) < R_threshold (kf_workers.py:1353) on a determinant: below
// lo it holds and above hi it fails for any log the kernels could compute (lo, hi = exp(thr) (1
// -+ eps), eps far above log_mant's and exp's rounding near thr; set_search_band computes them
// on the host); in between the log decides, as `log < T(thr)` exactly.
template <typename T>
struct DetBand {
    DetV<T> lo, hi;
    // 0: the band; 1: accept every valid determinant; 2: accept only a valid determinant that
    // underflowed to 0 (log -inf, below any finite threshold); 3: accept none (-inf or NaN)
    int mode;
    T thr;
    __device__ __forceinline__ explicit DetBand(const Ref15SearchArgs& a)
        : lo{T(a.band_lo_m), a.band_lo_e}, hi{T(a.band_hi_m), a.band_hi_e}, mode(a.band_mode), thr(T(a.threshold)) {}
    // d: a subset's max (valid, or NaN with kNanWins, which lies above hi)
    __device__ __forceinline__ bool accept(const DetV<T>& d) const {
        if (mode != 0) return d.valid() && (mode == 1 || (mode == 2 && d.m == T(0)));
        if (lo.gt(d)) return true;
        if (d.gt(hi)) return false;
        return log_mant(d.m, d.e) < thr;
    }
};

// Chains<T, M15>::logdet() accumulated one block at a time, in its order (pva chains, then aw
// chains) with its renormalisations, so the value is the same.
template <typename T>
struct LogdetAcc {
    T num = T(1), den = T(1);
    int ex = 0;
    bool ok = true;
    __device__ __forceinline__ void add_pva(const T (&P)[6], int c) {
        det3_scaled<T>(P, num, den, ok);
        if (sizeof(T) == 4 || c == M15::NP - 1) renorm(num, ex);
    }
    __device__ __forceinline__ void add_aw(const T (&P)[3]) {
        det2<T>(P, num, ok);
        if (sizeof(T) == 4) renorm(num, ex);
    }
    __device__ __forceinline__ T finish() {
        T prod = num * rcp_nr<kRefNewton>(den);
        renorm(prod, ex);
        const T ld = log_mant(prod, ex);
        return ok ? ld : quiet_nan<T>();
    }
    // the determinant itself (Chains::det_mant's value): no log.  A product that underflowed to 0
    // (log -inf) takes the lowest exponent, so it orders below every positive determinant.
    __device__ __forceinline__ DetV<T> det() {
        T prod = num * rcp_nr<kRefNewton>(den);
        renorm(prod, ex);
        return DetV<T>{ok ? prod : quiet_nan<T>(), ok && prod != T(0) ? ex : kNanLoses};
    }
};

// A stored node of the search: the covariance after a subset's events, its running max
// determinant (DetV: the max log-det before its log), the time of its last applied event and its
// subset mask.  The search scores a subset
// by its max log-det alone, which depends on the covariance alone, and the covariance does not
// depend on the measurements (nor, so, on the state): the state is not carried (kf_eval_combos
// carries it for the per-combination API).  The updates see a constant zero state (search_pva,
// search_aw), so their state half is dead code the compiler removes.
// SYM (Ref15SearchArgs::sym): the three pva chains, and the three aw chains, have the same
// constants and the same start, so in exact arithmetic the same covariance; the node holds one of
// each (rows 0..5 pva, 6..8 aw) and the search computes one of each, entering it into the
// log-dets once per chain it stands for.  (The every-chain kernels' separately compiled copies
// of a chain round alike in most subsets and one ulp apart in some.)
template <typename T, bool CUSTOM, bool SYM = false>
struct SearchNode {
    static constexpr int NP = SYM ? 1 : M15::NP, NA = SYM ? 1 : M15::NA;
    static constexpr int NR = 6 * NP + 3 * NA;  // covariance rows held (27, or 9)
    T P[NR];
    DetV<T> run;
    double prev;
    uint64_t mask;

    // The root (defined after search_child_to, whose operations it applies to the fixed events)
    __device__ __forceinline__ DetV<T> root(const Ref15SearchArgs& a, bool eval);
    __device__ __forceinline__ void load(const void* level, uint64_t p) {
        char* blk = level_block<T, SYM>(level, p);
        const uint32_t lane = uint32_t(p) & 63u;
#pragma unroll
        for (int i = 0; i < NR; ++i) P[i] = *level_row<T>(blk, lane, i);
        run.m = *level_row<T>(blk, lane, NR);
        run.e = *level_exp<T, SYM>(blk, lane);
        prev = *level_tail<T, SYM>(blk, lane, 0);
        mask = __builtin_bit_cast(uint64_t, *level_tail<T, SYM>(blk, lane, 1));
    }
    // the node as level K + 1's parent at colex rank r (the head kernel)
    __device__ __forceinline__ void store(void* level, uint64_t r) const {
        char* cb = level_block<T, SYM>(level, r);
        const uint32_t cl = uint32_t(r) & 63u;
#pragma unroll
        for (int i = 0; i < NR; ++i) *level_row<T>(cb, cl, i) = P[i];
        *level_row<T>(cb, cl, NR) = run.m;
        *level_exp<T, SYM>(cb, cl) = run.e;
        *level_tail<T, SYM>(cb, cl, 0) = prev;
        *level_tail<T, SYM>(cb, cl, 1) = __builtin_bit_cast(double, mask);
    }
    // largest free candidate in the subset (local index), -1 for the root
    __device__ __forceinline__ int max_event(int shift) const {
        const uint64_t loc = mask >> shift;
        return loc ? 63 - __builtin_clzll(loc) : -1;
    }
};

// a scored subset: every max log-det to subset_max (its one log), the acceptance test into
// (best, cnt) — on the determinant (DetBand) when no log was taken
template <typename T>
__device__ __forceinline__ void search_score(const Ref15SearchArgs& a, const DetBand<T>& band, uint64_t mask,
                                             const DetV<T>& fmax, uint64_t& best, uint64_t& cnt) {
    bool acc;
    if (a.subset_max) {
        const T ld = fmax.log();
        static_cast<T*>(a.subset_max)[mask] = ld;
        acc = ld < band.thr;
    } else {
        acc = band.accept(fmax);
    }
    if (acc) {  // max(log_det) < R_threshold (kf_workers.py:1353); NaN never passes
        const uint64_t key = __builtin_bitreverse64(mask);  // larger key = earlier in itertools order
        best = key > best ? key : best;
        ++cnt;
    }
}

// Event j applied to a node whose last applied event is at prev_in (kf_workers.py:36-82): a
// negative dt skips the event and keeps the time; the worker's final predict to target_end runs
// when the new time is before it.
// the search's events are read through ro() (the table above `ro`): scalar loads in the child loops
struct SearchEvent {
    ro_double* e;
    int type;
    bool step, final_predict;
    double dt, dte, prev;  // prev: the time after the event
};

__device__ __forceinline__ SearchEvent search_event(const Ref15SearchArgs& a, int j, double prev_in) {
    SearchEvent v;
    v.e = ro(a.ev) + j * 11;
    v.type = int(v.e[1]);
    v.dt = v.e[0] - prev_in;
    v.step = v.dt >= 0.0;  // kf_workers.py:38-40
    v.prev = v.step ? v.e[0] : prev_in;
    v.final_predict = v.prev < a.target_end - 1e-8;  // kf_workers.py:74-82
    v.dte = a.target_end - v.prev;
    return v;
}

// One chain of the 15-state filter through one event, Chains::event's operations for that
// chain (each chain's predict and update touch only that chain); the state is not carried
// (SearchNode), so xb is constant zeros and the state half is dead code after inlining.
template <typename T, bool CUSTOM>
__device__ __forceinline__ void search_pva(const SearchEvent& v, int ch, T (&Pb)[6], bool& ok, const RefConsts* kc) {
    using C15 = Chains<T, M15>;
    T qpva[3], Rp[6], rg;
    pva_noise<CUSTOM, M15>(kc, ch, qpva, Rp, rg);
    const T Rg[1] = {rg};
    if (!v.step) return;
    const T dt = T(v.dt);
    T xb[3] = {T(0), T(0), T(0)};
    C15::template chain_predict<3>(xb, Pb, dt, qpva);
    if (v.type == kGps) {
        const T zb[1] = {T(v.e[2 + ch])};
        ok = sel_update<3, 1, true, T, kRefNewton, true, kRefJoseph<T>, kRefGainR>(xb, Pb, zb, Rg) && ok;
    } else {
        const T acc = T(v.e[2 + M15::imu_acc(ch)]);
        const T V = fmaT(acc, dt, xb[1]);
        const T X = fmaT(V, dt, xb[0]);
        const T zb[3] = {X, V, acc};
        ok = sel_update<3, 3, true, T, kRefNewton, true, kRefJoseph<T>, kRefGainR>(xb, Pb, zb, Rp) && ok;
    }
}

template <typename T, bool CUSTOM>
__device__ __forceinline__ void search_aw(const SearchEvent& v, int ch, T (&Pa)[3], bool& ok, const RefConsts* kc) {
    using C15 = Chains<T, M15>;
    T qaw[2], Ra[3];
    aw_noise<CUSTOM, M15>(kc, ch, qaw, Ra);
    if (!v.step) return;
    T xa[2] = {T(0), T(0)};
    C15::template chain_predict<2>(xa, Pa, T(v.dt), qaw);
    if (v.type != kGps) {  // a GPS fix updates the pva chains only
        const T za[2] = {T(v.e[2 + M15::imu_att(ch)]), T(v.e[2 + M15::imu_rate(ch)])};
        ok = sel_update<2, 2, true, T, kRefNewton, true, kRefJoseph<T>, kRefGainR>(xa, Pa, za, Ra) && ok;
    }
}

// The log-dets of one subset: its record after the event (rec) and after the worker's final
// predict (fin), accumulated chain by chain in Chains::logdet's block order, so the numbers are
// kf_eval_combos's.
template <typename T, bool CUSTOM>
struct SearchScore {
    LogdetAcc<T> rec, fin;
    bool ok = true;
    const RefConsts* kc = nullptr;
    // chains ch .. ch + reps - 1 all holding Pb (reps = 3: the axis-symmetric search's one pva
    // chain standing for the three; their blocks enter the log-dets in the same order)
    __device__ __forceinline__ void add_pva(const SearchEvent& v, const T (&Pb)[6], int ch, int reps = 1) {
        using C15 = Chains<T, M15>;
        T qpva[3], Rp[6], rg;
        pva_noise<CUSTOM, M15>(kc, ch, qpva, Rp, rg);
#pragma unroll
        for (int r = 0; r < reps; ++r) rec.add_pva(Pb, ch + r);
        T Pf[6], xf[3] = {T(0), T(0), T(0)};
#pragma unroll
        for (int i = 0; i < 6; ++i) Pf[i] = Pb[i];
        C15::template chain_predict<3>(xf, Pf, T(v.dte), qpva);  // read by finish() only with v.final_predict
#pragma unroll
        for (int r = 0; r < reps; ++r) fin.add_pva(Pf, ch + r);
    }
    __device__ __forceinline__ void add_aw(const SearchEvent& v, const T (&Pa)[3], int ch, int reps = 1) {
        using C15 = Chains<T, M15>;
        T qaw[2], Ra[3];
        aw_noise<CUSTOM, M15>(kc, ch, qaw, Ra);
#pragma unroll
        for (int r = 0; r < reps; ++r) rec.add_aw(Pa);
        T Pf[3], xf[2] = {T(0), T(0)};
#pragma unroll
        for (int i = 0; i < 3; ++i) Pf[i] = Pa[i];
        C15::template chain_predict<2>(xf, Pf, T(v.dte), qaw);  // read by finish() only with v.final_predict
#pragma unroll
        for (int r = 0; r < reps; ++r) fin.add_aw(Pf);
    }
    // the running max determinant after the event (NaN for a failed filter, kf_eval_combos:
    // KF_ENOTSPD), and into fmax the subset's max with the final predict — the max log-dets'
    // determinants, no log taken
    __device__ __forceinline__ DetV<T> finish(const SearchEvent& v, const DetV<T>& run_in, DetV<T>& fmax) {
        DetV<T> run = run_in;
        if (v.step) {
            const DetV<T> d = rec.det();
            run = dmax(d, run_in);
            if (!ok) run.fail();
        }
        fmax = run;
        if (v.final_predict) {
            const DetV<T> d = fin.det();
            fmax = dmax(d, run);
        }
        return run;
    }
};

// Child j (> the parent's largest event) of node `par`, colex rank c at level a.k: scored into
// (best, cnt), and stored when a.child is set and the child has stored children (largest event
// <= n - 3).  With a.tail, the child holding event n - 2 is not stored: its only child (it plus
// event n - 1, level k + 1) is evaluated from the registers and scored into (best1, cnt1).
// Chain by chain: a chain's child covariance is stored (or carried through event n - 1) as soon
// as it is computed, so only one chain of the child and grandchild is live at a time.
// The parent's covariance as search_child reads it: from registers, or from a lane's LDS column
// (the parent-major kernel's LDS variant, which frees the registers that hold it across the
// loop over children).
// kChainFence: a scheduling barrier after each chain, so the compiler does not hoist the next
// chains' LDS reads over this one's arithmetic (which spilled the 3-wave LDS variant)
template <typename T>
struct ParRegs {
    static constexpr bool kChainFence = false;
    const T* P;
    __device__ __forceinline__ T operator()(int i) const { return P[i]; }
};
template <typename T>
struct ParLds {
    static constexpr bool kChainFence = true;
    const T* col;  // row i at col[i * 64]
    __device__ __forceinline__ T operator()(int i) const { return col[i * 64]; }
};

// Where search_child_to puts the child it computed: a level buffer's node (LevelSink: level k,
// stored for the next launch), or a lane's LDS column and registers (LdsSink: the pair kernel's
// level k, read back at once as the parent of level k + 1).  Either way the bits are the same.
template <typename T, bool SYM>
struct LevelSink {
    char* cb;
    uint32_t cl;
    bool on;
    __device__ __forceinline__ void row(int i, T v) const { *level_row<T>(cb, cl, i) = v; }
    __device__ __forceinline__ void node(int nr, const DetV<T>& run, double prev, uint64_t mask) const {
        *level_row<T>(cb, cl, nr) = run.m;
        *level_exp<T, SYM>(cb, cl) = run.e;
        *level_tail<T, SYM>(cb, cl, 0) = prev;
        *level_tail<T, SYM>(cb, cl, 1) = __builtin_bit_cast(double, mask);
    }
};
template <typename T>
struct LdsSink {
    T* col;  // row i at col[i * 64]
    bool on;
    DetV<T> run;
    double prev;
    uint64_t mask;
    __device__ __forceinline__ void row(int i, T v) const { col[i * 64] = v; }
    __device__ __forceinline__ void node(int, const DetV<T>& r, double p, uint64_t m) {
        run = r;
        prev = p;
        mask = m;
    }
};

// A class root's prefix nodes (SearchNode::root): the child's rows and scalars in registers,
// with its score's determinant (fmax) instead of a scoring
template <typename T, int NR>
struct RegSink {
    T P[NR];
    bool on;
    DetV<T> run, fmax;
    double prev;
    uint64_t mask;
    __device__ __forceinline__ void row(int i, T v) { P[i] = v; }
    __device__ __forceinline__ void node(int, const DetV<T>& r, double p, uint64_t m) {
        run = r;
        prev = p;
        mask = m;
    }
};

// SCORE = false: the child is not scored (nor is a tail computed); its max with the final predict
// goes to sk.fmax (RegSink)
template <typename T, bool CUSTOM, bool SYM, class PS, class SK, bool SCORE = true>
__device__ __forceinline__ void search_child_to(const Ref15SearchArgs& a, const DetBand<T>& band,
                                                const SearchNode<T, CUSTOM, SYM>& par, const PS& pp, int j, SK& sk,
                                                bool tail, uint64_t& best, uint64_t& cnt, uint64_t& best1,
                                                uint64_t& cnt1) {
    using Node = SearchNode<T, CUSTOM, SYM>;
    constexpr int RP = SYM ? M15::NP : 1, RA = SYM ? M15::NA : 1;  // chains each computed one stands for
    const SearchEvent vs = search_event(a, j, par.prev);
    const bool store = sk.on;
    SearchEvent vg;
    if (tail) vg = search_event(a, j + 1, vs.prev);
    SearchScore<T, CUSTOM> ss, sg;
    ss.kc = sg.kc = a.kc;
#pragma unroll
    for (int ch = 0; ch < Node::NP; ++ch) {
        T Pb[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) Pb[i] = pp(6 * ch + i);
        search_pva<T, CUSTOM>(vs, ch, Pb, ss.ok, a.kc);
        if (store) {
#pragma unroll
            for (int i = 0; i < 6; ++i) sk.row(6 * ch + i, Pb[i]);
        }
        ss.add_pva(vs, Pb, ch, RP);
        if (tail) {
            search_pva<T, CUSTOM>(vg, ch, Pb, sg.ok, a.kc);
            sg.add_pva(vg, Pb, ch, RP);
        }
        if constexpr (PS::kChainFence) __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int ch = 0; ch < Node::NA; ++ch) {
        T Pa[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) Pa[i] = pp(6 * Node::NP + 3 * ch + i);
        search_aw<T, CUSTOM>(vs, ch, Pa, ss.ok, a.kc);
        if (store) {
#pragma unroll
            for (int i = 0; i < 3; ++i) sk.row(6 * Node::NP + 3 * ch + i, Pa[i]);
        }
        ss.add_aw(vs, Pa, ch, RA);
        if (tail) {
            search_aw<T, CUSTOM>(vg, ch, Pa, sg.ok, a.kc);
            sg.add_aw(vg, Pa, ch, RA);
        }
        if constexpr (PS::kChainFence) __builtin_amdgcn_sched_barrier(0);
    }
    DetV<T> fmax;
    const DetV<T> run = ss.finish(vs, par.run, fmax);
    const uint64_t cmask = par.mask | (uint64_t(1) << (j + a.shift));
    if (store) sk.node(Node::NR, run, vs.prev, cmask);
    if constexpr (SCORE) {
        search_score(a, band, cmask, fmax, best, cnt);
        if (tail) {
            DetV<T> gmax;
            (void)sg.finish(vg, run, gmax);
            search_score(a, band, cmask | (uint64_t(1) << (j + 1 + a.shift)), gmax, best1, cnt1);
        }
    } else {
        sk.fmax = fmax;
    }
}

// The root: the search's fixed events (a.root_mask, none for a whole search) applied to the
// initial filter in index order as the worker applies a combination's events
// (kf_workers.py:36-71); record 0 is the logdet of the initial covariance (:32).  Each fixed
// event is applied with search_child_to's operations, from the node its predecessors made, so a
// class root is bit for bit the node the whole search computes for that subset (its prefixes are
// not scored: they belong to other classes).  With `eval`, returns the root subset's max log-det
// with the final predict (as a determinant) for the caller to score.
template <typename T, bool CUSTOM, bool SYM>
__device__ __forceinline__ DetV<T> SearchNode<T, CUSTOM, SYM>::root(const Ref15SearchArgs& a, bool eval) {
    Ref15<T, CUSTOM> r;
    r.kc = a.kc;
#pragma unroll
    for (int i = 0; i < 15; ++i) r.x[i] = T(a.init[i]);
#pragma unroll
    for (int i = 0; i < 27; ++i) r.blk(i) = T(a.init[15 + i]);
    run.m = r.det_mant(run.e);
    if (!run.valid()) run.fail();
    if (run.m == T(0)) run.e = kNanLoses;
    prev = a.prev_time;
    mask = 0;
#pragma unroll
    for (int i = 0; i < 6 * NP; ++i) P[i] = r.blk(i);
#pragma unroll
    for (int i = 0; i < 3 * NA; ++i) P[6 * NP + i] = r.blk(6 * M15::NP + i);
    DetV<T> fmax = run;
    if (a.root_mask) {
        const DetBand<T> band(a);
        for (uint64_t rest = a.root_mask; rest; rest &= rest - 1) {
            RegSink<T, NR> sk;
            sk.on = true;
            uint64_t b0 = 0, c0 = 0, b1 = 0, c1 = 0;
            // j = the candidate's index relative to the free ones (negative: a.ev + 11 j is the
            // fixed event's row of a.ev_all)
            search_child_to<T, CUSTOM, SYM, ParRegs<T>, RegSink<T, NR>, false>(
                a, band, *this, ParRegs<T>{P}, __builtin_ctzll(rest) - a.shift, sk, false, b0, c0, b1, c1);
#pragma unroll
            for (int i = 0; i < NR; ++i) P[i] = sk.P[i];
            run = sk.run;
            prev = sk.prev;
            mask = sk.mask;
            fmax = sk.fmax;
        }
    }
    (void)eval;
    return fmax;
}

template <typename T, bool CUSTOM, bool SYM, class PS>
__device__ __forceinline__ void search_child(const Ref15SearchArgs& a, const DetBand<T>& band,
                                             const SearchNode<T, CUSTOM, SYM>& par, const PS& pp, int j, uint64_t c,
                                             uint64_t& best, uint64_t& cnt, uint64_t& best1, uint64_t& cnt1) {
    const bool store = a.child && j < a.n_events - 2;
    LevelSink<T, SYM> sk{store ? level_block<T, SYM>(a.child, c) : nullptr, uint32_t(c) & 63u, store};
    search_child_to<T, CUSTOM, SYM>(a, band, par, pp, j, sk, a.tail && j == a.n_events - 2,  // wave-uniform (j is)
                                    best, cnt, best1, cnt1);
}

// one atomic pair per wave, and only from waves with an accepted subset; k = local level
__device__ __forceinline__ void search_publish(const Ref15SearchArgs& a, int k, uint64_t best, uint64_t cnt) {
    if (__builtin_amdgcn_ballot_w64(cnt != 0) != 0) {  // wave-uniform
        best = wave_max_u64(best);
        cnt = wave_sum_u64(cnt);
        if (__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)) == 0) {
            atomicMax(reinterpret_cast<unsigned long long*>(&a.best[a.k_base + k]), static_cast<unsigned long long>(best));
            atomicAdd(reinterpret_cast<unsigned long long*>(&a.n_acc[a.k_base + k]), static_cast<unsigned long long>(cnt));
        }
    }
}

// Parent-major: one lane per parent, its children in a wave-uniform loop over j (parents of a
// wave share their largest event except at run boundaries, so event j is the same for every
// active lane: scalar loads, a uniform GPS/IMU branch).  For the wide levels.
#ifndef KF_SEARCH_PM_WAVES
#define KF_SEARCH_PM_WAVES 2  // waves per SIMD of the register variant (its VGPR budget)
#endif
// Ref15SearchArgs::stop_best: lane i reads size stop_lo + i (vector loads: these counters were
// written by earlier launches' atomics); the same answer in every wave of the grid.  Called
// before any lane leaves the kernel.
__device__ __forceinline__ bool search_stopped(const Ref15SearchArgs& a) {
    if (!a.stop_best) return false;
    const int s = a.stop_lo + int(threadIdx.x & 63u);
    const uint64_t v = s <= a.stop_hi ? __atomic_load_n(a.stop_best + s, __ATOMIC_RELAXED) : 0;
    return __any(v != 0);
}

#ifndef KF_SEARCH_SYM_WAVES
#define KF_SEARCH_SYM_WAVES 3  // waves per SIMD of the axis-symmetric search kernels (A/B builds)
#endif
// PLDS: the parent's covariance lives in LDS (one 64-lane block per workgroup, [27][64] T),
// which fits the kernel in 3 waves per SIMD without spills; otherwise in registers.
template <typename T, bool PLDS, bool CUSTOM, bool SYM>
__global__ __launch_bounds__(PLDS ? 64 : kBlock) __attribute__((
    amdgpu_waves_per_eu(SYM ? KF_SEARCH_SYM_WAVES : PLDS ? 3 : KF_SEARCH_PM_WAVES))) void
ref15_search_pm_kernel(const Ref15SearchArgs a) {
    if (search_stopped(a)) return;
    constexpr int NT = PLDS ? 64 : kBlock;
    constexpr int NR = SearchNode<T, CUSTOM, SYM>::NR;
    const int64_t p = static_cast<int64_t>(blockIdx.x) * NT + threadIdx.x;
    if (uint64_t(p) >= a.n_par) return;
    const DetBand<T> band(a);
    SearchNode<T, CUSTOM, SYM> par;
    if (a.k == 1) {
        uint64_t rb = 0, rc = 0;  // a fixed root is itself one of the subsets searched
        const DetV<T> f = par.root(a, a.root_mask != 0);
        if (a.root_mask) search_score(a, band, a.root_mask, f, rb, rc);
        search_publish(a, 0, rb, rc);
    } else {
        par.load(a.par, uint64_t(p));
    }
    const int m = par.max_event(a.shift);
    const int j0 = wave_uniform(m) + 1;  // colex order: the first lane holds the smallest max
    uint64_t best = 0, cnt = 0, best1 = 0, cnt1 = 0;
    if constexpr (PLDS) {
        __shared__ T sP[NR * 64];
        T* col = sP + threadIdx.x;
#pragma unroll
        for (int i = 0; i < NR; ++i) col[i * 64] = par.P[i];  // read back by this lane only
        const ParLds<T> pp{col};
#pragma unroll 1
        for (int j = j0; j < a.n_events; ++j) {
            if (j <= m) continue;
            search_child<T, CUSTOM, SYM>(a, band, par, pp, j, uint64_t(p) + ro(a.binom)[j * (kMaxEvents + 1) + a.k], best,
                                         cnt, best1, cnt1);
        }
    } else {
        const ParRegs<T> pp{par.P};
#pragma unroll 1
        for (int j = j0; j < a.n_events; ++j) {
            if (j <= m) continue;
            search_child<T, CUSTOM, SYM>(a, band, par, pp, j, uint64_t(p) + ro(a.binom)[j * (kMaxEvents + 1) + a.k], best,
                                         cnt, best1, cnt1);
        }
    }
    search_publish(a, a.k, best, cnt);
    if (a.tail) search_publish(a, a.k + 1, best1, cnt1);
}

// Two levels per launch (KF_OPT_SEARCH_PAIR, the axis-symmetric search's parent-major levels):
// lane p's parent (level k - 1, stored), each of its children (level k) computed into the lane's
// LDS column — not stored — and, at once, that child's children (level k + 1) from the column,
// stored as the next launch's parents.  Each subset's operations are search_child's and a child
// reaches its children with the bits a stored node would carry, so every score and every stored
// node is the one-level search's; level k's nodes (half the level traffic) never reach HBM.  A
// child holding event n - 2 has one child (it plus n - 1), scored by its tail as size k + 1.
template <typename T, bool CUSTOM, bool SYM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(KF_SEARCH_SYM_WAVES))) void
ref15_search_pair_kernel(const Ref15SearchArgs a) {
    if (search_stopped(a)) return;
    constexpr int NR = SearchNode<T, CUSTOM, SYM>::NR;
    const int64_t p = static_cast<int64_t>(blockIdx.x) * 64 + threadIdx.x;
    if (uint64_t(p) >= a.n_par) return;
    const int n = a.n_events, k = a.k;
    const DetBand<T> band(a);
    SearchNode<T, CUSTOM, SYM> par;
    par.load(a.par, uint64_t(p));
    const int m = par.max_event(a.shift);
    const int j0 = wave_uniform(m) + 1;  // colex order: the first lane holds the smallest max
    __shared__ T sP[NR * 64];
    __shared__ T sC[NR * 64];
    T* col = sP + threadIdx.x;
    T* ccol = sC + threadIdx.x;
#pragma unroll
    for (int i = 0; i < NR; ++i) col[i * 64] = par.P[i];  // read back by this lane only
    const ParLds<T> pp{col}, cp{ccol};
    uint64_t best = 0, cnt = 0, best1 = 0, cnt1 = 0, best2 = 0, cnt2 = 0;
#pragma unroll 1
    for (int j = j0; j < n; ++j) {
        if (j <= m) continue;
        LdsSink<T> sk{ccol, j < n - 2};
        search_child_to<T, CUSTOM, SYM>(a, band, par, pp, j, sk, j == n - 2, best, cnt, best1, cnt1);
        if (j < n - 2) {  // wave-uniform
            SearchNode<T, CUSTOM, SYM> ch;
            ch.run = sk.run;
            ch.prev = sk.prev;
            ch.mask = sk.mask;
            const uint64_t c = uint64_t(p) + ro(a.binom)[j * (kMaxEvents + 1) + k];  // the child's rank at level k
#pragma unroll 1
            for (int j2 = j + 1; j2 < n; ++j2)
                search_child<T, CUSTOM, SYM>(a, band, ch, cp, j2, c + ro(a.binom)[j2 * (kMaxEvents + 1) + k + 1], best1,
                                             cnt1, best2, cnt2);
        }
    }
    search_publish(a, k, best, cnt);
    search_publish(a, k + 1, best1, cnt1);
    if (a.tail) search_publish(a, k + 2, best2, cnt2);
}

// The head of the search: levels 1 .. K (a.k = K) in ONE launch, one lane per subset of at most
// K free candidates — lanes in (size, colex rank) order — each run from the root through its
// events in index order with the level kernels' per-chain operations, so every score and every
// stored node is the level search's, bit for bit.  It replaces K launches whose first few hold a
// few dozen to a few thousand subsets each and sit at a launch-and-one-event floor of ~10 us
// (DESIGN.md §3).  Level K's subsets whose largest candidate is <= n - 3 are stored as level
// K + 1's parents; one whose largest is n - 2 also scores its child with n - 1 (the tail).
// a.n_child = sum_{k <= K} C(n, k).  Every lane stays to the end (the publish reductions read
// every lane).
// The binomials C(x, y), x <= n, y <= ymax, of the one-lane-per-subset kernels (head, end) in
// LDS: their colex unranking walks up to n candidates per lane, each step a binomial load that
// the next step depends on, so each step waits an LDS latency instead of an L1/L2 one.
// Dynamic LDS of search_binom_lds_bytes(n, ymax); every lane of the block calls it.
__host__ __device__ constexpr size_t search_binom_lds_bytes(int n, int ymax) {
    return sizeof(uint64_t) * size_t(n + 1) * size_t(ymax + 1);
}
__device__ __forceinline__ const uint64_t* search_binom_lds(const Ref15SearchArgs& a, int ymax) {
    extern __shared__ uint64_t sbinom[];
    const int n = a.n_events, w = ymax + 1, tot = (n + 1) * w;
    for (int i = int(threadIdx.x); i < tot; i += int(blockDim.x)) {
        const int x = i / w, y = i - x * w;
        sbinom[i] = a.binom[x * (kMaxEvents + 1) + y];
    }
    __syncthreads();
    return sbinom;
}

template <typename T, bool CUSTOM, bool SYM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SYM ? KF_SEARCH_SYM_WAVES : 3))) void ref15_search_head_kernel(
    const Ref15SearchArgs a) {
    using Node = SearchNode<T, CUSTOM, SYM>;
    constexpr int RP = SYM ? M15::NP : 1, RA = SYM ? M15::NA : 1;
    const int n = a.n_events, K = a.k;
    const uint64_t* C = search_binom_lds(a, K + 1);  // C(n, k) for k <= K, C(c, i) for i <= K
    auto binom = [&](int x, int y) -> uint64_t { return C[x * (K + 2) + y]; };
    const uint64_t g = uint64_t(blockIdx.x) * 64 + threadIdx.x;
    const bool live = g < a.n_child;
    int k = 1;
    uint64_t r = live ? g : 0;
    while (k < K && r >= binom(n, k)) {
        r -= binom(n, k);
        ++k;
    }
    // colex unranking: rank r = sum_i C(c_i, i) over the sorted members c_1 < ... < c_k
    uint64_t sub = 0;
    {
        uint64_t rr = r;
        int c = n - 1;
        for (int i = k; i >= 1; --i) {
            while (binom(c, i) > rr) --c;
            rr -= binom(c, i);
            sub |= uint64_t(1) << c;
            --c;
        }
    }
    uint64_t best = 0, cnt = 0, best1 = 0, cnt1 = 0;
    const DetBand<T> band(a);
    Node nd;
    {
        uint64_t rb = 0, rc = 0;  // a fixed root is itself one of the subsets searched (lane 0 scores it)
        const bool eval = a.root_mask != 0 && g == 0;
        const DetV<T> f = nd.root(a, eval);
        if (eval) search_score(a, band, a.root_mask, f, rb, rc);
        search_publish(a, 0, rb, rc);
    }
    DetV<T> fmax = nd.run;
#pragma unroll 1
    for (uint64_t m = sub; m; m &= m - 1) {
        const int j = __builtin_ctzll(m);
        SearchEvent vs = search_event(a, j, nd.prev);
        vs.final_predict = vs.final_predict && (m & (m - 1)) == 0;  // only the subset itself is scored
        SearchScore<T, CUSTOM> ss;
        ss.kc = a.kc;
#pragma unroll
        for (int ch = 0; ch < Node::NP; ++ch) {
            T Pb[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) Pb[i] = nd.P[6 * ch + i];
            search_pva<T, CUSTOM>(vs, ch, Pb, ss.ok, a.kc);
#pragma unroll
            for (int i = 0; i < 6; ++i) nd.P[6 * ch + i] = Pb[i];
            ss.add_pva(vs, Pb, ch, RP);
        }
#pragma unroll
        for (int ch = 0; ch < Node::NA; ++ch) {
            T Pa[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) Pa[i] = nd.P[6 * Node::NP + 3 * ch + i];
            search_aw<T, CUSTOM>(vs, ch, Pa, ss.ok, a.kc);
#pragma unroll
            for (int i = 0; i < 3; ++i) nd.P[6 * Node::NP + 3 * ch + i] = Pa[i];
            ss.add_aw(vs, Pa, ch, RA);
        }
        nd.run = ss.finish(vs, nd.run, fmax);
        nd.prev = vs.prev;
        nd.mask |= uint64_t(1) << (j + a.shift);
    }
    const int top = sub ? 63 - __builtin_clzll(sub) : -1;
    if (live) {
        search_score(a, band, nd.mask, fmax, best, cnt);
        if (k == K && a.child && top <= n - 3) nd.store(a.child, r);  // level K + 1's parent, at its colex rank
        if (k == K && a.tail && top == n - 2) {  // its only child, plus event n - 1 (size K + 1)
            const SearchEvent vg = search_event(a, n - 1, nd.prev);
            SearchScore<T, CUSTOM> sg;
            sg.kc = a.kc;
#pragma unroll
            for (int ch = 0; ch < Node::NP; ++ch) {
                T Pb[6];
#pragma unroll
                for (int i = 0; i < 6; ++i) Pb[i] = nd.P[6 * ch + i];
                search_pva<T, CUSTOM>(vg, ch, Pb, sg.ok, a.kc);
                sg.add_pva(vg, Pb, ch, RP);
            }
#pragma unroll
            for (int ch = 0; ch < Node::NA; ++ch) {
                T Pa[3];
#pragma unroll
                for (int i = 0; i < 3; ++i) Pa[i] = nd.P[6 * Node::NP + 3 * ch + i];
                search_aw<T, CUSTOM>(vg, ch, Pa, sg.ok, a.kc);
                sg.add_aw(vg, Pa, ch, RA);
            }
            DetV<T> gmax;
            (void)sg.finish(vg, nd.run, gmax);
            search_score(a, band, nd.mask | (uint64_t(1) << (n - 1 + a.shift)), gmax, best1, cnt1);
        }
    }
    // per size: a wave holds lanes of at most a few consecutive sizes
#pragma unroll 1
    for (int kk = 1; kk <= K; ++kk)
        if (__builtin_amdgcn_ballot_w64(live && k == kk) != 0)
            search_publish(a, kk, k == kk ? best : 0, k == kk ? cnt : 0);
    if (a.tail) search_publish(a, K + 1, best1, cnt1);
}

// The end of the search, sizes a.k .. a.k_end (free sizes) in ONE launch, extension-major: a
// subset S of size >= a.k is its (a.k - 1)-prefix P (its smallest members, a node of level
// a.k - 1) plus its extension E (the rest).  For an extension E whose smallest member is e, the
// prefixes are every (a.k - 1)-subset of 0 .. e - 1, which are level a.k - 1's colex ranks
// 0 .. C(e, a.k - 1) - 1, all stored (their largest member is <= n - 3) except, for E = {n - 1},
// the ranks from C(n - 2, a.k - 1) on, whose subsets level a.k - 1's tail scored.  So one wave
// takes one extension and 64 consecutive prefixes: its node loads are one parent block, its
// events and subset size are wave-uniform, and nothing is unranked.  Group i of the host's table
// is extension gblk[i] (a mask of free candidates, ordered by size), its waves start at
// gitem[i].  Every subset's score is the level search's, bit for bit (the level kernels' per-chain
// operations from the same stored node).  It replaces the last levels' launches, which hold a few
// thousand subsets or fewer and sit at the launch-and-one-event floor.
template <typename T, bool CUSTOM, bool SYM>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SYM ? KF_SEARCH_SYM_WAVES : 3))) void ref15_search_end_kernel(
    const Ref15SearchArgs a) {
    if (search_stopped(a)) return;
    using Node = SearchNode<T, CUSTOM, SYM>;
    constexpr int RP = SYM ? M15::NP : 1, RA = SYM ? M15::NA : 1;
    const int n = a.n_events, K0 = a.k;
    const uint64_t w = blockIdx.x;
    int lo = 0, hi = a.n_groups - 1;  // the last group whose first wave is <= w
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (a.gitem[mid] <= w) lo = mid;
        else hi = mid - 1;
    }
    const uint64_t ext = a.gblk[lo];
    const int e = __builtin_ctzll(ext);
    const int ex = e == n - 1 ? n - 2 : e;  // E = {n - 1}: the stored prefixes only
    const uint64_t n_pre = ro(a.binom)[ex * (kMaxEvents + 1) + K0 - 1];
    const uint64_t rp = (w - a.gitem[lo]) * 64 + threadIdx.x;
    const bool live = rp < n_pre;
    uint64_t best = 0, cnt = 0;
    const DetBand<T> band(a);
    Node nd;
    nd.load(a.par, live ? rp : 0);  // a stored node either way (rank 0 is)
    DetV<T> fmax = nd.run;
#pragma unroll 1
    for (uint64_t m = ext; m; m &= m - 1) {
        const int j = __builtin_ctzll(m);
        SearchEvent vs = search_event(a, j, nd.prev);
        vs.final_predict = vs.final_predict && (m & (m - 1)) == 0;  // only the subset itself is scored
        SearchScore<T, CUSTOM> ss;
        ss.kc = a.kc;
#pragma unroll
        for (int ch = 0; ch < Node::NP; ++ch) {
            T Pb[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) Pb[i] = nd.P[6 * ch + i];
            search_pva<T, CUSTOM>(vs, ch, Pb, ss.ok, a.kc);
#pragma unroll
            for (int i = 0; i < 6; ++i) nd.P[6 * ch + i] = Pb[i];
            ss.add_pva(vs, Pb, ch, RP);
        }
#pragma unroll
        for (int ch = 0; ch < Node::NA; ++ch) {
            T Pa[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) Pa[i] = nd.P[6 * Node::NP + 3 * ch + i];
            search_aw<T, CUSTOM>(vs, ch, Pa, ss.ok, a.kc);
#pragma unroll
            for (int i = 0; i < 3; ++i) nd.P[6 * Node::NP + 3 * ch + i] = Pa[i];
            ss.add_aw(vs, Pa, ch, RA);
        }
        nd.run = ss.finish(vs, nd.run, fmax);
        nd.prev = vs.prev;
        nd.mask |= uint64_t(1) << (j + a.shift);
    }
    if (live) search_score(a, band, nd.mask, fmax, best, cnt);
    search_publish(a, K0 - 1 + __builtin_popcountll(ext), best, cnt);
}

// Child-major: one wave per (parent block of 64, child event) work item, one child per lane,
// so no lane walks a long list of children (the narrow levels, where few parents have many
// children each).  Items are ordered by parent block, then j, and dealt to the XCDs in
// contiguous ranges, so the items that read one parent block run back to back on one XCD and
// re-read it from that XCD's L2.  Blocks are grouped by their first parent's largest event v
// (non-decreasing in colex order); a block of group v has items j = v + 1 .. n - 1.
// PAIR (the axis-symmetric search, KF_OPT_SEARCH_PAIR): levels k and k + 1 in one launch — each
// lane's child j (level k) computed into its LDS column, never stored, then that child's children
// j2 > j (level k + 1) from the column, stored as the next launch's parents, as the parent-major
// pair kernel does; the items keep this kernel's parallelism (a parent block per child event).
template <typename T, bool CUSTOM, bool SYM, bool PAIR = false>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(SYM ? KF_SEARCH_SYM_WAVES : 3))) void ref15_search_cm_kernel(const Ref15SearchArgs a,
                                                                                                     uint64_t n_items) {
    if (search_stopped(a)) return;
    const uint64_t per_xcd = (n_items + 7) / 8;
    const uint64_t item = uint64_t(blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    if (item >= n_items) return;
    const int n = a.n_events, k = a.k;
    ro_u64* C = ro(a.binom);
    auto binom = [&](int x, int y) -> uint64_t { return x < 0 ? (y == 0 ? 1 : 0) : C[x * (kMaxEvents + 1) + y]; };
    // the item's group (the host's table in the kernel arguments: a binary search over
    // constant-cache loads, instead of a walk whose every step waited on a binomial load)
    int v = -1;
    uint64_t blk = 0;
    int j = int(item);  // k == 1: item j is the root's child j
    if (k > 1) {
        int lo = 0, hi = a.n_groups - 1;  // the last group whose first item is <= item
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (a.gitem[mid] <= item) lo = mid;
            else hi = mid - 1;
        }
        v = a.v_lo + lo;
        const uint32_t r = uint32_t(item - a.gitem[lo]), w = uint32_t(n - 1 - v);  // r < 2^31 (host check)
        const uint32_t q = r / w;
        blk = a.gblk[lo] + q;
        j = v + 1 + int(r - q * w);
    }
    const uint64_t p = blk * 64 + threadIdx.x;
    if (p >= a.n_par) return;
    const DetBand<T> band(a);
    SearchNode<T, CUSTOM, SYM> par;
    if (k == 1) {
        uint64_t rb = 0, rc = 0;  // a fixed root is itself one of the subsets searched (item 0 scores it)
        const bool eval = a.root_mask != 0 && item == 0;
        const DetV<T> f = par.root(a, eval);
        if (eval) search_score(a, band, a.root_mask, f, rb, rc);
        search_publish(a, 0, rb, rc);
    } else {
        par.load(a.par, p);
    }
    uint64_t best = 0, cnt = 0, best1 = 0, cnt1 = 0;
    if constexpr (PAIR) {
        constexpr int NR = SearchNode<T, CUSTOM, SYM>::NR;
        __shared__ T sC[NR * 64];
        T* ccol = sC + threadIdx.x;
        uint64_t best2 = 0, cnt2 = 0;
        if (par.max_event(a.shift) < j) {
            LdsSink<T> sk{ccol, j < n - 2};
            // a child holding n - 2 has the one child adding n - 1: its tail, size k + 1
            search_child_to<T, CUSTOM, SYM>(a, band, par, ParRegs<T>{par.P}, j, sk, j == n - 2, best, cnt, best1, cnt1);
            if (j < n - 2) {  // wave-uniform (j is)
                SearchNode<T, CUSTOM, SYM> ch;
                ch.run = sk.run;
                ch.prev = sk.prev;
                ch.mask = sk.mask;
                const uint64_t c = p + binom(j, k);  // the child's rank at level k
#pragma unroll 1
                for (int j2 = j + 1; j2 < n; ++j2)
                    search_child<T, CUSTOM, SYM>(a, band, ch, ParLds<T>{ccol}, j2, c + binom(j2, k + 1), best1, cnt1,
                                                 best2, cnt2);
            }
        }
        search_publish(a, k, best, cnt);
        search_publish(a, k + 1, best1, cnt1);
        if (a.tail) search_publish(a, k + 2, best2, cnt2);
    } else {
        if (par.max_event(a.shift) < j)
            search_child<T, CUSTOM, SYM>(a, band, par, ParRegs<T>{par.P}, j, p + binom(j, k), best, cnt, best1, cnt1);
        search_publish(a, a.k, best, cnt);
        if (a.tail) search_publish(a, a.k + 1, best1, cnt1);
    }
}

// ------------------------------------------------------------------------------------
// Scheduler scoring and the rate-decimated greedy driver (kf_workers.py:99-213, 826-957).
// ------------------------------------------------------------------------------------
template <typename T, bool CUSTOM>
__device__ __forceinline__ T cov_trace(const Ref15<T, CUSTOM>& s) {
    T tr = T(0);
#pragma unroll
    for (int i = 0; i < 3; ++i) tr += s.pva[i][0] + s.pva[i][3] + s.pva[i][5];
#pragma unroll
    for (int i = 0; i < 3; ++i) tr += s.aw[i][0] + s.aw[i][2];
    return tr;
}

// trace of Scheduler.cov_matrix (kf_workers.py:112-147) for one candidate sensor.  The first
// row of both H_gps and H_imu is e_0 (pos_x), with R[0,0] = 3 (GPS) or 50 (IMU); a full update
// uses every row.  The state vector is not needed, so a zero one is carried through.
template <typename T, bool CUSTOM>
__device__ __forceinline__ Ref15<T, CUSTOM> posterior(const Ref15<T, CUSTOM>& s0, int type, bool full) {
    Ref15<T, CUSTOM> c = s0;
#pragma unroll
    for (int i = 0; i < 15; ++i) c.x[i] = T(0);
    if (!full) {
        T xb[3] = {T(0), T(0), T(0)};
        const T z[1] = {T(0)};
        T q[3], Rp[6], rg;
        pva_noise<CUSTOM, M15>(s0.kc, 0, q, Rp, rg);
        const T R[1] = {type == kGps ? rg : Rp[0]};
        sel_update<3, 1, true, T, kRefNewton, true, kRefJoseph<T>, kRefGainR>(xb, c.pva[0], z, R);
    } else if (type == kGps) {
        const T z[3] = {T(0), T(0), T(0)};
        c.update_gps(z);
    } else {
        T imu[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) imu[i] = T(0);
        c.update_imu(imu, T(0));
    }
    return c;
}

template <typename T, bool CUSTOM>
__device__ __forceinline__ T posterior_trace(const Ref15<T, CUSTOM>& s0, int type, bool full) {
    return cov_trace(posterior(s0, type, full));
}

// One scalar measurement of state k of a chain block with variance r: P -= P e_k e_k^T P / (P_kk + r)
// (Scheduler.cov_matrix's Sigma - K H Sigma for a one-row H, kf_workers.py:121-147)
template <int NB, typename T>
__device__ __forceinline__ void chain_scalar_update(T (&Pb)[NB * (NB + 1) / 2], int k, T r) {
    T g[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) g[i] = Pb[tri<NB>(i, k)];
    const T inv = T(1) / (g[k] + r);
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = i; j < NB; ++j) Pb[tri<NB>(i, j)] = fmaT(-g[i] * inv, g[j], Pb[tri<NB>(i, j)]);
}

// Scheduler.cov_matrix(S, Sigma, R, H) for any set S of measurement rows (kf_workers.py:121-138:
// H_hat = H[S], R_hat = R[S, S]).  H's rows select states and R is diagonal, so the rows are
// independent measurements and, P being block-diagonal over the chains, each chain takes its own
// rows: sequential scalar updates in row order give the joint update's value.  mask bit i = row
// i + 1 of the sensor's H (GPS: pos_x, pos_y, pos_z; IMU: state i).
template <typename T, bool CUSTOM>
__device__ __forceinline__ Ref15<T, CUSTOM> posterior_rows(const Ref15<T, CUSTOM>& s0, int type, uint32_t mask) {
    Ref15<T, CUSTOM> c = s0;
#pragma unroll
    for (int ch = 0; ch < M15::NP; ++ch) {
        T q[3], Rp[6], rg;
        pva_noise<CUSTOM, M15>(s0.kc, ch, q, Rp, rg);
        if (type == kGps) {
            if (mask >> ch & 1u) chain_scalar_update<3>(c.pva[ch], 0, rg);
        } else {
            const T r[3] = {Rp[0], Rp[3], Rp[5]};
#pragma unroll
            for (int k = 0; k < 3; ++k)
                if (mask >> M15::pva(ch, k) & 1u) chain_scalar_update<3>(c.pva[ch], k, r[k]);
        }
    }
    if (type != kGps) {
#pragma unroll
        for (int ch = 0; ch < M15::NA; ++ch) {
            T q[2], Ra[3];
            aw_noise<CUSTOM, M15>(s0.kc, ch, q, Ra);
            const T r[2] = {Ra[0], Ra[2]};
#pragma unroll
            for (int k = 0; k < 2; ++k)
                if (mask >> M15::aw(ch, k) & 1u) chain_scalar_update<2>(c.aw[ch], k, r[k]);
        }
    }
    return c;
}

// The greedy scheduler's gain (S = [1]): only the x-axis (pos, vel, acc) block changes, so the
// trace is the current one with that block's diagonal replaced — no copy of the whole state.
template <typename T, bool CUSTOM>
__device__ __forceinline__ T first_row_gain(const Ref15<T, CUSTOM>& s, int type) {
    T p[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) p[k] = s.pva[0][k];
    T xb[3] = {T(0), T(0), T(0)};
    const T z[1] = {T(0)};
    T q[3], Rp[6], rg;
    pva_noise<CUSTOM, M15>(s.kc, 0, q, Rp, rg);
    const T R[1] = {type == kGps ? rg : Rp[0]};
    sel_update<3, 1, true, T, kRefNewton, true, kRefJoseph<T>, kRefGainR>(xb, p, z, R);
    T tr = p[0] + p[3] + p[5];
#pragma unroll
    for (int i = 1; i < 3; ++i) tr += s.pva[i][0] + s.pva[i][3] + s.pva[i][5];
#pragma unroll
    for (int i = 0; i < 3; ++i) tr += s.aw[i][0] + s.aw[i][2];
    return tr;
}

template <typename T, bool CUSTOM>
__global__ __launch_bounds__(kBlock) void ref15_score_kernel(const Ref15ScoreArgs a) {
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(a.B) * uint32_t(sizeof(T));
    const uint32_t rb_post = a.post ? rb : 0u;
    Ref15<T, CUSTOM> s;
    s.kc = a.kc;
    s.load(a.x, a.P, rb, off);
    for (int c = 0; c < a.n_types; ++c) {
        const Ref15<T, CUSTOM> p = a.rows ? posterior_rows(s, int(a.types[c]), a.masks[c])
                                          : posterior(s, int(a.types[c]), a.full != 0);
        stb(a.gain, c, rb, off, cov_trace(p));
        p.store_cov(a.post, int64_t(c) * 27, rb_post, off);
    }
}

// Scheduler.random_schedule (kf_workers.py:188-193) is np.random.choice(len(queue)) on NumPy's
// global legacy RandomState: randint(0, n) by masked rejection on 32-bit MT19937 outputs (n = 1
// takes no output; otherwise mask = the smallest 2^k - 1 >= n - 1, outputs & mask until one is
// <= n - 1).  The caller hands each filter its column of the generator's raw outputs
// (words[n_words][B]); wp counts the ones taken.  Returns the draw, or -1 when the column ran out.
__device__ __forceinline__ int legacy_choice(const uint32_t* words, int n_words, int64_t B, int64_t f, int& wp, int n) {
    const uint32_t rng = uint32_t(n - 1);
    if (rng == 0) return 0;
    uint32_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    while (wp < n_words) {
        const uint32_t v = words[int64_t(wp++) * B + f] & mask;
        if (v <= rng) return int(v);
    }
    return -1;
}

// the r-th queued event of a queue that began at event `first`: every event from there on that is
// not padding was queued (a trigger ends the queue; an empty queue's trigger is its only event)
__device__ __forceinline__ int queued_event(const uint8_t* etype, int64_t B, int64_t f, int first, int r) {
    for (int ev = first;; ++ev)
        if (etype[int64_t(ev) * B + f] != 255 && r-- == 0) return ev;
}

// The greedy pick needs no scan of the queue: a candidate's gain depends only on its sensor
// type and the current covariance, so the first candidate with the largest gain is the first
// queued GPS fix or the first queued other event (ties: whichever came first; a NaN gain is
// never picked, and with none pickable the queue's first event is, as the reference's loop
// leaves best_i at its start).  Each lane tracks those two candidates (index, type, time) as
// events are queued, and reads the payload of the picked one only.
template <typename T, bool CUSTOM>
struct SchedLane {
    Ref15<T, CUSTOM> s;
    int32_t st;
    double prev, period;
    int q_len = 0, nsel = 0;
    // per class (0: GPS fix, 1: any other event) the first queued event's index (-1: none),
    // type and time; named scalars, not arrays (an array indexed by a runtime class went to
    // scratch memory)
    int qi0 = -1, qi1 = -1, qt0 = 0, qt1 = 0;
    double qtime0 = 0.0, qtime1 = 0.0;
    int q_first = 0, wp = 0;  // random selection: the queue's first event, generator outputs taken (-1: ran out)

    // event i (type ty at time ti) of filter f (kf_workers.py:870-957)
    __device__ __forceinline__ void event(const Ref15SchedArgs& a, int64_t f, int i, int ty, double ti) {
        if (ty == 255 || wp < 0) return;  // padding of a ragged stream; a random run out of draws
        const int64_t B = a.B;
        const bool gps = ty == kGps;
        const bool window = ti - prev < period;  // still inside the window: queue it
        if (window || q_len == 0) {  // a trigger with an empty queue is its own candidate
            if (q_len == 0) q_first = i;
            if (gps && qi0 < 0) {
                qi0 = i;
                qt0 = ty;
                qtime0 = ti;
            }
            if (!gps && qi1 < 0) {
                qi1 = i;
                qt1 = ty;
                qtime1 = ti;
            }
            ++q_len;
            if (window) return;
        }
        // greedy_schedule (kf_workers.py:195-213); with one class queued its first event is
        // the pick whatever the gain (a NaN gain leaves the queue's first, the same event)
        bool pick0 = qi0 >= 0;
        if (qi0 >= 0 && qi1 >= 0 && !a.words) {
            const T g0 = first_row_gain(s, kGps), g1 = first_row_gain(s, kImu);
            const bool v0 = g0 == g0, v1 = g1 == g1;
            if (v0 && v1) pick0 = g0 > g1 ? true : (g1 > g0 ? false : qi0 < qi1);
            else if (v0 != v1) pick0 = v0;
            else pick0 = qi0 < qi1;  // the queue's first
        }
        int sel = pick0 ? qi0 : qi1;
        double tsel = pick0 ? qtime0 : qtime1;
        int tsel_type = pick0 ? qt0 : qt1;
        if (a.words) {  // random_schedule: any queued event, drawn as the reference draws it
            const int r = legacy_choice(a.words, a.n_words, B, f, wp, q_len);
            if (r < 0) {
                wp = -1;
                return;
            }
            sel = queued_event(a.etype, B, f, q_first, r);
            tsel = a.t[int64_t(sel) * B + f];
            tsel_type = a.etype[int64_t(sel) * B + f];
        }
        q_len = 0;
        qi0 = qi1 = -1;
        T pay[9];
        // the selected event differs per lane: plain 64-bit addressing (a buffer descriptor per
        // lane would be a waterfall loop)
        // [T][9][B] rows, or [T][B][pay_rec] records (kf_run_scheduled_rec)
        const T* ps = static_cast<const T*>(a.payload) +
                      (a.pay_rec ? (int64_t(sel) * B + f) * a.pay_rec : int64_t(sel) * 9 * B + f);
        const int64_t pstep = a.pay_rec ? 1 : B;
#pragma unroll
        for (int k = 0; k < 9; ++k) pay[k] = ps[int64_t(k) * pstep];
        bool ok = true;
        s.template event<false>(tsel_type, T(tsel - prev), pay, false, T(0), ok);
        if (!ok) {
            st = kNotSpd;
            s.fill_nan();
        }
        if (a.traj) {
            T* tro = static_cast<T*>(a.traj) + int64_t(nsel) * 6 * B + f;
#pragma unroll
            for (int k = 0; k < 6; ++k) tro[int64_t(k) * B] = s.x[k];
        }
        if (a.logdet) static_cast<T*>(a.logdet)[int64_t(nsel) * B + f] = s.logdet();
        if (a.sel_time) a.sel_time[int64_t(nsel) * B + f] = tsel;
        ++nsel;
        prev = tsel;
    }
};

// random_schedule's picks alone (kf_sched_random_picks): the windows and the draws need only the
// event times and types (the windows open at the picked events' times, the draws consume the
// filter's generator outputs), so a lane per filter walks its stream with no filter arithmetic
// and writes the picked event indices and times; the caller runs the picked events through the
// event engine (for one filter over a long log: kf_run_events' time-parallel route).  Event
// types and times ride an 8-deep register ring; the generator outputs a 4-deep one.
template <int D>
__device__ __forceinline__ void ring_shift(int (&ty)[D], double (&tt)[D]) {
#pragma unroll
    for (int k = 0; k + 1 < D; ++k) {
        ty[k] = ty[k + 1];
        tt[k] = tt[k + 1];
    }
}
__global__ __launch_bounds__(kBlock) void ref15_random_picks_kernel(const Ref15SchedArgs a, int32_t* pick) {
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const int64_t B = a.B;
    constexpr int D = 8;
    int ty[D];
    double tt[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        ty[k] = k < a.T ? int(a.etype[int64_t(k) * B + f]) : 255;
        tt[k] = k < a.T ? a.t[int64_t(k) * B + f] : 0.0;
    }
    double prev = a.prev_time[f];
    const double period = 1.0 / (a.freq ? a.freq[f] : a.freq_all);  // kf_workers.py:880
    int q_len = 0, q_first = 0, nsel = 0, wp = 0;
    bool q_gap = false;  // a padding event inside the queue: the r-th queued event needs a scan
    for (int i = 0; i < a.T; ++i) {
        const int ty0 = ty[0];
        const double t0 = tt[0];
        ring_shift(ty, tt);
        const int nx = i + D;
        ty[D - 1] = nx < a.T ? int(a.etype[int64_t(nx) * B + f]) : 255;
        tt[D - 1] = nx < a.T ? a.t[int64_t(nx) * B + f] : 0.0;
        if (ty0 == 255) {  // padding: never queued (a queue it falls inside is no longer contiguous)
            q_gap = q_gap || q_len > 0;
            continue;
        }
        const bool window = t0 - prev < period;
        if (window || q_len == 0) {
            if (q_len == 0) {
                q_first = i;
                q_gap = false;
            }
            ++q_len;
            if (window) continue;
        }
        const int r = legacy_choice(a.words, a.n_words, B, f, wp, q_len);
        if (r < 0) {
            wp = -1;
            break;
        }
        const int sel = q_gap ? queued_event(a.etype, B, f, q_first, r) : q_first + r;
        const double ts = sel == i ? t0 : a.t[int64_t(sel) * B + f];
        pick[int64_t(nsel) * B + f] = sel;
        a.sel_time[int64_t(nsel) * B + f] = ts;
        ++nsel;
        prev = ts;
        q_len = 0;
    }
    a.n_sel[f] = nsel;
    a.words_used[f] = wp;
}

#ifndef KF_SCHED_WAVES
#define KF_SCHED_WAVES 2
#endif
// Any B: the next event's type and time are loaded one event ahead in registers.
template <typename T, bool CUSTOM>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KF_SCHED_WAVES))) void ref15_sched_kernel(
    const Ref15SchedArgs a) {
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    if (a.only && !a.only[f]) return;  // the two-pass run's fallback: flagged filters only
    const int64_t B = a.B;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(B) * uint32_t(sizeof(T));
    SchedLane<T, CUSTOM> L;
    L.s.kc = a.kc;
    L.s.load(a.x, a.P, rb, off);
    L.st = a.status[f];
    L.prev = a.prev_time[f];
    L.period = 1.0 / (a.freq ? a.freq[f] : a.freq_all);  // kf_workers.py:880
    int tyn = a.T > 0 ? a.etype[f] : 255;
    double tn = a.T > 0 ? a.t[f] : 0.0;
    for (int i = 0; i < a.T; ++i) {
        const int ty = tyn;
        const double ti = tn;
        if (i + 1 < a.T) {
            tyn = a.etype[int64_t(i + 1) * B + f];
            tn = a.t[int64_t(i + 1) * B + f];
        }
        L.event(a, f, i, ty, ti);
    }
    if (a.n_sel) a.n_sel[f] = L.nsel;
    if (a.words_used) a.words_used[f] = L.wp;
    L.s.store(a.x, a.P, rb, off);
    a.status[f] = L.st;
}

// B % 64 == 0: the event types and times travel HBM -> LDS by buffer_load ... lds, kSchedChunk
// events at a time into one of two per-wave images while the previous chunk is consumed (the
// queueing iterations are a few instructions each, so a register prefetch one event ahead
// waited a memory latency per event, and a deeper one did not fit the registers).
//   image: t rows [kSchedChunk][64] f64, then etype rows [kSchedChunk][64] u8
#ifndef KF_SCHED_CHUNK
#define KF_SCHED_CHUNK 16
#endif
constexpr int kSchedChunk = KF_SCHED_CHUNK;
constexpr int kSchedImg = kSchedChunk * 512 + kSchedChunk * 64;
template <typename T, bool CUSTOM>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(KF_SCHED_WAVES))) void ref15_sched_lds_kernel(
    const Ref15SchedArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[(kBlock / 64) * 2 * kSchedImg];
    const int lane = int(threadIdx.x & 63);
    const int wave = wave_uniform(int(threadIdx.x >> 6));
    const int64_t f0 = int64_t(blockIdx.x) * kBlock + int64_t(wave) * 64;
    if (f0 >= a.B) return;  // whole waves (B % 64 == 0)
    const int64_t f = f0 + lane;
    const int64_t B = a.B;
    unsigned char* const img0 = lds + wave * 2 * kSchedImg;
    const uint32_t off = uint32_t(f) * uint32_t(sizeof(T));
    const uint32_t rb = uint32_t(B) * uint32_t(sizeof(T));
    SchedLane<T, CUSTOM> L;
    L.s.kc = a.kc;
    L.s.load(a.x, a.P, rb, off);
    L.st = a.status[f];
    L.prev = a.prev_time[f];
    L.period = 1.0 / (a.freq ? a.freq[f] : a.freq_all);
    waitcnt<vmcnt_imm(0)>();
    // t: one 16-B-per-lane DMA moves two rows (lanes 0-31 row r, 32-63 row r + 1); etype: one
    // moves 16 rows of 64 bytes (4 lanes per row)
    const uint32_t voff_t = uint32_t(lane >> 5) * uint32_t(B) * 8u + uint32_t(lane & 31) * 16u;
    const uint32_t voff_e = uint32_t(lane >> 2) * uint32_t(B) + uint32_t(lane & 3) * 16u;
    auto issue = [&](int c, unsigned char* img) {
        const int r0 = c * kSchedChunk;
        const int nr = a.T - r0 < kSchedChunk ? a.T - r0 : kSchedChunk;  // rows of this chunk (>= 1)
#pragma unroll
        for (int k = 0; k < kSchedChunk / 2; ++k) {
            if (2 * k >= nr) break;  // wave-uniform
            const char* tb = reinterpret_cast<const char*>(a.t) + (int64_t(r0 + 2 * k) * B + f0) * 8;
            const uint32_t span = 2 * k + 1 < nr ? uint32_t(B) * 8u + 512u : 512u;
            lds_dma16(bytes_rsrc(tb, span), img + k * 1024, voff_t, 0);
        }
        const char* eb = reinterpret_cast<const char*>(a.etype) + int64_t(r0) * B + f0;
        lds_dma16(bytes_rsrc(eb, uint32_t(nr - 1) * uint32_t(B) + 64u), img + kSchedChunk * 512, voff_e, 0);
    };
    const int nch = (a.T + kSchedChunk - 1) / kSchedChunk;
    if (nch > 0) issue(0, img0);
    for (int c = 0; c < nch; ++c) {
        // this chunk's image has landed, the other image's reads are done (vmcnt also counts
        // the stores of the chunk before: once per chunk)
        waitcnt<0>();
        unsigned char* const img = img0 + (c & 1) * kSchedImg;
        if (c + 1 < nch) issue(c + 1, img0 + ((c + 1) & 1) * kSchedImg);
        const double* ti_img = reinterpret_cast<const double*>(img) + lane;
        const unsigned char* ty_img = img + kSchedChunk * 512 + lane;
        const int r0 = c * kSchedChunk;
        const int nr = a.T - r0 < kSchedChunk ? a.T - r0 : kSchedChunk;
#pragma unroll 1
        for (int d = 0; d < nr; ++d) L.event(a, f, r0 + d, int(ty_img[d * 64]), ti_img[d * 64]);
    }
    if (a.n_sel) a.n_sel[f] = L.nsel;
    if (a.words_used) a.words_used[f] = L.wp;
    L.s.store(a.x, a.P, rb, off);
    a.status[f] = L.st;
}


// ------------------------------------------------------------------------------------
// Two-pass scheduled filter.  The greedy pick (kf_workers.py:195-213) compares two posterior
// traces tr(P) - |P e_0|^2 / (P_00 + R) whose only difference is R: R_gps[0] for a fix, R_imu[0]
// for any other event.  Wherever the covariance is finite the pick is therefore decided by the
// constants alone — the larger R gives the larger trace — so the windows, the queue and the
// picks need no covariance at all.  Pass 1 (ref15_pick_kernel) runs them from the event times
// and types only (registers for a handful of scalars, 8 waves per SIMD) and writes each pick as
// code << 24 | event index (code: event type, both-classes-queued bit, fix-first bit) with its
// time.  Pass 2 (ref15_apply_kernel) runs the picked events as the fused kernel's apply does,
// the picked payload rows gathered HBM -> LDS by DMA one pick ahead, and at every pick made with
// both classes queued it evaluates the two gains on the covariance, as the fused kernel does: if
// the greedy rule disagrees (a NaN covariance, a rounding tie) the filter is flagged and left
// untouched, and the fused kernel reruns exactly those filters.  Outputs are the fused kernel's.
// ------------------------------------------------------------------------------------
constexpr int kPickBoth = 0x10, kPickGpsFirst = 0x20;

// payload element i of this lane in the apply pass's image, read from LDS where the update uses
// it.  Rows ([T][9][B]): [9][64] slots of kSlot bytes per lane.  Records ([T][B][rec],
// REC): the first 9 values of the lane's record as 16-B chunks, [chunk][64][16 B].
template <typename T, bool REC = false>
struct LdsGathered {
    const unsigned char* img;  // image base + this lane's slot (+ its value's offset in the slot)
    static constexpr int kSlot = REC || sizeof(T) == 8 ? 16 : 4;
    static constexpr int kChunks = (9 * int(sizeof(T)) + 15) / 16;  // REC: 16-B chunks per record
    __device__ __forceinline__ T operator[](int i) const {
        constexpr int W = int(sizeof(T));
        if constexpr (REC) return *reinterpret_cast<const T*>(img + ((i * W) >> 4) * 1024 + ((i * W) & 15));
        else return *reinterpret_cast<const T*>(img + i * 64 * kSlot);
    }
};

#ifndef KF_PICK_CHUNK
#define KF_PICK_CHUNK 8
#endif
#ifndef KF_APPLY_IMAGES
#define KF_APPLY_IMAGES 1  // payload images per wave of the two-pass apply (2: two-wave groups)
#endif
#ifndef KF_REC_IMAGES
#define KF_REC_IMAGES 1  // payload images per wave of the apply pass over payload records (2: A/B)
#endif
#ifndef KF_APPLY_PROBE
#define KF_APPLY_PROBE 0  // 1 / 2 / 3: apply-pass timing probes for in-process A/B builds (tools/ab_inproc.py)
#endif
// events per LDS image of the pick pass: its lanes hold a few scalars, so the LDS, not the
// registers, sets its waves per SIMD (8 events: 4 workgroups of 4 waves per CU)
constexpr int kPickChunk = KF_PICK_CHUNK;
constexpr int kPickImg = kPickChunk * 512 + kPickChunk * 64;
// The pick pass of one wave (filters f0 .. f0 + 63) with its two staging images at img0
// (2 * kPickImg bytes); returns this lane's pick count.  Every store is issued on return.
// RND: random_schedule's pick (a.words) instead of the greedy rule's; picks carry no
// both-classes bit, so the apply pass checks nothing and flags no filter.
template <bool RND = false>
__device__ __forceinline__ int pick_phase(const Ref15SchedArgs& a, int lane, int64_t f0, unsigned char* img0) {
    constexpr int kSchedChunk = kPickChunk, kSchedImg = kPickImg;  // the fused kernel's staging, resized
    static_assert(kSchedChunk % 2 == 0 && kSchedChunk <= 16, "t rows move in pairs; etype rows 4 lanes each");
    const int64_t f = f0 + lane;
    const int64_t B = a.B;
    double prev = a.prev_time[f];
    const double period = 1.0 / (a.freq ? a.freq[f] : a.freq_all);  // kf_workers.py:880
    int q_len = 0, nsel = 0, qi0 = -1, qi1 = -1, qt0 = 0, qt1 = 0;
    double qtime0 = 0.0, qtime1 = 0.0;
    int q_first = 0, wp = 0;  // RND: the queue's first event, generator outputs taken (-1: ran out)
    waitcnt<vmcnt_imm(0)>();
    const uint32_t voff_t = uint32_t(lane >> 5) * uint32_t(B) * 8u + uint32_t(lane & 31) * 16u;
    const uint32_t voff_e = uint32_t(lane >> 2) * uint32_t(B) + uint32_t(lane & 3) * 16u;
    auto issue = [&](int c, unsigned char* img) {
        const int r0 = c * kSchedChunk;
        const int nr = a.T - r0 < kSchedChunk ? a.T - r0 : kSchedChunk;
#pragma unroll
        for (int k = 0; k < kSchedChunk / 2; ++k) {
            if (2 * k >= nr) break;  // wave-uniform
            const char* tb = reinterpret_cast<const char*>(a.t) + (int64_t(r0 + 2 * k) * B + f0) * 8;
            const uint32_t span = 2 * k + 1 < nr ? uint32_t(B) * 8u + 512u : 512u;
            lds_dma16(bytes_rsrc(tb, span), img + k * 1024, voff_t, 0);
        }
        // 4 lanes per etype row: the lanes past this chunk's rows would write zeros (their rows
        // are out of the descriptor's range) beyond the image
        const char* eb = reinterpret_cast<const char*>(a.etype) + int64_t(r0) * B + f0;
        if (lane < 4 * kSchedChunk)
            lds_dma16(bytes_rsrc(eb, uint32_t(nr - 1) * uint32_t(B) + 64u), img + kSchedChunk * 512, voff_e, 0);
    };
    const int nch = (a.T + kSchedChunk - 1) / kSchedChunk;
    if (nch > 0) issue(0, img0);
    for (int c = 0; c < nch; ++c) {
        waitcnt<0>();
        unsigned char* const img = img0 + (c & 1) * kSchedImg;
        if (c + 1 < nch) issue(c + 1, img0 + ((c + 1) & 1) * kSchedImg);
        const double* ti_img = reinterpret_cast<const double*>(img) + lane;
        const unsigned char* ty_img = img + kSchedChunk * 512 + lane;
        const int r0 = c * kSchedChunk;
        const int nr = a.T - r0 < kSchedChunk ? a.T - r0 : kSchedChunk;
#pragma unroll 1
        for (int d = 0; d < nr; ++d) {
            const int ty = int(ty_img[d * 64]);
            const double ti = ti_img[d * 64];
            const int i = r0 + d;
            if (ty == 255 || (RND && wp < 0)) continue;  // padding of a ragged stream; out of draws
            const bool gps = ty == kGps;
            const bool window = ti - prev < period;  // SchedLane::event, kf_workers.py:870-957
            if (window || q_len == 0) {
                if (RND && q_len == 0) q_first = i;
                if (gps && qi0 < 0) {
                    qi0 = i;
                    qt0 = ty;
                    qtime0 = ti;
                }
                if (!gps && qi1 < 0) {
                    qi1 = i;
                    qt1 = ty;
                    qtime1 = ti;
                }
                ++q_len;
                if (window) continue;
            }
            const bool both = qi0 >= 0 && qi1 >= 0;
            const bool gps_first = qi0 >= 0 && (qi1 < 0 || qi0 < qi1);
            const bool pick0 = both ? (a.gps_wins > 0 ? true : a.gps_wins == 0 ? false : gps_first) : qi0 >= 0;
            int sel = pick0 ? qi0 : qi1;
            double tsel = pick0 ? qtime0 : qtime1;
            int code = (pick0 ? qt0 : qt1) | (both ? kPickBoth : 0) | (gps_first ? kPickGpsFirst : 0);
            if constexpr (RND) {
                const int r = legacy_choice(a.words, a.n_words, B, f, wp, q_len);
                if (r < 0) {
                    wp = -1;
                    continue;
                }
                sel = queued_event(a.etype, B, f, q_first, r);
                tsel = a.t[int64_t(sel) * B + f];
                code = a.etype[int64_t(sel) * B + f];
            }
            a.picks[int64_t(nsel) * B + f] = (uint32_t(code) << 24) | uint32_t(sel);
            if (a.sel_time && !a.rec_time) a.sel_time[int64_t(nsel) * B + f] = tsel;  // rec_time: the apply pass writes it
            ++nsel;
            prev = tsel;
            q_len = 0;
            qi0 = qi1 = -1;
        }
    }
    if (a.n_sel) a.n_sel[f] = nsel;
    if (RND && a.words_used) a.words_used[f] = wp;
    a.flags[f] = 0;
    return nsel;
}

template <int WAVES, bool RND = false>
__global__ __launch_bounds__(WAVES * 64) void ref15_pick_kernel(const Ref15SchedArgs a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[WAVES * 2 * kPickImg];
    const int lane = int(threadIdx.x & 63);
    const int wave = WAVES == 1 ? 0 : wave_uniform(int(threadIdx.x >> 6));
    const int64_t f0 = int64_t(blockIdx.x) * (WAVES * 64) + int64_t(wave) * 64;
    if (f0 >= a.B) return;  // whole waves (B % 64 == 0)
    const int nsel = pick_phase<RND>(a, lane, f0, lds + wave * 2 * kPickImg);
    if (a.wave_key) {  // the wave's longest pick list, for the apply pass's heaviest-first order
        int S = nsel;
#pragma unroll
        for (int sh = 32; sh >= 1; sh >>= 1) {
            const int o = __shfl_xor(S, sh, 64);
            S = o > S ? o : S;
        }
        if (lane == 0) {
            a.wave_key[f0 >> 6] = uint32_t(S);
            a.wave_id[f0 >> 6] = uint32_t(f0 >> 6);
        }
    }
}

// The one-launch run's wave order: its picks do not exist before the launch, so each wave is
// keyed by its highest processing frequency, which sets its pick count (bit patterns of
// positive floats sort as their values).
__global__ __launch_bounds__(kBlock) void ref15_rate_key_kernel(const Ref15SchedArgs a) {
    const int lane = int(threadIdx.x & 63);
    const int64_t f0 = int64_t(blockIdx.x) * kBlock + int64_t(threadIdx.x >> 6) * 64;
    if (f0 >= a.B) return;  // whole waves (B % 64 == 0)
    float fr = float(a.freq[f0 + lane]);
    fr = fr > 0.0f ? fr : 0.0f;  // NaN and non-positive rates sort last
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
        const float o = __shfl_xor(fr, sh, 64);
        fr = o > fr ? o : fr;
    }
    if (lane == 0) {
        a.wave_key[f0 >> 6] = __float_as_uint(fr);
        a.wave_id[f0 >> 6] = uint32_t(f0 >> 6);
    }
}

// PICK: the wave runs its pick pass first (one launch for both passes: a wave's streaming pick
// phase overlaps the other waves' compute-bound apply phases)
// REC: the payload is [T][B][pay_rec] records (kf_run_scheduled_rec): a lane's 9 values are one
// contiguous 72-B (f64) span, gathered as 16-B chunks, instead of 9 rows B elements apart
// RT: f64 records carry the event's time at rec[9] (KF_OPT_SCHED_REC_TIME): each pick's time
// comes with its gathered record (the 16-B chunk holding payload[8] already spans it) instead of
// a sel_time row read, and this pass writes sel_time; two payload images, so pick q + 1's record
// (and time) is in flight through event q
template <typename T, bool CUSTOM, int WAVES, bool PICK, bool REC = false, bool RT = false>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(3))) void ref15_apply_kernel(
    const Ref15SchedArgs a) {
    static_assert(!RT || (REC && sizeof(T) == 8 && !PICK), "record time: f64 records, two launches");
    constexpr int W = int(sizeof(T));
    // The picked payload is gathered per lane: the picks of a wave's lanes lie on different rows,
    // so with the [T][9][B] rows every gather instruction touches up to 64 cache lines and the
    // address unit, not HBM, bounds the pass.  f64 moves 16 B per lane (the aligned pair holding
    // the lane's value: one instruction per value instead of two dword ones), f32 4 B.  With
    // records (REC) a pick is 5 (f64) / 3 (f32) 16-B chunks of one span, and the pass moves its
    // bytes at the HBM's rate.  One payload image per wave:
    // the next pick's gather is issued once this event's update has read the image, and waited
    // for after the next predict.
    // NIMG = 2: two payload images, pick q + 1's gather issued before event q's predict (a whole
    // event of cover instead of one predict), at the LDS cost of fewer waves per CU
    // (records: 5-KB images, so two fit 12 waves per CU, KF_REC_IMAGES=2: measured no faster)
    constexpr int NIMG = RT ? 2 : PICK ? 1 : REC ? KF_REC_IMAGES : KF_APPLY_IMAGES;
    static_assert(NIMG == 1 || NIMG == 2, "payload images");
    using Gathered = LdsGathered<T, REC>;
    constexpr int GB = Gathered::kSlot;
    constexpr int PAY = REC ? Gathered::kChunks * 1024 : 9 * 64 * GB;  // payload image
    constexpr int NG = REC ? Gathered::kChunks : 9;                     // gather instructions per pick
    constexpr int TM = NIMG * PAY;         // pick times, two rows (q & 1)
    constexpr int PK = TM + 2 * 512;       // picks, three rows (q % 3), 64 u32 each
    constexpr int APPLY_LDS = PK + 3 * 256;
    constexpr int WAVE_LDS = PICK && 2 * kPickImg > APPLY_LDS ? 2 * kPickImg : APPLY_LDS;  // the pick phase's images alias
    constexpr int NST = RT ? 8 : 7;        // traj (6 rows), logdet (RT: sel_time); absent ones dropped by offset
    __shared__ __attribute__((aligned(16))) unsigned char lds[WAVES * WAVE_LDS];
    const int lane = int(threadIdx.x & 63);
    const int wave = WAVES == 1 ? 0 : wave_uniform(int(threadIdx.x >> 6));
    const int64_t slot = int64_t(blockIdx.x) * WAVES + wave;  // the wave's place in the launch
    if (slot * 64 >= a.B) return;  // whole waves (B % 64 == 0)
    // heaviest waves first where the pick pass sorted them (their list lengths differ by rate,
    // and the longest started last set the launch's tail)
    const int64_t f0 = (a.order ? int64_t(wave_uniform(int(a.order[slot]))) : slot) * 64;
    const int64_t f = f0 + lane;
    const int64_t B = a.B;
    unsigned char* const base = lds + wave * WAVE_LDS;
    const uint32_t off = uint32_t(f) * uint32_t(W);
    const uint32_t rb = uint32_t(B) * uint32_t(W);
    int nsel;
    if constexpr (PICK) {
        nsel = pick_phase(a, lane, f0, base);
        waitcnt<vmcnt_imm(0)>();  // its picks are read back below (this wave's own rows)
    } else {
        nsel = a.n_sel[f];
    }
    Ref15<T, CUSTOM> s;
    s.kc = a.kc;
    s.load(a.x, a.P, rb, off);
    int32_t st = a.status[f];
    double prev = a.prev_time[f];
    int S = nsel;  // the wave's longest pick list
#pragma unroll
    for (int sh = 32; sh >= 1; sh >>= 1) {
        const int o = __shfl_xor(S, sh, 64);
        S = o > S ? o : S;
    }
    S = wave_uniform(S);
    waitcnt<vmcnt_imm(0)>();
    // pick r's payload (NG VMEM): a lane past its list reads row 0.  Device pass only: the 16-B
    // form of the builtin is a gfx950 one, and the host pass would drop the kernel's stub.
    auto gather = [&](int r, uint32_t pick) {
#if defined(__HIP_DEVICE_COMPILE__)
        const int64_t col = W == 8 ? (f & ~int64_t(1)) : f;  // f64: the 16-B-aligned pair
        const uint32_t ev = pick & 0xFFFFFFu;
#if KF_APPLY_PROBE == 1  // timing probe (wrong results): every lane gathers lane 0's row
        const int64_t row = __shfl((r < nsel && ev < uint32_t(a.T)) ? int(ev) : 0, 0, 64);
#else
        const int64_t row = (r < nsel && ev < uint32_t(a.T)) ? int64_t(ev) : 0;
#endif
        if constexpr (REC) {  // the record's first kChunks 16-B chunks (within pay_rec * W bytes)
            const char* src = reinterpret_cast<const char*>(a.payload) + (row * B + f) * int64_t(a.pay_rec) * W;
#pragma unroll
            for (int c = 0; c < Gathered::kChunks; ++c)
                __builtin_amdgcn_global_load_lds(src + c * 16,
                                                 (__attribute__((address_space(3))) void*)(base + (r & (NIMG - 1)) * PAY + c * 1024),
                                                 16, 0, 0);
        } else {
            const char* src = reinterpret_cast<const char*>(a.payload) + (row * 9 * B + col) * W;
#pragma unroll
            for (int i = 0; i < 9; ++i)
#if KF_APPLY_PROBE == 2  // timing probe (wrong results): no payload gather
                if (r < 0)
#endif
                    __builtin_amdgcn_global_load_lds(src + int64_t(i) * B * W,
                                                     (__attribute__((address_space(3))) void*)(base + (r & (NIMG - 1)) * PAY + i * 64 * GB),
                                                     Gathered::kSlot, 0, 0);
        }
#else
        (void)r;
        (void)pick;
#endif
    };
    // pick r's time / row r of the picks (1 VMEM each, issued by every wave: past the list a
    // zero-length descriptor, so the waits below can be counted)
    auto issue_time = [&](int r) {
        const char* tb = reinterpret_cast<const char*>(a.sel_time) + (int64_t(r) * B + f0) * 8;
        if (lane < 32) lds_dma16(bytes_rsrc(tb, r < S ? 512u : 0u), base + TM + (r & 1) * 512, uint32_t(lane) * 16u, 0);
    };
    auto issue_picks = [&](int r) {
        const char* pb = reinterpret_cast<const char*>(a.picks) + (int64_t(r) * B + f0) * 4;
        if (lane < 16) lds_dma16(bytes_rsrc(pb, r < S ? 256u : 0u), base + PK + (r % 3) * 256, uint32_t(lane) * 16u, 0);
    };
    auto pick_row = [&](int r) { return reinterpret_cast<const uint32_t*>(base + PK + (r % 3) * 256)[lane]; };
    const unsigned char* const pay0 = base + lane * GB + (!REC && W == 8 ? (lane & 1) * 8 : 0);  // read where used
    if (S > 0) {
        issue_picks(0);
        issue_picks(1);
        if constexpr (!RT) issue_time(0);
        waitcnt<vmcnt_imm(0)>();
        gather(0, pick_row(0));
    }
    bool bad = false;
    for (int q = 0; q < S; ++q) {
        const Gathered pay{pay0 + (q & (NIMG - 1)) * PAY};
        if constexpr (NIMG == 1) {
            // time q and pick row q: older than pick row q + 1, gather q (NG) and event q - 1's stores
            if (q > 0) waitcnt<vmcnt_imm(1 + NG + NST)>();
        } else {
            // time q, pick row q + 1 and gather q: older than event q - 1's stores
            if (q > 0) waitcnt<vmcnt_imm(NST)>();
            // the other image was last read by event q - 1's update
            __builtin_amdgcn_s_waitcnt(lgkmcnt0_imm);
            asm volatile("" ::: "memory");
            if (q + 1 < S) gather(q + 1, pick_row(q + 1));
            // RT: the time is in record q (gather 0 is older than gather 1, when there is one)
            if (RT && q == 0) {
                if (S > 1) waitcnt<vmcnt_imm(NG)>();
                else waitcnt<vmcnt_imm(0)>();
            }
        }
        double tq;
        if constexpr (RT) tq = pay[9];
        else tq = reinterpret_cast<const double*>(base + TM + (q & 1) * 512)[lane];
        const uint32_t pick_c = pick_row(q);
        if constexpr (!RT) issue_time(q + 1);
        issue_picks(q + 2);  // into the slot row q - 1 held
        const bool live = q < nsel;
        const int code = int(pick_c >> 24);
#if KF_APPLY_PROBE == 3  // timing probe (wrong results): lane 0's event type for the wave
        const int type = __shfl(code & 7, 0, 64);
#else
        const int type = code & 7;
#endif
        if (live && !bad && (code & kPickBoth)) {
            // the greedy rule on this covariance (SchedLane::event): the pick pass's choice must
            // be the first candidate with the largest gain
            const T g0 = first_row_gain(s, kGps), g1 = first_row_gain(s, kImu);
            const bool v0 = g0 == g0, v1 = g1 == g1;
            const bool gps_first = (code & kPickGpsFirst) != 0;
            bool pick0;
            if (v0 && v1) pick0 = g0 > g1 ? true : (g1 > g0 ? false : gps_first);
            else if (v0 != v1) pick0 = v0;
            else pick0 = gps_first;
#if KF_APPLY_PROBE == 3
            bad = false && pick0;
#else
            bad = pick0 != (type == kGps);
#endif
        }
        const bool run = live && !bad;
        const T dt = T(tq - prev);
        if (run) s.predict(dt);  // Chains::event, split around the payload wait
        if constexpr (NIMG == 1) {
            // gather q: older than event q - 1's stores, time q + 1 and pick row q + 2
            if (q > 0) waitcnt<vmcnt_imm(NST + 2)>();
            else waitcnt<vmcnt_imm(2)>();
        } else if (!RT && q == 0) {
            // gather 0: older than gather 1 (when there is one), time 1 and pick row 2
            if (S > 1) waitcnt<vmcnt_imm(NG + 2)>();
            else waitcnt<vmcnt_imm(2)>();
        }
        if (run && (type == kGps || type == kImu)) {
            bool ok;
            if (type == kGps) {
                const T z[3] = {pay[0], pay[1], pay[2]};  // (easting, northing, altitude)
                ok = s.template update_gps<false>(z);
            } else {
                ok = s.template update_imu<false>(pay, dt);
            }
            if (!ok) {
                st = kNotSpd;
                s.fill_nan();
            }
        }
        if (run) prev = tq;
        // the image's reads are done: gather q + 1 into it (its pick row landed before gather q;
        // reading the payload into registers first, to issue the gather before the update, cost
        // 10 spilled registers and measured 5.98 vs 5.45 ms)
        if constexpr (NIMG == 1) {
            __builtin_amdgcn_s_waitcnt(lgkmcnt0_imm);
            asm volatile("" ::: "memory");
            if (q + 1 < S) gather(q + 1, pick_row(q + 1));
        }
        // a record's descriptor per pick (the records of the whole run exceed 32-bit offsets)
        const uint32_t vo = live ? off : kDropOffset;
        const auto r_tr = span_rsrc(a.traj, int64_t(q) * 6, rb, 6u);
#pragma unroll
        for (int k = 0; k < 6; ++k) stv(r_tr, uint32_t(k) * rb + vo, s.x[k]);
        stv(span_rsrc(a.logdet, q, rb, 1u), vo, s.logdet());
        if constexpr (RT) stv(span_rsrc(a.sel_time, q, rb, 1u), vo, tq);
    }
    a.flags[f] = bad ? 1 : 0;
    if (bad) return;  // the fused kernel reruns this filter from the handle's state
    s.store(a.x, a.P, rb, off);
    a.status[f] = st;
}

// kf_search_combos' counters (best[], n_acc[]) to the handle's mapped host buffer (vector
// stores, made visible to the host before the kernel ends): after a level of a non-exhaustive
// search (peek), and at the end, where they are also zeroed for the next search on the stream.
__global__ __launch_bounds__(256) void search_finish_kernel(uint64_t* counters, uint64_t* host, int n, bool zero) {
    const int i = int(threadIdx.x);
    if (i < n) {
        host[i] = counters[i];
        if (zero) counters[i] = 0;
    }
    __threadfence_system();
}
}  // namespace

// kernel<..., CUSTOM> for a launch: the reference's constants (kc == nullptr) or the handle's
#define KF_CUSTOM_DISPATCH(kc, ...)         \
    do {                                    \
        if (kc) {                           \
            constexpr bool CUSTOM = true;   \
            __VA_ARGS__;                    \
        } else {                            \
            constexpr bool CUSTOM = false;  \
            __VA_ARGS__;                    \
        }                                   \
    } while (0)

hipError_t launch_ref15_random_picks(const Ref15SchedArgs& a, int32_t* pick, hipStream_t stream) {
    if (a.B <= 0 || a.T < 0 || !a.words || !a.words_used || !a.n_sel || !a.sel_time || !pick) return hipErrorInvalidValue;
    ref15_random_picks_kernel<<<dim3(unsigned((a.B + kBlock - 1) / kBlock)), kBlock, 0, stream>>>(a, pick);
    return hipGetLastError();
}

hipError_t launch_ref15_score(bool f64, const Ref15ScoreArgs& a, hipStream_t stream) {
    const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
    KF_CUSTOM_DISPATCH(a.kc, {
        if (f64) ref15_score_kernel<double, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
        else ref15_score_kernel<float, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
    });
    return hipGetLastError();
}

hipError_t launch_ref15_scheduled(bool f64, const Ref15SchedArgs& a, hipStream_t stream) {
    const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
    // the LDS variants' descriptors: whole waves, and a chunk's row spans within 32-bit ranges
    const bool lds = a.B % 64 == 0 && uint64_t(a.B) * 8 * 2 < (uint64_t(1) << 32) &&
                     reinterpret_cast<uintptr_t>(a.t) % 16 == 0 && reinterpret_cast<uintptr_t>(a.etype) % 16 == 0 &&
                     uint64_t(a.B) * kSchedChunk < (uint64_t(1) << 32) && !a.regs;
    // two passes where legal (the host gives them workspace); the pick codes hold 24-bit indices
    // and the apply pass's record of one pick spans a 32-bit byte range
    const bool two = lds && !a.fused && a.picks && a.flags && a.n_sel && a.sel_time && a.T < (1 << 24) &&
                     uint64_t(a.B) * 6u * (f64 ? 8u : 4u) < (uint64_t(1) << 32) &&
                     reinterpret_cast<uintptr_t>(a.sel_time) % 16 == 0 &&
                     ((!f64 && !a.pay_rec) || reinterpret_cast<uintptr_t>(a.payload) % 16 == 0) &&
                     (!a.pay_rec || (int64_t(a.pay_rec) * (f64 ? 8 : 4)) % 16 == 0);
    if (two) {
        // four-wave groups (KF_OPT_SCHED_GROUP): one-wave groups, which free their slot when their
        // wave's pick list ends, measured slower on the bench row (5.51 vs 5.07 ms apply)
        const dim3 g1(static_cast<unsigned>(a.B / 64)), g4(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
        const bool rnd = a.words != nullptr;
        if (a.one_launch && !rnd) {
            Ref15SchedArgs c = a;  // heaviest first by rate where the filters have their own rates
            c.order = nullptr;
            c.rec_time = false;    // its pick phase's sel_time rows are its apply phase's times
            if (a.order && a.freq) {
                ref15_rate_key_kernel<<<g4, 256, 0, stream>>>(a);
                size_t tb = a.sort_tmp_bytes;
                const hipError_t e = sort_pairs_desc_u32(a.sort_tmp, &tb, a.wave_key, a.wave_key_sorted, a.wave_id,
                                                         a.order, static_cast<int>(a.B / 64), 32, stream);
                if (e != hipSuccess) return e;
                c.order = a.order;
            }
            KF_CUSTOM_DISPATCH(c.kc, {
                if (c.pay_rec) {
                    if (f64) ref15_apply_kernel<double, CUSTOM, 4, true, true><<<g4, 256, 0, stream>>>(c);
                    else ref15_apply_kernel<float, CUSTOM, 4, true, true><<<g4, 256, 0, stream>>>(c);
                } else {
                    if (f64) ref15_apply_kernel<double, CUSTOM, 4, true><<<g4, 256, 0, stream>>>(c);
                    else ref15_apply_kernel<float, CUSTOM, 4, true><<<g4, 256, 0, stream>>>(c);
                }
            });
        } else {
            if (rnd) ref15_pick_kernel<4, true><<<g4, 256, 0, stream>>>(a);
            else if (a.group_waves == 4) ref15_pick_kernel<4><<<g4, 256, 0, stream>>>(a);
            else ref15_pick_kernel<1><<<g1, 64, 0, stream>>>(a);
            if (a.order) {  // the waves by their longest pick list, descending (stable)
                int bits = 1;
                while ((1 << bits) <= a.T && bits < 31) ++bits;
                size_t tb = a.sort_tmp_bytes;
                const hipError_t e = sort_pairs_desc_u32(a.sort_tmp, &tb, a.wave_key, a.wave_key_sorted, a.wave_id,
                                                         a.order, static_cast<int>(a.B / 64), bits, stream);
                if (e != hipSuccess) return e;
            }
            KF_CUSTOM_DISPATCH(a.kc, {
                if (a.pay_rec) {  // payload records (kf_run_scheduled_rec): four-wave groups
                    if (f64 && a.rec_time) ref15_apply_kernel<double, CUSTOM, 4, false, true, true><<<g4, 256, 0, stream>>>(a);
                    else if (f64) ref15_apply_kernel<double, CUSTOM, 4, false, true><<<g4, 256, 0, stream>>>(a);
                    else ref15_apply_kernel<float, CUSTOM, 4, false, true><<<g4, 256, 0, stream>>>(a);
                } else
#if KF_APPLY_IMAGES == 2
                if (a.group_waves == 4) {  // two images: 8 waves per CU in LDS
                    const dim3 g2(static_cast<unsigned>((a.B + 127) / 128));
                    if (f64) ref15_apply_kernel<double, CUSTOM, 2, false><<<g2, 128, 0, stream>>>(a);
                    else ref15_apply_kernel<float, CUSTOM, 2, false><<<g2, 128, 0, stream>>>(a);
                } else
#endif
                if (a.group_waves == 4) {
                    if (f64) ref15_apply_kernel<double, CUSTOM, 4, false><<<g4, 256, 0, stream>>>(a);
                    else ref15_apply_kernel<float, CUSTOM, 4, false><<<g4, 256, 0, stream>>>(a);
                } else {
                    if (f64) ref15_apply_kernel<double, CUSTOM, 1, false><<<g1, 64, 0, stream>>>(a);
                    else ref15_apply_kernel<float, CUSTOM, 1, false><<<g1, 64, 0, stream>>>(a);
                }
            });
        }
        if (rnd) return hipGetLastError();  // random picks are never checked, so none is flagged
        Ref15SchedArgs b = a;  // the flagged filters (usually none: every lane leaves at once)
        b.only = a.flags;
        KF_CUSTOM_DISPATCH(a.kc, {
            if (f64) ref15_sched_kernel<double, CUSTOM><<<grid, kBlock, 0, stream>>>(b);
            else ref15_sched_kernel<float, CUSTOM><<<grid, kBlock, 0, stream>>>(b);
        });
        return hipGetLastError();
    }
    KF_CUSTOM_DISPATCH(a.kc, {
        if (lds) {
            if (f64) ref15_sched_lds_kernel<double, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
            else ref15_sched_lds_kernel<float, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
        } else {
            if (f64) ref15_sched_kernel<double, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
            else ref15_sched_kernel<float, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
        }
    });
    return hipGetLastError();
}

namespace {
template <typename T, class M, bool CUSTOM>
void ref_events_t(const RefArgs& a, hipStream_t stream, int variant) {
    if (variant == kEventsLds) {
        const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
        if (a.cov) ref_events_lds_kernel<T, M, true, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
        else ref_events_lds_kernel<T, M, false, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
    } else if (variant == kEventsChain) {
        const dim3 cgrid(static_cast<unsigned>((a.B * kGroup + kBlock - 1) / kBlock));
        ref_chain_kernel<T, M, false, CUSTOM><<<cgrid, kBlock, 0, stream>>>(a);
    } else if (variant == kEventsGated) {
        ref_chain_gated_kernel<T, M, CUSTOM><<<1, 64, 0, stream>>>(a);
    } else {
        const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
        ref_events_kernel<T, M, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
    }
}
template <typename T, class M, bool CUSTOM>
void ref_stream_t(const RefArgs& a, hipStream_t stream, int nv) {
    if (nv == 4) {
        const dim3 vgrid(static_cast<unsigned>((a.B * chain_lanes<4>() + kBlock - 1) / kBlock));
        ref_chain_kernel<T, M, true, CUSTOM, 4><<<vgrid, kBlock, 0, stream>>>(a);
    } else {
        const dim3 cgrid(static_cast<unsigned>((a.B * kGroup + kBlock - 1) / kBlock));
        ref_chain_kernel<T, M, true, CUSTOM><<<cgrid, kBlock, 0, stream>>>(a);
    }
}
}  // namespace

hipError_t launch_ref_events(int model, bool f64, const RefArgs& a, hipStream_t stream, int variant) {
    if (model != 15 && model != 8) return hipErrorInvalidValue;
    KF_CUSTOM_DISPATCH(a.kc, {
        if (model == 15) {
            if (f64) ref_events_t<double, M15, CUSTOM>(a, stream, variant);
            else ref_events_t<float, M15, CUSTOM>(a, stream, variant);
        } else {
            if (f64) ref_events_t<double, M8, CUSTOM>(a, stream, variant);
            else ref_events_t<float, M8, CUSTOM>(a, stream, variant);
        }
    });
    return hipGetLastError();
}

hipError_t launch_ref_stream(int model, bool f64, const RefArgs& a, hipStream_t stream, int nv) {
    if (a.s_len <= 0 || a.s_nchunks <= 0 || (nv != 1 && nv != 4)) return hipErrorInvalidValue;
    if (model != 15 && model != 8) return hipErrorInvalidValue;
    KF_CUSTOM_DISPATCH(a.kc, {
        if (model == 15) {
            if (f64) ref_stream_t<double, M15, CUSTOM>(a, stream, nv);
            else ref_stream_t<float, M15, CUSTOM>(a, stream, nv);
        } else {
            if (f64) ref_stream_t<double, M8, CUSTOM>(a, stream, nv);
            else ref_stream_t<float, M8, CUSTOM>(a, stream, nv);
        }
    });
    return hipGetLastError();
}

template <typename T, class M>
void stream_phase(int phase, const StreamArgs& a, hipStream_t stream) {
    constexpr int NCH = M::NP + M::NA;
    auto grid = [](int64_t n) { return dim3(static_cast<unsigned>((n + kBlock - 1) / kBlock)); };
    switch (phase) {
        case 0: stream_init_kernel<T, M><<<grid(a.C), kBlock, 0, stream>>>(a); break;
        case 1: stream_perturb_kernel<T, M><<<grid(4 * a.C), kBlock, 0, stream>>>(a); break;
        case kStreamPhaseScanTiles: {
            const dim3 g(unsigned((a.C + kScanTile - 1) / kScanTile), NCH);
            stream_scan_tiles_kernel<T, M><<<g, kScanTile, 0, stream>>>(a);
            break;
        }
        case kStreamPhaseTop:
            stream_top_kernel<T, M><<<dim3(1, NCH), kScanTile, 0, stream>>>(a);
            break;
        case kStreamPhaseStarts: {
            const dim3 g(unsigned((a.C + kScanTile - 1) / kScanTile), NCH);
            stream_starts_kernel<T, M><<<g, kScanTile, 0, stream>>>(a);
            break;
        }
        case kStreamPhaseLftMaps: {
            const int64_t lanes = a.C * a.np * lft_map_chains<M>(a.sym != 0) * kLftStride;
            if (a.kc) stream_lft_maps_kernel<T, M, true><<<grid(lanes), kBlock, 0, stream>>>(a);
            else stream_lft_maps_kernel<T, M, false><<<grid(lanes), kBlock, 0, stream>>>(a);
            break;
        }
        case kStreamPhaseLftStart: {
            const int64_t bc = a.g > 0 ? a.G : kBlock;
            // LDS variant: G / g threads walk, but the whole block stages the window maps (more
            // loads in flight; the extra threads leave after the staging)
            const unsigned walkers = a.g > 0 ? unsigned((a.G + a.g - 1) / a.g) : unsigned(kBlock);
            const unsigned want = a.start_threads > 0 ? unsigned(a.start_threads) : unsigned(kBlock);
            const unsigned threads = a.g > 0 ? (want > walkers && want <= unsigned(kBlock) ? want : walkers)
                                             : unsigned(kBlock);
            const bool fixed = a.g > 0 && (a.G + a.iters) * a.np <= kStartNu;
            const size_t lds = !(a.g > 0) ? 0
                               : fixed    ? size_t(kStartNu) * 36 * sizeof(double)
                                          : size_t(a.G + a.iters) * a.np * 36 * sizeof(double);
            const dim3 g(unsigned((a.C + bc - 1) / bc), NCH);
            if (fixed) stream_lft_start_kernel<T, M, true, true><<<g, threads, lds, stream>>>(a);
            else if (a.g > 0) stream_lft_start_kernel<T, M, true><<<g, threads, lds, stream>>>(a);
            else stream_lft_start_kernel<T, M, false><<<g, threads, 0, stream>>>(a);
            break;
        }
        case 5: stream_finish_kernel<T, M><<<1, 1024, 0, stream>>>(a); break;
        case kStreamPhaseRecords:
            if constexpr (M::NTRAJ % 2 == 0 && kStreamRecordPairs) {
                // (a caller's trajectory that is not aligned to a pair takes the one-entry kernel)
                if (a.dtab && reinterpret_cast<uintptr_t>(a.traj) % (2 * sizeof(T)) == 0) {
                    stream_records2_kernel<T, M><<<grid(a.S * (M::NTRAJ / 2)), kBlock, 0, stream>>>(a);
                    break;
                }
            }
            stream_records_kernel<T, M><<<grid(a.S * M::NTRAJ), kBlock, 0, stream>>>(a);
            break;
        default: break;
    }
}

hipError_t launch_stream_phase(int model, bool f64, int phase, const StreamArgs& a, hipStream_t stream) {
    if (a.C < 2 || phase < 0 || phase > kStreamPhaseRecords) return hipErrorInvalidValue;
    if (model == 15) {
        if (f64) stream_phase<double, M15>(phase, a, stream);
        else stream_phase<float, M15>(phase, a, stream);
    } else if (model == 8) {
        if (f64) stream_phase<double, M8>(phase, a, stream);
        else stream_phase<float, M8>(phase, a, stream);
    } else {
        return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

namespace {
// launch_stream_choose (kf_internal.h): one block; 64 segments of 1024 consecutive flags spread
// evenly over the stream (or every flag of a shorter one), coalesced byte loads, an LDS count
__global__ void __launch_bounds__(1024) stream_choose_kernel(StreamCheck* k, const uint8_t* up, int64_t T,
                                                             int share_den) {
    __shared__ int total;
    const int tid = int(threadIdx.x);
    if (tid == 0) total = 0;
    __syncthreads();
    constexpr int kSeg = 64, kSegLen = 1024;
    int cnt = 0;
    int64_t seen = 0;
    if (T <= int64_t(kSeg) * kSegLen) {
        for (int64_t i = tid; i < T; i += kSegLen) cnt += up[i] != 0;
        seen = T;
    } else {
        for (int j = 0; j < kSeg; ++j) cnt += up[(T - kSegLen) * j / (kSeg - 1) + tid] != 0;
        seen = int64_t(kSeg) * kSegLen;
    }
    atomicAdd(&total, cnt);
    __syncthreads();
    if (tid != 0) return;
    const int ok = k->ok;
    const bool look = int64_t(total) * share_den <= seen;
    k->skip_chain = (ok || look) ? 1 : 0;
    k->skip_gated = (ok || !look) ? 1 : 0;
}
}  // namespace

hipError_t launch_stream_choose(StreamCheck* check, const uint8_t* updated, int64_t T, int share_den,
                                hipStream_t stream) {
    if (!check || !updated || T <= 0 || share_den < 1) return hipErrorInvalidValue;
    stream_choose_kernel<<<1, 1024, 0, stream>>>(check, updated, T, share_den);
    return hipGetLastError();
}

hipError_t launch_ref_reset(int model, bool f64, const RefArgs& a, hipStream_t stream) {
    const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
    if (model != 15 && model != 8) return hipErrorInvalidValue;
    KF_CUSTOM_DISPATCH(a.kc, {
        if (model == 15) {
            if (f64) ref_reset_kernel<double, M15, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
            else ref_reset_kernel<float, M15, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
        } else {
            if (f64) ref_reset_kernel<double, M8, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
            else ref_reset_kernel<float, M8, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
        }
    });
    return hipGetLastError();
}

hipError_t launch_ref15_combos(bool f64, const Ref15ComboArgs& a, hipStream_t stream) {
    if (a.n_events > kMaxEvents) return hipErrorInvalidValue;
    const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
    KF_CUSTOM_DISPATCH(a.kc, {
        if (f64) ref15_combo_kernel<double, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
        else ref15_combo_kernel<float, CUSTOM><<<grid, kBlock, 0, stream>>>(a);
    });
    return hipGetLastError();
}


void set_search_band(Ref15SearchArgs& a, bool f64) {
    // the threshold as the kernels compare it (T(threshold)); (mantissa, exponent) pairs whose
    // mantissa T's rounding keeps far inside eps (a mantissa rounded up to 1 only makes the
    // kernels' (e, m) comparisons conservative)
    // |log det| of a 15 x 15 SPD matrix stays below 15 * 745 (every pivot is a finite double, a
    // float's log below 15 * 104): above 1e5 the test accepts every valid determinant; below
    // -1e5 only one that underflowed to 0 (its log is -inf), and none at -inf or NaN
    const double t = f64 ? a.threshold : double(float(a.threshold));
    a.band_mode = t == t ? (t > 1e5 ? 1 : (t < -1e5 ? (t == -HUGE_VAL ? 3 : 2) : 0)) : 3;
    a.band_lo_m = a.band_hi_m = 1.0;
    a.band_lo_e = a.band_hi_e = 0;
    if (a.band_mode != 0) return;
    // the band's half-width in log units: above the log's absolute rounding near t (a few ulps of
    // t in T) and this exp2's (q - fl carries q's rounding, 1e-16 |t|)
    const double eps = f64 ? std::fmax(1e-10, std::fabs(t) * 1e-14) : std::fmax(1e-4, std::fabs(t) * 1e-6);
    const double q = t * 1.4426950408889634074;  // thr / ln 2: e^thr = 2^fl * 2^(q - fl)
    const double fl = std::floor(q);
    const double mm = std::exp2(q - fl);
    int e1, e2;
    a.band_lo_m = std::frexp(mm * (1.0 - eps), &e1);
    a.band_hi_m = std::frexp(mm * (1.0 + eps), &e2);
    a.band_lo_e = int(fl) + e1;
    a.band_hi_e = int(fl) + e2;
}

hipError_t launch_search_finish(uint64_t* counters, uint64_t* host, int n, bool zero, hipStream_t stream) {
    if (n < 1 || n > 256) return hipErrorInvalidValue;
    search_finish_kernel<<<1, 256, 0, stream>>>(counters, host, n, zero);
    return hipGetLastError();
}

hipError_t launch_ref15_search_end(bool f64, const Ref15SearchArgs& a, hipStream_t stream) {
    if (a.n_events > kMaxEvents || a.k < 2 || a.k_end < a.k || a.k_end > a.n_events || !a.par || a.n_groups < 1 ||
        a.n_groups > 65 || a.gitem[a.n_groups] == 0 || a.gitem[a.n_groups] >= (1ull << 31))
        return hipErrorInvalidValue;
    // the extensions' table (group i: extension gblk[i], first wave gitem[i], then the total)
    const dim3 grid(unsigned(a.gitem[a.n_groups]));
    KF_CUSTOM_DISPATCH(a.kc, {
        if (a.sym) {
            if (f64) ref15_search_end_kernel<double, CUSTOM, true><<<grid, 64, 0, stream>>>(a);
            else ref15_search_end_kernel<float, CUSTOM, true><<<grid, 64, 0, stream>>>(a);
        } else {
            if (f64) ref15_search_end_kernel<double, CUSTOM, false><<<grid, 64, 0, stream>>>(a);
            else ref15_search_end_kernel<float, CUSTOM, false><<<grid, 64, 0, stream>>>(a);
        }
    });
    return hipGetLastError();
}

hipError_t launch_ref15_search_head(bool f64, const Ref15SearchArgs& a, hipStream_t stream) {
    if (a.n_events > kMaxEvents || a.n_events < 3 || a.k < 1 || a.k > a.n_events - 2 || a.n_child == 0 ||
        a.n_child >= (1ull << 31))
        return hipErrorInvalidValue;
    const dim3 grid(unsigned((a.n_child + 63) / 64));
    const size_t lds = search_binom_lds_bytes(a.n_events, a.k + 1);
    KF_CUSTOM_DISPATCH(a.kc, {
        if (a.sym) {
            if (f64) ref15_search_head_kernel<double, CUSTOM, true><<<grid, 64, lds, stream>>>(a);
            else ref15_search_head_kernel<float, CUSTOM, true><<<grid, 64, lds, stream>>>(a);
        } else {
            if (f64) ref15_search_head_kernel<double, CUSTOM, false><<<grid, 64, lds, stream>>>(a);
            else ref15_search_head_kernel<float, CUSTOM, false><<<grid, 64, lds, stream>>>(a);
        }
    });
    return hipGetLastError();
}

// The child-major kernel's work items: per group v of parent blocks, blocks x (n - 1 - v) child
// events; group v holds blocks [ceil(C(v, k-1)/64), ceil(C(v+1, k-1)/64)) (the stored parents
// have largest event <= n - 3).  Fills b's group table; false when the items overflow.
static bool cm_items(const Ref15SearchArgs& a, Ref15SearchArgs& b, uint64_t& items, uint64_t& waves) {
    const uint64_t* C = a.binom_host;
    const int n = a.n_events, k = a.k;
    b = a;
    items = 0;
    if (k == 1) {
        items = uint64_t(n);
        b.n_groups = 0;
    } else {
        b.v_lo = k - 2;
        int i = 0;
        for (int v = k - 2; v <= n - 3; ++v, ++i) {
            const uint64_t b0 = (C[v * (kMaxEvents + 1) + k - 1] + 63) / 64;
            const uint64_t b1 = (C[(v + 1) * (kMaxEvents + 1) + k - 1] + 63) / 64;
            b.gitem[i] = items;
            b.gblk[i] = b0;
            const uint64_t span = (b1 - b0) * uint64_t(n - 1 - v);
            if (span >= (1ull << 31)) return false;  // 32-bit item offsets in a group
            items += span;
        }
        b.n_groups = i;
        if (i == 0) return false;
    }
    waves = (items + 7) / 8 * 8;
    return waves < (1ull << 31);
}

hipError_t launch_ref15_search(bool f64, const Ref15SearchArgs& a, bool child_major, hipStream_t stream) {
    // the stored parents (kf_search_combos' cap); a level's children C(n, k) may be many more
    // (n = 40, k = 10: 8.5e8): child ranks and node addresses are 64-bit, and only the children
    // below C(n - 2, k) are stored
    if (a.n_events > kMaxEvents || a.k < 1 || a.k > a.n_events || a.n_par == 0 || a.n_par >= (1ull << 28))
        return hipErrorInvalidValue;
    if (child_major) {
        Ref15SearchArgs b;
        uint64_t items = 0, waves = 0;
        if (!cm_items(a, b, items, waves)) return hipErrorInvalidValue;
        KF_CUSTOM_DISPATCH(a.kc, {
            if (a.sym) {
                if (f64) ref15_search_cm_kernel<double, CUSTOM, true><<<dim3(unsigned(waves)), 64, 0, stream>>>(b, items);
                else ref15_search_cm_kernel<float, CUSTOM, true><<<dim3(unsigned(waves)), 64, 0, stream>>>(b, items);
            } else {
                if (f64) ref15_search_cm_kernel<double, CUSTOM, false><<<dim3(unsigned(waves)), 64, 0, stream>>>(b, items);
                else ref15_search_cm_kernel<float, CUSTOM, false><<<dim3(unsigned(waves)), 64, 0, stream>>>(b, items);
            }
        });
        return hipGetLastError();
    }
    KF_CUSTOM_DISPATCH(a.kc, {
        if (!a.pm_regs) {
            const dim3 grid(static_cast<unsigned>((a.n_par + 63) / 64));
            if (a.sym) {
                if (f64) ref15_search_pm_kernel<double, true, CUSTOM, true><<<grid, 64, 0, stream>>>(a);
                else ref15_search_pm_kernel<float, true, CUSTOM, true><<<grid, 64, 0, stream>>>(a);
            } else {
                if (f64) ref15_search_pm_kernel<double, true, CUSTOM, false><<<grid, 64, 0, stream>>>(a);
                else ref15_search_pm_kernel<float, true, CUSTOM, false><<<grid, 64, 0, stream>>>(a);
            }
        } else {
            const dim3 grid(static_cast<unsigned>((a.n_par + kBlock - 1) / kBlock));
            if (a.sym) {
                if (f64) ref15_search_pm_kernel<double, false, CUSTOM, true><<<grid, kBlock, 0, stream>>>(a);
                else ref15_search_pm_kernel<float, false, CUSTOM, true><<<grid, kBlock, 0, stream>>>(a);
            } else {
                if (f64) ref15_search_pm_kernel<double, false, CUSTOM, false><<<grid, kBlock, 0, stream>>>(a);
                else ref15_search_pm_kernel<float, false, CUSTOM, false><<<grid, kBlock, 0, stream>>>(a);
            }
        }
    });
    return hipGetLastError();
}

hipError_t launch_ref15_search_pair(bool f64, const Ref15SearchArgs& a, bool child_major, hipStream_t stream) {
    // levels k and k + 1 <= n of the axis-symmetric search, from level k - 1's stored parents
    if (!a.sym || a.n_events > kMaxEvents || a.k < 2 || a.k + 1 > a.n_events || a.n_par == 0 ||
        a.n_par >= (1ull << 28) || !a.par)
        return hipErrorInvalidValue;
    if (child_major) {
        Ref15SearchArgs b;
        uint64_t items = 0, waves = 0;
        if (!cm_items(a, b, items, waves)) return hipErrorInvalidValue;
        KF_CUSTOM_DISPATCH(a.kc, {
            if (f64) ref15_search_cm_kernel<double, CUSTOM, true, true><<<dim3(unsigned(waves)), 64, 0, stream>>>(b, items);
            else ref15_search_cm_kernel<float, CUSTOM, true, true><<<dim3(unsigned(waves)), 64, 0, stream>>>(b, items);
        });
        return hipGetLastError();
    }
    const dim3 grid(static_cast<unsigned>((a.n_par + 63) / 64));
    KF_CUSTOM_DISPATCH(a.kc, {
        if (f64) ref15_search_pair_kernel<double, CUSTOM, true><<<grid, 64, 0, stream>>>(a);
        else ref15_search_pair_kernel<float, CUSTOM, true><<<grid, 64, 0, stream>>>(a);
    });
    return hipGetLastError();
}

}  // namespace kfmi
