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
//   logdet   LDL^T(P): sum of log pivots via frexp mantissa product (no sqrt, one log)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "kf_internal.h"

namespace kfmi {
namespace {

constexpr int32_t kNotSpd = -3;  // KF_ENOTSPD

// Upper-triangle packed row-major index of (i, j) in an N x N symmetric matrix.
template <int N>
__host__ __device__ constexpr int tri(int i, int j) {
    return i <= j ? i * N - i * (i - 1) / 2 + (j - i) : j * N - j * (j - 1) / 2 + (i - j);
}

__device__ __forceinline__ double rcp(double d) {
    double r = __builtin_amdgcn_rcp(d);  // v_rcp_f64, then two Newton steps -> ~1 ulp
    double e = __builtin_fma(-d, r, 1.0);
    r = __builtin_fma(r, e, r);
    e = __builtin_fma(-d, r, 1.0);
    return __builtin_fma(r, e, r);
}
__device__ __forceinline__ float rcp(float d) {
    float r = __builtin_amdgcn_rcpf(d);
    float e = __builtin_fmaf(-d, r, 1.0f);
    return __builtin_fmaf(r, e, r);
}

__device__ __forceinline__ double log_pos(double v) { return log(v); }
__device__ __forceinline__ float log_pos(float v) { return __logf(v); }

template <typename T>
__device__ __forceinline__ T quiet_nan();
template <>
__device__ __forceinline__ double quiet_nan<double>() { return __builtin_nan(""); }
template <>
__device__ __forceinline__ float quiet_nan<float>() { return __builtin_nanf(""); }

// log det of an SPD N x N matrix (packed upper) via LDL^T.  Returns NaN if a pivot is
// not > 0 (covariance lost positive definiteness).
template <int N, typename T>
__device__ __forceinline__ T logdet_ldl(const T (&P)[N * (N + 1) / 2]) {
    T L[N][N];
    T d[N];
    T dinv[N];
    bool ok = true;
    T mant = T(1);
    int ex = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        T v[N];
        T dj = P[tri<N>(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) {
            v[k] = L[j][k] * d[k];
            dj = __builtin_fma(-L[j][k], v[k], dj);
        }
        ok = ok && (dj > T(0));
        d[j] = dj;
        int e;
        mant *= frexp(dj, &e);
        ex += e;
        if (j + 1 < N) {
            dinv[j] = rcp(dj);
#pragma unroll
            for (int i = j + 1; i < N; ++i) {
                T s = P[tri<N>(i, j)];
#pragma unroll
                for (int k = 0; k < j; ++k) s = __builtin_fma(-L[i][k], v[k], s);
                L[i][j] = s * dinv[j];
            }
        }
    }
    const T ld = log_pos(mant) + T(ex) * T(0.69314718055994530942);
    return ok ? ld : quiet_nan<T>();
}

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
            x[i] = __builtin_fma(hdt2, u[i], __builtin_fma(dt, x[D + i], x[i]));
            x[D + i] = __builtin_fma(dt, u[i], x[D + i]);
        }
        // With P = [[A, Bm], [Bm^T, C]]:  Bm' = Bm + dt C,  A' = A + dt (Bm' + Bm^T),  C' = C.
        T Bn[D][D];
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int j = 0; j < D; ++j)
                Bn[i][j] = __builtin_fma(dt, P[tri<N>(D + i, D + j)], P[tri<N>(i, D + j)]);
#pragma unroll
        for (int i = 0; i < D; ++i)
#pragma unroll
            for (int j = i; j < D; ++j)
                P[tri<N>(i, j)] = __builtin_fma(dt, Bn[i][j] + P[tri<N>(j, D + i)], P[tri<N>(i, j)]);
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
    // Returns false when S is not positive definite.
    __device__ static __forceinline__ bool update(T (&x)[N], T (&P)[NT], const T (&z)[M],
                                                  const T (&R)[MT]) {
        // LDL^T of S = H P H^T + R
        T L[M][M];
        T d[M];
        T dinv[M];
        bool ok = true;
#pragma unroll
        for (int j = 0; j < M; ++j) {
            T v[M];
            T dj = P[tri<N>(j, j)] + R[tri<M>(j, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) {
                v[k] = L[j][k] * d[k];
                dj = __builtin_fma(-L[j][k], v[k], dj);
            }
            ok = ok && (dj > T(0));
            d[j] = dj;
            dinv[j] = rcp(dj);
#pragma unroll
            for (int i = j + 1; i < M; ++i) {
                T s = P[tri<N>(i, j)] + R[tri<M>(i, j)];
#pragma unroll
                for (int k = 0; k < j; ++k) s = __builtin_fma(-L[i][k], v[k], s);
                L[i][j] = s * dinv[j];
            }
        }
        // K row i solves S k = (P H^T)_i = P[i, 0:m]
        T K[N][M];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            T w[M];
#pragma unroll
            for (int a = 0; a < M; ++a) {
                T s = P[tri<N>(i, a)];
#pragma unroll
                for (int b = 0; b < a; ++b) s = __builtin_fma(-L[a][b], w[b], s);
                w[a] = s;
            }
#pragma unroll
            for (int a = M - 1; a >= 0; --a) {
                T s = w[a] * dinv[a];
#pragma unroll
                for (int b = a + 1; b < M; ++b) s = __builtin_fma(-L[b][a], K[i][b], s);
                K[i][a] = s;
            }
        }
        // x += K (z - H x)
        T y[M];
#pragma unroll
        for (int a = 0; a < M; ++a) y[a] = z[a] - x[a];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            T s = x[i];
#pragma unroll
            for (int a = 0; a < M; ++a) s = __builtin_fma(K[i][a], y[a], s);
            x[i] = s;
        }
        // Joseph: E = K R - (I - K H) P H^T   (n x m)
        T E[N][M];
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
            for (int a = 0; a < M; ++a) {
                T yia = P[tri<N>(i, a)];
                T kr = T(0);
#pragma unroll
                for (int b = 0; b < M; ++b) {
                    yia = __builtin_fma(-K[i][b], P[tri<N>(b, a)], yia);
                    kr = __builtin_fma(K[i][b], R[tri<M>(b, a)], kr);
                }
                E[i][a] = kr - yia;
            }
        // P' = Y + E K^T with Y = (I - K H) P; upper triangle only.  Rows >= m are written in
        // place (their old values are read only by themselves); rows < m are staged because
        // every Y needs them.
        T top[M][N];
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
            for (int j = i; j < N; ++j) {
                T s = P[tri<N>(i, j)];
#pragma unroll
                for (int b = 0; b < M; ++b) s = __builtin_fma(-K[i][b], P[tri<N>(b, j)], s);
#pragma unroll
                for (int a = 0; a < M; ++a) s = __builtin_fma(E[i][a], K[j][a], s);
                if (i < M)
                    top[i][j] = s;
                else
                    P[tri<N>(i, j)] = s;
            }
#pragma unroll
        for (int i = 0; i < M; ++i)
#pragma unroll
            for (int j = i; j < N; ++j) P[tri<N>(i, j)] = top[i][j];
        return ok;
    }
};

template <typename T>
__device__ __forceinline__ T ldg(const void* p, int64_t idx) {
    return reinterpret_cast<const T*>(p)[idx];
}
template <typename T>
__device__ __forceinline__ void stg(void* p, int64_t idx, T v) {
    reinterpret_cast<T*>(p)[idx] = v;
}

template <int D, typename T>
__device__ __forceinline__ void load_state(const CvArgs& a, int64_t f, T (&x)[2 * D],
                                           T (&P)[Cv<D, T>::NT]) {
#pragma unroll
    for (int i = 0; i < 2 * D; ++i) x[i] = ldg<T>(a.x, i * a.B + f);
#pragma unroll
    for (int k = 0; k < Cv<D, T>::NT; ++k) P[k] = ldg<T>(a.P, k * a.B + f);
}

template <int D, typename T>
__device__ __forceinline__ void store_state(const CvArgs& a, int64_t f, const T (&x)[2 * D],
                                            const T (&P)[Cv<D, T>::NT]) {
#pragma unroll
    for (int i = 0; i < 2 * D; ++i) stg<T>(a.x, i * a.B + f, x[i]);
#pragma unroll
    for (int k = 0; k < Cv<D, T>::NT; ++k) stg<T>(a.P, k * a.B + f, P[k]);
}

template <int D, typename T>
__device__ __forceinline__ void fill_nan(T (&x)[2 * D], T (&P)[D * (2 * D + 1)]) {
#pragma unroll
    for (int i = 0; i < 2 * D; ++i) x[i] = quiet_nan<T>();
#pragma unroll
    for (int k = 0; k < Cv<D, T>::NT; ++k) P[k] = quiet_nan<T>();
}

// ------------------------------------------------------------------------------------
// The fused hot path: T predict(+update) steps in one launch.
// ------------------------------------------------------------------------------------
// GENERAL = false: the bench / fusion configuration (scalar dt, control present, no mask,
// trajectory and logdet written) with no runtime checks; GENERAL = true: every optional
// stream decided at run time by a wave-uniform branch.
template <int D, typename T, bool GENERAL>
__global__ __launch_bounds__(kBlock) void cv_run_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    constexpr int N = K::N, M = K::M;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const int64_t B = a.B;
    const bool HAS_DTS = GENERAL && a.dt_steps != nullptr;
    const bool HAS_U = !GENERAL || a.u != nullptr;
    const bool HAS_MASK = GENERAL && a.mask != nullptr;
    const bool TRAJ = !GENERAL || a.traj != nullptr;
    const bool LOGDET = !GENERAL || a.logdet != nullptr;

    T x[N], P[K::NT];
    load_state<D, T>(a, f, x, P);
    int32_t st = a.status[f];
    T R[K::MT];
#pragma unroll
    for (int k = 0; k < K::MT; ++k) R[k] = T(a.r[k]);

    const int k_upd = a.update_every;
    const int U = a.T / k_upd;
    // Software pipeline: the control of step t+1 and the fix of the next update are loaded
    // before step t computes, so their HBM latency hides under a full step of VALU work.
    T u_nxt[D], z_nxt[M];
#pragma unroll
    for (int i = 0; i < D; ++i) u_nxt[i] = (HAS_U && a.T > 0) ? ldg<T>(a.u, i * B + f) : T(0);
#pragma unroll
    for (int i = 0; i < M; ++i) z_nxt[i] = U > 0 ? ldg<T>(a.z, i * B + f) : T(0);
    int s = 0;         // index of the next update
    int until_upd = k_upd;

    for (int t = 0; t < a.T; ++t) {
        T u[D];
#pragma unroll
        for (int i = 0; i < D; ++i) u[i] = u_nxt[i];
        if (HAS_U) {
            const int tn = t + 1 < a.T ? t + 1 : t;
#pragma unroll
            for (int i = 0; i < D; ++i) u_nxt[i] = ldg<T>(a.u, (int64_t(tn) * D + i) * B + f);
        }
        const double dtd = HAS_DTS ? a.dt_steps[t] : a.dt;
        const T dt = T(dtd);
        K::predict(x, P, dt, u, T(a.q_pos * dtd), T(a.q_vel * dtd));

        if (--until_upd == 0) {
            until_upd = k_upd;
            T z[M];
#pragma unroll
            for (int i = 0; i < M; ++i) z[i] = z_nxt[i];
            const bool use = !HAS_MASK || a.mask[int64_t(s) * B + f] != 0;
            const int sn = s + 1 < U ? s + 1 : s;
#pragma unroll
            for (int i = 0; i < M; ++i) z_nxt[i] = ldg<T>(a.z, (int64_t(sn) * M + i) * B + f);
            if (use && !K::update(x, P, z, R)) {
                st = kNotSpd;
                fill_nan<D, T>(x, P);
            }
            ++s;
        }
        if (TRAJ) {
#pragma unroll
            for (int i = 0; i < N; ++i) stg<T>(a.traj, (int64_t(t) * N + i) * B + f, x[i]);
        }
        if (LOGDET) {
            const T ld = logdet_ldl<N, T>(P);
            if (!(ld == ld)) st = kNotSpd;
            stg<T>(a.logdet, int64_t(t) * B + f, ld);
        }
    }
    store_state<D, T>(a, f, x, P);
    a.status[f] = st;
}

// Single predict step (kf_predict): optional per-filter dt and logdet of the prediction.
template <int D, typename T>
__global__ __launch_bounds__(kBlock) void cv_predict_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    T x[K::N], P[K::NT];
    load_state<D, T>(a, f, x, P);
    T u[D];
#pragma unroll
    for (int i = 0; i < D; ++i) u[i] = a.u ? ldg<T>(a.u, i * a.B + f) : T(0);
    const double dtd = a.dt_filter ? a.dt_filter[f] : a.dt;
    K::predict(x, P, T(dtd), u, T(a.q_pos * dtd), T(a.q_vel * dtd));
    store_state<D, T>(a, f, x, P);
    if (a.logdet) {
        const T ld = logdet_ldl<K::N, T>(P);
        stg<T>(a.logdet, f, ld);
        if (!(ld == ld)) a.status[f] = kNotSpd;
    }
}

// Single GPS update (kf_update).
template <int D, typename T>
__global__ __launch_bounds__(kBlock) void cv_update_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    T x[K::N], P[K::NT];
    load_state<D, T>(a, f, x, P);
    T R[K::MT];
#pragma unroll
    for (int k = 0; k < K::MT; ++k) R[k] = T(a.r[k]);
    T z[K::M];
#pragma unroll
    for (int i = 0; i < K::M; ++i) z[i] = ldg<T>(a.z, i * a.B + f);
    int32_t st = a.status[f];
    if (!a.mask || a.mask[f] != 0) {
        if (!K::update(x, P, z, R)) {
            st = kNotSpd;
            fill_nan<D, T>(x, P);
        }
    }
    store_state<D, T>(a, f, x, P);
    if (a.logdet) {
        const T ld = logdet_ldl<K::N, T>(P);
        if (!(ld == ld)) st = kNotSpd;
        stg<T>(a.logdet, f, ld);
    }
    a.status[f] = st;
}

// x = x0 (or 0), P = diag(p0_pos I, p0_vel I), status = OK.
template <int D, typename T>
__global__ __launch_bounds__(kBlock) void cv_reset_kernel(const CvArgs a) {
    using K = Cv<D, T>;
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    T x[K::N], P[K::NT];
#pragma unroll
    for (int i = 0; i < K::N; ++i) x[i] = a.x0 ? ldg<T>(a.x0, i * a.B + f) : T(0);
#pragma unroll
    for (int k = 0; k < K::NT; ++k) P[k] = T(0);
#pragma unroll
    for (int i = 0; i < D; ++i) {
        P[tri<K::N>(i, i)] = T(a.p0_pos);
        P[tri<K::N>(D + i, D + i)] = T(a.p0_vel);
    }
    store_state<D, T>(a, f, x, P);
    a.status[f] = 0;
}

// ------------------------------------------------------------------------------------
// Synthetic GPS+IMU streams: Philox4x32-10 (Salmon et al., SC'11), counter = (t, draw,
// filter lo, filter hi), key = seed.  Generated in fp64, rounded once to T.
// ------------------------------------------------------------------------------------
struct U4 {
    uint32_t v[4];
};

__device__ __forceinline__ U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                            uint32_t k0, uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = uint64_t(M0) * c0;
        const uint64_t p1 = uint64_t(M1) * c2;
        const uint32_t n0 = uint32_t(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n1 = uint32_t(p1);
        const uint32_t n2 = uint32_t(p0 >> 32) ^ c3 ^ k1;
        const uint32_t n3 = uint32_t(p0);
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += W0;
        k1 += W1;
    }
    return U4{{c0, c1, c2, c3}};
}

// Two independent N(0,1) from one Philox block (53-bit uniforms, Box-Muller).
__device__ __forceinline__ void normal2(const U4& r, double& n0, double& n1) {
    const uint64_t a = (uint64_t(r.v[0]) << 21) ^ (r.v[1] >> 11);
    const uint64_t b = (uint64_t(r.v[2]) << 21) ^ (r.v[3] >> 11);
    const double u1 = (double(a & ((1ull << 53) - 1)) + 0.5) * 0x1.0p-53;
    const double u2 = (double(b & ((1ull << 53) - 1)) + 0.5) * 0x1.0p-53;
    const double rad = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincos(6.283185307179586476925 * u2, &sn, &cs);
    n0 = rad * cs;
    n1 = rad * sn;
}

__device__ __forceinline__ double uniform01(const U4& r) {
    const uint64_t a = (uint64_t(r.v[0]) << 21) ^ (r.v[1] >> 11);
    return (double(a & ((1ull << 53) - 1)) + 0.5) * 0x1.0p-53;
}

template <int D, typename T>
__global__ __launch_bounds__(kBlock) void cv_synth_kernel(const SynthArgs a) {
    const int64_t f = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x;
    if (f >= a.B) return;
    const uint64_t g = uint64_t(a.filter_offset + f);
    const uint32_t g0 = uint32_t(g), g1 = uint32_t(g >> 32);
    const uint32_t k0 = uint32_t(a.seed), k1 = uint32_t(a.seed >> 32);
    const double sd_gps = 1.7320508075688772;  // sqrt(3): R_gps variance (kf_workers.py:583)
    double p[D], v[D];
    // initial truth and first fix: counter t = 0xFFFFFFFF
#pragma unroll
    for (int i = 0; i < D; ++i) {
        const U4 ru = philox4x32_10(0xFFFFFFFFu, uint32_t(i), g0, g1, k0, k1);
        p[i] = -1000.0 + 2000.0 * uniform01(ru);
        const U4 rn = philox4x32_10(0xFFFFFFFFu, uint32_t(8 + i), g0, g1, k0, k1);
        double n0, n1;
        normal2(rn, n0, n1);
        v[i] = 10.0 * n0;
        stg<T>(a.x0, i * a.B + f, T(p[i] + sd_gps * n1));  // position = first GPS fix
        stg<T>(a.x0, (D + i) * a.B + f, T(0));               // other states 0 (kf_workers.py:655-659)
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
            stg<T>(a.u, (int64_t(t) * D + i) * a.B + f, T(acc + imu));
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
                stg<T>(a.z, (int64_t(s) * D + i) * a.B + f, T(p[i] + sd_gps * n[2 * D + i]));
            ++s;
        }
    }
}

template <int D, typename T>
hipError_t launch_run(const CvArgs& a, dim3 grid, hipStream_t st) {
    const bool fast = a.dt_steps == nullptr && a.u != nullptr && a.mask == nullptr &&
                      a.traj != nullptr && a.logdet != nullptr;
    if (fast)
        cv_run_kernel<D, T, false><<<grid, kBlock, 0, st>>>(a);
    else
        cv_run_kernel<D, T, true><<<grid, kBlock, 0, st>>>(a);
    return hipGetLastError();
}

template <int D, typename T>
hipError_t launch_cv_t(Op op, const CvArgs& a, hipStream_t st) {
    const dim3 grid(static_cast<unsigned>((a.B + kBlock - 1) / kBlock));
    switch (op) {
        case Op::Run: return launch_run<D, T>(a, grid, st);
        case Op::Predict: cv_predict_kernel<D, T><<<grid, kBlock, 0, st>>>(a); break;
        case Op::Update: cv_update_kernel<D, T><<<grid, kBlock, 0, st>>>(a); break;
        case Op::Reset: cv_reset_kernel<D, T><<<grid, kBlock, 0, st>>>(a); break;
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_cv(int axes, bool f64, Op op, const CvArgs& a, hipStream_t stream) {
    if (axes == 2) return f64 ? launch_cv_t<2, double>(op, a, stream) : launch_cv_t<2, float>(op, a, stream);
    return f64 ? launch_cv_t<3, double>(op, a, stream) : launch_cv_t<3, float>(op, a, stream);
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
