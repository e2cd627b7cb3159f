// Shared device arithmetic and memory helpers of the gfx950 KF kernels (kf_cv.hip, kf_ref15.hip).
// Everything is lane-local: one filter per lane, small matrices fully unrolled into VGPRs.
#pragma once

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

namespace kfmi {
namespace dev {

constexpr int32_t kNotSpd = -3;  // KF_ENOTSPD

// Upper-triangle packed row-major index of (i, j) in an N x N symmetric matrix.
template <int N>
__host__ __device__ constexpr int tri(int i, int j) {
    return i <= j ? i * N - i * (i - 1) / 2 + (j - i) : j * N - j * (j - 1) / 2 + (i - j);
}

__device__ __forceinline__ double fmaT(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fmaT(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

template <typename T>
__device__ __forceinline__ T quiet_nan();
template <>
__device__ __forceinline__ double quiet_nan<double>() { return __builtin_nan(""); }
template <>
__device__ __forceinline__ float quiet_nan<float>() { return __builtin_nanf(""); }

// 1/d: the hardware approximation (v_rcp_f64 / v_rcp_f32) refined by NEWTON Newton steps.
template <int NEWTON>
__device__ __forceinline__ double rcp_nr(double d) {
    double r = __builtin_amdgcn_rcp(d);
#pragma unroll
    for (int i = 0; i < NEWTON; ++i) r = fmaT(r, fmaT(-d, r, 1.0), r);
    return r;
}
template <int NEWTON>
__device__ __forceinline__ float rcp_nr(float d) {
    float r = __builtin_amdgcn_rcpf(d);
#pragma unroll
    for (int i = 0; i < NEWTON; ++i) r = fmaT(r, fmaT(-d, r, 1.0f), r);
    return r;
}
// Same, but NaN unless d > 0: a non-positive pivot of S poisons everything derived from it.
template <int NEWTON, typename T>
__device__ __forceinline__ T rcp_pos(T d) {
    const T r = rcp_nr<NEWTON>(d);
    return d > T(0) ? r : quiet_nan<T>();
}

// log(m) + e ln 2 for a mantissa m in [0.5, 1) (the frexp-normalised pivot product).
// fp64: reduce to m' in [sqrt(1/2), sqrt(2)), then log m' = 2 atanh(s), s = (m'-1)/(m'+1),
// |s| < 0.1716, summed to s^21 (truncation < 1e-17) — ~25 VALU ops instead of the ~100 of
// the general double-double log().  fp32: the hardware log (v_log_f32).
__device__ __forceinline__ double log_mant(double m, int e) {
    const bool lo = m < 0.70710678118654752440;
    m = lo ? m + m : m;
    e = lo ? e - 1 : e;
    const double f = m - 1.0;
    const double s = f * rcp_nr<2>(2.0 + f);
    const double s2 = s * s;
    double p = 1.0 / 21;
    p = fmaT(p, s2, 1.0 / 19);
    p = fmaT(p, s2, 1.0 / 17);
    p = fmaT(p, s2, 1.0 / 15);
    p = fmaT(p, s2, 1.0 / 13);
    p = fmaT(p, s2, 1.0 / 11);
    p = fmaT(p, s2, 1.0 / 9);
    p = fmaT(p, s2, 1.0 / 7);
    p = fmaT(p, s2, 1.0 / 5);
    p = fmaT(p, s2, 1.0 / 3);
    const double two_s = s + s;
    const double lm = fmaT(two_s * s2, p, two_s);
    return fmaT(double(e), 0.69314718055994530942, lm);
}
__device__ __forceinline__ float log_mant(float m, int e) {
    return fmaT(float(e), 0.69314718055994530942f, __logf(m));
}

// Accumulate the LDL^T pivots of an SPD N x N matrix (packed upper) into a running
// (mantissa, binary exponent) product, renormalised every 3 pivots so fp32 cannot overflow.
// ok becomes false if a pivot is not > 0 (covariance lost positive definiteness).
template <int N, typename T>
__device__ __forceinline__ void ldl_pivot_product(const T (&P)[N * (N + 1) / 2], T& prod, int& ex, bool& ok) {
    T L[N][N];
    T d[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
        T v[N];
        T dj = P[tri<N>(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) {
            v[k] = L[j][k] * d[k];
            dj = fmaT(-L[j][k], v[k], dj);
        }
        ok = ok && (dj > T(0));
        d[j] = dj;
        prod *= dj;
        if (j % 3 == 2 || j == N - 1) {
            int e;
            prod = frexp(prod, &e);
            ex += e;
        }
        if (j + 1 < N) {
            const T dinv = rcp_nr<1>(dj);  // a bad pivot already makes `ok` false
#pragma unroll
            for (int i = j + 1; i < N; ++i) {
                T s = P[tri<N>(i, j)];
#pragma unroll
                for (int k = 0; k < j; ++k) s = fmaT(-L[i][k], v[k], s);
                L[i][j] = s * dinv;
            }
        }
    }
}

// Division-free determinants of small SPD blocks for the log-det, with the LDL pivots' test of
// positive definiteness (every leading minor > 0, Sylvester).  3 x 3 by one fraction-free
// elimination step with pivot a (the LDL order): a * det = (ad - b^2)(af - c^2) - (ae - bc)^2,
// so num accumulates a * det and den accumulates a; the caller divides once.  The pivot
// product d0 d1 d2 of LDL^T is the same quantity (d0 = a, d1 = (ad - b^2)/a,
// d2 = num/(a (ad - b^2))) without its two reciprocals per block.
template <typename T>
__device__ __forceinline__ void det3_scaled(const T (&P)[6], T& num, T& den, bool& ok) {
    const T a = P[0], b = P[1], c = P[2], d = P[3], e = P[4], f = P[5];
    const T m2 = fmaT(-b, b, a * d);
    const T g = fmaT(-c, c, a * f);
    const T h = fmaT(-b, c, a * e);
    const T n = fmaT(-h, h, m2 * g);
    ok = ok && (a > T(0)) && (m2 > T(0)) && (n > T(0));
    num *= n;
    den *= a;
}
template <typename T>
__device__ __forceinline__ void det2(const T (&P)[3], T& num, bool& ok) {
    const T m2 = fmaT(-P[1], P[1], P[0] * P[2]);
    ok = ok && (P[0] > T(0)) && (m2 > T(0));
    num *= m2;
}
// renormalise a running product: prod = mantissa in [0.5, 1), exponent into ex
template <typename T>
__device__ __forceinline__ void renorm(T& prod, int& ex) {
    int e;
    prod = frexp(prod, &e);
    ex += e;
}

// log det of an SPD N x N matrix (packed upper) via LDL^T; NaN unless positive definite.
template <int N, typename T>
__device__ __forceinline__ T logdet_ldl(const T (&P)[N * (N + 1) / 2]) {
    T prod = T(1);
    int ex = 0;
    bool ok = true;
    ldl_pivot_product<N, T>(P, prod, ex, ok);
    const T ld = log_mant(prod, ex);  // prod was frexp-normalised at the last pivot
    return ok ? ld : quiet_nan<T>();
}

// Measurement update of an N-state filter whose observation selects the FIRST M states,
// H = [I_M 0] (a row selection: no multiply), R packed upper M x M (DIAG_R: off-diagonal zero):
//   S = P[0:M,0:M] + R, LDL^T(S) in-lane, K = P H^T S^-1 by substitution per row,
//   x += K (z - x[0:M]),
//   Joseph: P+ = (I-KH) P (I-KH)^T + K R K^T = (P - K G^T) + E K^T, G = P H^T, E = K S - G.
// Returns false when S is not positive definite (x and P are then NaN).  NEWTON: Newton steps
// on each pivot reciprocal (1 leaves a ~2^-46 relative gain error, which Joseph's form turns
// into a second-order term of P+ and x carries at ~1e-14; the BASELINE kernels keep 2 so the
// block and general constant-velocity kernels stay bit-identical).
// POISON = false: a non-positive pivot is only reported (return value), for callers that
// replace the whole filter with NaN themselves (saves a select per reciprocal).
// NV > 1: NV state vectors share the covariance (filters that differ only in their state, as
// kf_run_stream's map variants do): S, K and P+ are computed once, every x_v[v] is updated with
// the same K, each term in the same order as the single-state update.
// JOSEPH = false: the reference models' own form P+ = (I-KH)P = P - K G^T (kf_workers.py:711,
// hw5_2.py:358, 376), upper triangle only: the same rows without the E K^T term.
// GAIN_R (H = I, M == N, diagonal R): P+ = K R.  I - K = (S - P) S^-1 = R S^-1, so
// (I - K)P = R S^-1 P, the transpose of P S^-1 R = K R, and the product is symmetric: one multiply
// per entry and no cancellation (P - K P subtracts nearly equal terms where P >> R).
template <int N, int M, bool DIAG_R, typename T, int NEWTON = 2, bool POISON = true, int NV = 1, bool JOSEPH = true,
          bool GAIN_R = false>
__device__ __forceinline__ bool sel_update_nv(T (&xv)[NV][N], T (&P)[N * (N + 1) / 2], const T (&zv)[NV][M],
                                              const T (&R)[M * (M + 1) / 2]) {
    constexpr int MT = M * (M + 1) / 2;
    // S = H P H^T + R, then its LDL^T
    T S[MT];
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = i; j < M; ++j)
            S[tri<M>(i, j)] = (i == j || !DIAG_R) ? P[tri<N>(i, j)] + R[tri<M>(i, j)] : P[tri<N>(i, j)];
    T L[M][M];
    T d[M];
    T dinv[M];
    bool ok = true;
#pragma unroll
    for (int j = 0; j < M; ++j) {
        T v[M];
        T dj = S[tri<M>(j, j)];
#pragma unroll
        for (int k = 0; k < j; ++k) {
            v[k] = L[j][k] * d[k];
            dj = fmaT(-L[j][k], v[k], dj);
        }
        ok = ok && (dj > T(0));
        d[j] = dj;
        dinv[j] = POISON ? rcp_pos<NEWTON>(dj) : rcp_nr<NEWTON>(dj);
#pragma unroll
        for (int i = j + 1; i < M; ++i) {
            T s = S[tri<M>(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) s = fmaT(-L[i][k], v[k], s);
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
            for (int b = 0; b < a; ++b) s = fmaT(-L[a][b], w[b], s);
            w[a] = s;
        }
#pragma unroll
        for (int a = M - 1; a >= 0; --a) {
            T s = w[a] * dinv[a];
#pragma unroll
            for (int b = a + 1; b < M; ++b) s = fmaT(-L[b][a], K[i][b], s);
            K[i][a] = s;
        }
    }
    // x += K (z - H x)
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        T y[M];
#pragma unroll
        for (int a = 0; a < M; ++a) y[a] = zv[v][a] - xv[v][a];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            T s = xv[v][i];
#pragma unroll
            for (int a = 0; a < M; ++a) s = fmaT(K[i][a], y[a], s);
            xv[v][i] = s;
        }
    }
    if constexpr (GAIN_R && M == N && DIAG_R) {
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
            for (int j = i; j < N; ++j) P[tri<N>(i, j)] = K[i][j] * R[tri<M>(j, j)];
        return ok;
    }
    // Joseph: P+ = (I-KH) P (I-KH)^T + K R K^T = (P - K G^T) + E K^T with G = P H^T and
    // E = K S - G, an identity for ANY K (E is the residual of the gain equation K S = G,
    // so an error dK in the gain enters P+ only as dK S dK^T).  Upper triangle only, row
    // by row; row i's E is formed just before it is used so only m values of E are live.
    // Rows >= m are written in place (their old values are read only by themselves); rows
    // < m hold G and feed every row, so their new values are staged until the end.
    T top[M][N];
#pragma unroll
    for (int i = 0; i < N; ++i) {
        T E[M];
        if constexpr (JOSEPH) {
#pragma unroll
            for (int a = 0; a < M; ++a) {
                T e = -P[tri<N>(i, a)];
#pragma unroll
                for (int b = 0; b < M; ++b) e = fmaT(K[i][b], S[tri<M>(b, a)], e);
                E[a] = e;
            }
        }
#pragma unroll
        for (int j = i; j < N; ++j) {
            T s = P[tri<N>(i, j)];
#pragma unroll
            for (int b = 0; b < M; ++b) s = fmaT(-K[i][b], P[tri<N>(b, j)], s);
            if constexpr (JOSEPH) {
#pragma unroll
                for (int a = 0; a < M; ++a) s = fmaT(E[a], K[j][a], s);
            }
            if (i < M)
                top[i][j] = s;
            else
                P[tri<N>(i, j)] = s;
        }
    }
#pragma unroll
    for (int i = 0; i < M; ++i)
#pragma unroll
        for (int j = i; j < N; ++j) P[tri<N>(i, j)] = top[i][j];
    return ok;
}

template <int N, int M, bool DIAG_R, typename T, int NEWTON = 2, bool POISON = true, bool JOSEPH = true,
          bool GAIN_R = false>
__device__ __forceinline__ bool sel_update(T (&x)[N], T (&P)[N * (N + 1) / 2], const T (&z)[M],
                                           const T (&R)[M * (M + 1) / 2]) {
    T xv[1][N], zv[1][M];
#pragma unroll
    for (int i = 0; i < N; ++i) xv[0][i] = x[i];
#pragma unroll
    for (int a = 0; a < M; ++a) zv[0][a] = z[a];
    const bool ok = sel_update_nv<N, M, DIAG_R, T, NEWTON, POISON, 1, JOSEPH, GAIN_R>(xv, P, zv, R);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = xv[0][i];
    return ok;
}

// Addressing: every access goes through a raw buffer descriptor built from wave-uniform
// scalars — the base of one [B]-long row (component i of step t) and the row's byte length —
// plus the lane's 32-bit byte offset (buffer_load ... offen).  No 64-bit address lives in
// VGPRs, and the hardware range check turns an out-of-row access into a dropped store /
// zero load instead of a fault.  B * sizeof(T) < 2^31 is enforced by kf_alloc.
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* base, int64_t r, uint32_t row_bytes) {
    const char* p = reinterpret_cast<const char*>(base) + r * int64_t(row_bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(p), 0, row_bytes, 0x00020000);
}

// A descriptor over rows [r0, r0 + nrows) of a [.][B] array, for lanes that address different
// rows: the lane's row goes into voffset (row * row_bytes + off) so the descriptor stays
// wave-uniform (a per-lane descriptor costs a waterfall loop per access).  A masked lane uses
// kDropOffset: beyond every span, so its store is dropped and its load returns 0.
constexpr uint32_t kDropOffset = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(const void* base, int64_t r0, uint32_t row_bytes,
                                                            uint32_t nrows) {
    const char* p = reinterpret_cast<const char*>(base) + r0 * int64_t(row_bytes);
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(p), 0, base ? row_bytes * nrows : 0u, 0x00020000);
}
__device__ __forceinline__ double ldv(__amdgpu_buffer_rsrc_t r, uint32_t voff, double) {
    return __builtin_bit_cast(double, (v2u)__builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0));
}
__device__ __forceinline__ float ldv(__amdgpu_buffer_rsrc_t r, uint32_t voff, float) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, voff, 0, 0));
}
__device__ __forceinline__ void stv(__amdgpu_buffer_rsrc_t r, uint32_t voff, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), r, voff, 0, 0);
}
__device__ __forceinline__ void stv(__amdgpu_buffer_rsrc_t r, uint32_t voff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), r, voff, 0, 0);
}

// Cache policy of the once-touched input streams (u, z: read once per launch).  nt (aux = 2):
// round 1 measured it mixed across processes (profiles/r01_ab/nt_streams_ab.txt); late round 2's
// in-process A/Bs, arms in both orders, give config 3 -0.6..-0.8 %, config 5 -0.5..-0.7 %,
// configs 2 and 4 within noise on slow-placement boxes and config 3 / 5 -2.1 / -2.2 % on a
// fast one (profiles/r02_ab/load_nt_ab*.txt), so nt is the default.
// -DKF_STREAM_CPOL=0 builds the default-policy variant.
#ifndef KF_STREAM_CPOL
#define KF_STREAM_CPOL 2
#endif
__device__ __forceinline__ double ldb_stream(const void* base, int64_t r, uint32_t row_bytes, uint32_t off, double) {
    return __builtin_bit_cast(double, (v2u)__builtin_amdgcn_raw_buffer_load_b64(row_rsrc(base, r, row_bytes), off, 0,
                                                                                KF_STREAM_CPOL));
}
__device__ __forceinline__ float ldb_stream(const void* base, int64_t r, uint32_t row_bytes, uint32_t off, float) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(row_rsrc(base, r, row_bytes), off, 0,
                                                                          KF_STREAM_CPOL));
}
__device__ __forceinline__ void stb_stream(void* base, int64_t r, uint32_t row_bytes, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), row_rsrc(base, r, row_bytes), off, 0,
                                          KF_STREAM_CPOL);
}
__device__ __forceinline__ void stb_stream(void* base, int64_t r, uint32_t row_bytes, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), row_rsrc(base, r, row_bytes), off, 0,
                                          KF_STREAM_CPOL);
}

// LDS-DMA: 64 lanes x 16 B from a row-span descriptor (the lane's chunk at voff + soff) to the
// wave-uniform LDS address `lds` + lane * 16 (buffer_load_dwordx4 ... lds).
// Cache policy of the LDS-DMA input loads.  nt (-DKF_DMA_CPOL=2) made the ref15 event kernel
// 2 % slower and left sched, bf and config 1 unchanged (profiles/r02_ab/dma_nt_ab.txt).
#ifndef KF_DMA_CPOL
#define KF_DMA_CPOL 0
#endif
__device__ __forceinline__ void lds_dma16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, uint32_t voff, int soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0,
                                             KF_DMA_CPOL);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bytes_rsrc(const void* p, uint32_t nbytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, p ? nbytes : 0u, 0x00020000);
}
__device__ __forceinline__ void stb_u8(void* base, int64_t r, uint32_t row_bytes, uint32_t off, uint8_t v) {
    __builtin_amdgcn_raw_buffer_store_b8(v, row_rsrc(base, r, row_bytes), off, 0, 0);
}
__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <int IMM>
__device__ __forceinline__ void waitcnt() { __builtin_amdgcn_s_waitcnt(IMM); }

template <typename T>
__device__ __forceinline__ T ldb(const void* base, int64_t r, uint32_t row_bytes, uint32_t off);
template <>
__device__ __forceinline__ double ldb<double>(const void* base, int64_t r, uint32_t row_bytes, uint32_t off) {
    return __builtin_bit_cast(double, (v2u)__builtin_amdgcn_raw_buffer_load_b64(row_rsrc(base, r, row_bytes), off, 0, 0));
}
template <>
__device__ __forceinline__ float ldb<float>(const void* base, int64_t r, uint32_t row_bytes, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(row_rsrc(base, r, row_bytes), off, 0, 0));
}
template <>
__device__ __forceinline__ uint8_t ldb<uint8_t>(const void* base, int64_t r, uint32_t row_bytes, uint32_t off) {
    return __builtin_amdgcn_raw_buffer_load_b8(row_rsrc(base, r, row_bytes), off, 0, 0);
}
__device__ __forceinline__ void stb(void* base, int64_t r, uint32_t row_bytes, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), row_rsrc(base, r, row_bytes), off, 0, 0);
}
__device__ __forceinline__ void stb(void* base, int64_t r, uint32_t row_bytes, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), row_rsrc(base, r, row_bytes), off, 0, 0);
}
// Per-step record rows of the fused run (trajectory, log-det): written once, read by nobody in the
// launch, tens of GB per launch — stored non-temporal.  In-process A/Bs on two boxes
// (profiles/r02_ab/store_nt_ab*.txt): config 3 -1.2..-1.6%, config 2 -1.9..-2.3%, config 5
// -0.9%, config 4 -0.4%.  Other stores keep the default policy (state and buffers that a later
// launch reads back can still hit the caches).  -DKF_REC_CPOL=0 restores the default.
#ifndef KF_REC_CPOL
#define KF_REC_CPOL 2
#endif
__device__ __forceinline__ void stb_rec(void* base, int64_t r, uint32_t row_bytes, uint32_t off, double v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, v), row_rsrc(base, r, row_bytes), off, 0,
                                          KF_REC_CPOL);
}
__device__ __forceinline__ void stb_rec(void* base, int64_t r, uint32_t row_bytes, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned int, v), row_rsrc(base, r, row_bytes), off, 0,
                                          KF_REC_CPOL);
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

__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
    const uint64_t a = (uint64_t(hi) << 21) ^ (lo >> 11);
    return (double(a & ((1ull << 53) - 1)) + 0.5) * 0x1.0p-53;  // (0, 1)
}

// Two independent N(0,1) from one Philox block (53-bit uniforms, Box-Muller).
__device__ __forceinline__ void normal2(const U4& r, double& n0, double& n1) {
    const double u1 = u53(r.v[0], r.v[1]);
    const double u2 = u53(r.v[2], r.v[3]);
    const double rad = sqrt(-2.0 * log(u1));
    double sn, cs;
    sincos(6.283185307179586476925 * u2, &sn, &cs);
    n0 = rad * cs;
    n1 = rad * sn;
}


}  // namespace dev
}  // namespace kfmi
