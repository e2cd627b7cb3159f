// Internal interface between the C ABI (kf_capi.cpp) and the gfx950 kernels (kf_cv.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kfmi {

// Everything one launch of a constant-velocity kernel needs.  Passed by value (kernarg
// segment), so wave-uniform values land in SGPRs.
struct CvArgs {
    int64_t B;               // filters in this handle
    int T;                   // time steps in this launch (kf_run), 1 for predict/update
    int update_every;        // k: update after step t when (t+1) % k == 0
    double dt;               // scalar dt (used when dt_steps == nullptr)
    const double* dt_steps;  // [T] per-step dt or nullptr
    const double* dt_filter; // [B] per-filter dt (kf_predict only) or nullptr
    void* x;                 // [n][B]
    void* P;                 // [n(n+1)/2][B]
    int32_t* status;         // [B]
    const void* u;           // [T][c][B] or nullptr (zero control)
    const void* x0;          // [n][B] reset state (Op::Reset) or nullptr (zeros)
    const void* z;           // [U][m][B]
    const uint8_t* mask;     // [U][B] or nullptr
    void* traj;              // [T][n][B] or nullptr
    void* logdet;            // [T][B] or nullptr
    double q_pos, q_vel;     // Q = diag(q_pos dt, q_vel dt)
    double r[6];             // R upper triangle, packed row-major (m <= 3)
    double p0_pos, p0_vel;   // reset covariance
};

struct SynthArgs {
    int64_t B;
    int64_t filter_offset;
    uint64_t seed;
    int T;
    int update_every;
    double dt;
    void* x0;                // [n][B]
    void* u;                 // [T][c][B]
    void* z;                 // [U][m][B]
};

enum class Op { Run, Predict, Update, Reset };

// Launchers (kf_cv.hip).  Return hipSuccess or the launch error.
hipError_t launch_cv(int axes, bool f64, Op op, const CvArgs& a, hipStream_t stream);
hipError_t launch_synth(int axes, bool f64, const SynthArgs& a, hipStream_t stream);

constexpr int kBlock = 256;  // 4 wave64 per workgroup

}  // namespace kfmi
