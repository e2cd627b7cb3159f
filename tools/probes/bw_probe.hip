// Bandwidth probe for the kf_run access pattern with the arithmetic removed: what HBM rate
// can a stream of [T][c][B] SoA rows (per step: 6 row loads, 7 row stores, 8 B per lane)
// reach on this GPU, versus a tiled layout and a plain copy.  Diagnostic tool, not product.
//   hipcc --offload-arch=gfx950 -O3 -o bw_probe tools/probes/bw_probe.hip && ./bw_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// SoA rows: in [T][6][B], out [T][7][B]; lane f touches element f of each row.
__global__ __launch_bounds__(256) void soa_stream(const double* __restrict__ in, double* __restrict__ out,
                                                  long B, int T) {
    long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    double acc = 0;
    for (int t = 0; t < T; ++t) {
        double v[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = in[(long(t) * 6 + i) * B + f];
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += v[i];
#pragma unroll
        for (int i = 0; i < 7; ++i) out[(long(t) * 7 + i) * B + f] = acc + i;
    }
}
// Tiled: in [T][B/64][6][64], out [T][B/64][7][64]: a wave's per-step rows are contiguous.
__global__ __launch_bounds__(256) void tiled_stream(const double* __restrict__ in, double* __restrict__ out,
                                                    long B, int T) {
    long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    long w = f / 64, l = f % 64, W = B / 64;
    double acc = 0;
    for (int t = 0; t < T; ++t) {
        double v[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = in[((long(t) * W + w) * 6 + i) * 64 + l];
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += v[i];
#pragma unroll
        for (int i = 0; i < 7; ++i) out[((long(t) * W + w) * 7 + i) * 64 + l] = acc + i;
    }
}
// Filter-block major: in [B/256][T][6][256], out [B/256][T][7][256]: a workgroup's whole
// launch is one contiguous span, so the pages it touches are few and consecutive.
__global__ __launch_bounds__(256) void blocked_stream(const double* __restrict__ in, double* __restrict__ out,
                                                      long B, int T) {
    long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    const double* ib = in + long(blockIdx.x) * T * 6 * 256 + threadIdx.x;
    double* ob = out + long(blockIdx.x) * T * 7 * 256 + threadIdx.x;
    double acc = 0;
    for (int t = 0; t < T; ++t) {
        double v[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = ib[(long(t) * 6 + i) * 256];
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += v[i];
#pragma unroll
        for (int i = 0; i < 7; ++i) ob[(long(t) * 7 + i) * 256] = acc + i;
    }
}
// SoA rows moved 16 B per lane: lane pairs (2j, 2j+1) swap one value with DPP (quad_perm
// [1,0,3,2]) so the even lane moves row r of filters (2j, 2j+1) and the odd lane row r+1.
__device__ __forceinline__ double swap_pair(double v) {
    int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
    int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <bool PAIR_LOADS>
__global__ __launch_bounds__(256) void soa_stream_pair(const double* __restrict__ in, double* __restrict__ out,
                                                       long B, int T) {
    long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    const bool odd = f & 1;
    const long fe = f & ~1L;  // the pair's even filter
    double acc = 0;
    for (int t = 0; t < T; ++t) {
        double v[6];
        if (PAIR_LOADS) {
#pragma unroll
            for (int i = 0; i < 6; i += 2) {
                // even lane loads row i of (fe, fe+1), odd lane row i+1
                const double2 w = *reinterpret_cast<const double2*>(&in[(long(t) * 6 + i + (odd ? 1 : 0)) * B + fe]);
                const double mine = odd ? w.y : w.x;     // this lane's filter in the row it loaded
                const double other = odd ? w.x : w.y;    // the partner's filter
                const double got = swap_pair(other);     // partner sends me my filter of its row
                v[i] = odd ? got : mine;
                v[i + 1] = odd ? mine : got;
            }
        } else {
#pragma unroll
            for (int i = 0; i < 6; ++i) v[i] = in[(long(t) * 6 + i) * B + f];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += v[i];
        double o[7];
#pragma unroll
        for (int i = 0; i < 7; ++i) o[i] = acc + i;
#pragma unroll
        for (int i = 0; i < 6; i += 2) {
            const double send = odd ? o[i] : o[i + 1];   // what the partner stores for me
            const double recv = swap_pair(send);
            double2 w;
            w.x = odd ? recv : o[i];        // even: (row i: fe, fe+1); odd: (row i+1: fe, fe+1)
            w.y = odd ? o[i + 1] : recv;
            *reinterpret_cast<double2*>(&out[(long(t) * 7 + i + (odd ? 1 : 0)) * B + fe]) = w;
        }
        out[(long(t) * 7 + 6) * B + f] = o[6];
    }
}
// Non-temporal stores of the SoA pattern.
__global__ __launch_bounds__(256) void soa_stream_nt(const double* __restrict__ in, double* __restrict__ out,
                                                     long B, int T) {
    long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    double acc = 0;
    for (int t = 0; t < T; ++t) {
        double v[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = __builtin_nontemporal_load(&in[(long(t) * 6 + i) * B + f]);
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += v[i];
#pragma unroll
        for (int i = 0; i < 7; ++i) __builtin_nontemporal_store(acc + i, &out[(long(t) * 7 + i) * B + f]);
    }
}
// Read-only and write-only SoA variants.
__global__ __launch_bounds__(256) void soa_read(const double* __restrict__ in, double* __restrict__ out, long B, int T) {
    long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    double acc = 0;
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += in[(long(t) * 6 + i) * B + f];
    out[f] = acc;
}
__global__ __launch_bounds__(256) void soa_write(const double* __restrict__ in, double* __restrict__ out, long B, int T) {
    long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    double a = in[f];
    for (int t = 0; t < T; ++t)
#pragma unroll
        for (int i = 0; i < 7; ++i) out[(long(t) * 7 + i) * B + f] = a + t + i;
}
// Plain float4 copy (calibration).
__global__ __launch_bounds__(256) void copy4(const float4* __restrict__ in, float4* __restrict__ out, long n) {
    for (long i = long(blockIdx.x) * 256 + threadIdx.x; i < n; i += long(gridDim.x) * 256) out[i] = in[i];
}

int main(int argc, char** argv) {
    const long B = argc > 1 ? atol(argv[1]) : (1L << 20);
    const int T = argc > 2 ? atoi(argv[2]) : 256;
    const size_t in_bytes = size_t(T) * 6 * B * 8, out_bytes = size_t(T) * 7 * B * 8;
    double *in, *out;
    CK(hipMalloc(&in, in_bytes));
    CK(hipMalloc(&out, out_bytes));
    CK(hipMemset(in, 0, in_bytes));
    CK(hipMemset(out, 0, out_bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    dim3 grid((B + 255) / 256);
    auto timeit = [&](const char* name, auto launch, double bytes) {
        for (int r = 0; r < 2; ++r) launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-14s %8.3f ms  %7.0f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    timeit("soa_stream", [&] { soa_stream<<<grid, 256>>>(in, out, B, T); }, double(in_bytes + out_bytes));
    timeit("soa_pair_ldst", [&] { soa_stream_pair<true><<<grid, 256>>>(in, out, B, T); }, double(in_bytes + out_bytes));
    timeit("soa_pair_st", [&] { soa_stream_pair<false><<<grid, 256>>>(in, out, B, T); }, double(in_bytes + out_bytes));
    timeit("soa_stream_nt", [&] { soa_stream_nt<<<grid, 256>>>(in, out, B, T); }, double(in_bytes + out_bytes));
    timeit("soa_stream", [&] { soa_stream<<<grid, 256>>>(in, out, B, T); }, double(in_bytes + out_bytes));
    timeit("tiled_stream", [&] { tiled_stream<<<grid, 256>>>(in, out, B, T); }, double(in_bytes + out_bytes));
    timeit("blocked_stream", [&] { blocked_stream<<<grid, 256>>>(in, out, B, T); }, double(in_bytes + out_bytes));
    timeit("soa_read", [&] { soa_read<<<grid, 256>>>(in, out, B, T); }, double(in_bytes));
    timeit("soa_write", [&] { soa_write<<<grid, 256>>>(in, out, B, T); }, double(out_bytes));
    const long n4 = long(in_bytes / 16);
    timeit("copy_float4", [&] { copy4<<<2048, 256>>>((const float4*)in, (float4*)out, n4); }, 2.0 * double(in_bytes));
    return 0;
}
