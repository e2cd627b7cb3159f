// Access-pattern probe for kf_run's SoA streams, arithmetic removed: does the HBM rate of the
// [T][c][B] row stream depend on the row PITCH (rows padded by a few KB so the 13 rows a wave
// touches per step start on different channels/banks), on keeping the waves of a workgroup in
// lockstep (s_barrier per step, 1024-thread workgroups), or on a persistent grid?
// Diagnostic tool, not product.
//   hipcc --offload-arch=gfx950 -O3 -o bw_pitch tools/probes/bw_pitch.hip && ./bw_pitch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

// in [T][6][pitch], out [T][7][pitch]; lane f touches element f of each row; inputs of step
// t+1 are loaded before step t's stores (as the product kernels pipeline them).
template <int WG, bool SYNC>
__global__ __launch_bounds__(WG) void soa_pitch(const double* __restrict__ in, double* __restrict__ out,
                                                long B, long pitch, int T) {
    long f = long(blockIdx.x) * WG + threadIdx.x;
    const bool live = f < B;
    f = live ? f : 0;
    double acc = 0;
    double v[6], w[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] = in[long(i) * pitch + f];
    for (int t = 0; t < T; ++t) {
        const int tn = t + 1 < T ? t + 1 : t;
#pragma unroll
        for (int i = 0; i < 6; ++i) w[i] = in[(long(tn) * 6 + i) * pitch + f];
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += v[i];
        if (live) {
#pragma unroll
            for (int i = 0; i < 7; ++i) out[(long(t) * 7 + i) * pitch + f] = acc + i;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = w[i];
        if (SYNC) __syncthreads();
    }
}

// Persistent grid: G workgroups walk the filter blocks g, g + G, ...
__global__ __launch_bounds__(256) void soa_persist(const double* __restrict__ in, double* __restrict__ out,
                                                   long B, long pitch, int T) {
    for (long blk = blockIdx.x; blk * 256 < B; blk += gridDim.x) {
        const long f = blk * 256 + threadIdx.x;
        double acc = 0;
        double v[6], w[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = in[long(i) * pitch + f];
        for (int t = 0; t < T; ++t) {
            const int tn = t + 1 < T ? t + 1 : t;
#pragma unroll
            for (int i = 0; i < 6; ++i) w[i] = in[(long(tn) * 6 + i) * pitch + f];
#pragma unroll
            for (int i = 0; i < 6; ++i) acc += v[i];
#pragma unroll
            for (int i = 0; i < 7; ++i) out[(long(t) * 7 + i) * pitch + f] = acc + i;
#pragma unroll
            for (int i = 0; i < 6; ++i) v[i] = w[i];
        }
    }
}

// float4 copy, 4 independent 16-B loads in flight per lane (calibration of the box's copy rate)
__global__ __launch_bounds__(256) void copy4x4(const float4* __restrict__ in, float4* __restrict__ out, long n) {
    const long base = (long(blockIdx.x) * 256 * 4) + threadIdx.x;
    float4 r[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) r[j] = base + j * 256 < n ? in[base + j * 256] : float4{};
#pragma unroll
    for (int j = 0; j < 4; ++j)
        if (base + j * 256 < n) out[base + j * 256] = r[j];
}

int main(int argc, char** argv) {
    const long B = argc > 1 ? atol(argv[1]) : (1L << 20);
    const int T = argc > 2 ? atoi(argv[2]) : 256;
    const long max_pad = 2 * 262144 + 512;
    const long pmax = B + max_pad;
    const size_t in_alloc = size_t(T) * 6 * pmax * 8, out_alloc = size_t(T) * 7 * pmax * 8;
    double *in, *out;
    CK(hipMalloc(&in, in_alloc));
    CK(hipMalloc(&out, out_alloc));
    CK(hipMemset(in, 0, in_alloc));
    CK(hipMemset(out, 0, out_alloc));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = double(T) * 13 * B * 8;
    auto timeit = [&](const char* name, long pad, auto launch, double nbytes) {
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
        printf("%-16s pad %7ld el  %8.3f ms  %7.0f GB/s\n", name, pad, ms, nbytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    const long pads[] = {0, 32, 64, 256, 512, 4096, 65536, 262144 + 32, 262144 + 512};
    for (long pad : pads) {
        const long pitch = B + pad;
        timeit("soa_pitch", pad, [&] { soa_pitch<256, false><<<(B + 255) / 256, 256>>>(in, out, B, pitch, T); }, bytes);
    }
    for (long pad : {0L, 512L}) {
        const long pitch = B + pad;
        timeit("soa_wg1024", pad, [&] { soa_pitch<1024, false><<<(B + 1023) / 1024, 1024>>>(in, out, B, pitch, T); }, bytes);
        timeit("soa_wg1024_sync", pad, [&] { soa_pitch<1024, true><<<(B + 1023) / 1024, 1024>>>(in, out, B, pitch, T); }, bytes);
        timeit("soa_wg256_sync", pad, [&] { soa_pitch<256, true><<<(B + 255) / 256, 256>>>(in, out, B, pitch, T); }, bytes);
        for (int g : {512, 1024, 2048})
            timeit(g == 512 ? "persist512" : g == 1024 ? "persist1024" : "persist2048", pad,
                   [&] { soa_persist<<<g, 256>>>(in, out, B, pitch, T); }, bytes);
    }
    timeit("soa_pitch", 0, [&] { soa_pitch<256, false><<<(B + 255) / 256, 256>>>(in, out, B, B, T); }, bytes);
    const long n4 = long(size_t(T) * 6 * B * 8 / 16);
    timeit("copy4x4", 0, [&] { copy4x4<<<(n4 + 1023) / 1024, 256>>>((const float4*)in, (float4*)out, n4); },
           2.0 * double(n4) * 16);
    return 0;
}
