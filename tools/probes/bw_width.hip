// Access-width probe for kf_run's SoA streams, arithmetic removed: the [T][6][B] -> [T][7][B]
// row stream (config 3/4's 6 input and 7 output rows per step) with K adjacent filters per
// lane, i.e. 4-B (fp32, K = 1) up to 16-B (K = 4) accesses per lane and 256 B to 1 KB per
// wave instruction.  Does the fp32 kernels' 256-B wave access cost HBM rate against fp64's
// 512 B?  Diagnostic tool, not product.
//   hipcc --offload-arch=gfx950 -O3 -o bw_width tools/probes/bw_width.hip && ./bw_width
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <typename V>
__device__ __forceinline__ V addv(V a, V b) { return a + b; }
template <>
__device__ __forceinline__ float2 addv(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
template <>
__device__ __forceinline__ float4 addv(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
template <>
__device__ __forceinline__ double2 addv(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }

// V = the K filters of one lane; rows hold B/K vectors; next step's inputs load before this step's stores
template <typename V>
__global__ __launch_bounds__(256) void soa_width(const V* __restrict__ in, V* __restrict__ out, long BV, int T) {
    const long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= BV) return;
    V v[6], w[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] = in[long(i) * BV + f];
    V acc = v[0];
    for (int t = 0; t < T; ++t) {
        const int tn = t + 1 < T ? t + 1 : t;
#pragma unroll
        for (int i = 0; i < 6; ++i) w[i] = in[(long(tn) * 6 + i) * BV + f];
#pragma unroll
        for (int i = 0; i < 6; ++i) acc = addv(acc, v[i]);
#pragma unroll
        for (int i = 0; i < 7; ++i) out[(long(t) * 7 + i) * BV + f] = acc;
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = w[i];
    }
}

int main(int argc, char** argv) {
    const long B = argc > 1 ? atol(argv[1]) : (1L << 20);
    const int T = argc > 2 ? atoi(argv[2]) : 256;
    const size_t in_alloc = size_t(T) * 6 * B * 8, out_alloc = size_t(T) * 7 * B * 8;
    void *in, *out;
    CK(hipMalloc(&in, in_alloc));
    CK(hipMalloc(&out, out_alloc));
    CK(hipMemset(in, 0, in_alloc));
    CK(hipMemset(out, 0, out_alloc));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch, double nbytes) {
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
        printf("%-22s %8.3f ms  %7.0f GB/s\n", name, ms, nbytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    const double b32 = double(T) * 13 * B * 4, b64 = double(T) * 13 * B * 8;
    for (int rep = 0; rep < 2; ++rep) {
        timeit("f32 x1 (4 B/lane)", [&] { soa_width<float><<<(B + 255) / 256, 256>>>((const float*)in, (float*)out, B, T); }, b32);
        timeit("f32 x2 (8 B/lane)", [&] { soa_width<float2><<<(B / 2 + 255) / 256, 256>>>((const float2*)in, (float2*)out, B / 2, T); }, b32);
        timeit("f32 x4 (16 B/lane)", [&] { soa_width<float4><<<(B / 4 + 255) / 256, 256>>>((const float4*)in, (float4*)out, B / 4, T); }, b32);
        timeit("f64 x1 (8 B/lane)", [&] { soa_width<double><<<(B + 255) / 256, 256>>>((const double*)in, (double*)out, B, T); }, b64);
        timeit("f64 x2 (16 B/lane)", [&] { soa_width<double2><<<(B / 2 + 255) / 256, 256>>>((const double2*)in, (double2*)out, B / 2, T); }, b64);
    }
    return 0;
}
