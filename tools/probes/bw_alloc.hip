// Does the per-process HBM rate split (consecutive processes alternate between a
// ~4.97 and a ~5.46 TB/s state on the same SoA stream) depend on how the buffers are allocated?
// Same [T][6][B] -> [T][7][B] stream as bw_pitch's soa_pitch, buffers from
//   plain      hipMalloc, one buffer per stream
//   contig     hipExtMallocWithFlags(hipDeviceMallocContiguous)
//   arena      one hipMalloc holding both streams, 2 MiB aligned
// each timed 3x in an interleaved order.  Diagnostic tool, not product.
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/bw_alloc tools/probes/bw_alloc.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__global__ __launch_bounds__(256) void soa(const double* __restrict__ in, double* __restrict__ out, long B, int T) {
    const long f = long(blockIdx.x) * 256 + threadIdx.x;
    if (f >= B) return;
    double acc = 0, v[6], w[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) v[i] = in[long(i) * B + f];
    for (int t = 0; t < T; ++t) {
        const int tn = t + 1 < T ? t + 1 : t;
#pragma unroll
        for (int i = 0; i < 6; ++i) w[i] = in[(long(tn) * 6 + i) * B + f];
#pragma unroll
        for (int i = 0; i < 6; ++i) acc += v[i];
#pragma unroll
        for (int i = 0; i < 7; ++i) out[(long(t) * 7 + i) * B + f] = acc + i;
#pragma unroll
        for (int i = 0; i < 6; ++i) v[i] = w[i];
    }
}

int main(int argc, char** argv) {
    const long B = argc > 1 ? atol(argv[1]) : (1L << 20);
    const int T = argc > 2 ? atoi(argv[2]) : 256;
    const int mode = argc > 3 ? atoi(argv[3]) : 0;  // 0: allocation kinds, 1: offsets within one arena
    const size_t nin = size_t(T) * 6 * B * 8, nout = size_t(T) * 7 * B * 8;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = double(T) * 13 * B * 8;
    auto timeit = [&](const char* name, long arg, const double* in, double* out) {
        auto launch = [&] { soa<<<(B + 255) / 256, 256>>>(in, out, B, T); };
        launch();
        CK(hipDeviceSynchronize());
        const int reps = 10;
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-7s %10ld  %8.3f ms  %7.0f GB/s  in %p out %p\n", name, arg, ms, bytes / (ms * 1e-3) / 1e9,
               (const void*)in, (void*)out);
        fflush(stdout);
    };
    const size_t MiB = size_t(1) << 20;
    const size_t a2 = (nin + 2 * MiB - 1) & ~(2 * MiB - 1);
    if (mode == 0) {
        double *pin[3], *pout[3];
        void* arena = nullptr;
        CK(hipMalloc(&pin[0], nin));
        CK(hipMalloc(&pout[0], nout));
        CK(hipExtMallocWithFlags((void**)&pin[1], nin, hipDeviceMallocContiguous));
        CK(hipExtMallocWithFlags((void**)&pout[1], nout, hipDeviceMallocContiguous));
        CK(hipMalloc(&arena, a2 + nout));
        pin[2] = (double*)arena;
        pout[2] = (double*)((char*)arena + a2);
        const char* names[3] = {"plain", "contig", "arena"};
        for (int m = 0; m < 3; ++m) {
            CK(hipMemset(pin[m], 0, nin));
            CK(hipMemset(pout[m], 0, nout));
        }
        for (int rep = 0; rep < 3; ++rep)
            for (int m = 0; m < 3; ++m) timeit(names[m], rep, pin[m], pout[m]);
        return 0;
    }
    if (mode == 3) {
        // order check: one arena allocated FIRST, then two plain buffers, then each timed 3x
        char* ar = nullptr;
        CK(hipMalloc((void**)&ar, a2 + nout));
        double *pin = nullptr, *pout = nullptr;
        CK(hipMalloc(&pin, nin));
        CK(hipMalloc(&pout, nout));
        CK(hipMemset(ar, 0, a2 + nout));
        CK(hipMemset(pin, 0, nin));
        CK(hipMemset(pout, 0, nout));
        for (int rep = 0; rep < 3; ++rep) {
            timeit("arena1st", rep, (const double*)ar, (double*)(ar + a2));
            timeit("plain2nd", rep, pin, pout);
        }
        return 0;
    }
    if (mode == 2) {
        // walk one arena through the device memory: time it, free it, keep an 8 GiB spacer, repeat
        for (int step = 0; step < 12; ++step) {
            char* ar = nullptr;
            CK(hipMalloc((void**)&ar, a2 + nout));
            CK(hipMemset(ar, 0, a2 + nout));
            timeit("walk", step, (const double*)ar, (double*)(ar + a2));
            CK(hipFree(ar));
            void* spacer = nullptr;
            CK(hipMalloc(&spacer, 8 * 1024 * MiB));
        }
        return 0;
    }
    // one arena; the output stream at a2 + delta (and the input at in_off)
    const long deltas[] = {0, 4096, 65536, 256 << 10, 1 << 20, 2 << 20, 3 << 20, 4 << 20, 6 << 20, 8 << 20, 12 << 20,
                           16 << 20, 33 << 20};
    char* arena = nullptr;
    const size_t slack = 64 * MiB;
    CK(hipMalloc((void**)&arena, a2 + nout + slack));
    CK(hipMemset(arena, 0, a2 + nout + slack));
    for (int rep = 0; rep < 2; ++rep) {
        for (long d : deltas) timeit("out+", d, (const double*)arena, (double*)(arena + a2 + d));
        for (long d : {4096L, 1L << 20, 2L << 20, 5L << 20}) timeit("in+", d, (const double*)(arena + d), (double*)(arena + a2 + 32 * MiB));
    }
    return 0;
}
