// v_mfma_f64_16x16x4_f64 throughput vs the number of independent accumulators
// a wave cycles through (dependency distance), at one and two waves per SIMD.
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma_dep.hip -o tools/mfma_dep
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NACC>
__global__ void k_dep(double* sink, int iters) {
    d4 c[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) c[q] = d4{0, 0, 0, 0};
    const double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3 + 1.0;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[q], 0, 0, 0);
    double s = 0;
#pragma unroll
    for (int q = 0; q < NACC; ++q) s += c[q][0] + c[q][3];
    if (s == 1.2345) sink[0] = s;
}

// v_mfma_f64_4x4x4_4b_f64 (16 blocks of... 4 blocks of 4x4x4): 512 flops each
template <int NACC>
__global__ void k_dep4(double* sink, int iters) {
    double c[NACC];
#pragma unroll
    for (int q = 0; q < NACC; ++q) c[q] = 0.0;
    const double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3 + 1.0;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[q], 0, 0, 0);
    double s = 0;
#pragma unroll
    for (int q = 0; q < NACC; ++q) s += c[q];
    if (s == 1.2345) sink[0] = s;
}

int main() {
    double* sink; CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int total = 16384;  // MFMAs per wave
    auto run = [&](auto kern, int nacc, int threads) -> int {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, dim3(256), dim3(threads), 0, 0, sink, total / nacc);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
        }
        const int wps = threads / 256;  // waves per SIMD
        printf("acc %2d waves/SIMD %d: %.4f ms = %.1f ns per MFMA per SIMD\n", nacc, wps, best,
               best * 1e6 / (total * wps));
        return 0;
    };
    for (int t : {256, 512}) {
        run(k_dep4<1>, 1, t); run(k_dep4<4>, 4, t); run(k_dep4<8>, 8, t);
    }
    for (int t : {256, 512, 1024}) {
        run(k_dep<1>, 1, t); run(k_dep<2>, 2, t); run(k_dep<4>, 4, t); run(k_dep<8>, 8, t); run(k_dep<16>, 16, t);
    }
    return 0;
}
