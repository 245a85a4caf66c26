// v_mfma_f64_16x16x4_f64 rate with constant vs random operands (power / clock
// effect of toggling data), two waves per SIMD, K2's 16 independent
// accumulators, ~0.5 ms per launch.  K2 (k_m3_cp) issues 8192 MFMAs per SIMD
// in ~0.29 ms = 35 ns each; tools/mfma_dep.hip (constant operands) gives 27 ns.
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma_power.hip -o tools/mfma_power
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

// RND: operands from a per-lane table of 32 random doubles (registers), so
// every MFMA sees fresh mantissas; otherwise one constant pair
template <bool RND>
__global__ __launch_bounds__(512) void k_pow(const double* __restrict__ tab, double* sink, int iters) {
    d4 c[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) c[q] = d4{0, 0, 0, 0};
    double va[8], vb[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        va[q] = RND ? tab[(threadIdx.x * 16 + q) & 4095] : 1.0 + 1e-3 * threadIdx.x;
        vb[q] = RND ? tab[(blockIdx.x * 64 + threadIdx.x * 16 + 8 + q) & 4095] : 0.5;
    }
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int q = 0; q < 16; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(va[q & 7], vb[(q * 3) & 7], c[q], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += c[q][0] + c[q][3];
    if (s == 1.2345) sink[0] = s;
}

int main() {
    double *sink, *tab;
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&tab, 4096 * 8));
    std::vector<double> h(4096);
    std::mt19937_64 g(1);
    std::normal_distribution<double> nd;
    for (auto& x : h) x = nd(g);
    CK(hipMemcpy(tab, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int total : {8192, 16384, 65536}) {  // MFMAs per wave
        for (int rnd = 0; rnd < 2; ++rnd) {
            float best = 1e9, worst = 0;
            for (int rep = 0; rep < 5; ++rep) {
                CK(hipEventRecord(e0));
                if (rnd) hipLaunchKernelGGL(k_pow<true>, dim3(256), dim3(512), 0, 0, tab, sink, total / 16);
                else hipLaunchKernelGGL(k_pow<false>, dim3(256), dim3(512), 0, 0, tab, sink, total / 16);
                CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
                if (ms > worst) worst = ms;
            }
            // two waves per SIMD: 2 * total MFMAs per SIMD
            printf("%s operands, %6d MFMA/wave: best %.4f ms worst %.4f ms = %.1f ns per MFMA per SIMD (%.1f TF/s)\n",
                   rnd ? "random  " : "constant", total, best, worst, best * 1e6 / (2.0 * total),
                   2.0 * total * 1024 * 2048.0 / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
