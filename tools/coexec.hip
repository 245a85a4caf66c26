// Does f64 MFMA co-execute with VALU on one SIMD?  One 512-thread workgroup
// per CU (two waves per SIMD): waves 0-3 run role A, waves 4-7 role B, each a
// fixed instruction count; the kernel time of A+B against A alone and B
// alone says whether the two share the SIMD's issue or datapath.
//   roles: 0 idle, 1 v_mfma_f64_16x16x4 (4 independent accumulators),
//          2 v_fma_f64 (8 independent chains), 3 v_add_u32/v_xor (int),
//          4 v_fma_f32 (8 chains)
// build: hipcc --offload-arch=gfx950 -O3 tools/coexec.hip -o tools/coexec
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int ROLE>
__device__ double work(int iters, double seed) {
    double out = 0.0;
    if (ROLE == 1) {
        d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        double a = seed, b = seed * 0.5;
        for (int i = 0; i < iters; ++i) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
        }
        out = c0[0] + c1[1] + c2[2] + c3[3];
    } else if (ROLE == 2) {
        double x[8];
        for (int q = 0; q < 8; ++q) x[q] = seed + q;
        for (int i = 0; i < iters * 8; ++i)
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = __builtin_fma(x[q], 0.999999, 1e-7);
        for (int q = 0; q < 8; ++q) out += x[q];
    } else if (ROLE == 3) {
        // 32-bit integer adds, 8 independent chains (asm: no strength reduction)
        unsigned x[8];
        for (int q = 0; q < 8; ++q) x[q] = (unsigned)(seed * 1000) + q;
        for (int i = 0; i < iters * 8; ++i)
#pragma unroll
            for (int q = 0; q < 8; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[q]) : "v"(x[(q + 1) & 7]));
        for (int q = 0; q < 8; ++q) out += x[q];
    } else if (ROLE == 5) {
        // v_mov_b64 (64-bit moves), 8 chains
        double x[8];
        for (int q = 0; q < 8; ++q) x[q] = seed + q;
        for (int i = 0; i < iters * 8; ++i)
#pragma unroll
            for (int q = 0; q < 8; ++q) asm volatile("v_mov_b64 %0, %1" : "=v"(x[q]) : "v"(x[(q + 3) & 7]));
        for (int q = 0; q < 8; ++q) out += x[q];
    } else if (ROLE == 6) {
        // v_cndmask_b32 (the compact-E selects), 8 chains
        unsigned x[8];
        for (int q = 0; q < 8; ++q) x[q] = (unsigned)(seed * 1000) + q;
        for (int i = 0; i < iters * 8; ++i)
#pragma unroll
            for (int q = 0; q < 8; ++q) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[q]) : "v"(x[(q + 1) & 7]));
        for (int q = 0; q < 8; ++q) out += x[q];
    } else if (ROLE == 7) {
        // v_mfma_f32_16x16x4_f32, 4 independent accumulators (config 5's K5/K2)
        typedef float f4 __attribute__((ext_vector_type(4)));
        f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
        float a = (float)seed, b = (float)seed * 0.5f;
        for (int i = 0; i < iters * 2; ++i) {  // asm volatile: the builtin loop was folded away
            asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c0) : "v"(a), "v"(b));
            asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c1) : "v"(b), "v"(a));
            asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c2) : "v"(a), "v"(a));
            asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(c3) : "v"(b), "v"(b));
        }
        out = c0[0] + c1[1] + c2[2] + c3[3];
    } else if (ROLE == 4) {
        float x[8];
        for (int q = 0; q < 8; ++q) x[q] = (float)seed + q;
        for (int i = 0; i < iters * 8; ++i)
#pragma unroll
            for (int q = 0; q < 8; ++q) x[q] = __builtin_fmaf(x[q], 0.999f, 1e-7f);
        for (int q = 0; q < 8; ++q) out += x[q];
    }
    return out;
}

template <int RA, int RB>
__global__ __launch_bounds__(512) void k_co(double* sink, int ia, int ib) {
    const int w = threadIdx.x >> 6;
    const double seed = threadIdx.x * 1e-3 + blockIdx.x;
    double v = (w < 4) ? work<RA>(ia, seed) : work<RB>(ib, seed);
    if (v == 1.2345) sink[0] = v;
}

int main() {
    double* sink; CK(hipMalloc(&sink, 64));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int IM = 2048;   // MFMA loop: 4 MFMA per iteration
    const int IV = 1024;   // VALU loop: 64 ops per iteration
    auto run = [&](auto kern, const char* name) -> int {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, dim3(256), dim3(512), 0, 0, sink, IM, IV);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
        }
        printf("%-28s %.4f ms\n", name, best);
        return 0;
    };
    run(k_co<1, 0>, "mfma | idle");
    run(k_co<0, 2>, "idle | fma_f64");
    run(k_co<1, 2>, "mfma | fma_f64");
    run(k_co<0, 3>, "idle | int");
    run(k_co<1, 3>, "mfma | int");
    run(k_co<0, 4>, "idle | fma_f32");
    run(k_co<1, 4>, "mfma | fma_f32");
    run(k_co<2, 2>, "fma_f64 | fma_f64");
    run(k_co<1, 1>, "mfma | mfma");
    run(k_co<0, 5>, "idle | mov_b64");
    run(k_co<1, 5>, "mfma | mov_b64");
    run(k_co<0, 6>, "idle | cndmask");
    run(k_co<1, 6>, "mfma | cndmask");
    run(k_co<3, 3>, "int | int");
    run(k_co<7, 0>, "mfma32 | idle");
    run(k_co<7, 4>, "mfma32 | fma_f32");
    run(k_co<7, 3>, "mfma32 | int");
    run(k_co<7, 2>, "mfma32 | fma_f64");
    run(k_co<7, 7>, "mfma32 | mfma32");
    return 0;
}
