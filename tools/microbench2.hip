// f64 compute ceilings on gfx950: MFMA 16x16x4, MFMA 4x4x4 (16 blocks), VALU v_fma_f64,
// and MFMA-waves + VALU-waves co-resident.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NACC>
__device__ void mfma_loop(double* out, int iters) {
    d4 c[NACC];
    for (int q = 0; q < NACC; ++q) c[q] = d4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int q = 0; q < NACC; ++q) c[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b + q, c[q], 0, 0, 0);
    double s = 0;
    for (int q = 0; q < NACC; ++q) s += c[q][0];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__device__ void valu_loop(double* out, int iters) {
    double x[16];
    for (int q = 0; q < 16; ++q) x[q] = threadIdx.x + q;
    const double a = 1.0000001, b = 1e-9;
    for (int i = 0; i < iters; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) x[q] = fma(x[q], a, b);
    double s = 0;
    for (int q = 0; q < 16; ++q) s += x[q];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mfma4(double* o, int it) { mfma_loop<4>(o, it); }
__global__ __launch_bounds__(256) void k_mfma8(double* o, int it) { mfma_loop<8>(o, it); }
__global__ __launch_bounds__(256) void k_valu(double* o, int it) { valu_loop(o, it); }
// waves 0,1 MFMA; waves 2,3 VALU  (co-resident on different SIMDs? waves map to SIMDs round robin)
__global__ __launch_bounds__(512) void k_mix(double* o, int itm, int itv) {
    if ((threadIdx.x >> 6) & 1) valu_loop(o, itv); else mfma_loop<4>(o, itm);
}
int main() {
    double* out; CK(hipMalloc(&out, 8192 * 512 * 8));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto time = [&](auto launch) { float ms = 0; for (int r = 0; r < 3; ++r) { hipEventRecord(e0); launch(); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);} return ms; };
    for (int blocks : {256, 1024, 2048}) {
        const int it = 2048;
        float ms = time([&] { hipLaunchKernelGGL(k_mfma4, dim3(blocks), dim3(256), 0, 0, out, it); });
        printf("mfma4  blocks %4d: %.1f TF/s\n", blocks, blocks * 4.0 * it * 4 * 2048 / (ms * 1e-3) / 1e12);
        ms = time([&] { hipLaunchKernelGGL(k_mfma8, dim3(blocks), dim3(256), 0, 0, out, it); });
        printf("mfma8  blocks %4d: %.1f TF/s\n", blocks, blocks * 4.0 * it * 8 * 2048 / (ms * 1e-3) / 1e12);
        ms = time([&] { hipLaunchKernelGGL(k_valu, dim3(blocks), dim3(256), 0, 0, out, it * 4); });
        printf("valu   blocks %4d: %.1f TF/s\n", blocks, blocks * 256.0 * it * 4 * 16 * 2 / (ms * 1e-3) / 1e12);
        const int itm = 2048, itv = 2048 * 4;
        ms = time([&] { hipLaunchKernelGGL(k_mix, dim3(blocks), dim3(512), 0, 0, out, itm, itv); });
        const double fm = blocks * 4.0 * itm * 4 * 2048, fv = blocks * 256.0 * itv * 16 * 2;
        printf("mix    blocks %4d: %.1f TF/s total (mfma part %.1f, valu part %.1f if fully overlapped)\n", blocks,
               (fm + fv) / (ms * 1e-3) / 1e12, fm / (ms * 1e-3) / 1e12, fv / (ms * 1e-3) / 1e12);
    }
    return 0;
}
