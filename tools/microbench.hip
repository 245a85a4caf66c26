// Calibration microbenchmarks for the roofline (run on the GPU box):
//  (1) streaming: 1R+1W copy and the K5 mix (4 read + 5 write streams), d2v per lane
//  (2) v_mfma_f64_16x16x4_f64 throughput, 4 independent accumulators per wave
// build: hipcc --offload-arch=gfx950 -O3 tools/microbench.hip -o tools/microbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d2v __attribute__((ext_vector_type(2)));
typedef double d4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_copy(const d2v* __restrict__ a, d2v* __restrict__ b, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L) b[i] = a[i];
}
__global__ void k_mix(const d2v* __restrict__ a0, const d2v* __restrict__ a1, const d2v* __restrict__ a2,
                      const d2v* __restrict__ a3, d2v* b0, d2v* b1, d2v* b2, d2v* b3, d2v* b4, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += gridDim.x * 256L) {
        d2v x = a0[i], y = a1[i], z = a2[i], w = a3[i];
        b0[i] = x + y; b1[i] = y + z; b2[i] = z + w; b3[i] = w + x; b4[i] = x - w;
    }
}
__global__ __launch_bounds__(256) void k_mfma(double* out, int iters) {
    d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double a = threadIdx.x * 1e-3, b = blockIdx.x * 1e-3;
    for (int i = 0; i < iters; ++i) {
        c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
        c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
        c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
        c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
    out[blockIdx.x * 256 + threadIdx.x] = c0[0] + c1[1] + c2[2] + c3[3];
}
int main() {
    const long n = 1L << 26;  // d2v elements per stream = 1 GiB
    std::vector<d2v*> buf(9);
    for (auto& p : buf) { CK(hipMalloc(&p, n * 16)); CK(hipMemset(p, 0, n * 16)); }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    for (int grid : {2048, 4096, 8192}) {
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, buf[0], buf[1], n);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        }
        printf("copy grid %5d: %.1f GB/s\n", grid, 2.0 * n * 16 / (ms * 1e-3) / 1e9);
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_mix, dim3(grid), dim3(256), 0, 0, buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], buf[7], buf[8], n);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        }
        printf("mix4r5w grid %5d: %.1f GB/s\n", grid, 9.0 * n * 16 / (ms * 1e-3) / 1e9);
    }
    double* out; CK(hipMalloc(&out, 2048 * 256 * 8));
    for (int blocks : {256, 512, 1024}) {
        const int iters = 4096;
        float ms = 0;
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out, iters);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
        }
        const double flops = (double)blocks * 4 /*waves*/ * iters * 4 * 2048.0;
        printf("mfma f64 16x16x4 blocks %d: %.1f TF/s\n", blocks, flops / (ms * 1e-3) / 1e12);
    }
    return 0;
}
