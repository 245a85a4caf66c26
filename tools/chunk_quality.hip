// Per-chunk streaming speed (in-place read+write of 256 MB chunks) of a few
// 6 GiB allocations: is HBM placement quality a property of physical regions?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d2v __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)
__global__ __launch_bounds__(256) void k_rw(d2v* p, long n) {
    for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
        d2v v = p[e]; p[e] = v * 1.0000001;
    }
}
int main() {
    const size_t pool = (size_t)6 << 30, chunk = (size_t)256 << 20;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    std::vector<char*> pools(4);
    for (auto& p : pools) { CK(hipMalloc(&p, pool)); CK(hipMemset(p, 0, pool)); }
    for (int k = 0; k < 4; ++k) {
        printf("pool %d:", k);
        for (size_t c = 0; c < pool / chunk; ++c) {
            float best = 1e9, ms;
            for (int r = 0; r < 3; ++r) {
                hipEventRecord(e0);
                hipLaunchKernelGGL(k_rw, dim3(8192), dim3(256), 0, 0, (d2v*)(pools[k] + c * chunk), (long)(chunk / 16));
                hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf(" %.2f", 2.0 * chunk / (best * 1e-3) / 1e12);
        }
        printf("\n");
    }
    // whole-pool 5-stream K5-like speed for reference is in aos_pattern
    for (auto p : pools) hipFree(p);
    return 0;
}
