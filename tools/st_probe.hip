// soft_threshold (K6, soft_threshold.m:2) at 512^3 fp64: chunk order / block
// size / loads-in-flight variants, and the same access pattern as a copy.
// Build: hipcc -O3 --offload-arch=gfx950 tools/st_probe.hip -o tools/st_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef double d2v __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ double st1(double x, double lam) {
    const double s = x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
    return s * fmax(fabs(x) - lam, 0.0);
}
// MAP 0: block b -> chunk b; 1: XCD-major (block b runs on XCD b % 8: chunk (b%8)*per + b/8);
// 2: chunks of consecutive blocks 1 MB apart (b%64 * nch/64 + b/64)
template <int U, int BS, int MAP, bool COPY>
__global__ __launch_bounds__(BS) void st(const d2v* __restrict__ X, int64_t n2, double lam, d2v* __restrict__ Y, int64_t nch) {
    int64_t b = blockIdx.x;
    if (MAP == 1) { const int64_t per = nch / 8; b = (b % 8) * per + b / 8; }
    if (MAP == 2) { const int64_t per = nch / 64; b = (b % 64) * per + b / 64; }
    const int64_t base = b * U * BS;
    d2v v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(X + base + u * BS + threadIdx.x);
#pragma unroll
    for (int u = 0; u < U; ++u) {
        d2v o = v[u];
        if (!COPY) { o.x = st1(v[u].x, lam); o.y = st1(v[u].y, lam); }
        __builtin_nontemporal_store(o, Y + base + u * BS + threadIdx.x);
    }
}

int main() {
    const int64_t N = 512LL * 512 * 512, n2 = N / 2;
    d2v *x, *y;
    CK(hipMalloc(&x, N * 8)); CK(hipMalloc(&y, N * 8));
    CK(hipMemset(x, 0, N * 8));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](auto launch, const char* name) {
        launch(); (void)hipDeviceSynchronize();
        float best = 1e9;
        for (int rep = 0; rep < 20; ++rep) {
            (void)hipEventRecord(e0); launch(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("%-30s %.4f ms  %.2f TB/s\n", name, best, 2.0 * N * 8 / (best * 1e-3) / 1e12);
    };
#define V(U, BS, MAP, COPY) timeit([&] { const int64_t nch = n2 / (U * BS); hipLaunchKernelGGL((st<U, BS, MAP, COPY>), dim3((unsigned)nch), dim3(BS), 0, 0, x, n2, 0.5, y, nch); }, #COPY " " #U "x" #BS " map" #MAP);
    V(8, 256, 0, false) V(8, 256, 1, false) V(8, 256, 2, false)
    V(4, 256, 0, false) V(16, 256, 0, false) V(8, 512, 0, false) V(4, 1024, 0, false)
    V(16, 256, 1, false) V(4, 512, 1, false)
    V(8, 256, 0, true) V(8, 256, 1, true) V(16, 256, 0, true)
    return 0;
}
