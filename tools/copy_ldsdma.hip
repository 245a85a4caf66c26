// HBM copy ceiling with LDS-DMA loads: is a read+write stream faster when the
// loads go global -> LDS (global_load_lds_dwordx4, nontemporal) instead of
// into registers?  (north star: >= 80 % of 8 TB/s on unfold + soft_threshold;
// a float4 register copy peaks at ~6.29 TB/s, MI355X_MICROARCH.md)
// Build: hipcc -O3 --offload-arch=gfx950 tools/copy_ldsdma.hip -o tools/copy_ldsdma
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef double d2v __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// register copy: U 16-B nt loads per thread before the stores
template <int U>
__global__ __launch_bounds__(256) void copy_reg(const d2v* __restrict__ X, int64_t n2, d2v* __restrict__ Y) {
    for (int64_t base = (int64_t)blockIdx.x * U * 256; base < n2; base += (int64_t)gridDim.x * U * 256) {
        d2v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(X + base + u * 256 + threadIdx.x);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], Y + base + u * 256 + threadIdx.x);
    }
}

// LDS-DMA copy: each wave moves U KiB per step through its own two LDS
// buffers (the loads of step s+1 are in flight while step s is stored)
template <int U, int AUX>
__global__ __launch_bounds__(256) void copy_lds(const d2v* __restrict__ X, int64_t n2, d2v* __restrict__ Y) {
    __shared__ __attribute__((aligned(16))) d2v buf[4][2][U][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t per = (int64_t)U * 64;  // d2v per wave-step
    const int64_t wave = (int64_t)blockIdx.x * 4 + w, nw = (int64_t)gridDim.x * 4;
    const int64_t steps = n2 / per;  // n2 is a multiple of per here
    auto issue = [&](int64_t s, int b) {
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_global_load_lds((const void*)(X + s * per + u * 64 + lane), (void*)&buf[w][b][u][0], 16, 0, AUX);
    };
    int b = 0;
    int64_t s = wave;
    if (s < steps) issue(s, 0);
    for (; s < steps; s += nw) {
        const int64_t sn = s + nw;
        if (sn < steps) issue(sn, b ^ 1);
        // wait for this step's U loads (the next step's U may stay in flight)
        if (sn < steps) __builtin_amdgcn_s_waitcnt(0x0f70 | (U & 0xf) | ((U >> 4) << 14));  // vmcnt(U)
        else __builtin_amdgcn_s_waitcnt(0x0f70);                                            // vmcnt(0)
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(buf[w][b][u][lane], Y + s * per + u * 64 + lane);
        __builtin_amdgcn_wave_barrier();
        b ^= 1;
    }
}

int main() {
    const int64_t n = 512LL * 512 * 512;  // doubles (1 GiB)
    const int64_t n2 = n / 2;
    d2v *X, *Y;
    CK(hipMalloc(&X, n * 8));
    CK(hipMalloc(&Y, n * 8));
    CK(hipMemset(X, 0, n * 8));
    CK(hipMemset(Y, 0, n * 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timeit = [&](const char* name, auto launch) -> int {
        float best = 1e9;
        for (int rep = 0; rep < 12; ++rep) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 2 && ms < best) best = ms;
        }
        printf("%-28s %.4f ms  %.3f TB/s (%.1f %% of 8)\n", name, best, 2.0 * n * 8 / (best * 1e-3) / 1e12,
               100.0 * 2.0 * n * 8 / (best * 1e-3) / 8e12);
        return 0;
    };
    for (int g : {2048, 4096, 8192}) {
        char nm[64];
        snprintf(nm, sizeof nm, "reg U=8 grid=%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL(copy_reg<8>, dim3(g), dim3(256), 0, 0, X, n2, Y); });
        snprintf(nm, sizeof nm, "lds U=4 nt grid=%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_lds<4, 2>), dim3(g), dim3(256), 0, 0, X, n2, Y); });
        snprintf(nm, sizeof nm, "lds U=8 nt grid=%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_lds<8, 2>), dim3(g), dim3(256), 0, 0, X, n2, Y); });
        snprintf(nm, sizeof nm, "lds U=8 default grid=%d", g);
        timeit(nm, [&] { hipLaunchKernelGGL((copy_lds<8, 0>), dim3(g), dim3(256), 0, 0, X, n2, Y); });
    }
    // correctness of the LDS path: copy a ramp
    {
        d2v* h = (d2v*)malloc(n * 8);
        for (int64_t i = 0; i < n2; ++i) h[i] = d2v{(double)i, (double)-i};
        CK(hipMemcpy(X, h, n * 8, hipMemcpyHostToDevice));
        CK(hipMemset(Y, 0, n * 8));
        hipLaunchKernelGGL((copy_lds<8, 2>), dim3(4096), dim3(256), 0, 0, X, n2, Y);
        CK(hipMemcpy(h, Y, n * 8, hipMemcpyDeviceToHost));
        int64_t bad = 0;
        for (int64_t i = 0; i < n2; ++i) bad += (h[i].x != (double)i) || (h[i].y != (double)-i);
        printf("lds copy check: %lld mismatches\n", (long long)bad);
        free(h);
    }
    return 0;
}
