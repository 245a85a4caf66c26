// Variants of the two HBM-bound API kernels (north star: >= 80 % of 8 TB/s on
// unfold + soft_threshold): soft_threshold (K6, soft_threshold.m:2) and the
// batched transpose behind unfold modes 2/3 (unfold.m:8,10), 512^3 fp64.
// Build: hipcc -O3 --offload-arch=gfx950 -ffp-contract=off tools/prim_stream.hip -o tools/prim_stream
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef double d2v __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__device__ __forceinline__ double st1(double x, double lam) {
    const double s = x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
    return s * fmax(fabs(x) - lam, 0.0);
}

// V0: the current kernel (grid-stride, one 16-B load per iteration, nt)
__global__ __launch_bounds__(256) void st_v0(const double* __restrict__ X, int64_t n, double lam,
                                             double* __restrict__ Y) {
    const int64_t n2 = n >> 1, stride = (int64_t)gridDim.x * 256;
    const d2v* X2 = reinterpret_cast<const d2v*>(X);
    d2v* Y2 = reinterpret_cast<d2v*>(Y);
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n2; e += stride) {
        const d2v v = __builtin_nontemporal_load(X2 + e);
        d2v o; o.x = st1(v.x, lam); o.y = st1(v.y, lam);
        __builtin_nontemporal_store(o, Y2 + e);
    }
}

// V1..: U 16-B loads per thread issued before any store; block owns a
// contiguous chunk of U*BS d2v; NT = nontemporal loads/stores
template <int U, int BS, int NT>
__global__ __launch_bounds__(BS) void st_vu(const double* __restrict__ X, int64_t n, double lam,
                                            double* __restrict__ Y) {
    const int64_t n2 = n >> 1;
    const d2v* X2 = reinterpret_cast<const d2v*>(X);
    d2v* Y2 = reinterpret_cast<d2v*>(Y);
    for (int64_t base = (int64_t)blockIdx.x * U * BS; base < n2; base += (int64_t)gridDim.x * U * BS) {
        d2v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + u * BS + threadIdx.x;
            if (e < n2) v[u] = NT ? __builtin_nontemporal_load(X2 + e) : X2[e];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + u * BS + threadIdx.x;
            d2v o; o.x = st1(v[u].x, lam); o.y = st1(v[u].y, lam);
            if (e < n2) {
                if (NT) __builtin_nontemporal_store(o, Y2 + e); else Y2[e] = o;
            }
        }
    }
}

// plain copy (the ceiling for this access pattern)
template <int U, int BS>
__global__ __launch_bounds__(BS) void copy_vu(const d2v* __restrict__ X, int64_t n2, d2v* __restrict__ Y) {
    for (int64_t base = (int64_t)blockIdx.x * U * BS; base < n2; base += (int64_t)gridDim.x * U * BS) {
        d2v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + u * BS + threadIdx.x;
            if (e < n2) v[u] = X[e];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t e = base + u * BS + threadIdx.x;
            if (e < n2) Y[e] = v[u];
        }
    }
}

// ---------------------------------------------------------------- transpose
// T0: current (64x64 tile, LDS [64][65], 16-B global accesses both sides)
constexpr int TT = 64;
__global__ __launch_bounds__(256) void tr_v0(const double* __restrict__ in, double* __restrict__ out,
                                             int64_t rows, int64_t cols) {
    __shared__ double tile[TT][TT + 1];
    const int64_t b = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.x * TT, c0 = (int64_t)blockIdx.y * TT;
    const double* src = in + b * rows * cols;
    double* dst = out + b * rows * cols;
    const int th = threadIdx.x;
    {
        const int rr = 2 * (th & 31), cc = th >> 5;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int c = cc + 8 * m;
            const d2v v = *reinterpret_cast<const d2v*>(src + (c0 + c) * rows + r0 + rr);
            tile[c][rr] = v.x;
            tile[c][rr + 1] = v.y;
        }
    }
    __syncthreads();
    {
        const int cc = 2 * (th & 31), rr = th >> 5;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int r = rr + 8 * m;
            *reinterpret_cast<d2v*>(dst + (r0 + r) * cols + c0 + cc) = d2v{tile[cc][r], tile[cc + 1][r]};
        }
    }
}

// T1: 64 x 64 tile, XOR-swizzled LDS (no padding), loads all issued first,
// TB threads (256 or 512); S tiles per block along columns (more bytes in flight)
template <int TB>
__global__ __launch_bounds__(TB) void tr_v1(const double* __restrict__ in, double* __restrict__ out,
                                            int64_t rows, int64_t cols) {
    __shared__ d2v tile[TT][TT / 2];  // [c][r/2] pairs, swizzled on the pair index
    const int64_t b = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.x * TT, c0 = (int64_t)blockIdx.y * TT;
    const double* src = in + b * rows * cols;
    double* dst = out + b * rows * cols;
    const int th = threadIdx.x;
    constexpr int M = 64 * 32 / TB;  // d2v per thread
    d2v v[M];
    const int rp = th & 31, cc = th >> 5;  // pair index (r = 2 rp), column
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int c = cc + (TB / 32) * m;
        v[m] = *reinterpret_cast<const d2v*>(src + (c0 + c) * rows + r0 + 2 * rp);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int c = cc + (TB / 32) * m;
        tile[c][rp ^ (c & 31)] = v[m];
    }
    __syncthreads();
    // out row r = r0 + rr, cols c0 + 2cp, +1: needs (c=2cp, r) and (c=2cp+1, r)
    const int cp = th & 31, rr0 = th >> 5;
#pragma unroll
    for (int m = 0; m < M; ++m) {
        const int r = rr0 + (TB / 32) * m;
        const int c = 2 * cp;
        const d2v a = tile[c][(r >> 1) ^ (c & 31)];
        const d2v bb = tile[c + 1][(r >> 1) ^ ((c + 1) & 31)];
        const double x = (r & 1) ? a.y : a.x, y = (r & 1) ? bb.y : bb.x;
        *reinterpret_cast<d2v*>(dst + (r0 + r) * cols + c0 + c) = d2v{x, y};
    }
}

// T2: TR x TC tile (TR rows contiguous in the input, TC contiguous in the output), LDS
// [TC][TR+1], 256 threads, all loads issued before the LDS stores
template <int TR, int TC>
__global__ __launch_bounds__(256) void tr_v2(const double* __restrict__ in, double* __restrict__ out,
                                             int64_t rows, int64_t cols) {
    __shared__ double tile[TC][TR + 1];
    const int64_t b = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.x * TR, c0 = (int64_t)blockIdx.y * TC;
    const double* src = in + b * rows * cols;
    double* dst = out + b * rows * cols;
    const int th = threadIdx.x;
    constexpr int PR = TR / 2, CPP = 256 / PR, ML = TC / CPP;  // loads
    d2v v[ML];
    const int rp = th % PR, cc = th / PR;
#pragma unroll
    for (int m = 0; m < ML; ++m)
        v[m] = *reinterpret_cast<const d2v*>(src + (c0 + cc + CPP * m) * rows + r0 + 2 * rp);
#pragma unroll
    for (int m = 0; m < ML; ++m) {
        tile[cc + CPP * m][2 * rp] = v[m].x;
        tile[cc + CPP * m][2 * rp + 1] = v[m].y;
    }
    __syncthreads();
    constexpr int PC = TC / 2, RPP = 256 / PC, MS = TR / RPP;  // stores
    const int cp = th % PC, rr = th / PC;
#pragma unroll
    for (int m = 0; m < MS; ++m) {
        const int r = rr + RPP * m;
        *reinterpret_cast<d2v*>(dst + (r0 + r) * cols + c0 + 2 * cp) = d2v{tile[2 * cp][r], tile[2 * cp + 1][r]};
    }
}

// T3: T0 with the column tile fastest in blockIdx.x (groups of blocks write whole output rows)
template <int TR, int TC>
__global__ __launch_bounds__(256) void tr_v3(const double* __restrict__ in, double* __restrict__ out,
                                             int64_t rows, int64_t cols, int nct) {
    __shared__ double tile[TC][TR + 1];
    const int64_t ct = blockIdx.x % nct, rt = blockIdx.x / nct;
    const int64_t r0 = rt * TR, c0 = ct * TC;
    const double* src = in;
    double* dst = out;
    const int th = threadIdx.x;
    constexpr int PR = TR / 2, CPP = 256 / PR, ML = TC / CPP;
    d2v v[ML];
    const int rp = th % PR, cc = th / PR;
#pragma unroll
    for (int m = 0; m < ML; ++m)
        v[m] = *reinterpret_cast<const d2v*>(src + (c0 + cc + CPP * m) * rows + r0 + 2 * rp);
#pragma unroll
    for (int m = 0; m < ML; ++m) {
        tile[cc + CPP * m][2 * rp] = v[m].x;
        tile[cc + CPP * m][2 * rp + 1] = v[m].y;
    }
    __syncthreads();
    constexpr int PC = TC / 2, RPP = 256 / PC, MS = TR / RPP;
    const int cp = th % PC, rr = th / PC;
#pragma unroll
    for (int m = 0; m < MS; ++m) {
        const int r = rr + RPP * m;
        *reinterpret_cast<d2v*>(dst + (r0 + r) * cols + c0 + 2 * cp) = d2v{tile[2 * cp][r], tile[2 * cp + 1][r]};
    }
}

template <typename F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    f();
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < reps; ++r) {
        hipEventRecord(a);
        f();
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
    }
    hipEventDestroy(a); hipEventDestroy(b);
    return best;
}

int main() {
    const int64_t n1 = 512, n2 = 512, n3 = 512, N = n1 * n2 * n3;
    double *X, *Y;
    CK(hipMalloc(&X, N * 8));
    CK(hipMalloc(&Y, N * 8));
    std::vector<double> h(N);
    for (int64_t e = 0; e < N; ++e) h[e] = (double)((e * 2654435761u) % 2001) - 1000.0;
    CK(hipMemcpy(X, h.data(), N * 8, hipMemcpyHostToDevice));
    const double bytes = 2.0 * N * 8;
    auto rep = [&](const char* name, float ms) {
        printf("{\"kernel\": \"%s\", \"ms\": %.4f, \"GBs\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    };
    const int R = 20;
    rep("st_v0_8192", timeit([&] { hipLaunchKernelGGL(st_v0, dim3(8192), dim3(256), 0, 0, X, N, 1.8, Y); }, R));
#define ST(U, BS, NT, G)                                                                         \
    rep("st_u" #U "_bs" #BS "_nt" #NT "_g" #G, timeit([&] {                                       \
        hipLaunchKernelGGL((st_vu<U, BS, NT>), dim3(G), dim3(BS), 0, 0, X, N, 1.8, Y); }, R));
    const int64_t n2v = N / 2;
    ST(4, 256, 0, 65536) ST(4, 256, 1, 65536) ST(8, 256, 0, 32768) ST(8, 256, 1, 32768)
    ST(4, 256, 0, 2048) ST(8, 256, 0, 2048) ST(4, 512, 0, 32768) ST(2, 256, 0, 131072)
    ST(16, 256, 0, 16384) ST(4, 1024, 0, 16384)
#define CP(U, BS, G) \
    rep("copy_u" #U "_bs" #BS "_g" #G, timeit([&] { hipLaunchKernelGGL((copy_vu<U, BS>), dim3(G), dim3(BS), 0, 0, (const d2v*)X, n2v, (d2v*)Y); }, R));
    CP(4, 256, 65536) CP(8, 256, 32768) CP(1, 256, 262144)
    (void)n2v;
    // unfold mode 2: per t, (n1 x n2) -> (n2 x n1): rows = n1, cols = n2, batch n3
    rep("tr_v0_mode2", timeit([&] { hipLaunchKernelGGL(tr_v0, dim3(n1 / TT, n2 / TT, n3), dim3(256), 0, 0, X, Y, n1, n2); }, R));
    rep("tr_v1_256_mode2", timeit([&] { hipLaunchKernelGGL(tr_v1<256>, dim3(n1 / TT, n2 / TT, n3), dim3(256), 0, 0, X, Y, n1, n2); }, R));
    rep("tr_v1_512_mode2", timeit([&] { hipLaunchKernelGGL(tr_v1<512>, dim3(n1 / TT, n2 / TT, n3), dim3(512), 0, 0, X, Y, n1, n2); }, R));
    rep("tr_v1_1024_mode2", timeit([&] { hipLaunchKernelGGL(tr_v1<1024>, dim3(n1 / TT, n2 / TT, n3), dim3(1024), 0, 0, X, Y, n1, n2); }, R));
    // unfold mode 3: (n1 n2) x n3 -> n3 x (n1 n2)
    rep("tr_v0_mode3", timeit([&] { hipLaunchKernelGGL(tr_v0, dim3(n1 * n2 / TT, n3 / TT, 1), dim3(256), 0, 0, X, Y, n1 * n2, n3); }, R));
    rep("tr_v1_256_mode3", timeit([&] { hipLaunchKernelGGL(tr_v1<256>, dim3(n1 * n2 / TT, n3 / TT, 1), dim3(256), 0, 0, X, Y, n1 * n2, n3); }, R));
    rep("tr_v1_512_mode3", timeit([&] { hipLaunchKernelGGL(tr_v1<512>, dim3(n1 * n2 / TT, n3 / TT, 1), dim3(512), 0, 0, X, Y, n1 * n2, n3); }, R));
    rep("tr_v2_128x64_mode3", timeit([&] { hipLaunchKernelGGL((tr_v2<128, 64>), dim3(n1 * n2 / 128, n3 / 64, 1), dim3(256), 0, 0, X, Y, n1 * n2, n3); }, R));
    rep("tr_v2_64x128_mode3", timeit([&] { hipLaunchKernelGGL((tr_v2<64, 128>), dim3(n1 * n2 / 64, n3 / 128, 1), dim3(256), 0, 0, X, Y, n1 * n2, n3); }, R));
    rep("tr_v2_128x128_mode3", timeit([&] { hipLaunchKernelGGL((tr_v2<128, 128>), dim3(n1 * n2 / 128, n3 / 128, 1), dim3(256), 0, 0, X, Y, n1 * n2, n3); }, R));
    rep("tr_v2_64x64_mode3", timeit([&] { hipLaunchKernelGGL((tr_v2<64, 64>), dim3(n1 * n2 / 64, n3 / 64, 1), dim3(256), 0, 0, X, Y, n1 * n2, n3); }, R));
    rep("tr_v2_128x64_mode2", timeit([&] { hipLaunchKernelGGL((tr_v2<128, 64>), dim3(n1 / 128, n2 / 64, n3), dim3(256), 0, 0, X, Y, n1, n2); }, R));
    rep("tr_v2_64x128_mode2", timeit([&] { hipLaunchKernelGGL((tr_v2<64, 128>), dim3(n1 / 64, n2 / 128, n3), dim3(256), 0, 0, X, Y, n1, n2); }, R));
    rep("tr_v3_64x64_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<64, 64>), dim3(n1 * n2 / 64 * (n3 / 64)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 64)); }, R));
    rep("tr_v3_32x128_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<32, 128>), dim3(n1 * n2 / 32 * (n3 / 128)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 128)); }, R));
    rep("tr_v3_128x64_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<128, 64>), dim3(n1 * n2 / 128 * (n3 / 64)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 64)); }, R));
    rep("tr_v3_64x128_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<64, 128>), dim3(n1 * n2 / 64 * (n3 / 128)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 128)); }, R));
    rep("tr_v3_16x256_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<16, 256>), dim3(n1 * n2 / 16 * (n3 / 256)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 256)); }, R));
    rep("tr_v3_32x256_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<32, 256>), dim3(n1 * n2 / 32 * (n3 / 256)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 256)); }, R));
    rep("tr_v3_16x512_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<16, 512>), dim3(n1 * n2 / 16), dim3(256), 0, 0, X, Y, n1 * n2, n3, 1); }, R));
    rep("tr_v3_32x64_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<32, 64>), dim3(n1 * n2 / 32 * (n3 / 64)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 64)); }, R));
    rep("tr_v3_16x128_mode3", timeit([&] { hipLaunchKernelGGL((tr_v3<16, 128>), dim3(n1 * n2 / 16 * (n3 / 128)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 128)); }, R));
    rep("tr_v3_64x64_mode2b", timeit([&] { for (int t = 0; t < 1; ++t) hipLaunchKernelGGL((tr_v3<64, 64>), dim3(n1 / 64 * (n2 / 64)), dim3(256), 0, 0, X, Y, n1, n2, (int)(n2 / 64)); }, R));
    // second pair of buffers (placement sensitivity)
    {
        double *X2b, *Y2b;
        CK(hipMalloc(&X2b, N * 8)); CK(hipMalloc(&Y2b, N * 8));
        CK(hipMemcpy(X2b, h.data(), N * 8, hipMemcpyHostToDevice));
        rep("alloc2_st_u8_nt1", timeit([&] { hipLaunchKernelGGL((st_vu<8, 256, 1>), dim3(32768), dim3(256), 0, 0, X2b, N, 1.8, Y2b); }, R));
        rep("alloc2_tr_v0_mode2", timeit([&] { hipLaunchKernelGGL(tr_v0, dim3(n1 / TT, n2 / TT, n3), dim3(256), 0, 0, X2b, Y2b, n1, n2); }, R));
        rep("alloc2_tr_v0_mode3", timeit([&] { hipLaunchKernelGGL(tr_v0, dim3(n1 * n2 / TT, n3 / TT, 1), dim3(256), 0, 0, X2b, Y2b, n1 * n2, n3); }, R));
        rep("alloc2_tr_v2_128x64_mode3", timeit([&] { hipLaunchKernelGGL((tr_v2<128, 64>), dim3(n1 * n2 / 128, n3 / 64, 1), dim3(256), 0, 0, X2b, Y2b, n1 * n2, n3); }, R));
        rep("alloc2_copy_u1", timeit([&] { hipLaunchKernelGGL((copy_vu<1, 256>), dim3(262144), dim3(256), 0, 0, (const d2v*)X2b, N / 2, (d2v*)Y2b); }, R));
    }
    // correctness of tr_v1 against tr_v0 (mode 3)
    double* Z;
    CK(hipMalloc(&Z, N * 8));
    hipLaunchKernelGGL(tr_v0, dim3(n1 * n2 / TT, n3 / TT, 1), dim3(256), 0, 0, X, Z, n1 * n2, n3);
    hipLaunchKernelGGL((tr_v3<64, 64>), dim3(n1 * n2 / 64 * (n3 / 64)), dim3(256), 0, 0, X, Y, n1 * n2, n3, (int)(n3 / 64));
    CK(hipDeviceSynchronize());
    std::vector<double> a(N), bb(N);
    CK(hipMemcpy(a.data(), Y, N * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(bb.data(), Z, N * 8, hipMemcpyDeviceToHost));
    int64_t bad = 0;
    for (int64_t e = 0; e < N; ++e) bad += a[e] != bb[e];
    printf("{\"tr_v3_mismatches\": %ld}\n", (long)bad);
    return 0;
}
