// unfold mode 3 (permute [3 1 2], unfold.m:10) at 512^3 fp64 as a tall
// transpose in (rows = n1*n2, cols = n3, column-major) -> out (rows x cols,
// row-major): tile-shape / order / nontemporal variants against a plain copy.
// Build: hipcc -O3 --offload-arch=gfx950 tools/unfold3_probe.hip -o tools/unfold3_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
typedef double d2v __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <bool NT> __device__ __forceinline__ d2v ldv(const d2v* p) { return NT ? __builtin_nontemporal_load(p) : *p; }
template <bool NT> __device__ __forceinline__ void stv(d2v v, d2v* p) { if (NT) __builtin_nontemporal_store(v, p); else *p = v; }

// TR x TC tiles, column tile fastest (the library's k_transpose_tall)
template <int TR, int TC, bool NT, bool XCD>
__global__ __launch_bounds__(256) void tall(const double* __restrict__ in, double* __restrict__ out,
                                            int64_t rows, int64_t cols, int64_t nct) {
    __shared__ double tile[TC][TR + 1];
    int64_t b = blockIdx.x;
    if (XCD) {  // consecutive tiles on one XCD: block b runs on XCD b % 8
        const int64_t nb = gridDim.x, per = nb / 8;
        b = (b % 8) * per + b / 8;
    }
    const int64_t ct = b % nct, rt = b / nct;
    const int64_t r0 = rt * TR, c0 = ct * TC;
    const int th = threadIdx.x;
    constexpr int PR = TR / 2, CPP = 256 / PR, ML = TC / CPP;
    d2v v[ML];
    const int rp = th % PR, cc = th / PR;
#pragma unroll
    for (int m = 0; m < ML; ++m) v[m] = ldv<NT>(reinterpret_cast<const d2v*>(in + (c0 + cc + CPP * m) * rows + r0 + 2 * rp));
#pragma unroll
    for (int m = 0; m < ML; ++m) { tile[cc + CPP * m][2 * rp] = v[m].x; tile[cc + CPP * m][2 * rp + 1] = v[m].y; }
    __syncthreads();
    constexpr int PC = TC / 2, RPP = 256 / PC, MS = TR / RPP;
    const int cp = th % PC, rr = th / PC;
#pragma unroll
    for (int m = 0; m < MS; ++m) {
        const int r = rr + RPP * m;
        stv<NT>(d2v{tile[2 * cp][r], tile[2 * cp + 1][r]}, reinterpret_cast<d2v*>(out + (r0 + r) * cols + c0 + 2 * cp));
    }
}

// full-width slabs: a block moves TR rows x all cols (cols == C): the output
// slab is one contiguous TR*C*8-byte range; loads in two halves of C/2
template <int TR, int C, bool NT>
__global__ __launch_bounds__(512) void slab(const double* __restrict__ in, double* __restrict__ out, int64_t rows) {
    __shared__ double tile[C][TR + 1];
    const int64_t r0 = (int64_t)blockIdx.x * TR;
    const int th = threadIdx.x;
    constexpr int PR = TR / 2, CPP = 512 / PR, ML = C / CPP;  // column pairs per pass
    const int rp = th % PR, cc = th / PR;
    constexpr int H = ML > 16 ? 16 : ML;
#pragma unroll
    for (int m0 = 0; m0 < ML; m0 += H) {
        d2v v[H];
#pragma unroll
        for (int m = 0; m < H; ++m) v[m] = ldv<NT>(reinterpret_cast<const d2v*>(in + (int64_t)(cc + CPP * (m0 + m)) * rows + r0 + 2 * rp));
#pragma unroll
        for (int m = 0; m < H; ++m) { tile[cc + CPP * (m0 + m)][2 * rp] = v[m].x; tile[cc + CPP * (m0 + m)][2 * rp + 1] = v[m].y; }
    }
    __syncthreads();
    // out slab: TR*C doubles contiguous; thread th moves pairs e = th + 512 k
    d2v* o2 = reinterpret_cast<d2v*>(out + r0 * C);
#pragma unroll 4
    for (int e = th; e < TR * C / 2; e += 512) {
        const int r = (2 * e) / C, c = (2 * e) % C;
        stv<NT>(d2v{tile[c][r], tile[c + 1][r]}, o2 + e);
    }
}

// batched (mode 2): matrix b = blockIdx / per, tiles as in `tall`
template <int TR, int TC, bool NT>
__global__ __launch_bounds__(256) void bat(const double* __restrict__ in, double* __restrict__ out,
                                           int64_t rows, int64_t cols, int64_t nct, int64_t per) {
    __shared__ double tile[TC][TR + 1];
    const int64_t mb = blockIdx.x / per, b = blockIdx.x - mb * per;
    const double* src = in + mb * rows * cols;
    double* dst = out + mb * rows * cols;
    const int64_t ct = b % nct, rt = b / nct;
    const int64_t r0 = rt * TR, c0 = ct * TC;
    const int th = threadIdx.x;
    constexpr int PR = TR / 2, CPP = 256 / PR, ML = TC / CPP;
    d2v v[ML];
    const int rp = th % PR, cc = th / PR;
#pragma unroll
    for (int m = 0; m < ML; ++m) v[m] = ldv<NT>(reinterpret_cast<const d2v*>(src + (c0 + cc + CPP * m) * rows + r0 + 2 * rp));
#pragma unroll
    for (int m = 0; m < ML; ++m) { tile[cc + CPP * m][2 * rp] = v[m].x; tile[cc + CPP * m][2 * rp + 1] = v[m].y; }
    __syncthreads();
    constexpr int PC = TC / 2, RPP = 256 / PC, MS = TR / RPP;
    const int cp = th % PC, rr = th / PC;
#pragma unroll
    for (int m = 0; m < MS; ++m) {
        const int r = rr + RPP * m;
        stv<NT>(d2v{tile[2 * cp][r], tile[2 * cp + 1][r]}, reinterpret_cast<d2v*>(dst + (r0 + r) * cols + c0 + 2 * cp));
    }
}

template <int U, int BS>
__global__ __launch_bounds__(BS) void copy_vu(const d2v* __restrict__ X, int64_t n2, d2v* __restrict__ Y) {
    for (int64_t base = (int64_t)blockIdx.x * U * BS; base < n2; base += (int64_t)gridDim.x * U * BS) {
        d2v v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(X + base + u * BS + threadIdx.x);
#pragma unroll
        for (int u = 0; u < U; ++u) __builtin_nontemporal_store(v[u], Y + base + u * BS + threadIdx.x);
    }
}

int main() {
    const int64_t n = 512, rows = n * n, cols = n, N = rows * cols;
    double *in, *out;
    CK(hipMalloc(&in, N * 8)); CK(hipMalloc(&out, N * 8));
    std::vector<double> h(N);
    for (int64_t e = 0; e < N; ++e) h[e] = (double)e;
    CK(hipMemcpy(in, h.data(), N * 8, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto check = [&](const char* name) {
        std::vector<double> o(N);
        (void)hipMemcpy(o.data(), out, N * 8, hipMemcpyDeviceToHost);
        int64_t bad = 0;
        for (int64_t r = 0; r < rows; r += 997) for (int64_t c = 0; c < cols; ++c) bad += o[r * cols + c] != h[c * rows + r];
        if (bad) printf("  %s: %lld WRONG\n", name, (long long)bad);
        (void)hipMemset(out, 0, N * 8);
    };
    auto timeit = [&](auto launch, const char* name, bool chk) {
        launch(); (void)hipDeviceSynchronize();
        if (chk) { check(name); launch(); (void)hipDeviceSynchronize(); }
        float best = 1e9;
        for (int rep = 0; rep < 20; ++rep) {
            (void)hipEventRecord(e0); launch(); (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms; (void)hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
        }
        printf("%-34s %.4f ms  %.2f TB/s\n", name, best, 2.0 * N * 8 / (best * 1e-3) / 1e12);
    };
    timeit([&] { hipLaunchKernelGGL((copy_vu<8, 256>), dim3(2048), dim3(256), 0, 0, (const d2v*)in, N / 2, (d2v*)out); }, "copy (ceiling)", false);
#define TALL(TR, TC, NT, X) timeit([&] { const int64_t nct = cols / TC; hipLaunchKernelGGL((tall<TR, TC, NT, X>), dim3((unsigned)((rows / TR) * nct)), dim3(256), 0, 0, in, out, rows, cols, nct); }, "tall " #TR "x" #TC " nt" #NT " xcd" #X, true);
    TALL(32, 128, false, false)
    TALL(32, 128, true, false)
    TALL(128, 64, true, false)
    TALL(128, 64, false, false)
    TALL(128, 32, true, false)
    TALL(256, 32, true, false)
    TALL(256, 16, true, false)
    TALL(64, 32, true, false)
    TALL(128, 64, true, true)
    TALL(256, 32, true, true)
    // mode 2: batched 512 x 512 transposes (rows n1, cols n2, batch n3)
#define BAT(TR, TC, NT) timeit([&] { const int64_t nct = n / TC, per = (n / TR) * nct; hipLaunchKernelGGL((bat<TR, TC, NT>), dim3((unsigned)(per * n)), dim3(256), 0, 0, in, out, n, n, nct, per); }, "mode2 " #TR "x" #TC " nt" #NT, false);
    BAT(64, 64, false)
    BAT(64, 64, true)
    BAT(128, 64, true)
    BAT(64, 128, true)
    BAT(32, 128, true)
    BAT(128, 32, true)
    return 0;
}
