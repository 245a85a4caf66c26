// K5's exact memory pattern without compute on K pools held at once (same
// physical placements for every variant): does the traversal's concurrent
// footprint decide the placement sensitivity?
//   GM: group-major (a workgroup's 4 ij-tiles x all t-tiles contiguous)
//   TM: t-major (t-tile outermost; resident workgroups sweep adjacent blocks)
//   LIN: elementwise grid-stride over the same 5 fields (no tiles)
// reads D, YL, E, YO; writes E, YL, YO in place and T.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d2v __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int LAY>
__device__ inline long tbase(long g, long tt, long ntt, long ngrp) {
    if (LAY == 0) return ((((g >> 2) * ntt + tt) << 2) + (g & 3)) << 8;
    return (((tt * ngrp + (g >> 2)) << 2) + (g & 3)) << 8;
}

template <int LAY>
__global__ __launch_bounds__(256) void k_pat(double* base, long fstride, long tiles, long ntt) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long tile = (long)blockIdx.x * 4 + wid;
    d2v* F[5];
    for (int f = 0; f < 5; ++f) F[f] = reinterpret_cast<d2v*>(base + f * fstride);
    const long ngrp = tiles / 4;
    auto off = [&](long tt) { return (tbase<LAY>(tile, tt, ntt, ngrp) >> 1) + lane; };
    d2v xa[4][2], xb[4][2];
    auto ld = [&](long tt, d2v (&nx)[4][2]) {
        const long o = off(tt);
        for (int p = 0; p < 2; ++p)
            for (int f = 0; f < 4; ++f) nx[f][p] = F[f][o + 64 * p];
    };
    auto body = [&](long tt, d2v (&c)[4][2], d2v (&n)[4][2], bool pf) {
        if (pf) { ld(tt + 1, n); __builtin_amdgcn_sched_barrier(0); }
        const long o = off(tt);
        for (int p = 0; p < 2; ++p) {
            F[1][o + 64 * p] = c[0][p] + c[1][p];
            F[2][o + 64 * p] = c[2][p] - c[3][p];
            F[3][o + 64 * p] = c[0][p] * c[2][p];
            F[4][o + 64 * p] = c[1][p] - c[3][p];
        }
    };
    ld(0, xa);
    long tt = 0;
    for (; tt + 2 < ntt; tt += 2) { body(tt, xa, xb, true); body(tt + 1, xb, xa, true); }
    if (tt + 1 < ntt) { body(tt, xa, xb, true); body(tt + 1, xb, xa, false); }
    else body(tt, xa, xb, false);
}

// compact-E variant: reads D, YL, YO + the tile's 256 B slot (8 B per lane,
// lanes 32..63 duplicate), writes YL, YO, T + the slot (lanes 0..31)
__global__ __launch_bounds__(256) void k_ce(double* base, long fstride, long tiles, long ntt) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long tile = (long)blockIdx.x * 4 + wid;
    d2v* F[5];
    for (int f = 0; f < 5; ++f) F[f] = reinterpret_cast<d2v*>(base + f * fstride);
    double* CE = base + 5 * fstride;  // slots: 32 doubles per tile
    auto off = [&](long tt) { return (tbase<0>(tile, tt, ntt, tiles / 4) >> 1) + lane; };
    auto so = [&](long tt) { return (tbase<0>(tile, tt, ntt, tiles / 4) >> 8) * 32 + (lane & 31); };
    struct R { d2v x[3][2]; double c; };
    R xa, xb;
    auto ld = [&](long tt, R& n) {
        const long o = off(tt);
        for (int p = 0; p < 2; ++p) { n.x[0][p] = F[0][o + 64 * p]; n.x[1][p] = F[1][o + 64 * p]; n.x[2][p] = F[3][o + 64 * p]; }
        n.c = CE[so(tt)];
    };
    auto body = [&](long tt, R& c, R& n, bool pf) {
        if (pf) { ld(tt + 1, n); __builtin_amdgcn_sched_barrier(0); }
        const long o = off(tt);
        for (int p = 0; p < 2; ++p) {
            F[1][o + 64 * p] = c.x[0][p] + c.x[1][p];
            F[3][o + 64 * p] = c.x[2][p] - c.x[1][p];
            F[4][o + 64 * p] = c.x[0][p] * c.x[2][p];
        }
        if (lane < 32) CE[so(tt)] = c.c + 1.0;
    };
    ld(0, xa);
    long tt = 0;
    for (; tt + 2 < ntt; tt += 2) { body(tt, xa, xb, true); body(tt + 1, xb, xa, true); }
    if (tt + 1 < ntt) { body(tt, xa, xb, true); body(tt + 1, xb, xa, false); }
    else body(tt, xa, xb, false);
}

__global__ __launch_bounds__(256) void k_lin(double* base, long fstride, long tiles, long ntt) {
    d2v* F[5];
    for (int f = 0; f < 5; ++f) F[f] = reinterpret_cast<d2v*>(base + f * fstride);
    const long n2 = tiles * ntt * 128;
    for (long e = (long)blockIdx.x * 256 + threadIdx.x; e < n2; e += (long)gridDim.x * 256) {
        d2v a = F[0][e], b = F[1][e], c = F[2][e], d = F[3][e];
        F[1][e] = a + b; F[2][e] = c - d; F[3][e] = a * c; F[4][e] = b - d;
    }
}

int main() {
    const long ntt = 32, tiles = 16384;  // 512^3 doubles
    const long N = tiles * ntt * 256;    // doubles per field
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto time = [&](auto kern, int grid, double* base, long fstride, const char* name, int rep, double bytes = 8.0 * N * 8) {
        float ms = 0, best = 1e9;
        for (int r = 0; r < 4; ++r) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, base, fstride, tiles, ntt);
            hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("pool %d %-4s %.3f ms  %.2f TB/s\n", rep, name, best, bytes / (best * 1e-3) / 1e12);
    };
    const int K = 6;
    const long fstride = N + 32;  // 256 B stagger
    std::vector<double*> pools(K);
    for (auto& p : pools) { CK(hipMalloc(&p, 6 * fstride * 8)); CK(hipMemset(p, 0, 6 * fstride * 8)); }
    for (int k = 0; k < K; ++k) {
        time(k_pat<0>, tiles / 4, pools[k], fstride, "GM", k);
        time(k_ce, tiles / 4, pools[k], fstride, "CE", k, 6.0 * N * 8 + 2.0 * N);
    }
    for (auto p : pools) hipFree(p);
    return 0;
}
