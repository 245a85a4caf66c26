// K5's derived-Y_O memory pattern (read D, Y_L and two compact-E slots;
// write Y_L, T and one slot per 16x16 tile; one wave per ij-tile walking its
// t-tiles) without K5's arithmetic, under the structural choices K5 has to
// make: waves per SIMD (capped with dynamic LDS), prefetch depth (register
// sets in flight), a workgroup barrier per t-tile, and a dependent f64 chain
// of NF operations per element standing in for the compute latency.
// build: hipcc --offload-arch=gfx950 -O3 tools/k5_floor.hip -o tools/k5_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d2v __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ inline long tbase(long g, long tt, long ntt) { return ((((g >> 2) * ntt + tt) << 2) + (g & 3)) << 8; }

template <int DEPTH, bool SYNC, int NF, int NM = 0, int NI = 0>
__global__ __launch_bounds__(256) void k_floor(const double* D, double* YL, double* T, double* CEa,
                                               const double* CEb, long tiles, long ntt, double* sink) {
    extern __shared__ double pad[];
    const int lane = threadIdx.x & 63;
    const long tile = (long)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const d2v* D2 = reinterpret_cast<const d2v*>(D);
    d2v* Y2 = reinterpret_cast<d2v*>(YL);
    d2v* T2 = reinterpret_cast<d2v*>(T);
    struct R { d2v d[2], y[2]; double ca, cb; };
    R r[DEPTH + 1];
    auto off = [&](long tt) { return (tbase(tile, tt, ntt) >> 1) + lane; };
    auto so = [&](long tt) { return (tbase(tile, tt, ntt) >> 8) * 32 + (lane & 31); };
    auto ld = [&](long tt, R& x) {
        const long o = off(tt);
        x.d[0] = D2[o]; x.d[1] = D2[o + 64];
        x.y[0] = Y2[o]; x.y[1] = Y2[o + 64];
        x.ca = CEa[so(tt)]; x.cb = CEb[so(tt)];
    };
    double acc = 0.0;
    typedef double d4 __attribute__((ext_vector_type(4)));
    d4 m0 = {0, 0, 0, 0}, m1 = m0, m2 = m0, m3 = m0;
    unsigned iu = lane;
#pragma unroll
    for (int q = 0; q < DEPTH; ++q) ld(q < ntt ? q : ntt - 1, r[q]);
    for (long t0 = 0; t0 < ntt; t0 += DEPTH + 1) {
#pragma unroll
        for (int u = 0; u <= DEPTH; ++u) {
            const long tt = t0 + u;
            if (tt >= ntt) break;
            R& c = r[u];
            R& n = r[(u + DEPTH) % (DEPTH + 1)];
            const long tn = tt + DEPTH < ntt ? tt + DEPTH : ntt - 1;
            ld(tn, n);
            __builtin_amdgcn_sched_barrier(0);
            const long o = off(tt);
            d2v a0 = c.d[0] + c.y[0], a1 = c.d[1] - c.y[1];
            double e = c.ca + c.cb;
#pragma unroll
            for (int f = 0; f < NF; ++f) {
                a0 = a0 * 0.999 + e;
                a1 = a1 * 1.001 - e;
                e = e * 0.5 + a0[0];
            }
#pragma unroll
            for (int q = 0; q < NM / 4; ++q) {
                m0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[0], a1[1], m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[1], a1[0], m1, 0, 0, 0);
                m2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[0], a0[0], m2, 0, 0, 0);
                m3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[1], a0[1], m3, 0, 0, 0);
            }
#pragma unroll
            for (int q = 0; q < NI; ++q) asm volatile("v_add_u32 %0, %0, %1" : "+v"(iu) : "v"(lane));
            Y2[o] = a0; Y2[o + 64] = a1;
            T2[o] = a1; T2[o + 64] = a0;
            if (lane < 32) CEa[so(tt)] = e;
            acc += e;
            if (SYNC) __syncthreads();
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (acc == 1.2345 || m0[0] + m1[1] + m2[2] + m3[3] == 1.5 || iu == 77u) sink[0] = pad[0];
}

int main() {
    const long n = 512, ntt = n / 16, tiles = n * n / 16;
    const size_t N = (size_t)tiles * ntt * 256;
    double *D, *YL, *T, *CEa, *CEb, *sink;
    CK(hipMalloc(&D, N * 8)); CK(hipMalloc(&YL, N * 8)); CK(hipMalloc(&T, N * 8));
    CK(hipMalloc(&CEa, N)); CK(hipMalloc(&CEb, N)); CK(hipMalloc(&sink, 64));
    CK(hipMemset(D, 0, N * 8)); CK(hipMemset(YL, 0, N * 8)); CK(hipMemset(T, 0, N * 8));
    CK(hipMemset(CEa, 0, N)); CK(hipMemset(CEb, 0, N));
    const double bytes = 4.0 * N * 8 + 3.0 * N;  // 4 dense streams + 3 slot accesses per tile
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto run = [&](auto kern, const char* name, size_t lds) -> int {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, dim3(tiles / 4), dim3(256), lds, 0, D, YL, T, CEa, CEb, tiles, ntt, sink);
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (ms < best) best = ms;
        }
        printf("%-34s lds %6zu: %.3f ms  %.2f TB/s\n", name, lds, best, bytes / (best * 1e-3) / 1e12);
        return 0;
    };
    const size_t L2W = 68 * 1024, L3W = 52 * 1024, L1W = 120 * 1024, L0 = 0;
#define RUN(DP, SY, NF, LDS) run(k_floor<DP, SY, NF>, "depth " #DP " sync " #SY " nf " #NF, LDS)
#define RUNM(DP, SY, NF, NM, NI, LDS) run(k_floor<DP, SY, NF, NM, NI>, "depth " #DP " sync " #SY " nf " #NF " mfma " #NM " int " #NI, LDS)
    RUN(1, true, 0, L2W); RUN(2, true, 0, L2W); RUN(1, true, 0, L1W);
    RUNM(1, true, 0, 32, 0, L2W); RUNM(2, true, 0, 32, 0, L2W); RUNM(1, true, 0, 32, 0, L1W); RUNM(3, true, 0, 32, 0, L1W);
    RUNM(1, true, 24, 32, 0, L2W); RUNM(1, true, 24, 32, 150, L2W); RUNM(2, true, 24, 32, 150, L2W);
    RUNM(1, true, 24, 32, 150, L1W); RUNM(3, true, 24, 32, 150, L1W);
    RUNM(1, false, 24, 32, 150, L2W);
    return 0;
}
