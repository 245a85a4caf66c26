// K5's memory pattern without compute: 4 read + 4 write d2v streams, a wave owns
// one ij-tile = a contiguous stream of ntt*2 KB per array, tile tt+1 prefetched.
// Variants: waves per CU (occupancy via LDS padding), rotation, nontemporal.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef double d2v __attribute__((ext_vector_type(2)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <int NT, int ROT, int GS>
__global__ __launch_bounds__(256) void k_pat(const d2v* __restrict__ a0, const d2v* __restrict__ a1,
                                             const d2v* __restrict__ a2, const d2v* __restrict__ a3,
                                             d2v* b0, d2v* b1, d2v* b2, d2v* b3, long tiles, long ntt) {
    extern __shared__ double pad[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const long tile = (long)blockIdx.x * 4 + wid;
    if (tile >= tiles) return;
    if (lane == 999) pad[0] = 0;  // keep dynamic LDS (occupancy knob)
    // group-major layout: GS consecutive tiles interleaved per t-tile
    const long grp = tile / GS, gi = tile % GS;
    const long rot = ROT ? ((long)blockIdx.x * 7) % ntt : 0;
    auto ph = [&](long tt) { long x = tt + rot; return x >= ntt ? x - ntt : x; };
    auto off = [&](long tt) { return ((grp * ntt + ph(tt)) * GS + gi) * 128 + lane; };
    d2v nx[4][2];
    auto ld = [&](long tt) {
        const long o = off(tt);
        for (int p = 0; p < 2; ++p) {
            if (NT & 1) {
                nx[0][p] = __builtin_nontemporal_load(a0 + o + 64 * p);
                nx[1][p] = __builtin_nontemporal_load(a1 + o + 64 * p);
                nx[2][p] = __builtin_nontemporal_load(a2 + o + 64 * p);
                nx[3][p] = __builtin_nontemporal_load(a3 + o + 64 * p);
            } else {
                nx[0][p] = a0[o + 64 * p]; nx[1][p] = a1[o + 64 * p];
                nx[2][p] = a2[o + 64 * p]; nx[3][p] = a3[o + 64 * p];
            }
        }
    };
    ld(0);
    for (long tt = 0; tt < ntt; ++tt) {
        d2v c[4][2];
        for (int q = 0; q < 4; ++q) { c[q][0] = nx[q][0]; c[q][1] = nx[q][1]; }
        if (tt + 1 < ntt) ld(tt + 1);
        const long o = off(tt);
        for (int p = 0; p < 2; ++p) {
            d2v x = c[0][p] + c[1][p], y = c[2][p] - c[3][p], z = c[0][p] * c[2][p], w = c[1][p] - c[3][p];
            if (NT & 2) {
                __builtin_nontemporal_store(x, b0 + o + 64 * p); __builtin_nontemporal_store(y, b1 + o + 64 * p);
                __builtin_nontemporal_store(z, b2 + o + 64 * p); __builtin_nontemporal_store(w, b3 + o + 64 * p);
            } else {
                b0[o + 64 * p] = x; b1[o + 64 * p] = y; b2[o + 64 * p] = z; b3[o + 64 * p] = w;
            }
        }
    }
}

int main() {
    const long ntt = 32, tiles = 16384;  // 512^3 doubles
    const long n2 = tiles * ntt * 128;   // d2v per array
    std::vector<d2v*> buf(8);
    for (auto& p : buf) { CK(hipMalloc(&p, n2 * 16 + 4096)); CK(hipMemset(p, 0, n2 * 16)); }
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const double bytes = 8.0 * n2 * 16;
    auto run = [&](auto kern, size_t lds, const char* name) {
        hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        float ms = 0, best = 1e9;
        for (int r = 0; r < 5; ++r) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(tiles / 4), dim3(256), lds, 0, buf[0], buf[1], buf[2], buf[3], buf[4], buf[5], buf[6], buf[7], tiles, ntt);
            hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        printf("%-28s lds %6zu: %.3f ms  %.2f TB/s\n", name, lds, best, bytes / (best * 1e-3) / 1e12);
    };
    for (size_t lds : {(size_t)40 << 10, (size_t)64 << 10}) {
        run(k_pat<0, 0, 1>, lds, "plain GS1");
        run(k_pat<0, 1, 1>, lds, "plain GS1 rot");
        run(k_pat<3, 0, 1>, lds, "nt GS1");
        run(k_pat<0, 0, 4>, lds, "plain GS4");
        run(k_pat<1, 0, 4>, lds, "ntload GS4");
        run(k_pat<2, 0, 4>, lds, "ntstore GS4");
        run(k_pat<3, 0, 4>, lds, "nt GS4");
        run(k_pat<3, 0, 16>, lds, "nt GS16");
        run(k_pat<0, 0, 1>, lds, "plain GS1 again");
    }
    return 0;
}
