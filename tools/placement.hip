// K5's HBM access pattern (read D, Y_L and the compact-E slot; write Y_L in
// place, T and the slot; one wave per ij-tile walking its t-tiles with the
// next tile prefetched — exactly k_pool_probe of k_admm.hip) at 512^3, timed
// on EIGHT candidate allocations held at once, per placement strategy:
//   pool256   one allocation, tensors 1 GiB + 256 B apart (the library's pool)
//   pool2M    one allocation, tensors 1 GiB + 2 MiB + 256 B apart
//   separate  one hipMalloc per tensor
//   record    one allocation, D/Y_L/T tiles of one (ij-tile, t-tile)
//             adjacent: 6 KiB records in the group-major tile order
// The spread inside a strategy is the placement sensitivity.
//   hipcc --offload-arch=gfx950 -O3 tools/placement.hip -o tools/placement.bin
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

constexpr long N = 512L * 512 * 512;  // doubles per tensor
constexpr long NTT = 32, TILES4 = 16384, SLOT = 32;

// group-major tile base (doubles), as common.h tm_tile_base
__device__ __forceinline__ long tm_base(long tile, long tt) {
    return (((tile >> 2) * NTT + tt) * 4 + (tile & 3)) << 8;
}

// REC: field f of tile ordinal b at b * 768 + f * 256 doubles
template <bool REC>
__global__ __launch_bounds__(256) void k_pat(double* D, double* YL, double* T, double* CE) {
    const int lane = threadIdx.x & 63;
    const long tile = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    auto addr = [&](int f, long tt) -> d2v* {
        const long b = tm_base(tile, tt);
        if (REC) return reinterpret_cast<d2v*>(D + (b >> 8) * 768 + f * 256);
        return reinterpret_cast<d2v*>((f == 0 ? D : f == 1 ? YL : T) + b);
    };
    struct R {
        d2v x[2][2];
        double ce;
    };
    R xa, xb;
    auto load = [&](long tt, R& nx) {
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int f = 0; f < 2; ++f) nx.x[f][p] = addr(f, tt)[lane + 64 * p];
        nx.ce = CE[(tm_base(tile, tt) >> 8) * SLOT + (lane & 31)];
    };
    auto body = [&](long tt, R& c, R& n, bool pf) {
        if (pf) {
            load(tt + 1, n);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            addr(1, tt)[lane + 64 * p] = c.x[0][p] + c.x[1][p];
            addr(2, tt)[lane + 64 * p] = c.x[0][p] - c.x[1][p];
        }
        CE[(tm_base(tile, tt) >> 8) * SLOT + (lane & 31)] = c.ce + 1.0;
    };
    load(0, xa);
    long tt = 0;
    for (; tt + 2 < NTT; tt += 2) {
        body(tt, xa, xb, true);
        body(tt + 1, xb, xa, true);
    }
    body(tt, xa, xb, true);
    body(tt + 1, xb, xa, false);
}

struct Cand {
    std::vector<void*> allocs;
    double *D, *YL, *T, *CE;
};

static Cand make(int strat) {
    Cand c;
    const size_t tb = N * 8, sb = (N / 256) * SLOT * 8;
    auto al = [&](size_t b) {
        void* p;
        CK(hipMalloc(&p, b));
        c.allocs.push_back(p);
        return static_cast<char*>(p);
    };
    if (strat == 0 || strat == 1) {
        const size_t st = tb + (strat == 0 ? 256 : (2u << 20) + 256);
        char* p = al(3 * st + sb + 4096);
        c.D = (double*)p;
        c.YL = (double*)(p + st);
        c.T = (double*)(p + 2 * st);
        c.CE = (double*)(p + 3 * st);
    } else if (strat == 2) {
        c.D = (double*)al(tb);
        c.YL = (double*)al(tb);
        c.T = (double*)al(tb);
        c.CE = (double*)al(sb);
    } else {
        char* p = al(3 * tb + sb + 4096);
        c.D = c.YL = c.T = (double*)p;
        c.CE = (double*)(p + 3 * tb);
    }
    for (void* a : c.allocs) (void)a;
    CK(hipMemset(c.D, 0, 8));
    return c;
}

int main(int argc, char** argv) {
    const int ncand = argc > 1 ? std::atoi(argv[1]) : 8;
    const char* names[4] = {"pool256", "pool2M", "separate", "record"};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int strat = 0; strat < 4; ++strat) {
        std::vector<Cand> cs;
        for (int q = 0; q < ncand; ++q) cs.push_back(make(strat));
        std::vector<double> med;
        for (auto& c : cs) {
            std::vector<float> t;
            for (int rep = 0; rep < 6; ++rep) {
                CK(hipEventRecord(e0, 0));
                if (strat == 3)
                    hipLaunchKernelGGL(k_pat<true>, dim3(TILES4 / 4), dim3(256), 0, 0, c.D, c.YL, c.T, c.CE);
                else
                    hipLaunchKernelGGL(k_pat<false>, dim3(TILES4 / 4), dim3(256), 0, 0, c.D, c.YL, c.T, c.CE);
                CK(hipGetLastError());
                CK(hipEventRecord(e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            med.push_back(t[t.size() / 2]);
        }
        double lo = *std::min_element(med.begin(), med.end()), hi = *std::max_element(med.begin(), med.end());
        std::printf("%-9s ms:", names[strat]);
        for (double m : med) std::printf(" %.4f", m);
        std::printf("  | min %.4f max %.4f spread %.1f%%\n", lo, hi, 100.0 * (hi - lo) / lo);
        std::fflush(stdout);
        for (auto& c : cs)
            for (void* a : c.allocs) CK(hipFree(a));
    }
    return 0;
}
