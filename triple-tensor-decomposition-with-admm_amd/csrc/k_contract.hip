// Mode contractions (MTTKRP) and the small R x R linear algebra of
// update_A / update_B / update_C (triple_decomp_ADMM.m:73-95).
//
//  update_A  (X1*F.')*pinv(F*F.'+l2 I)   = M1 * inv((B^TB)o(C^TC) + l2 I)
//            M1(i,k) = sum_j W(i,j,k) B^(j,k)        (W from K5, dimension tree)
//  update_B  (X2*G')*pinv(G*G'+l2 I)     = M2 * inv((A^TA)o(C^TC) + l2 I)
//            M2(j,k) = sum_i W(i,j,k) A^(i,k)        (new A, old C — same W)
//  update_C  (X3*H')*pinv(H*H'+1e-9 I)   = M3 * inv((A^TA)o(B^TB) + 1e-9 I)
//            M3(t,k) = sum_ij T(ij,t) A^(i,k) B^(j,k)   MFMA, this file's K2
// F*F.' = (B^TB) o (C^TC) is the Hadamard identity of the Khatri-Rao design
// matrices built by buildF/G/H (buildF.m:17-21): F, G, H are never formed.
#include "kernels.h"

namespace tritd {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ d4 mfma4(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// M1(i,k) = sum_j Wk[k][j*n1p + i] * Bh[j][k]; block = 64 rows x 4 j-slices
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_m1(const double* __restrict__ Wk,
                                            const double* __restrict__ Bh, double* M1,
                                            int64_t n1p, int64_t n2, int64_t plane, int RP,
                                            const int* stop) {
    if (*stop) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + lane;
    const int k = blockIdx.y;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (i < n1p) {
        const double* wp = Wk + (int64_t)k * plane + i;
        const double* bp = Bh + k;
        int64_t j = w;
        for (; j + 12 < n2; j += 16) {  // 4 independent chains, j = w + 4m
            a0 = fma(wp[j * n1p], bp[j * RP], a0);
            a1 = fma(wp[(j + 4) * n1p], bp[(j + 4) * RP], a1);
            a2 = fma(wp[(j + 8) * n1p], bp[(j + 8) * RP], a2);
            a3 = fma(wp[(j + 12) * n1p], bp[(j + 12) * RP], a3);
        }
        for (; j < n2; j += 4) a0 = fma(wp[j * n1p], bp[j * RP], a0);
    }
    __shared__ double red[4][64];
    red[w][lane] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (w == 0 && i < n1p) M1[i * RP + k] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

void launch_m1(const Geom& g, const double* Wk, const double* Bh, double* M1, const int* stop,
               hipStream_t st) {
    hipLaunchKernelGGL(k_m1, dim3((unsigned)cdiv(g.n1p, 64), g.RP), dim3(256), 0, st, Wk, Bh, M1,
                       g.n1p, g.n2, g.plane, g.RP, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// M2(j,k) = sum_i Wk[k][j*n1p + i] * AhT[k][i]; one wave per (j, k)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_m2(const double* __restrict__ Wk,
                                            const double* __restrict__ AhT, double* M2,
                                            int64_t n1p, int64_t n2, int64_t plane, int RP,
                                            const int* stop) {
    if (*stop) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t j = blockIdx.x;
    const int k = blockIdx.y * 4 + w;
    if (k >= RP) return;
    const double* wp = Wk + (int64_t)k * plane + j * n1p;
    const double* ap = AhT + (int64_t)k * n1p;
    double acc = 0.0;
    for (int64_t i = lane; i < n1p; i += 64) acc = fma(wp[i], ap[i], acc);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) M2[j * RP + k] = acc;
}

void launch_m2(const Geom& g, const double* Wk, const double* AhT, double* M2, const int* stop,
               hipStream_t st) {
    hipLaunchKernelGGL(k_m2, dim3((unsigned)g.n2, (unsigned)cdiv(g.RP, 4)), dim3(256), 0, st, Wk,
                       AhT, M2, g.n1p, g.n2, g.plane, g.RP, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// M3 partials: part[y][t][k] = sum over the block's ij-chunks of T(ij,t) KR(ij,k)
//   grid.x = t-blocks of 64, grid.y = split index; chunk = 64 ij (4 ij-tiles)
//   LDS: T tile [64 t][66] (pad 2 -> conflict-free ds_read_b64 of the B operand)
//        KR tile [64 ij][SKR]  (SKR = RP or RP+16 so 2*SKR = 32 mod 64)
//   MFMA: D(k, t) += sum_ij KR(ij,k) T(ij,t); K-step s covers ij = 4s..4s+3
//   The next chunk's T is prefetched into registers during the MFMAs.
// ---------------------------------------------------------------------------
constexpr int M3_TS = 66;

template <int RP>
struct M3Cfg {
    static constexpr int MT = RP / 16;
    static constexpr int KSPLIT = (MT == 3) ? 1 : 4 / MT;  // waves sharing one k-tile
    static constexpr int SKR = (RP % 32 == 0) ? RP + 16 : RP;
    static constexpr int LDS_T = 64 * M3_TS;
    static constexpr int LDS_KR = 64 * SKR;
};

template <int RP>
__global__ __launch_bounds__(256, 2) void k_m3(const double* __restrict__ T,
                                               const double* __restrict__ Ah,
                                               const double* __restrict__ Bh, double* part,
                                               int64_t n1p, int64_t n3p, int64_t ntt,
                                               int64_t tiles, int split, const int* stop) {
    if (*stop) return;
    using C = M3Cfg<RP>;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    double* sT = lds;             // [64][M3_TS]
    double* sK = lds + C::LDS_T;  // [64][SKR]

    const int th = threadIdx.x, lane = th & 63, wid = th >> 6;
    const int il = lane & 15, tg = lane >> 4;
    const int64_t t0 = (int64_t)blockIdx.x * 64;
    const int64_t nchunk = cdiv(tiles, 4);
    const int64_t qper = n1p >> 4;

    const int mt = (C::MT == 3) ? wid : wid % C::MT;
    const int kpart = (C::MT == 3) ? 0 : wid / C::MT;
    const bool wave_on = wid < C::MT * C::KSPLIT;

    d4 acc[4];
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[n] = d4{0.0, 0.0, 0.0, 0.0};

    // T staging from the tile-major layout: the chunk's 4 ij-tiles x the
    // block's 4 t-tiles are 16 contiguous 2 KB tiles = 2048 d2v; thread th in
    // round m takes d2v idx = m*256 + th (1 KB contiguous per wave-instruction)
    typedef double d2v __attribute__((ext_vector_type(2)));
    const d2v* T2 = reinterpret_cast<const d2v*>(T);
    d2v pre[8];
    auto load_T = [&](int64_t c) {
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int idx = m * 256 + th;
            const int q = idx >> 7, w = idx & 127;
            const int64_t g = c * 4 + (q & 3), tt = (int64_t)blockIdx.x * 4 + (q >> 2);
            if (g < tiles && tt < ntt)
                pre[m] = T2[(g * ntt + tt) * 128 + w];
            else
                pre[m] = d2v{0.0, 0.0};
        }
    };
    auto store_T = [&]() {
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int idx = m * 256 + th;
            const int q = idx >> 7, w = idx & 127;
            const int gi = q & 3, ti = q >> 2, p = w >> 6, l = w & 63;
            const int row = 16 * ti + (l >> 4) + 8 * p, col = 16 * gi + (l & 15);
            sT[row * M3_TS + col] = pre[m][0];        // r = 2p
            sT[(row + 4) * M3_TS + col] = pre[m][1];  // r = 2p + 1
        }
    };

    int64_t c = blockIdx.y;
    if (c < nchunk) load_T(c);
    for (; c < nchunk; c += split) {
        __syncthreads();  // previous chunk's LDS reads are done
        store_T();
        // KR tile: entry e -> (ij = e / RP, k = e % RP)
        for (int e = th; e < 64 * RP; e += 256) {
            const int ijl = e / RP, k = e - ijl * RP;
            const int64_t tile = c * 4 + (ijl >> 4);
            double v = 0.0;
            if (tile < tiles) {
                const int64_t j = tile / qper;
                const int64_t i = ((tile - j * qper) << 4) + (ijl & 15);
                v = Ah[i * RP + k] * Bh[j * RP + k];
            }
            sK[ijl * C::SKR + k] = v;
        }
        __syncthreads();
        if (c + split < nchunk) load_T(c + split);  // prefetch, lands during the MFMAs
        if (wave_on) {
#pragma unroll 4
            for (int s = kpart; s < 16; s += C::KSPLIT) {
                const double av = sK[(4 * s + tg) * C::SKR + 16 * mt + il];
#pragma unroll
                for (int n = 0; n < 4; ++n) {
                    const double bv = sT[(16 * n + il) * M3_TS + 4 * s + tg];
                    acc[n] = mfma4(av, bv, acc[n]);
                }
            }
        }
    }

    // combine the KSPLIT waves that share a k-tile (fixed order), write partial
    __syncthreads();
    double* red = lds;  // reuse: [4 waves][4 n][4 rr][64 lanes]
    if (C::KSPLIT > 1) {
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) red[((wid * 4 + n) * 4 + rr) * 64 + lane] = acc[n][rr];
        __syncthreads();
    }
    if (wave_on && kpart == 0) {
        double* out = part + (int64_t)blockIdx.y * n3p * RP;
#pragma unroll
        for (int n = 0; n < 4; ++n)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                double v = acc[n][rr];
                if (C::KSPLIT > 1)
                    for (int q = 1; q < C::KSPLIT; ++q)
                        v += red[(((wid + q * C::MT) * 4 + n) * 4 + rr) * 64 + lane];
                const int64_t t = t0 + 16 * n + il;
                const int k = 16 * mt + tg + 4 * rr;
                if (t < n3p) out[t * RP + k] = v;
            }
    }
}

// M3[t][k] = sum_y part[y][t][k]  (fixed order)
__global__ __launch_bounds__(256) void k_m3_reduce(const double* __restrict__ part, double* M3,
                                                   int64_t count, int split, const int* stop) {
    if (*stop) return;
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= count) return;
    double s = 0.0;
    for (int y = 0; y < split; ++y) s += part[(int64_t)y * count + e];
    M3[e] = s;
}

int m3_split(const Geom& g) {
    const int64_t nchunk = cdiv(g.tiles, 4);
    const int64_t tb = cdiv(g.n3p, 64);
    int64_t split = cdiv(512, tb);  // ~2 workgroups per CU
    if (split > nchunk) split = nchunk;
    if (split < 1) split = 1;
    return (int)split;
}

void launch_m3(const Geom& g, const double* T, const double* Ah, const double* Bh, double* part,
               double* M3, const int* stop, hipStream_t st) {
    const int split = m3_split(g);
    const dim3 grid((unsigned)cdiv(g.n3p, 64), (unsigned)split);
#define M3_CASE(RPV)                                                                          \
    case RPV: {                                                                               \
        const size_t lds = (M3Cfg<RPV>::LDS_T + M3Cfg<RPV>::LDS_KR) * sizeof(double);         \
        static bool attr_set = false;                                                         \
        if (!attr_set) {                                                                      \
            TRITD_HIP(hipFuncSetAttribute((const void*)k_m3<RPV>,                             \
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
            attr_set = true;                                                                  \
        }                                                                                     \
        hipLaunchKernelGGL(k_m3<RPV>, grid, dim3(256), lds, st, T, Ah, Bh, part, g.n1p, g.n3p, \
                           g.ntt, g.tiles, split, stop);                                    \
    } break;
    switch (g.RP) {
        M3_CASE(16)
        M3_CASE(32)
        M3_CASE(48)
        M3_CASE(64)
        default:
            throw Error(TRITD_ERR_UNSUPPORTED, "rank not supported by M3");
    }
#undef M3_CASE
    TRITD_CHECK_LAUNCH();
    const int64_t count = g.n3p * g.RP;
    hipLaunchKernelGGL(k_m3_reduce, dim3((unsigned)cdiv(count, 256)), dim3(256), 0, st, part, M3,
                       count, split, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Gram: G[k][k'] = sum_i X[i][k] X[i][k'] (rows in 256/RP interleaved groups)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gram(const double* __restrict__ X, int64_t rows, int RP,
                                              double* G, const int* stop) {
    if (stop && *stop) return;
    const int k = blockIdx.x;
    const int groups = 256 / RP;
    const int kk = threadIdx.x % RP, grp = threadIdx.x / RP;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    if (grp < groups) {
        const int64_t st = groups;
        int64_t i = grp;
        for (; i + 3 * st < rows; i += 4 * st) {
            a0 = fma(X[i * RP + k], X[i * RP + kk], a0);
            a1 = fma(X[(i + st) * RP + k], X[(i + st) * RP + kk], a1);
            a2 = fma(X[(i + 2 * st) * RP + k], X[(i + 2 * st) * RP + kk], a2);
            a3 = fma(X[(i + 3 * st) * RP + k], X[(i + 3 * st) * RP + kk], a3);
        }
        for (; i < rows; i += st) a0 = fma(X[i * RP + k], X[i * RP + kk], a0);
    }
    __shared__ double red[256];
    red[threadIdx.x] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (grp == 0) {
        double s = red[kk];
        for (int q = 1; q < groups; ++q) s += red[q * RP + kk];
        G[k * RP + kk] = s;
    }
}

void launch_gram(int RP, const double* X, int64_t rows, double* G, const int* stop,
                 hipStream_t st) {
    hipLaunchKernelGGL(k_gram, dim3(RP), dim3(256), 0, st, X, rows, RP, G, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Ginv = inv(P o Q + alpha I): in-place Gauss-Jordan in LDS, one block,
// thread (column c = th&63, rows h, h+4, ...).  The Gram is SPD (ridge
// alpha > 0) so no pivoting is needed; the smallest Gauss-Jordan pivot
// (= smallest LDL^T pivot) is compared with MATLAB's pinv tolerance
// max(size)*eps(max sigma) and flags[0] is raised when pinv could truncate
// (triple_decomp_ADMM.m:78,86,93 use pinv).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_solve(const double* __restrict__ P,
                                               const double* __restrict__ Q, int RP, int R,
                                               double alpha, double* Ginv, int* flags,
                                               const int* stop) {
    if (*stop) return;
    __shared__ double M[64][65];
    const int th = threadIdx.x;
    const int c = th & 63, h = th >> 6;
    const bool colok = c < R;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const int i = h + 4 * m;
        if (i < R && colok) {
            double v = P[i * RP + c] * Q[i * RP + c];
            if (i == c) v = v + alpha;
            M[i][c] = v;
        }
    }
    __syncthreads();
    double minpiv = 1e308, maxpiv = 0.0;
    for (int p = 0; p < R; ++p) {
        const double piv = M[p][p];
        minpiv = fmin(minpiv, piv);
        maxpiv = fmax(maxpiv, piv);
        const double d = 1.0 / piv;
        const double prv = colok ? ((c == p) ? d : M[p][c] * d) : 0.0;  // new pivot row
        double f[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            const int i = h + 4 * m;
            f[m] = (i < R) ? M[i][p] : 0.0;
        }
        __syncthreads();
        if (colok) {
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int i = h + 4 * m;
                if (i < R) {
                    if (i == p)
                        M[i][c] = prv;
                    else
                        M[i][c] = ((c == p) ? 0.0 : M[i][c]) - f[m] * prv;
                }
            }
        }
        __syncthreads();
    }
    for (int e = th; e < RP * RP; e += 256) {
        const int i = e / RP, cc = e - i * RP;
        Ginv[e] = (i < R && cc < R) ? M[i][cc] : 0.0;
    }
    if (th == 0) {
        // eps(x) = 2^(floor(log2 x) - 52)
        const double tol = (double)R * ldexp(1.0, ilogb(maxpiv) - 52);
        if (!(minpiv > 1e3 * tol)) atomicOr(flags, 1);
    }
}

void launch_solve(int RP, int R, const double* P, const double* Q, double alpha, double* Ginv,
                  int* flags, const int* stop, hipStream_t st) {
    if (R > 64) throw Error(TRITD_ERR_UNSUPPORTED, "R > 64 solve");
    hipLaunchKernelGGL(k_solve, dim3(1), dim3(256), 0, st, P, Q, RP, R, alpha, Ginv, flags, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Y = M * Ginv (rows x RP), optional transposed copy YT[k*ldT + i]
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_apply(const double* __restrict__ M, int64_t rows,
                                               const double* __restrict__ Ginv, int RP, double* Y,
                                               double* YT, int64_t ldT, const int* stop) {
    if (stop && *stop) return;
    __shared__ double g[64 * 64];
    for (int e = threadIdx.x; e < RP * RP; e += 256) g[e] = Ginv[e];
    __syncthreads();
    const int rpb = 256 / RP;  // rows per pass
    const int k = threadIdx.x % RP, rl = threadIdx.x / RP;
    for (int64_t i = (int64_t)blockIdx.x * 16 + rl; i < (int64_t)blockIdx.x * 16 + 16; i += rpb) {
        if (i >= rows) break;
        double s = 0.0;
        for (int q = 0; q < RP; ++q) s = fma(M[i * RP + q], g[q * RP + k], s);
        Y[i * RP + k] = s;
        if (YT) YT[(int64_t)k * ldT + i] = s;
    }
}

void launch_apply(int RP, const double* M, int64_t rows, const double* Ginv, double* Y, double* YT,
                  int64_t ldT, const int* stop, hipStream_t st) {
    hipLaunchKernelGGL(k_apply, dim3((unsigned)cdiv(rows, 16)), dim3(256), 0, st, M, rows, Ginv,
                       RP, Y, YT, ldT, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Virtual-shard all-reduce: sum in shard order, broadcast back.
// ---------------------------------------------------------------------------
struct VsumArgs {
    double* b[16];
};
__global__ void k_vsum(VsumArgs a, int nb, int64_t count) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (e >= count) return;
    double s = a.b[0][e];
    for (int p = 1; p < nb; ++p) s += a.b[p][e];
    for (int p = 0; p < nb; ++p) a.b[p][e] = s;
}

void launch_vsum(double* const* bufs, int nbufs, int64_t count, hipStream_t st) {
    if (nbufs > 16) throw Error(TRITD_ERR_ARG, "at most 16 virtual shards");
    VsumArgs a;
    for (int p = 0; p < nbufs; ++p) a.b[p] = bufs[p];
    hipLaunchKernelGGL(k_vsum, dim3((unsigned)cdiv(count, 256)), dim3(256), 0, st, a, nbufs, count);
    TRITD_CHECK_LAUNCH();
}

}  // namespace tritd
