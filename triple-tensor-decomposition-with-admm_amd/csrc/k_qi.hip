// Qi-model variant of the ADMM factor updates (opts.model = 'qi'; SURVEY.md
// §8f rank 4).  The executed reference uses the rank-r^2 CP builders of
// fast_robust_triple_tensor/buildF.m; origin_triple_tensor/buildF.m:2-6,
// buildG.m:7-11 and buildH.m:7-11 instead build the design matrices of Qi's
// 3-index triple product
//     L(i,j,t) = sum_{p,q,s} A(i,q,s) B(p,j,s) C(p,q,t)
// (the sum origin_triple_tensor/triple_product.m:8-19 spells out).  With the
// factor matrices of common.h (Ah(i,q+rs) = A(i,q,s), Bh(j,p+rs) = B(p,j,s),
// Ch(t,p+rq) = C(p,q,t)) and W = T x3 Ch (the same W K5 produces for CP):
//   F(q+rs, jt) = sum_p B(p,j,s) C(p,q,t):  M1(i,q+rs) = sum_j sum_p W(ij,p+rq) Bh(j,p+rs)
//   G(p+rs, it) = sum_q A(i,q,s) C(p,q,t):  M2(j,p+rs) = sum_i sum_q W(ij,p+rq) Ah(i,q+rs)
//   H(p+rq, ij) = sum_s A(i,q,s) B(p,j,s):  M3(t,k)    = sum_ij T(ij,t) H(k,ij)   (K2 on H)
//   L(ij,t)     = sum_k H(k,ij) Ch(t,k)                                           (K5 on H)
// and the design Grams come from the factor Grams without forming F, G, H:
//   F F'[(q,s),(q',s')] = sum_{p,p'} (Bh'Bh)[p+rs][p'+rs'] (Ch'Ch)[p+rq][p'+rq']
//   G G'[(p,s),(p',s')] = sum_{q,q'} (Ah'Ah)[q+rs][q'+rs'] (Ch'Ch)[p+rq][p'+rq']
//   H H'[(p,q),(p',q')] = sum_{s,s'} (Ah'Ah)[q+rs][q'+rs'] (Bh'Bh)[p+rs][p'+rs']
// H is materialised once per iteration (n1p*n2*RP doubles, row-major by ij)
// and fed to K2 and K5 as their Khatri-Rao operand (K5Args::ahj/bhj).
// All sums run in a fixed order (deterministic); memory-bound and small next
// to K5/K2.
#include "kernels.h"

namespace tritd {

// H[(j*n1p + i)*RP + k], k = p + r*q: one thread per element, k fastest
__global__ __launch_bounds__(256) void k_qi_h(const double* __restrict__ Ah,
                                              const double* __restrict__ Bh, double* H,
                                              int64_t n1p, int64_t n2, int r, int RP,
                                              const int* stop) {
    if (stop && *stop) return;
    const int R = r * r;
    const int64_t total = n1p * n2 * RP;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * 256) {
        const int k = (int)(e % RP);
        const int64_t ij = e / RP;
        const int64_t j = ij / n1p, i = ij - j * n1p;
        double v = 0.0;
        if (k < R) {
            const int p = k % r, q = k / r;
            const double* a = Ah + i * RP + q;
            const double* b = Bh + j * RP + p;
            for (int s = 0; s < r; ++s) v = fma(a[r * s], b[r * s], v);
        }
        H[e] = v;
    }
}

void launch_qi_h(const Geom& g, int r, const double* Ah, const double* Bh, double* H,
                 const int* stop, hipStream_t st) {
    const int64_t total = g.n1p * g.n2 * g.RP;
    const int64_t blocks = std::min<int64_t>(cdiv(total, 256), 8192);
    hipLaunchKernelGGL(k_qi_h, dim3((unsigned)blocks), dim3(256), 0, st, Ah, Bh, H, g.n1p, g.n2, r,
                       g.RP, stop);
    TRITD_CHECK_LAUNCH();
}

// M1(i, q+rs): block = 64 rows i x one q, the 4 waves take j = w mod 4
// (fixed-order LDS sum), lane = row i, r accumulators (s).
__global__ __launch_bounds__(256) void k_m1_qi(const double* __restrict__ Wk,
                                               const double* __restrict__ Bh, double* M1,
                                               int64_t n1p, int64_t n2, int64_t plane, int r,
                                               int RP, const int* stop) {
    if (*stop) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + lane;
    const int q = blockIdx.y;
    double acc[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = 0.0;
    if (i < n1p) {
        for (int64_t j = w; j < n2; j += 4) {
            const double* bj = Bh + j * RP;
            for (int p = 0; p < r; ++p) {
                const double x = Wk[(int64_t)(p + r * q) * plane + j * n1p + i];
#pragma unroll
                for (int s = 0; s < 8; ++s)
                    if (s < r) acc[s] = fma(x, bj[p + r * s], acc[s]);
            }
        }
    }
    __shared__ double red[4][8][64];
#pragma unroll
    for (int s = 0; s < 8; ++s) red[w][s][lane] = acc[s];
    __syncthreads();
    if (w == 0 && i < n1p) {
        for (int s = 0; s < r; ++s)
            M1[i * RP + q + r * s] =
                ((red[0][s][lane] + red[1][s][lane]) + red[2][s][lane]) + red[3][s][lane];
        if (q == 0)
            for (int k = r * r; k < RP; ++k) M1[i * RP + k] = 0.0;
    }
}

void launch_m1_qi(const Geom& g, int r, const double* Wk, const double* Bh, double* M1,
                  const int* stop, hipStream_t st) {
    if (r > 8) throw Error(TRITD_ERR_UNSUPPORTED, "Qi model: r <= 8");
    hipLaunchKernelGGL(k_m1_qi, dim3((unsigned)cdiv(g.n1p, 64), (unsigned)r), dim3(256), 0, st, Wk,
                       Bh, M1, g.n1p, g.n2, g.plane, r, g.RP, stop);
    TRITD_CHECK_LAUNCH();
}

// M2(j, p+rs): one wave per (j, p), lanes over i, r accumulators (s),
// butterfly sum over the lanes.
__global__ __launch_bounds__(256) void k_m2_qi(const double* __restrict__ Wk,
                                               const double* __restrict__ AhT, double* M2,
                                               int64_t n1p, int64_t n2, int64_t plane, int r,
                                               int RP, const int* stop) {
    if (*stop) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t j = blockIdx.x;
    const int p = blockIdx.y * 4 + w;
    if (p >= r) return;
    double acc[8];
#pragma unroll
    for (int s = 0; s < 8; ++s) acc[s] = 0.0;
    for (int64_t i = lane; i < n1p; i += 64) {
        for (int q = 0; q < r; ++q) {
            const double x = Wk[(int64_t)(p + r * q) * plane + j * n1p + i];
#pragma unroll
            for (int s = 0; s < 8; ++s)
                if (s < r) acc[s] = fma(x, AhT[(int64_t)(q + r * s) * n1p + i], acc[s]);
        }
    }
#pragma unroll
    for (int s = 0; s < 8; ++s) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) acc[s] += __shfl_xor(acc[s], off);
    }
    if (lane == 0) {
        for (int s = 0; s < r; ++s) M2[j * RP + p + r * s] = acc[s];
        if (p == 0)
            for (int k = r * r; k < RP; ++k) M2[j * RP + k] = 0.0;
    }
}

void launch_m2_qi(const Geom& g, int r, const double* Wk, const double* AhT, double* M2,
                  const int* stop, hipStream_t st) {
    if (r > 8) throw Error(TRITD_ERR_UNSUPPORTED, "Qi model: r <= 8");
    hipLaunchKernelGGL(k_m2_qi, dim3((unsigned)g.n2, (unsigned)cdiv(r, 4)), dim3(256), 0, st, Wk,
                       AhT, M2, g.n1p, g.n2, g.plane, r, g.RP, stop);
    TRITD_CHECK_LAUNCH();
}

// Design Gram of the Qi builders from two factor Grams (RP x RP, row-major),
// out[(u+rv)][(u'+rv')] with the contracted pair (c, c') of the mode:
//   mode 0 (F F', out (q,s)): X[c+rv][c'+rv'] * Y[c+ru][c'+ru']   X=Bh'Bh, Y=Ch'Ch
//   mode 1 (G G', out (p,s)): X[c+rv][c'+rv'] * Y[u+rc][u'+rc']   X=Ah'Ah, Y=Ch'Ch
//   mode 2 (H H', out (p,q)): X[v+rc][v'+rc'] * Y[u+rc][u'+rc']   X=Ah'Ah, Y=Bh'Bh
// Zero outside the leading R x R block (the solve pads with the identity).
__global__ __launch_bounds__(256) void k_qi_gram(const double* __restrict__ X,
                                                 const double* __restrict__ Y, double* out, int r,
                                                 int RP, int mode, const int* stop) {
    if (stop && *stop) return;
    const int R = r * r;
    for (int e = threadIdx.x; e < RP * RP; e += 256) {
        const int a = e / RP, b = e % RP;
        double v = 0.0;
        if (a < R && b < R) {
            const int u = a % r, vv = a / r, u2 = b % r, v2 = b / r;
            for (int c = 0; c < r; ++c)
                for (int c2 = 0; c2 < r; ++c2) {
                    double x, y;
                    if (mode == 0) {
                        x = X[(c + r * vv) * RP + c2 + r * v2];
                        y = Y[(c + r * u) * RP + c2 + r * u2];
                    } else if (mode == 1) {
                        x = X[(c + r * vv) * RP + c2 + r * v2];
                        y = Y[(u + r * c) * RP + u2 + r * c2];
                    } else {
                        x = X[(vv + r * c) * RP + v2 + r * c2];
                        y = Y[(u + r * c) * RP + u2 + r * c2];
                    }
                    v = fma(x, y, v);
                }
        }
        out[e] = v;
    }
}

void launch_qi_gram(int RP, int r, int mode, const double* X, const double* Y, double* out,
                    const int* stop, hipStream_t st) {
    hipLaunchKernelGGL(k_qi_gram, dim3(1), dim3(256), 0, st, X, Y, out, r, RP, mode, stop);
    TRITD_CHECK_LAUNCH();
}

__global__ __launch_bounds__(256) void k_fill(double* x, int64_t n, double v) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
        x[e] = v;
}

void launch_fill(double* x, int64_t n, double v, hipStream_t st) {
    hipLaunchKernelGGL(k_fill, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 1024)), dim3(256), 0,
                       st, x, n, v);
    TRITD_CHECK_LAUNCH();
}

}  // namespace tritd
