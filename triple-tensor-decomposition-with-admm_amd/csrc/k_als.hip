// Kernels of the ALS variant, fast_robust_triple_tensor/triple_decomp_ALS.m
// (DESIGN.md §8).
//
// One ALS iteration k reads the fixed data tensor X twice:
//   k_als_fit   Xhat = triple_product(A,B,C)            triple_decomp_ALS.m:15 (never stored)
//               ||X(:) - Xhat(:)||^2                     :16
//               W(ij,k) = sum_t X(ij,t) C^(t,k)          mode-1/2 half of :26-27 and :31-32
//               (C^ is the C of iteration k for both: B is updated with the
//               new A but the old C, :30-32)
//   K2 (k_m3)   X3 * H'                                  :36-37, over the TX copy of X
// plus the small M1 / M2 / Gram / solve / apply kernels the ADMM shares.
// k_als_fit is K5 without the ADMM elementwise chain: one wave per ij-tile
// walking its t-tiles (X tile-major, common.h), tile tt+1 prefetched while
// tile tt is computed, L and W on v_mfma_f64_16x16x4_f64 with C^ staged per
// workgroup in LDS.  Algorithmic traffic N*8 B read + W written.
#include "kernels.h"

namespace tritd {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

static constexpr int FIT_WAVES = 4;

__device__ __forceinline__ d4 als_mfma4(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// sign() of MATLAB without branches: 1, -1, 0 for +-0, NaN for NaN
__device__ __forceinline__ double nc_sign(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : x); }

template <int RP, bool NCV>
__global__ __launch_bounds__(64 * FIT_WAVES) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_als_fit(AlsFitArgs a) {
    if (*a.stop) return;
    constexpr int KS = RP / 4;    // K-steps of the L MFMA
    constexpr int MT = RP / 16;   // k-tiles of W
    constexpr int LDC = RP + 16;  // padded row stride of the [t][k] slice
    constexpr int SK = 17;        // odd [k][t] row stride: conflict-free staging writes (k_admm.hip)
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int il = lane & 15;
    const int tg = lane >> 4;
    const int64_t tile = (int64_t)blockIdx.x * FIT_WAVES + wid;
    const bool active = tile < a.tiles;
    const int64_t qper = a.n1p >> 4;
    const int64_t j = active ? tile / qper : 0;
    const int64_t i = active ? ((tile - j * qper) << 4) + il : 0;
    const int64_t ntt = a.ntt;

    __shared__ double sCT[2][RP * SK];   // L operand  C^(t0 + l&15, 4s + l>>4)
    __shared__ double sC[2][16 * LDC];   // W operand  C^(t0 + 4r + l>>4, 16m + l&15)
    constexpr int SP = 16 * RP / 2;
    constexpr int NS = (SP + 64 * FIT_WAVES - 1) / (64 * FIT_WAVES);
    d2v sv[NS];
    auto stage_load = [&](int64_t tt) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * FIT_WAVES;
            if (SP % (64 * FIT_WAVES) == 0 || e < SP)
                sv[q] = *reinterpret_cast<const d2v*>(a.Ch + (tt << 4) * RP + 2 * e);
        }
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * FIT_WAVES;
            if (SP % (64 * FIT_WAVES) == 0 || e < SP) {
                const int row = (2 * e) / RP, k = (2 * e) % RP;
                sC[buf][row * LDC + k] = sv[q][0];
                sC[buf][row * LDC + k + 1] = sv[q][1];
                sCT[buf][k * SK + row] = sv[q][0];
                sCT[buf][(k + 1) * SK + row] = sv[q][1];
            }
        }
    };

    double kr[KS];  // (A^ o B^)(ij, 4s + l>>4): the Khatri-Rao row of this lane's ij
    {
        // unconditional loads, all issued first (k_admm.hip: the KR gather)
        double av[KS], bv[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + tg;
            av[s] = a.Ah[i * RP + k];
            bv[s] = a.Bh[j * RP + k];
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) kr[s] = active ? av[s] * bv[s] : 0.0;
    }
    d4 wacc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) wacc[m] = d4{0.0, 0.0, 0.0, 0.0};
    double ss = 0.0;
    const d2v* X2 = reinterpret_cast<const d2v*>(a.X);

    // Two named register sets, the t-walk unrolled by two (a copy cur = next
    // would make the compiler wait for the prefetch at the copy; k_admm.hip).
    struct Regs {
        d2v x[2];
        d2v e[NCV ? 3 : 1][2];  // NCV: O, Lam, Gam of the same tile
    };
    const d2v* Oi2 = reinterpret_cast<const d2v*>(a.O_in);
    d2v* Oo2 = reinterpret_cast<d2v*>(a.O_out);
    d2v* L2 = reinterpret_cast<d2v*>(a.Lam);
    d2v* G2 = reinterpret_cast<d2v*>(a.Gam);
    auto load = [&](int64_t tt, Regs& nx) {
        const int64_t o = (tm_tile_base(tile, tt, ntt) >> 1) + lane;
        nx.x[0] = X2[o];
        nx.x[1] = X2[o + 64];
        if constexpr (NCV) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                nx.e[0][h] = Oi2[o + 64 * h];
                nx.e[1][h] = L2[o + 64 * h];
                nx.e[2][h] = G2[o + 64 * h];
            }
        }
    };
    auto body = [&](int64_t tt, int buf, Regs& cx, Regs& nx, bool pf) {
        if (pf) {
            stage_load(tt + 1);
            load(tt + 1, nx);
            __builtin_amdgcn_sched_barrier(0);
        }
        const double* cT = sCT[buf];
        const double* cR = sC[buf];
        d4 lacc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < KS; ++s) lacc = als_mfma4(cT[(4 * s + tg) * SK + il], kr[s], lacc);
        double xr[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) xr[r] = cx.x[r >> 1][r & 1];
        if constexpr (NCV) {
            // test.m:36,44,47,48,62 in MATLAB's operator order (-ffp-contract=off)
            const int64_t o = (tm_tile_base(tile, tt, ntt) >> 1) + lane;
            d2v on[2], ln[2], gn[2];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double x = xr[r], L = lacc[r];
                const double O = cx.e[0][r >> 1][r & 1], Lm = cx.e[1][r >> 1][r & 1],
                             Gm = cx.e[2][r >> 1][r & 1];
                const double Y = ((x - O) + a.rho * (L + Lm / a.rho)) / a.onep;
                const double xy = x - Y;
                const double z = xy + Gm / a.rho;
                const double On = nc_sign(z) * fmax(fabs(z) - a.tau, 0.0);
                const double d = xy - On;
                on[r >> 1][r & 1] = On;
                ln[r >> 1][r & 1] = Lm + a.rho * (L - Y);
                gn[r >> 1][r & 1] = Gm + a.rho * d;
                ss += d * d;
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                Oo2[o + 64 * h] = on[h];
                L2[o + 64 * h] = ln[h];
                G2[o + 64 * h] = gn[h];
            }
        } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double d = xr[r] - lacc[r];  // X(:) - Xhat(:)
                ss += d * d;
            }
        }
        // W^T(k, ij) += sum_t C^(t,k) X(t, ij): the C/D register r of the X
        // tile (t = t0 + 4r + l>>4, ij = l&15) is directly the B operand
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int m = 0; m < MT; ++m)
                wacc[m] = als_mfma4(cR[(4 * r + tg) * LDC + 16 * m + il], xr[r], wacc[m]);
        if (pf) stage_store(buf ^ 1);
        __syncthreads();
        __builtin_amdgcn_sched_barrier(0);
    };

    Regs xa, xb;
    xa.x[0] = xa.x[1] = xb.x[0] = xb.x[1] = d2v{0.0, 0.0};
#pragma unroll
    for (int q = 0; q < (NCV ? 3 : 1); ++q)
        xa.e[q][0] = xa.e[q][1] = xb.e[q][0] = xb.e[q][1] = d2v{0.0, 0.0};
    load(0, xa);
    stage_load(0);
    stage_store(0);
    __syncthreads();
    int64_t tt = 0;
    for (; tt + 2 < ntt; tt += 2) {
        body(tt, 0, xa, xb, true);
        body(tt + 1, 1, xb, xa, true);
    }
    if (tt + 1 < ntt) {
        body(tt, 0, xa, xb, true);
        body(tt + 1, 1, xb, xa, false);
    } else {
        body(tt, 0, xa, xb, false);
    }
    if (active) {
        const int64_t wbase = (tile << 4) + il;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
                a.Wk[(int64_t)(16 * m + tg + 4 * rr) * a.plane + wbase] = wacc[m][rr];
    }
    // fixed-order block reduction (pairs: the second is 0, k_reduce_pairs)
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off);
    __shared__ double red[FIT_WAVES];
    if (lane == 0) red[wid] = ss;
    __syncthreads();
    if (threadIdx.x == 0) {
        double x = 0.0;
        for (int w = 0; w < FIT_WAVES; ++w) x += red[w];
        a.partial[2 * blockIdx.x] = x;
        a.partial[2 * blockIdx.x + 1] = 0.0;
    }
}

int als_fit_grid(const Geom& g) { return (int)cdiv(g.tiles, FIT_WAVES); }

void launch_als_fit(const Geom& g, const AlsFitArgs& a, hipStream_t st) {
    const dim3 grid(als_fit_grid(g)), block(64 * FIT_WAVES);
#define FIT_CASE(RPV)                                                                  \
    case RPV:                                                                          \
        if (a.ncvx)                                                                    \
            hipLaunchKernelGGL((k_als_fit<RPV, true>), grid, block, 0, st, a);         \
        else                                                                           \
            hipLaunchKernelGGL((k_als_fit<RPV, false>), grid, block, 0, st, a);        \
        break;
    switch (g.RP) {
        FIT_CASE(16)
        FIT_CASE(32)
        FIT_CASE(48)
        FIT_CASE(64)
        default: throw Error(TRITD_ERR_UNSUPPORTED, "rank not supported by the ALS fit kernel");
    }
#undef FIT_CASE
    TRITD_CHECK_LAUNCH();
}

// errHist(k) = norm(X(:) - Xhat(:)) / Xnorm and the stop test of
// triple_decomp_ALS.m:16,20-23.  ctrl[0] = stop (set BEFORE the update of
// iteration k, so the update kernels of k early-exit and A, B, C stay those
// of iteration k), ctrl[1] = entries of errHist.
__global__ void k_als_finish(const double* ss, double Xnorm, int k, double tol, double* errHist,
                             int* ctrl) {
    if (ctrl[0]) return;
    const double e = sqrt(ss[0]) / Xnorm;
    errHist[k - 1] = e;
    ctrl[1] = k;
    if (k > 1 && fabs(e - errHist[k - 2]) < tol * errHist[k - 2]) ctrl[0] = 1;
}

void launch_als_finish(const double* ss, double Xnorm, int k, double tol, double* errHist,
                       int* ctrl, hipStream_t st) {
    hipLaunchKernelGGL(k_als_finish, dim3(1), dim3(1), 0, st, ss, Xnorm, k, tol, errHist, ctrl);
    TRITD_CHECK_LAUNCH();
}

// Reweighted shrink of the A update of test.m:82-92 (after the ridge-1e-12
// solve and apply): W_A = 1./((abs(A1) + epsilon).^(theta - p)) (:86),
// A1 = sign(A1).*max(abs(A1) - gamma_A.*W_A, 0) (:89, weighted_soft_threshold
// :97-101); written to Ah and its transposed copy AhT.  Zero pads stay zero.
__global__ __launch_bounds__(256) void k_ncvx_shrink(double* Ah, double* AhT, int64_t n1p, int RP,
                                                     double gamma, double eps, double expo,
                                                     const int* stop) {
    if (*stop) return;
    const int64_t n = n1p * RP;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        const double x = Ah[e];
        const double w = 1.0 / pow(fabs(x) + eps, expo);
        const double v = nc_sign(x) * fmax(fabs(x) - gamma * w, 0.0);
        Ah[e] = v;
        const int64_t i = e / RP, k = e - i * RP;
        AhT[k * n1p + i] = v;
    }
}

void launch_ncvx_shrink(const Geom& g, double* Ah, double* AhT, double gamma, double eps,
                        double expo, const int* stop, hipStream_t st) {
    const int64_t n = g.n1p * g.RP;
    hipLaunchKernelGGL(k_ncvx_shrink, dim3((unsigned)std::min<int64_t>(cdiv(n, 256), 2048)),
                       dim3(256), 0, st, Ah, AhT, g.n1p, g.RP, gamma, eps, expo, stop);
    TRITD_CHECK_LAUNCH();
}

// Tile-major -> TX (the B-operand order of K2, common.h), tile by tile:
// TX slot (s, l) at (s>>1)*128 + 2l + (s&1) holds (i%16 = 4s + l>>4,
// t%16 = l&15).  One-off per ALS solve (X is fixed).
__global__ __launch_bounds__(256) void k_tm_to_tx(const double* __restrict__ src,
                                                  double* __restrict__ dst, int64_t Ntm) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < Ntm;
         e += (int64_t)gridDim.x * 256) {
        const int w = (int)(e & 255);
        const int s = ((w >> 7) << 1) | (w & 1), l = (w & 127) >> 1;
        const int il = 4 * s + (l >> 4), tl = l & 15;  // element of this TX slot
        const int r = tl >> 2, lm = ((tl & 3) << 4) | il;   // its TM slot
        dst[e] = src[(e & ~(int64_t)255) + ((r >> 1) << 7) + (lm << 1) + (r & 1)];
    }
}

void launch_tm_to_tx(const Geom& g, const double* src, double* dst, hipStream_t st) {
    int64_t b = cdiv(g.Ntm, 256);
    if (b > 16384) b = 16384;
    hipLaunchKernelGGL(k_tm_to_tx, dim3((unsigned)b), dim3(256), 0, st, src, dst, g.Ntm);
    TRITD_CHECK_LAUNCH();
}

}  // namespace tritd
