// K5 — the fused ADMM update of one iteration.
//
// Replaces, per element of the shard, the whole chain
//   triple_product(A,B,C)                        triple_product.m:6 (L, never stored)
//   R1, R2, O                                    triple_decomp_ADMM.m:41-43
//   R3, E = sign(R3).*max(|R3|-lambda/muO,0)     :46-47 (soft_threshold.m:2)
//   resL, resO, Y_L, Y_O                         :50-53
//   ||resL||^2, ||resO||^2                       :59
//   T_next = D - O + (1/muL_next)*Y_L            :33 of the NEXT iteration
//   W(ij,k) = sum_t T_next(ij,t) C^(t,k)         mode-1/2 half of update_A/update_B (:78,:86)
// in one pass: reads D, Y_L, E, Y_O and writes E, Y_L, Y_O, T (8 N-streams)
// plus W (N*R/n3 elements).  O is never read inside the loop (E, not O, feeds
// :42), so it is not stored: T_{k+1} = (D - O_k) + Y_L/muL_{k+1} determines it
// and k_o_fixup rebuilds O_k = (D + Y_L/muL_{k+1}) - T_{k+1} when the caller
// asks for it (relative error ~1e-16).
//
// Work decomposition: a wave owns one ij-tile (16 consecutive rows i of one
// fibre j) and walks all its t-tiles of 16.  The big tensors are tile-major
// (common.h): the wave's data is one contiguous stream, each 16x16 tile two
// fully coalesced 1 KB dwordx4 sweeps per tensor, and tile tt+1 is
// prefetched into registers while tile tt is computed.  Per t-tile:
//   L^T(t,ij)  = C^(t,:) . KR(ij,:)^T          RP/4 x v_mfma_f64_16x16x4_f64
//   elementwise update in the MFMA C/D layout  (row t = t0+(l>>4)+4r, col ij = l&15)
//   W^T(k,ij) += C^T(k,t) . T(t,ij)            (RP/16)*4 MFMAs; the C/D register
//                                              of T *is* the B operand (no shuffle)
// W^T accumulates in registers over the whole t range, so W leaves the chip
// once.
//
// Elementwise arithmetic follows MATLAB's expression order exactly; the file
// is compiled with -ffp-contract=off so no statement is fused into an FMA.
#include "kernels.h"

namespace tritd {

typedef double d4 __attribute__((ext_vector_type(4)));

static constexpr int K5_WAVES = 4;

__device__ __forceinline__ double matlab_sign(double x) {
    // sign(): 1 / -1 / 0, NaN stays NaN
    return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
}

__device__ __forceinline__ d4 mfma4(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

typedef double d2v __attribute__((ext_vector_type(2)));

template <int RP, bool PRO>
__global__ __launch_bounds__(64 * K5_WAVES) void k5_fused(K5Args a) {
    if (*a.stop) return;
    constexpr int KS = RP / 4;   // MFMA K-steps for L
    constexpr int MT = RP / 16;  // k-tiles of W
    constexpr int LDC = RP + 16; // row stride of the [t][k] C^ slice (2*LDC = 32 mod 64: no bank conflicts)
    const int lane = threadIdx.x & 63;
    const int wid = threadIdx.x >> 6;
    const int il = lane & 15;
    const int tg = lane >> 4;
    const int64_t tile = (int64_t)blockIdx.x * K5_WAVES + wid;
    const bool active = tile < a.tiles;
    const int64_t qper = a.n1p >> 4;
    const int64_t j = active ? tile / qper : 0;
    const int64_t i = active ? ((tile - j * qper) << 4) + il : 0;
    const int64_t ntt = a.ntt;
    // this lane's d2v slots inside the wave's stream: tile tt, pair p at
    // stream + tt*128 + p*64 + lane   (in units of d2v)
    const int64_t sbase = tile * ntt * 128 + lane;

    // C^ rows of one t-tile, staged once per workgroup (double buffered):
    //   sCT[k][16]  (L operand: C^(t0+l&15, 4s+(l>>4)))
    //   sC [16][LDC] (W operand: C^(t0+4r+(l>>4), 16m+(l&15)))
    __shared__ double sCT[2][RP * 16];
    __shared__ double sC[2][16 * LDC];
    // per-wave 16x16 transpose buffer for T (stored in the M3 B-operand order)
    __shared__ double tsm[K5_WAVES][16 * 17];
    double* ts = tsm[wid];
    auto stage = [&](int64_t tt, int buf) {
        // 16 rows x RP of Ch (row-major [t][RP]), 2 doubles per thread-step
        for (int e = threadIdx.x; e < 16 * RP / 2; e += 64 * K5_WAVES) {
            const int row = (2 * e) / RP, k = (2 * e) % RP;
            const double* src = a.Ch + ((tt << 4) + row) * RP + k;
            const double v0 = src[0], v1 = src[1];
            sC[buf][row * LDC + k] = v0;
            sC[buf][row * LDC + k + 1] = v1;
            sCT[buf][k * 16 + row] = v0;
            sCT[buf][(k + 1) * 16 + row] = v1;
        }
    };

    double kr[KS];
    if (!PRO) {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + tg;
            kr[s] = active ? a.Ah[i * RP + k] * a.Bh[j * RP + k] : 0.0;
        }
    }
    d4 wacc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) wacc[m] = d4{0.0, 0.0, 0.0, 0.0};

    double ssL = 0.0, ssO = 0.0;
    const IterScalars sc = a.s;
    const d2v* D2 = reinterpret_cast<const d2v*>(a.D);
    d2v* O2 = reinterpret_cast<d2v*>(a.O);
    d2v* E2 = reinterpret_cast<d2v*>(a.E);
    d2v* YL2 = reinterpret_cast<d2v*>(a.YL);
    d2v* YO2 = reinterpret_cast<d2v*>(a.YO);
    d2v* T2 = reinterpret_cast<d2v*>(a.T);

    // register double buffer: [0] = D, [1] = Y_L, [2] = E (PRO: O), [3] = Y_O
    d2v nx[4][2];
    auto load = [&](int64_t tt) {
        if (!active) return;
        const int64_t o = sbase + tt * 128;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            nx[0][p] = D2[o + 64 * p];
            nx[1][p] = YL2[o + 64 * p];
            if (PRO) {
                nx[2][p] = O2[o + 64 * p];
            } else {
                nx[2][p] = E2[o + 64 * p];
                nx[3][p] = YO2[o + 64 * p];
            }
        }
    };
#pragma unroll
    for (int q = 0; q < 4; ++q) nx[q][0] = nx[q][1] = d2v{0.0, 0.0};
    load(0);
    stage(0, 0);
    __syncthreads();
    for (int64_t tt = 0; tt < ntt; ++tt) {
        const int buf = (int)(tt & 1);
        d2v cx[4][2];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            cx[q][0] = nx[q][0];
            cx[q][1] = nx[q][1];
        }
        if (tt + 1 < ntt) {
            load(tt + 1);
            stage(tt + 1, buf ^ 1);
        }
        const int64_t o = sbase + tt * 128;
        const double* cT = sCT[buf];
        const double* cR = sC[buf];
        double tr[4];
        if (PRO) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const double d = cx[0][p][q], yl = cx[1][p][q], ov = cx[2][p][q];
                    const double tn = (d - ov) + sc.invL * yl;  // :33
                    tr[2 * p + q] = tn;
                }
            }
        } else {
            d4 lacc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < KS; ++s) lacc = mfma4(cT[(4 * s + tg) * 16 + il], kr[s], lacc);
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                d2v En2, YLn2, YOn2;
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const int r = 2 * p + q;
                    const double d = cx[0][p][q], yl = cx[1][p][q], e = cx[2][p][q],
                                 yo = cx[3][p][q];
                    const double L = lacc[r];
                    const double R1 = (d - L) + sc.invL * yl;               // :41
                    const double R2 = e - sc.invO * yo;                     // :42
                    const double On = (sc.muL * R1 + sc.muO * R2) / sc.den; // :43
                    const double R3 = On + sc.invO * yo;                    // :46
                    const double En = matlab_sign(R3) * fmax(fabs(R3) - sc.thr, 0.0);  // :47
                    const double rL = (d - L) - On;                         // :50
                    const double rO = On - En;                              // :51
                    const double YLn = yl + sc.muL * rL;                    // :52
                    const double YOn = yo + sc.muO * rO;                    // :53
                    const double Tn = (d - On) + sc.invL_next * YLn;        // :33 (k+1)
                    ssL += rL * rL;
                    ssO += rO * rO;
                    En2[q] = En;
                    YLn2[q] = YLn;
                    YOn2[q] = YOn;
                    tr[r] = Tn;
                }
                if (active) {
                    E2[o + 64 * p] = En2;
                    YL2[o + 64 * p] = YLn2;
                    YO2[o + 64 * p] = YOn2;
                }
            }
        }
        // T -> "TX" order (common.h): lane l, slot s holds T(ij = 4s+(l>>4), t = l&15)
#pragma unroll
        for (int r = 0; r < 4; ++r) ts[(tg + 4 * r) * 17 + il] = tr[r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (active) {
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                d2v tv;
                tv[0] = ts[il * 17 + 4 * (2 * p) + tg];
                tv[1] = ts[il * 17 + 4 * (2 * p + 1) + tg];
                T2[o + 64 * p] = tv;
            }
        }
        // W^T(k, ij) += sum_t C^(t,k) T(t, ij): K-step r covers t = t0+4r+(l>>4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                wacc[m] = mfma4(cR[(4 * r + tg) * LDC + 16 * m + il], tr[r], wacc[m]);
        }
        __syncthreads();  // C^ buffer `buf` and the T transpose buffer are free again
    }
    if (active) {
        // W^T C/D layout: row k = 16m + tg + 4rr, col ij = il
        const int64_t wbase = (tile << 4) + il;
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
                a.Wk[(int64_t)(16 * m + tg + 4 * rr) * a.plane + wbase] = wacc[m][rr];
    }

    if (!PRO) {
        // fixed-order block reduction of the residual norms
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            ssL += __shfl_xor(ssL, off);
            ssO += __shfl_xor(ssO, off);
        }
        __shared__ double red[2][K5_WAVES];
        if (lane == 0) {
            red[0][wid] = ssL;
            red[1][wid] = ssO;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double x = 0.0, y = 0.0;
            for (int w = 0; w < K5_WAVES; ++w) {
                x += red[0][w];
                y += red[1][w];
            }
            a.partial[2 * blockIdx.x] = x;
            a.partial[2 * blockIdx.x + 1] = y;
        }
    }
}

int k5_grid(const Geom& g) { return (int)cdiv(g.tiles, K5_WAVES); }

void launch_k5(const Geom& g, const K5Args& a, bool prologue, hipStream_t st) {
    const dim3 grid(k5_grid(g)), block(64 * K5_WAVES);
#define K5_CASE(RPV)                                                           \
    case RPV:                                                                  \
        if (prologue)                                                          \
            hipLaunchKernelGGL((k5_fused<RPV, true>), grid, block, 0, st, a);  \
        else                                                                   \
            hipLaunchKernelGGL((k5_fused<RPV, false>), grid, block, 0, st, a); \
        break;
    switch (g.RP) {
        K5_CASE(16)
        K5_CASE(32)
        K5_CASE(48)
        K5_CASE(64)
        default:
            throw Error(TRITD_ERR_UNSUPPORTED, "rank not supported by K5");
    }
#undef K5_CASE
    TRITD_CHECK_LAUNCH();
}

// Sum n (x, y) pairs in a fixed order: per-thread strided sums, then a
// fixed tree.  One block.
__global__ __launch_bounds__(256) void k_reduce_pairs(const double* __restrict__ p, int n,
                                                      double* out, const int* stop) {
    if (stop && *stop) return;
    __shared__ double sx[256], sy[256];
    double x = 0.0, y = 0.0;
    for (int b = threadIdx.x; b < n; b += 256) {
        x += p[2 * b];
        y += p[2 * b + 1];
    }
    sx[threadIdx.x] = x;
    sy[threadIdx.x] = y;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            sx[threadIdx.x] += sx[threadIdx.x + w];
            sy[threadIdx.x] += sy[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out[0] = sx[0];
        out[1] = sy[0];
    }
}

void launch_reduce_pairs(const double* partial, int n, double* out, const int* stop,
                         hipStream_t st) {
    hipLaunchKernelGGL(k_reduce_pairs, dim3(1), dim3(256), 0, st, partial, n, out, stop);
    TRITD_CHECK_LAUNCH();
}

// ctrl[0] = stop flag, ctrl[1] = iterations completed (k of :68)
__global__ void k_finish(const double* ss, double normD, int k, double tol, double* errHist,
                         double* errL, double* errO, int* ctrl) {
    if (ctrl[0]) return;
    const double eL = sqrt(ss[0]) / normD;  // norm(resL(:))/normD
    const double eO = sqrt(ss[1]) / normD;  // norm(resO(:))/normD
    const double e = eL + eO;               // :59
    errHist[k - 1] = e;
    errL[k - 1] = eL;
    errO[k - 1] = eO;
    ctrl[1] = k;
    if (k > 1 && fabs(e - errHist[k - 2]) < tol * errHist[k - 2]) ctrl[0] = 1;  // :63
}

void launch_finish(const double* ss, double normD, int k, double tol, double* errHist, double* errL,
                   double* errO, int* ctrl, hipStream_t st) {
    hipLaunchKernelGGL(k_finish, dim3(1), dim3(1), 0, st, ss, normD, k, tol, errHist, errL, errO,
                       ctrl);
    TRITD_CHECK_LAUNCH();
}

// O_k = (D + (1/muL_{k+1}) Y_L) - T_{k+1}: D, Y_L, O in tile-major order,
// T in the TX order of the same tile (common.h)
__global__ __launch_bounds__(256) void k_o_fixup(const double* __restrict__ D,
                                                 const double* __restrict__ YL,
                                                 const double* __restrict__ T, double invL_next,
                                                 double* __restrict__ O, int64_t Np) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < Np; e += (int64_t)gridDim.x * 256) {
        const int w = (int)(e & 255);
        const int p = w >> 7, l = (w & 127) >> 1, q = w & 1;
        const int r = 2 * p + q;
        const int il = l & 15, tl = (l >> 4) + 4 * r;  // element of this TM slot
        const int s = il >> 2, lx = ((il & 3) << 4) | tl;  // its TX slot
        const int64_t tx = (e & ~(int64_t)255) + ((s >> 1) << 7) + (lx << 1) + (s & 1);
        O[e] = (D[e] + invL_next * YL[e]) - T[tx];
    }
}

void launch_o_fixup(const Geom& g, const double* D, const double* YL, const double* T,
                    double invL_next, double* O, hipStream_t st) {
    int64_t b = cdiv(g.Np, 256);
    if (b > 16384) b = 16384;
    hipLaunchKernelGGL(k_o_fixup, dim3((unsigned)b), dim3(256), 0, st, D, YL, T, invL_next, O, g.Np);
    TRITD_CHECK_LAUNCH();
}

}  // namespace tritd
