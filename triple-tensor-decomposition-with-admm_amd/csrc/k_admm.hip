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
#ifndef K5_NT
#define K5_NT 0  // nontemporal hints on the streamed tensors: bit 0 loads, bit 1 stores
#endif
#ifndef K5_EXP
#define K5_EXP 0  // timing experiments only (tools/): drop parts of the t-tile work
#endif

__device__ __forceinline__ double matlab_sign(double x) {
    // sign(): 1 / -1 / 0 (also for -0), NaN stays NaN; selects only, no
    // branches (a divergent branch would break the K5 loop's exact vmcnt waits)
    const double s = x == 0.0 ? 0.0 : __builtin_copysign(1.0, x);
    return __builtin_isnan(x) ? x : s;
}

__device__ __forceinline__ d4 mfma4(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d2v ld2(const d2v* p) {
    if (K5_NT & 1) return __builtin_nontemporal_load(p);
    return *p;
}
__device__ __forceinline__ void st2(d2v v, d2v* p) {
    if (K5_NT & 2)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

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
    // this lane's d2v slot of pair p in t-tile tt: tm_tile_base(tile, tt)/2 + 64p + lane

    // C^ rows of one t-tile, staged once per workgroup (double buffered):
    //   sCT[k][16]  (L operand: C^(t0+l&15, 4s+(l>>4)))
    //   sC [16][LDC] (W operand: C^(t0+4r+(l>>4), 16m+(l&15)))
    __shared__ double sCT[2][RP * 16];
    __shared__ double sC[2][16 * LDC];
    // per-wave 16x16 transpose buffer for T (stored in the M3 B-operand order)
    __shared__ double tsm[K5_WAVES][16 * 17];
    double* ts = tsm[wid];
    // Rotated t-walk: resident workgroups start at different t-tiles so that
    // their concurrent streams do not advance in lockstep 64 KB apart (HBM
    // channel hot-spotting).  Any fixed order is deterministic.
    const int64_t rot = a.rot ? ((int64_t)blockIdx.x * 7) % ntt : 0;
    auto phys = [&](int64_t tt) { int64_t x = tt + rot; return x >= ntt ? x - ntt : x; };
    // Staging is split so that its global loads are issued before the tile
    // prefetch and its LDS writes come after this t-tile's compute: vmcnt is
    // in-order, so a wait on a load issued after the prefetch would also wait
    // for the prefetch (measured: the prefetch was serialized every t-tile).
    constexpr int SP = 16 * RP / 2;                 // (v0,v1) pairs per slice
    constexpr int NS = (SP + 64 * K5_WAVES - 1) / (64 * K5_WAVES);
    d2v sv[NS];
    auto stage_load = [&](int64_t tt) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * K5_WAVES;
            if (SP % (64 * K5_WAVES) == 0 || e < SP)
                sv[q] = *reinterpret_cast<const d2v*>(a.Ch + (phys(tt) << 4) * RP + 2 * e);
        }
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * 64 * K5_WAVES;
            if (SP % (64 * K5_WAVES) == 0 || e < SP) {
                const int row = (2 * e) / RP, k = (2 * e) % RP;
                sC[buf][row * LDC + k] = sv[q][0];
                sC[buf][row * LDC + k + 1] = sv[q][1];
                sCT[buf][k * 16 + row] = sv[q][0];
                sCT[buf][(k + 1) * 16 + row] = sv[q][1];
            }
        }
    };
    auto stage = [&](int64_t tt, int buf) {
        stage_load(tt);
        stage_store(buf);
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

    // Two register sets [0] = D, [1] = Y_L, [2] = E (PRO: O), [3] = Y_O.  The
    // t-walk is unrolled by two so that the sets alternate by name: a copy
    // cur = next would make the compiler wait for the prefetch at the copy.
    // Inside the walk nothing depends on `active` (a wave past the last tile
    // streams the zero-filled group padding, see common.h), so the
    // steady-state loop has no control-flow joins and the in-order vmcnt
    // waits stay exact.
    auto load = [&](int64_t tt, d2v (&nx)[4][2]) {
        const int64_t o = (tm_tile_base(tile, phys(tt), ntt) >> 1) + lane;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            nx[0][p] = ld2(D2 + o + 64 * p);
            nx[1][p] = ld2(YL2 + o + 64 * p);
            if (PRO) {
                nx[2][p] = ld2(O2 + o + 64 * p);
            } else {
                nx[2][p] = ld2(E2 + o + 64 * p);
                nx[3][p] = ld2(YO2 + o + 64 * p);
            }
        }
    };
    // one t-tile: cx holds its data; if `pf`, tile tt+1 is prefetched into nx
    // and its C^ slice staged into buffer buf^1
    auto body = [&](int64_t tt, int buf, d2v (&cx)[4][2], d2v (&nx)[4][2], bool pf) {
        if (pf) {
            stage_load(tt + 1);
            load(tt + 1, nx);
            // keep the prefetch at the top: the scheduler otherwise sinks it
            // next to the stores (less register pressure, no latency hiding)
            __builtin_amdgcn_sched_barrier(0);
        }
        const int64_t o = (tm_tile_base(tile, phys(tt), ntt) >> 1) + lane;
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
            if (!(K5_EXP & 1))
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
                st2(En2, E2 + o + 64 * p);
                st2(YLn2, YL2 + o + 64 * p);
                st2(YOn2, YO2 + o + 64 * p);
            }
        }
        // T -> "TX" order (common.h): lane l, slot s holds T(ij = 4s+(l>>4), t = l&15)
        if (K5_EXP & 8) {
#pragma unroll
            for (int p = 0; p < 2; ++p) st2(d2v{tr[2 * p], tr[2 * p + 1]}, T2 + o + 64 * p);
        } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) ts[(tg + 4 * r) * 17 + il] = tr[r];
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            d2v tv;
            tv[0] = ts[il * 17 + 4 * (2 * p) + tg];
            tv[1] = ts[il * 17 + 4 * (2 * p + 1) + tg];
            st2(tv, T2 + o + 64 * p);
        }
        }
        // W^T(k, ij) += sum_t C^(t,k) T(t, ij): K-step r covers t = t0+4r+(l>>4)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if (!(K5_EXP & 2)) {
#pragma unroll
            for (int m = 0; m < MT; ++m)
                wacc[m] = mfma4(cR[(4 * r + tg) * LDC + 16 * m + il], tr[r], wacc[m]);
            } else {
                for (int m = 0; m < MT; ++m) wacc[m][0] += tr[r];
            }
        }
        if (pf) stage_store(buf ^ 1);  // buf^1 was last read in t-tile tt-1
        if (!(K5_EXP & 4)) __syncthreads();  // C^ buffer `buf` and the T transpose buffer are free again
    };

    d2v xa[4][2], xb[4][2];
#pragma unroll
    for (int q = 0; q < 4; ++q) xa[q][0] = xa[q][1] = xb[q][0] = xb[q][1] = d2v{0.0, 0.0};
    load(0, xa);
    stage(0, 0);
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
__device__ __forceinline__ void finish_body(const double* ss, double normD, int k, double tol,
                                            double* errHist, double* errL, double* errO, int* ctrl) {
    const double eL = sqrt(ss[0]) / normD;  // norm(resL(:))/normD
    const double eO = sqrt(ss[1]) / normD;  // norm(resO(:))/normD
    const double e = eL + eO;               // :59
    errHist[k - 1] = e;
    errL[k - 1] = eL;
    errO[k - 1] = eO;
    ctrl[1] = k;
    if (k > 1 && fabs(e - errHist[k - 2]) < tol * errHist[k - 2]) ctrl[0] = 1;  // :63
}

__global__ void k_finish(const double* ss, double normD, int k, double tol, double* errHist,
                         double* errL, double* errO, int* ctrl) {
    if (ctrl[0]) return;
    finish_body(ss, normD, k, tol, errHist, errL, errO, ctrl);
}

__global__ __launch_bounds__(256) void k_reduce_finish(const double* __restrict__ p, int n,
                                                       double normD, int k, double tol,
                                                       double* errHist, double* errL, double* errO,
                                                       int* ctrl) {
    if (ctrl[0]) return;
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
        const double ss[2] = {sx[0], sy[0]};
        finish_body(ss, normD, k, tol, errHist, errL, errO, ctrl);
    }
}

void launch_reduce_finish(const double* partial, int n, double normD, int k, double tol,
                          double* errHist, double* errL, double* errO, int* ctrl, hipStream_t st) {
    hipLaunchKernelGGL(k_reduce_finish, dim3(1), dim3(256), 0, st, partial, n, normD, k, tol,
                       errHist, errL, errO, ctrl);
    TRITD_CHECK_LAUNCH();
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
    int64_t b = cdiv(g.Ntm, 256);
    if (b > 16384) b = 16384;
    hipLaunchKernelGGL(k_o_fixup, dim3((unsigned)b), dim3(256), 0, st, D, YL, T, invL_next, O, g.Ntm);
    TRITD_CHECK_LAUNCH();
}

// Placement probe: K5's exact HBM pattern (read D, Y_L, E, Y_O; write E, Y_L,
// Y_O in place and T; one wave per ij-tile walking its t-tiles, prefetched)
// without the arithmetic.  K5 is HBM-bound (dropping all its compute leaves
// its time unchanged) and its bandwidth depends on where the pool landed
// physically; the session times candidate pools with this and keeps the
// fastest.  Contents are overwritten with garbage.
__global__ __launch_bounds__(256) void k_pool_probe(double* D, double* E, double* YL, double* YO,
                                                    double* T, int64_t tiles4, int64_t ntt) {
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (tile >= tiles4) return;
    d2v* P[5] = {reinterpret_cast<d2v*>(D), reinterpret_cast<d2v*>(YL), reinterpret_cast<d2v*>(E),
                 reinterpret_cast<d2v*>(YO), reinterpret_cast<d2v*>(T)};
    auto off = [&](int64_t tt) { return (tm_tile_base(tile, tt, ntt) >> 1) + lane; };
    d2v xa[4][2], xb[4][2];
    auto load = [&](int64_t tt, d2v (&nx)[4][2]) {
        const int64_t o = off(tt);
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int f = 0; f < 4; ++f) nx[f][p] = P[f][o + 64 * p];
    };
    auto body = [&](int64_t tt, d2v (&c)[4][2], d2v (&n)[4][2], bool pf) {
        if (pf) {
            load(tt + 1, n);
            __builtin_amdgcn_sched_barrier(0);
        }
        const int64_t o = off(tt);
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            P[1][o + 64 * p] = c[0][p] + c[1][p];
            P[2][o + 64 * p] = c[2][p] - c[3][p];
            P[3][o + 64 * p] = c[1][p] - c[3][p];
            P[4][o + 64 * p] = c[0][p] - c[2][p];
        }
    };
    load(0, xa);
    int64_t tt = 0;
    for (; tt + 2 < ntt; tt += 2) {
        body(tt, xa, xb, true);
        body(tt + 1, xb, xa, true);
    }
    if (tt + 1 < ntt) {
        body(tt, xa, xb, true);
        body(tt + 1, xb, xa, false);
    } else {
        body(tt, xa, xb, false);
    }
}

void launch_pool_probe(const Geom& g, double* D, double* E, double* YL, double* YO, double* T,
                       hipStream_t st) {
    hipLaunchKernelGGL(k_pool_probe, dim3((unsigned)(g.tiles4 / 4)), dim3(256), 0, st, D, E, YL, YO,
                       T, g.tiles4, g.ntt);
    TRITD_CHECK_LAUNCH();
}

}  // namespace tritd
