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
#include <algorithm>
#include <atomic>
#include <string>
#include <cstdlib>
#include <utility>

#include "finish.h"
#include "kernels.h"
#include "sweep.h"
#include "wtrace.h"

namespace tritd {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ d4 mfma4(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// M1(i,k) = sum_j Wk[k][j*n1p + i] * Bh[j][k]; block = 64 rows x M1_WAVES
// j-slices (j = w mod M1_WAVES), 8 independent load/FMA chains per lane,
// fixed-order LDS sum of the slices.  16 slices for short shards: each wave
// issues ~n2/128 batches of 8 loads, so a 64-row shard (8 GPUs at n1 = 512:
// 64 blocks) is not latency-bound on a few long per-wave chains.
// (A j-split over more workgroups for 64-row shards, joined by a last-arriver
// ticket, cost more than it saved: the device-scope fences it needs write
// back and invalidate L2 on gfx950 and slowed every following kernel.)
// ---------------------------------------------------------------------------
// SETS > 1: W arrives as the partial sets of a t-split K5 walk (k5_tsplit,
// set c at Wk + c*sstride) and is summed here in set order — the same
// additions, in the same order, as the separate reduction launch it replaces.
template <int M1_WAVES, bool SETS>
__global__ __launch_bounds__(64 * M1_WAVES) void k_m1(const double* __restrict__ Wk,
                                                      const double* __restrict__ Bh, double* M1,
                                                      int64_t n1p, int64_t n2, int64_t plane, int RP,
                                                      const int* stop, int sets, int64_t sstride,
                                                      FinishArgs fin) {
    // the extra column of workgroups: the previous iteration's norm
    // reduction and stop test in its first one (the others exit).  The
    // contraction below may run before or after it: it writes only M1 (the
    // stop flag gates the kernels that follow)
    if (fin.on && blockIdx.x == gridDim.x - 1) {
        if (blockIdx.y == 0) reduce_finish_wg<64 * M1_WAVES>(fin);
        return;
    }
    if (*stop) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 64 + lane;
    const int k = blockIdx.y;
    constexpr int JS = M1_WAVES;
    double acc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = 0.0;
    if (i < n1p) {
        const double* wp = Wk + (int64_t)k * plane + i;
        const double* bp = Bh + k;
        auto wv = [&](int64_t o) {
            double x = wp[o];
            if constexpr (SETS)
                for (int c = 1; c < sets; ++c) x += wp[c * sstride + o];
            return x;
        };
        int64_t j = w;
        for (; j + 7 * JS < n2; j += 8 * JS) {  // 8 independent chains, j = w + JS*u
#pragma unroll
            for (int u = 0; u < 8; ++u) acc[u] = fma(wv((j + JS * u) * n1p), bp[(j + JS * u) * RP], acc[u]);
        }
        for (; j < n2; j += JS) acc[0] = fma(wv(j * n1p), bp[j * RP], acc[0]);
    }
    __shared__ double red[JS][64];
    red[w][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    __syncthreads();
    if (w == 0 && i < n1p) {
        double t = red[0][lane];
#pragma unroll
        for (int q = 1; q < JS; ++q) t += red[q][lane];
        M1[i * RP + k] = t;
    }
}

void launch_m1(const Geom& g, const double* Wk, const double* Bh, double* M1, const int* stop,
               hipStream_t st, const FinishArgs& fin) {
    // 4 slices when the row blocks alone fill the chip (512 rows: 36 vs 39 us
    // with 16), 16 for short shards (64 rows: 64 blocks)
    // (16-byte-load variants, two rows per lane, measured neutral or slower
    // in the solver: DESIGN.md §4)
    const dim3 grid((unsigned)cdiv(g.n1p, 64) + (fin.on ? 1 : 0), g.RP);
    const int sets = g.tsplit;
    const int64_t ss = (int64_t)g.RP * g.plane;
#define M1_LAUNCH(NW, S) \
    hipLaunchKernelGGL((k_m1<NW, S>), grid, dim3(64 * NW), 0, st, Wk, Bh, M1, g.n1p, g.n2, g.plane, g.RP, stop, sets, ss, fin)
    if (g.n1p >= 256) {  // (two rows per lane with 16-B loads halves the waves: 72 vs 36 us)
        if (sets > 1) M1_LAUNCH(4, true); else M1_LAUNCH(4, false);
    } else {
        if (sets > 1) M1_LAUNCH(16, true); else M1_LAUNCH(16, false);
    }
#undef M1_LAUNCH
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// M2(j,k) = sum_i Wk[k][j*n1p + i] * AhT[k][i]; one wave per (j, k)
// ---------------------------------------------------------------------------
// side: workgroup 0 runs update_B's R x R solve (sweep.h) beside the
// contraction (one GPU: its A^TA needs no all-reduce); the grid is 1-D,
// workgroup b >= side.on takes (j, k-group) = ((b - on) % n2, (b - on) / n2)
// NWV waves per workgroup: 8, so the side solve's sweep runs 8 rows per
// lane (its barrier-bound pivot steps are the part of M2 + solve that
// outlasts the contraction)
#ifndef TRITD_M2_NW
#define TRITD_M2_NW 8
#endif
template <int RP, int NWV, bool SETS = false>
__global__ __launch_bounds__(64 * NWV) void k_m2(const double* __restrict__ Wk,
                                                 const double* __restrict__ AhT, double* M2,
                                                 int64_t n1p, int64_t n2, int64_t plane,
                                                 const int* stop, SideSolve side, int sets,
                                                 int64_t sstride) {
    if (*stop) return;
    if constexpr (RP <= 64 && RP % NWV == 0) {
        if (side.on && blockIdx.x == 0) {
            __shared__ double srow[2 * NWV * 64 + RP];
            side_solve<RP, NWV>(side, srow, srow + 2 * NWV * 64);
            return;
        }
    }
    const int64_t b = (int64_t)blockIdx.x - side.on;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t j = b % n2;
    const int k = (int)(b / n2) * NWV + w;
    if (k >= RP) return;
    // 16-B loads (n1p % 16 == 0): lane sums rows 2l, 2l+1, 2l+128, ... in two chains
    const d2v* wp = reinterpret_cast<const d2v*>(Wk + (int64_t)k * plane + j * n1p);
    const d2v* ap = reinterpret_cast<const d2v*>(AhT + (int64_t)k * n1p);
    double a0 = 0.0, a1 = 0.0;
    for (int64_t q = lane; q < (n1p >> 1); q += 64) {
        d2v x = wp[q];
        const d2v y = ap[q];
        if constexpr (SETS)  // t-split partial sets of W, summed in set order (k_m1)
            for (int c = 1; c < sets; ++c) x += wp[c * (sstride >> 1) + q];
        a0 = fma(x.x, y.x, a0);
        a1 = fma(x.y, y.y, a1);
    }
    double acc = a0 + a1;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) M2[j * RP + k] = acc;
}

void launch_m2(const Geom& g, const double* Wk, const double* AhT, double* M2, const int* stop,
               hipStream_t st, const SideSolve& side) {
    constexpr int NV = TRITD_M2_NW;
    static_assert(NV >= 1 && NV <= 16, "TRITD_M2_NW: 1..16 waves per workgroup");
    // k_m2 instantiates the side solve only where RP % NV == 0; anywhere else
    // workgroup 0 would fall through to the contraction with b = -1
    if (side.on && (g.RP > 64 || g.RP % NV != 0))
        throw Error(TRITD_ERR_ARG, "M2 side solve: RP <= 64 and a multiple of TRITD_M2_NW only");
    const dim3 grid((unsigned)(g.n2 * cdiv(g.RP, NV) + side.on)), blk(64 * NV);
    const int sets = g.tsplit;
    const int64_t ss = (int64_t)g.RP * g.plane;
#define M2_CASE(RPV)                                                                                  \
    case RPV:                                                                                         \
        if (sets > 1)                                                                                 \
            hipLaunchKernelGGL((k_m2<RPV, NV, true>), grid, blk, 0, st, Wk, AhT, M2, g.n1p, g.n2, g.plane, \
                               stop, side, sets, ss);                                                 \
        else                                                                                          \
            hipLaunchKernelGGL((k_m2<RPV, NV, false>), grid, blk, 0, st, Wk, AhT, M2, g.n1p, g.n2, g.plane, \
                               stop, side, sets, ss);                                                 \
        break;
    switch (g.RP) {
        M2_CASE(16)
        M2_CASE(32)
        M2_CASE(48)
        M2_CASE(64)
        M2_CASE(128)
        M2_CASE(256)
#undef M2_CASE
        default: throw Error(TRITD_ERR_UNSUPPORTED, "M2: RP not supported");
    }
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// K2 — mode-3 MTTKRP  M3(t,k) = sum_ij T(ij,t) A^(i,k) B^(j,k)  (update_C, :93)
//
// T arrives in the "TX" fragment order written by K5 (common.h): for
// ij-tile g and t-tile tt, lane l's two d2v hold T(ij = 16g + 4s + (l>>4),
// t = 16tt + (l&15)) for s = 0..3 — exactly the B operand of
// v_mfma_f64_16x16x4_f64 for the K-steps s of D(k,t) += KR(ij,k) T(ij,t).
// So each wave streams T from HBM straight into registers (1 KB contiguous
// per wave-instruction, next ij-tile prefetched), builds its KR operands
// from L2-resident A^/B^ rows, and runs (RP/16)*4*4 MFMAs per ij-tile.
// Wave = (t-block of 64 t, contiguous ij-tile range); the 4 waves of a
// workgroup share the t-block and are summed through LDS in fixed order;
// the per-workgroup partials are summed by k_m3_reduce in fixed order.
// ---------------------------------------------------------------------------

template <int RP, int LDA>  // LDA: row stride of the factor rows and the slabs (RP, or 128/256 in 64-column passes)
__global__ __launch_bounds__(256, 2) void k_m3(const double* __restrict__ T,
                                               const double* __restrict__ Ah,
                                               const double* __restrict__ Bh, double* part,
                                               int64_t n1p, int64_t n3p, int64_t ntt,
                                               int64_t tiles, int S, const int* stop,
                                               int64_t ahj, int64_t bhj) {
    constexpr int lda = LDA;
    if (*stop) return;
    constexpr int MT = RP / 16;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int il = lane & 15, tg = lane >> 4;
    const int64_t wave = (int64_t)blockIdx.x * 4 + wid;
    const int64_t tb = wave / S;
    const int64_t sidx = wave - tb * S;
    const int64_t g0 = tiles * sidx / S, g1 = tiles * (sidx + 1) / S;
    const int64_t qper = n1p >> 4;
    const d2v* T2 = reinterpret_cast<const d2v*>(T);

    d4 acc[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = d4{0.0, 0.0, 0.0, 0.0};

    d2v nb[4][2];
    auto loadB = [&](int64_t g) {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int64_t tt = tb * 4 + n;
#pragma unroll
            for (int p = 0; p < 2; ++p)
                nb[n][p] = (tt < ntt) ? __builtin_nontemporal_load(T2 + (tm_tile_base(g, tt, ntt) >> 1) + 64 * p + lane)
                                      : d2v{0.0, 0.0};
        }
    };
    if (g0 < g1) loadB(g0);
    for (int64_t g = g0; g < g1; ++g) {
        d2v b[4][2];
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            b[n][0] = nb[n][0];
            b[n][1] = nb[n][1];
        }
        if (g + 1 < g1) loadB(g + 1);
        const int64_t j = g / qper;
        const int64_t i0 = (g - j * qper) << 4;
        const double* Aj = Ah + j * ahj;  // Qi model: rows of H (kernels.h)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const int k = 16 * m + il;
            const double bh = Bh[j * bhj + k];
            double a[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) a[s] = Aj[(i0 + 4 * s + tg) * lda + k] * bh;
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int n = 0; n < 4; ++n) acc[m][n] = mfma4(a[s], b[n][s >> 1][s & 1], acc[m][n]);
        }
    }

    // fixed-order sum of the 4 waves: (w2,w3) -> (w0,w1), then w1 -> w0
    constexpr int PER = MT * 16;  // doubles per lane
    if (wid >= 2) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    lds[((wid - 2) * PER + (m * 4 + n) * 4 + rr) * 64 + lane] = acc[m][n][rr];
    }
    __syncthreads();
    if (wid < 2) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    acc[m][n][rr] += lds[(wid * PER + (m * 4 + n) * 4 + rr) * 64 + lane];
    }
    __syncthreads();
    if (wid == 1) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) lds[((m * 4 + n) * 4 + rr) * 64 + lane] = acc[m][n][rr];
    }
    __syncthreads();
    if (wid == 0) {
        double* out = part + (int64_t)(sidx >> 2) * n3p * lda;  // slabs of n3p x lda
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const double v = acc[m][n][rr] + lds[((m * 4 + n) * 4 + rr) * 64 + lane];
                    const int64_t t = tb * 64 + 16 * n + il;
                    const int k = 16 * m + tg + 4 * rr;
                    if (t < n3p) out[t * lda + k] = v;
                }
    }
}

// CP model (A^/B^ rows, not Qi's H): the same contraction with each wave
// holding ONE ij-tile row block i0..i0+15 and walking fibres j.  Its A^ rows
// stay in registers for the whole walk, so the Khatri-Rao operand of a step
// is ar * B^(j,k) (4 loads + 16 multiplies), and those loads go out in the
// same batch as the next step's T prefetch, one step ahead.  (The generic
// kernel above loads its A^ operand after issuing the T prefetch; vmcnt is
// in-order, so waiting on the operand also waited on the prefetch and
// exposed the HBM latency every ij-tile.)
// Wave = (t-block of 64 t, i-tile, part jp of the fibres); S waves per
// t-block (padded to a multiple of 4, surplus waves contribute zeros).
#if TRITD_WTRACE
WT_DECL(g_wt_k2)
#endif
template <int RP, int LDA>
__global__ __launch_bounds__(256, 2) void k_m3_cp(const double* __restrict__ T,
                                                  const double* __restrict__ Ah,
                                                  const double* __restrict__ Bh, double* part,
                                                  int64_t n2, int64_t n3p, int64_t ntt,
                                                  int64_t qper, int64_t J, int S,
                                                  const int* stop, SideSolve side) {
    if (*stop) return;
    // side job: workgroup 0 runs the R x R solve of update_C (sweep.h)
    if (side.on && blockIdx.x == 0) {
        extern __shared__ __attribute__((aligned(16))) double slds[];
        side_solve<RP>(side, slds, slds + 2 * 4 * 64);
        return;
    }
    const int64_t bid = (int64_t)blockIdx.x - side.on;
    WT_BEGIN();
    constexpr int MT = RP / 16;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int il = lane & 15, tg = lane >> 4;
    const int64_t wave = bid * 4 + wid;
    const int64_t tb = wave / S;
    const int64_t sidx = wave - tb * S;
    const bool live = sidx < qper * J;
    const int64_t itile = live ? sidx % qper : 0;
    const int64_t jp = live ? sidx / qper : 0;
    const int64_t j0 = n2 * jp / J, j1 = live ? n2 * (jp + 1) / J : j0;
    const int64_t i0 = itile << 4;
    const d2v* T2 = reinterpret_cast<const d2v*>(T);

    // A^(i0 + 4s + tg, 16m + il) at arl[(4m + s) * 64 + lane]: in LDS, not
    // registers (the accumulators and two prefetch sets fill the 256 VGPRs);
    // the region is reused by the final reduction
    double* arl = lds + wid * (MT * 4 * 64);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int s = 0; s < 4; ++s) arl[(4 * m + s) * 64 + lane] = Ah[(i0 + 4 * s + tg) * LDA + 16 * m + il];
    d4 acc[MT][4];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = d4{0.0, 0.0, 0.0, 0.0};

    struct Nx {
        d2v b[4][2];   // T(ij = i0 + 4s + (l>>4), t = 16(4tb+n) + (l&15)), s = 2p + q
        double bh[MT]; // B^(j, 16m + l&15)
    };
    // t-tiles past the last are clamped (their columns of acc are never stored)
    auto load = [&](int64_t j, Nx& x) {
#pragma unroll
        for (int m = 0; m < MT; ++m) x.bh[m] = Bh[j * LDA + 16 * m + il];
        const int64_t g = j * qper + itile;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
            const int64_t tt = tb * 4 + n < ntt ? tb * 4 + n : ntt - 1;
            const int64_t o = (tm_tile_base(g, tt, ntt) >> 1) + lane;
#pragma unroll
            for (int p = 0; p < 2; ++p) x.b[n][p] = __builtin_nontemporal_load(T2 + o + 64 * p);
        }
    };
    auto mm = [&](const Nx& c) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const double a = arl[(4 * m + s) * 64 + lane] * c.bh[m];
#pragma unroll
                for (int n = 0; n < 4; ++n) acc[m][n] = mfma4(a, c.b[n][s >> 1][s & 1], acc[m][n]);
            }
    };
    // one fibre per step: take the batch issued a step ago, issue the next
    Nx cur, nxt;
    if (j0 < j1) load(j0, nxt);
    for (int64_t j = j0; j < j1; ++j) {
        cur = nxt;
        if (j + 1 < j1) load(j + 1, nxt);
        mm(cur);
    }

    // fixed-order sum of the 4 waves: (w2,w3) -> (w0,w1), then w1 -> w0
    constexpr int PER = MT * 16;  // doubles per lane
    __syncthreads();  // every wave is done with its A^ rows in LDS
    if (wid >= 2) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    lds[((wid - 2) * PER + (m * 4 + n) * 4 + rr) * 64 + lane] = acc[m][n][rr];
    }
    __syncthreads();
    if (wid < 2) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                    acc[m][n][rr] += lds[(wid * PER + (m * 4 + n) * 4 + rr) * 64 + lane];
    }
    __syncthreads();
    if (wid == 1) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) lds[((m * 4 + n) * 4 + rr) * 64 + lane] = acc[m][n][rr];
    }
    __syncthreads();
    if (wid == 0) {
        double* out = part + (int64_t)(sidx >> 2) * n3p * LDA;  // slabs of n3p x LDA
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < 4; ++n)
#pragma unroll
                for (int rr = 0; rr < 4; ++rr) {
                    const double v = acc[m][n][rr] + lds[((m * 4 + n) * 4 + rr) * 64 + lane];
                    const int64_t t = tb * 64 + 16 * n + il;
                    const int k = 16 * m + tg + 4 * rr;
                    if (t < n3p) out[t * LDA + k] = v;
                }
    }
    WT_END(g_wt_k2, bid * 4 + wid);
}

// M3[t][k] = sum_y part[y][t][k]  (fixed order); 4 slices per output summed in LDS
__global__ __launch_bounds__(256) void k_m3_reduce(const double* __restrict__ part, double* M3,
                                                   int64_t count, int nparts, const int* stop) {
    if (*stop) return;
    const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * 64 + lane;
    double s = 0.0;
    if (nparts <= 4 * 16) {  // (512^3: 64 parts) every load issued before the in-order sum
        double v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int y = q + 4 * u;
            v[u] = (e < count && y < nparts) ? part[(int64_t)y * count + e] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) s += v[u];
    } else if (e < count) {
        for (int y = q; y < nparts; y += 4) s += part[(int64_t)y * count + e];
    }
    __shared__ double red[4][64];
    red[q][lane] = s;
    __syncthreads();
    if (q == 0 && e < count) M3[e] = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
}

// generic kernel: waves per t-block (multiple of 4)
int m3_split(const Geom& g) {
    const int64_t ntb = cdiv(g.ntt, 4);
    int64_t S = 2048 / ntb;  // about two waves per SIMD
    if (S > g.tiles) S = g.tiles;
    S = (S + 3) / 4 * 4;
    if (S < 4) S = 4;
    return (int)S;
}

// CP kernel: J fibre parts per i-tile, S = qper*J waves per t-block padded to 4
struct M3Cp {
    int64_t qper, J;
    int S;
};
static M3Cp m3_cp_split(const Geom& g) {
    M3Cp c;
    c.qper = g.n1p >> 4;
    const int64_t ntb = cdiv(g.ntt, 4);
    // about two waves per SIMD while that leaves every wave >= 64 fibre steps
    // (the whole 512^3 problem); shorter walks (mode-1 shards of 256 rows
    // and less) run one wave per SIMD: the prologue, the reduction epilogue
    // and the partial slabs are per wave, and the grid then leaves room for
    // the side solve's workgroup instead of displacing a compute one
    // (shard timings, 64-row shard: K2 + reduce 63.9 -> 55.8 us; 128 rows
    // 97.3 -> 88.0; 256 rows 161 -> 157; 512 rows 2048 waves stay ~1 % ahead)
    // (config 3 with 2 048 / 4 096 waves instead: 0.052 / 0.068 vs 0.048 ms,
    // profiles/round3/ab_c3_m3_waves.txt)
    const int64_t J2 = 2048 / (ntb * c.qper);
    const int64_t waves = (J2 >= 1 && g.n2 / J2 >= 64) ? 2048 : 1024;
    int64_t J = waves / (ntb * c.qper);
    if (J < 1) J = 1;
    if (J > g.n2) J = g.n2;
    c.J = J;
    c.S = (int)((c.qper * J + 3) / 4 * 4);
    return c;
}

// the CP model's K2 (k_m3_cp); Qi's H rows change with j (k_m3)
static bool m3_use_cp(int64_t ahj) { return ahj == 0; }

static int current_device() {
    int d = 0;
    TRITD_HIP(hipGetDevice(&d));
    return d;
}

int m3_parts(const Geom& g) {
    const int a = m3_split(g) / 4, b = m3_cp_split(g).S / 4;
    return a > b ? a : b;
}

void launch_m3(const Geom& g, const double* T, const double* Ah, const double* Bh, double* part,
               double* M3, const int* stop, hipStream_t st, int64_t ahj, int64_t bhj,
               const SideSolve& side) {
    if (bhj < 0) bhj = g.RP;
    const bool cp = m3_use_cp(ahj);
    if (side.on && (!cp || g.RP > 64)) throw Error(TRITD_ERR_ARG, "K2 side solve: CP kernel, RP <= 64 only");
    const M3Cp cs = m3_cp_split(g);
    const int S = cp ? cs.S : m3_split(g);
    const int64_t ntb = cdiv(g.ntt, 4);
    const dim3 grid((unsigned)(ntb * S / 4));
    // RP <= 64 in one pass; RP = 128 / 256 (fp64 r = 9..16) as 64-column
    // passes over the same T (their columns of the factor rows and of the
    // partial slabs, whose row stride stays RP)
#define M3_CASE(RPV, LDAV, KOFF)                                                              \
    {                                                                                         \
        const size_t lds = (size_t)2 * (RPV / 16) * 16 * 64 * sizeof(double);                \
        static std::atomic<uint64_t> attr_set{0}; /* per device (bit), device-set threads */  \
        const uint64_t dbit = (uint64_t)1 << (current_device() & 63);                          \
        if (!(attr_set.load(std::memory_order_acquire) & dbit)) {                               \
            TRITD_HIP(hipFuncSetAttribute((const void*)k_m3<RPV, LDAV>,                       \
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
            TRITD_HIP(hipFuncSetAttribute((const void*)k_m3_cp<RPV, LDAV>,                    \
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
            attr_set.fetch_or(dbit, std::memory_order_acq_rel);                                \
        }                                                                                     \
        if (cp) {                                                                             \
            hipLaunchKernelGGL((k_m3_cp<RPV, LDAV>), dim3(grid.x + side.on), dim3(256), lds, st, T, \
                               Ah + (KOFF), Bh + (KOFF), part + (KOFF), g.n2, g.n3p, g.ntt, cs.qper, \
                               cs.J, S, stop, side);                                 \
        } else {                                                                              \
            hipLaunchKernelGGL((k_m3<RPV, LDAV>), grid, dim3(256), lds, st, T, Ah + (KOFF),   \
                               Bh + (KOFF), part + (KOFF), g.n1p, g.n3p, g.ntt, g.tiles, S, stop, ahj, bhj); \
        }                                                                                     \
    }
    switch (g.RP) {
        case 16: M3_CASE(16, 16, 0) break;
        case 32: M3_CASE(32, 32, 0) break;
        case 48: M3_CASE(48, 48, 0) break;
        case 64: M3_CASE(64, 64, 0) break;
        case 128:
            for (int k0 = 0; k0 < 128; k0 += 64) M3_CASE(64, 128, k0)
            break;
        case 256:
            for (int k0 = 0; k0 < 256; k0 += 64) M3_CASE(64, 256, k0)
            break;
        default:
            throw Error(TRITD_ERR_UNSUPPORTED, "rank not supported by M3");
    }
#undef M3_CASE
    TRITD_CHECK_LAUNCH();
    const int64_t count = g.n3p * g.RP;
    hipLaunchKernelGGL(k_m3_reduce, dim3((unsigned)cdiv(count, 64)), dim3(256), 0, st, part, M3,
                       count, S / 4, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Gram: G[k][k'] = sum_i X[i][k] X[i][k'] (rows in 256/RP interleaved groups)
// ---------------------------------------------------------------------------
// G = X^T X (RP x RP) of a row-major rows x RP factor — the Hadamard-Gram
// factors A^TA, B^TB, C^TC of update_A/B/C (:77,86,93 build F F^T etc.;
// SURVEY.md §0.3).  One workgroup per 16 x 16 tile of G: the rows go to
// v_mfma_f64_16x16x4_f64 four at a time (A[m][k] = X(i0+k, 16ta+m),
// B[k][n] = X(i0+k, 16tb+n)), the NW waves take every NW-th K-step and are
// summed through LDS in fixed order (deterministic).  Out-of-range rows load
// as zero.  Latency-bound at these sizes; the old per-column VALU loop took
// 29 us at 512 x 64, this takes a few.
// NW waves per workgroup (16: every wave's K-steps in flight at once — 512
// rows are 128 K-steps, 8 per wave, one load round instead of eight).
template <int NW>
__global__ __launch_bounds__(64 * NW) void k_gram(const double* __restrict__ X, int64_t rows, int RP,
                                                  double* G, const int* stop) {
    if (stop && *stop) return;
    constexpr int U = 8;  // K-steps per wave per round: loads first
    const int nt = RP >> 4;
    const int ta = blockIdx.x / nt, tb = blockIdx.x - (blockIdx.x / nt) * nt;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int m = lane & 15, kq = lane >> 4;
    const double* xa = X + 16 * ta + m;
    const double* xb = X + 16 * tb + m;
    const int64_t steps = (rows + 3) >> 2;
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
    for (int64_t s = w; s < steps; s += U * NW) {  // K-steps s, s+NW, ..., s+(U-1)NW
        double a[U], b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = 4 * (s + NW * u) + kq;
            const bool in = i < rows;
            a[u] = in ? xa[i * RP] : 0.0;
            b[u] = in ? xb[i * RP] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc = mfma4(a[u], b[u], acc);
    }
    __shared__ double part[NW - 1][4][64];
    if (w > 0)
#pragma unroll
        for (int r = 0; r < 4; ++r) part[w - 1][r][lane] = acc[r];
    __syncthreads();
    if (w == 0) {
        // C/D element r of lane l: G(16ta + (l>>4) + 4r, 16tb + (l&15)); waves summed in order
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double v = acc[r];
#pragma unroll
            for (int q = 0; q < NW - 1; ++q) v += part[q][r][lane];
            G[(int64_t)(16 * ta + kq + 4 * r) * RP + 16 * tb + m] = v;
        }
    }
}

// side = true: four-wave workgroups, for a Gram on the side stream beside a
// grid of 256-thread workgroups that fills the chip (K2 / K5): a 1024-thread
// workgroup fits only where four of theirs retired on one CU at once, and
// waited for the whole grid (config 5: Gram B 4.9 ms beside K2, solve C
// after it on the critical path)
void launch_gram(int RP, const double* X, int64_t rows, double* G, const int* stop,
                 hipStream_t st, bool side) {
    const dim3 grid((RP / 16) * (RP / 16));
    if (side)
        hipLaunchKernelGGL(k_gram<4>, grid, dim3(64 * 4), 0, st, X, rows, RP, G, stop);
    else
        hipLaunchKernelGGL(k_gram<16>, grid, dim3(64 * 16), 0, st, X, rows, RP, G, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// The symmetric Gauss-Jordan sweep (sweep.h: sweep_all; the R x R solves
// inside M2/K2/K5 and the fallback of k_solve_ns below).
// The R x R matrix is embedded in RP x RP with an identity pad.  It is SPD
// (ridge alpha > 0), so Gauss-Jordan needs no pivoting, and its symmetric
// form (the sweep operator) keeps the matrix symmetric at every step, so
// column P == row P.  Wave w holds rows 8w..8w+7, lane c column c.
// Sweep on P, D = a_PP:
//   a_PP <- -1/D,  a_iP <- a_iP/D,  a_Pc <- a_Pc/D,  a_ic <- a_ic - a_iP*(a_Pc/D)
// after all pivots the matrix is -inv(.).  The off-pivot update is the
// Gauss-Jordan update term for term; written m*a - f*t with (m, t) = (1, s)
// or (0, -1/D) it needs no selects and rounds identically.  Per step, every
// wave publishes its candidate of row P (only the owner's is read), one
// barrier, double-buffered by step parity (8 rows per lane, RP/8 waves).  The smallest pivot (= smallest
// LDL^T pivot) is compared with MATLAB's pinv tolerance max(size)*eps(max
// sigma); within 1e3x of it, pinv could truncate (triple_decomp_ADMM.m:78,86,93
// use pinv) and the solve requests the pinv fallback of pinv.h.
// Register-pressure notes (each measured): the pivot loop is unrolled via an
// index sequence (a runtime pivot would index the register array); there is
// no divergent branch and no per-element runtime mask inside or after the
// sweep (either made the compiler keep every step's values and spill).
// ---------------------------------------------------------------------------


// ---------------------------------------------------------------------------
// Ginv = inv(P o Q + alpha I) for RP <= 64 by Newton-Schulz refinement of the
// previous inverse of the same Gram slot (the output buffer's contents on
// entry), with the symmetric Gauss-Jordan sweep above as the fallback.
//
// The Grams of consecutive ADMM iterations differ little once the factors
// settle, so X0 = the last inverse is already close: E = I - G X0 is small
// and X <- X + X E squares it per step (E' = E^2).  Every step is two RP^3
// GEMMs on v_mfma_f64_16x16x4_f64 (one 16x16 tile per wave, operands in
// LDS) and one fixed-order norm, ~0.5 us each, against the sweep's RP
// dependent pivot steps of ~0.3 us.  The loop stops once the update is
// below the rounding floor: after an update whose ||E||_F < 1e-7 (the new
// error is ~||E||^2 < 1e-14), or as soon as ||E|| stops halving (cond(G) *
// eps reached; the last X is kept).  With ||E0||_F >= 1/2 (early iterations,
// a zero or stale buffer, a NaN) the kernel runs the sweep instead, so the
// result is an inverse to working accuracy either way.
//
// pinv fallback request (triple_decomp_ADMM.m:78,86,93 use pinv; pinv.h):
// the sweep path compares its LDL^T pivots as k_solve does; the Newton path
// uses the bounds sigma_min >= 1/||X||_F and sigma_max <= ||G||_F, i.e. it
// requests whenever the sweep could (and up to sqrt(R) earlier).  Either way
// the fallback computes pinv itself and raises TRITD_FLAG_PINV_TOL only when
// pinv drops a value, so the flag does not depend on which test asked.
//
// Waves: RP/4 (the sweep runs 4 rows per lane); the Newton GEMMs use the
// first (RP/16)^2 of them.
// ---------------------------------------------------------------------------
template <int RP>
__global__ __launch_bounds__(RP * 16) void k_solve_ns(const double* __restrict__ P,
                                                     const double* __restrict__ Q, int R,
                                                     double alpha, double* Ginv, int* flags,
                                                     const int* stop, FinishArgs fin) {
    if (fin.on) {  // the previous iteration's finish first (launch_solve)
        reduce_finish_wg<RP * 16>(fin);
        __syncthreads();
    }
    if (*stop) return;
    __builtin_amdgcn_s_setprio(3);  // beside K2 / K5 on the side stream: win issue
    constexpr int NWV = RP / 4, NT = RP / 16, LD = RP + 1, KS = RP / 4, RW = 4;
    constexpr int NTH = 64 * NWV;
    __shared__ double Gs[RP * LD], Xs[RP * LD], Es[RP * LD];
    __shared__ double rowbuf[2 * NWV * 64];
    __shared__ double pivs[RP];
    __shared__ double red[2][NWV];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m = lane & 15, kq = lane >> 4;
    const bool tw = w < NT * NT;  // this wave owns a 16 x 16 tile of the GEMMs
    const int ta = tw ? w / NT : 0, tb = tw ? w - (w / NT) * NT : 0;
    double gss = 0.0;  // ||G||_F^2 partial
    {
        constexpr int NE = RP * RP / NTH;  // = RP/16 elements per thread
        static_assert(RP * RP % NTH == 0, "k_solve_ns: element split");
        double pv[NE], qv[NE], xv[NE];
#pragma unroll
        for (int q = 0; q < NE; ++q) {  // every load issued before the first use
            const int e = tid + q * NTH;
            pv[q] = P[e];
            qv[q] = Q[e];
            xv[q] = Ginv[e];
        }
#pragma unroll
        for (int q = 0; q < NE; ++q) {
            const int e = tid + q * NTH;
            const int i = e / RP, c = e - (e / RP) * RP;
            const bool in = i < R && c < R;
            const double pq = pv[q] * qv[q];
            const double g = in ? ((i == c) ? pq + alpha : pq) : ((i == c) ? 1.0 : 0.0);
            Gs[i * LD + c] = g;
            Xs[i * LD + c] = in ? xv[q] : ((i == c) ? 1.0 : 0.0);
            if (in) gss = fma(g, g, gss);
        }
    }
    auto wave_sum = [&](double v) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
        return v;
    };
    // C = A B for this wave's tile (A, B in LDS, row stride LD)
    auto gemm = [&](const double* A, const double* B) {
        double a[KS], b[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            a[s] = A[(16 * ta + m) * LD + 4 * s + kq];
            b[s] = B[(4 * s + kq) * LD + 16 * tb + m];
        }
        d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < KS; ++s) acc = mfma4(a[s], b[s], acc);
        return acc;
    };
    // C/D element r of lane l: (16 ta + (l>>4) + 4 r, 16 tb + (l&15))
    auto at = [&](int r) { return (16 * ta + kq + 4 * r) * LD + 16 * tb + m; };
    __syncthreads();
    bool sweep = false;
    double nprev = 0.0;
    for (int it = 0;; ++it) {
        double ss = 0.0;
        if (tw) {
            const d4 t = gemm(Gs, Xs);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * ta + kq + 4 * r, col = 16 * tb + m;
                const double ev = ((row == col) ? 1.0 : 0.0) - t[r];
                Es[at(r)] = ev;
                ss = fma(ev, ev, ss);
            }
        }
        ss = wave_sum(ss);
        if (lane == 0) red[0][w] = ss;
        __syncthreads();
        double n2 = 0.0;
#pragma unroll
        for (int q = 0; q < NWV; ++q) n2 += red[0][q];  // same order in every thread
        const double n = sqrt(n2);
        if (it == 0 && !(n < 0.5)) {  // no usable start: sweep
            sweep = true;
            break;
        }
        if (it > 0 && !(n < 0.5 * nprev)) break;  // rounding floor: keep X
        if (tw) {
            const d4 u = gemm(Xs, Es);
            double xv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) xv[r] = Xs[at(r)];
            __syncthreads();  // every wave has read Xs, Es and red
#pragma unroll
            for (int r = 0; r < 4; ++r) Xs[at(r)] = xv[r] + u[r];
        } else {
            __syncthreads();
        }
        __syncthreads();
        nprev = n;
        if (n < 1e-7 || it >= 7) break;  // the update left ~n^2 < 1e-14
    }
    double minpiv = 0.0, maxpiv = 0.0;  // sweep: LDL^T pivots; Newton: sigma bounds
    if (sweep) {
        // Gauss-Jordan sweep of G (k_solve with 4 rows per lane); -inv lands in Xs
        const int c = lane, cc = c < RP ? c : 0;
        double a[RW];
#pragma unroll
        for (int q = 0; q < RW; ++q) a[q] = Gs[(RW * w + q) * LD + cc];
        rowbuf[w * 64 + c] = a[0];
        __syncthreads();
        sweep_all<RP, RW>(a, rowbuf, pivs, c, w, std::make_integer_sequence<int, RP>{});
        if (c < RP)
#pragma unroll
            for (int q = 0; q < RW; ++q) Xs[(RW * w + q) * LD + c] = -a[q];
        __syncthreads();
    }
    double xss = 0.0;
    for (int e = tid; e < RP * RP; e += NTH) {
        const int i = e / RP, j = e - (e / RP) * RP;
        const bool in = i < R && j < R;
        const double x = in ? Xs[i * LD + j] : 0.0;
        Ginv[e] = x;
        xss = fma(x, x, xss);
    }
    bool near;
    if (sweep) {
        near = pivots_near_cutoff(pivs, R);
    } else {
        xss = wave_sum(xss);
        gss = wave_sum(gss);
        if (lane == 0) {
            red[0][w] = xss;
            red[1][w] = gss;
        }
        __syncthreads();
        double x2 = 0.0, g2 = 0.0;  // every thread, same order
        for (int q = 0; q < NWV; ++q) {
            x2 += red[0][q];
            g2 += red[1][q];
        }
        minpiv = 1.0 / sqrt(x2);
        maxpiv = sqrt(g2);
        const double tol = (double)R * ldexp(1.0, ilogb(maxpiv) - 52);  // pinv: R*eps(sigma_max)
        near = !(minpiv > 1e3 * tol);
    }
    pinv_request<NTH>(near, P, Q, R, RP, alpha, Ginv);
}

// ---------------------------------------------------------------------------
// Register sweep of one 16 x 16 diagonal block (k_solve_mw's owner step):
// lane c holds column c (the 4 lane groups of the wave sweep identical
// copies), pivot rows shared through LDS; the pivots are recorded for the
// pinv-tolerance check.
// ---------------------------------------------------------------------------
constexpr int SB = 16;  // pivots per block (a 32-wide register sweep does not fit the 128 VGPRs of a 1024-thread block)

template <int P>
__device__ __forceinline__ void sweep32_step(double (&a)[SB], double* rowp, double* pv, int c) {
    rowp[c] = a[P];  // lanes of equal c write equal values
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const double piv = rowp[P];
    pv[P] = piv;
    const double d = 1.0 / piv;
    const bool pc = (c == P);
    const double s = rowp[c] * d;
    const double m = pc ? 0.0 : 1.0;
    const double t = pc ? -d : s;
#pragma unroll
    for (int i = 0; i < SB; ++i) a[i] = m * a[i] - rowp[i] * t;
    a[P] = t;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_sched_barrier(0);
}
template <int... Ps>
__device__ __forceinline__ void sweep32_all(double (&a)[SB], double* rowp, double* pv, int c,
                                            std::integer_sequence<int, Ps...>) {
    (sweep32_step<Ps>(a, rowp, pv, c), ...);
}


// ---------------------------------------------------------------------------
// Ginv = inv(P o Q + alpha I) at RP = 128 / 256 across NB = RP/16 workgroups
// (k_solve_mw): a blocked symmetric sweep with S split into row strips.  (A
// one-workgroup form that kept S in one CU moved all of it through that CU's
// LDS/L2 port on every block step: 0.75 ms at RP = 256, on the critical path
// of config 5's update_B, triple_decomp_ADMM.m:86; this form 0.15 ms.)
// Here workgroup b owns rows [16b, 16b+16) in its LDS (32 KB at 256) and
// block step K is:
//   owner (b = K): M = inv(S_KK) (one wave, register sweep: the sequential
//     sweep's pivots, kept for the pinv-tolerance test), X = M S_K,: (f64
//     MFMA), S_K,: <- X except S_KK <- -M; publishes X and its 16 pivots
//     (global scratch of its Ginv buffer) and then step word K = epoch;
//   others: wait for step word K, then S_I,j -= S_IK X_Kj (f64 MFMA, the old
//     S_IK from registers) and S_IK <- (X_K,I)^T.
// The arithmetic per block is the sequential sweep's blocked form (same
// blocks, same order per block as the one-workgroup kernel it replaced).  Cross-workgroup order: the owner's stores, an agent-
// scope release fence, a barrier and a release store of the step word; the
// waiter's acquire load of it, a barrier and an agent-scope acquire fence in
// every thread.  Only workgroup 0 reads the stop flag; a stopped launch
// publishes step word 0 with the stop bit, so all workgroups agree (a flag
// set mid-launch by another stream could not split them).  The workgroups
// depend only on earlier steps (acyclic), so a workgroup dispatched late —
// the GPU busy with K5 on another stream — delays the chain but cannot
// deadlock it; a wait longer than ~1 s still gives up (flags bit 2, which
// the session turns into an error) rather than hang the GPU.
// Epochs (host counter, < 2^31, never 0) make the step words single-use
// without a reset.
// ---------------------------------------------------------------------------
constexpr int MW_NT = 256;  // 4 waves per workgroup
constexpr unsigned MW_STOP = 0x80000000u;

// Safety net, not a schedule: the workgroups of a launch depend only on
// earlier steps, so a slow peer (late dispatch, preemption) only delays the
// chain.  A wait of ~1 s of polls gives up instead of hanging the device: it
// raises flags bit 2 (sync() turns it into an error) and the solver's stop
// flag, so every later kernel of the enqueued iterations skips its work
// rather than running on a half-swept inverse.
__device__ __forceinline__ unsigned mw_wait(const unsigned* w, unsigned epoch, int* flags,
                                            const int* stop) {
    unsigned v = 0;
    for (int n = 0;; ++n) {
        v = __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if ((v & ~MW_STOP) == epoch) return v;
        if (n > (1 << 22)) {
            atomicOr(flags, 2);
            atomicExch(const_cast<int*>(stop), 1);
            return MW_STOP;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

template <int RP>
__global__ __launch_bounds__(MW_NT) void k_solve_mw(const double* __restrict__ P,
                                                  const double* __restrict__ Q, int R,
                                                  double alpha, double* Ginv, int* flags,
                                                  const int* stop, unsigned epoch) {
    constexpr int NB = RP / SB, LD = RP + 2, TPW = NB / (MW_NT / 64);  // column tiles per wave
    static_assert(NB % (MW_NT / 64) == 0, "column tiles split evenly over the waves");
    __shared__ double St[SB * LD];  // this workgroup's strip of S
    __shared__ double Ml[SB * (SB + 1)];
    __shared__ double rowp[64];
    __shared__ double pvl[SB];
    __shared__ unsigned state;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m = lane & 15, kq = lane >> 4;
    const int b = blockIdx.x, i0 = SB * b;
    double* Xg = Ginv + 2 * (int64_t)RP * RP;  // [NB][SB][RP]: X of every step (pinv.h scratch, free here)
    double* pivg = Ginv + ginv_piv(RP);
    unsigned* sync = reinterpret_cast<unsigned*>(Ginv + ginv_sync(RP));
    // the launch's stop decision, workgroup 0's alone
    if (b == 0 && tid == 0) state = (*stop) ? MW_STOP : 0u;
    if (b == 0) {
        __syncthreads();
        if (state) {
            if (tid == 0) __hip_atomic_store(&sync[0], epoch | MW_STOP, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
    }
    // strip rows i0..i0+15 of S = P o Q + alpha I (R x R block), identity pad
    for (int e = tid; e < SB * RP; e += MW_NT) {
        const int r = e / RP, c = e - (e / RP) * RP, i = i0 + r;
        double v;
        if (i < R && c < R) {
            v = P[(int64_t)i * RP + c] * Q[(int64_t)i * RP + c];
            if (i == c) v = v + alpha;
        } else {
            v = (i == c) ? 1.0 : 0.0;
        }
        St[r * LD + c] = v;
    }
    __syncthreads();
    for (int K = 0; K < NB; ++K) {
        const int k0 = SB * K;
        double* XK = Xg + (int64_t)K * SB * RP;
        if (b == K) {
            // M = inv(S_KK): wave 0 sweeps the block in registers (sweep32_all)
            if (w == 0) {
                const int cc = lane & (SB - 1);
                double a[SB];
#pragma unroll
                for (int i = 0; i < SB; ++i) a[i] = St[i * LD + k0 + cc];
                sweep32_all(a, rowp, pvl, cc, std::make_integer_sequence<int, SB>{});
#pragma unroll
                for (int i = 0; i < SB; ++i) Ml[i * (SB + 1) + cc] = -a[i];
            }
            __syncthreads();
            // X = M S_K,: : tile jt, A[m][k] = M(m, 4s+k), B[k][n] = S(k0+4s+k, 16jt+n)
            d4 x[TPW];
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const int jt = w + (MW_NT / 64) * u;
                d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int s4 = 0; s4 < SB / 4; ++s4)
                    acc = mfma4(Ml[m * (SB + 1) + 4 * s4 + kq], St[(4 * s4 + kq) * LD + 16 * jt + m], acc);
                x[u] = acc;
            }
            __syncthreads();  // every B operand read before the strip is overwritten
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const int jt = w + (MW_NT / 64) * u;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = kq + 4 * r, col = 16 * jt + m;
                    XK[row * RP + col] = x[u][r];
                    St[row * LD + col] = (jt == K) ? -Ml[row * (SB + 1) + m] : x[u][r];
                }
            }
            if (tid < SB) pivg[k0 + tid] = pvl[tid];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            __syncthreads();
            if (tid == 0) __hip_atomic_store(&sync[K], epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (tid == 0) state = mw_wait(&sync[K], epoch, flags, stop);
            // old S_IK as the A operands (A[m][k] = -S(i0+m, k0+4s+k)) before any write
            double a[SB / 4];
#pragma unroll
            for (int s4 = 0; s4 < SB / 4; ++s4) a[s4] = -St[m * LD + k0 + 4 * s4 + kq];
            __syncthreads();
            if (state & MW_STOP) return;  // stopped launch (or a timed-out wait)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
            for (int u = 0; u < TPW; ++u) {
                const int jt = w + (MW_NT / 64) * u;
                if (jt == K) {
                    // S_IK <- (X_K,I)^T: element (row kq+4r, col k0+m) = X(m, i0+kq+4r)
#pragma unroll
                    for (int r = 0; r < 4; ++r) St[(kq + 4 * r) * LD + k0 + m] = XK[m * RP + i0 + kq + 4 * r];
                } else {
                    d4 acc;
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[r] = St[(kq + 4 * r) * LD + 16 * jt + m];
#pragma unroll
                    for (int s4 = 0; s4 < SB / 4; ++s4)
                        acc = mfma4(a[s4], XK[(4 * s4 + kq) * RP + 16 * jt + m], acc);
#pragma unroll
                    for (int r = 0; r < 4; ++r) St[(kq + 4 * r) * LD + 16 * jt + m] = acc[r];
                }
            }
            __syncthreads();
        }
    }
    // S = -inv: Ginv rows i0.. = -S, pad zeroed
    for (int e = tid; e < SB * RP; e += MW_NT) {
        const int r = e / RP, c = e - (e / RP) * RP, i = i0 + r;
        Ginv[(int64_t)i * RP + c] = (i < R && c < R) ? -St[r * LD + c] : 0.0;
    }
    // the last owner has acquired every earlier step, so it sees every pivot
    if (b == NB - 1) {
        __shared__ double pall[RP];
        for (int p = tid; p < RP; p += MW_NT) pall[p] = pivg[p];
        __syncthreads();
        pinv_request<MW_NT>(pivots_near_cutoff(pall, R), P, Q, R, RP, alpha, Ginv);
    }
}

// Process-wide epoch counter.  Sessions may be driven from several host
// threads (ctypes releases the GIL; a device group runs one thread per
// device), so the increment is atomic: every launch gets an epoch no other
// launch has had for 2^31 launches, and each Ginv buffer's step words
// therefore never see the same epoch twice in a row.
static std::atomic<unsigned> g_mw_epoch{0};
static unsigned mw_epoch() {
    for (;;) {
        const unsigned e = (g_mw_epoch.fetch_add(1, std::memory_order_relaxed) + 1) & ~MW_STOP;
        if (e != 0) return e;
    }
}

// RP <= 64: Newton-Schulz refinement of the previous inverse with the
// per-pivot sweep as fallback (k_solve_ns); RP = 128 / 256: the multi-
// workgroup blocked sweep (k_solve_mw).
void launch_solve(int RP, int R, const double* P, const double* Q, double alpha, double* Ginv,
                  int* flags, const int* stop, hipStream_t st, const FinishArgs* fin) {
    FinishArgs f;  // on = 0: no finish
    if (fin) {
        if (RP > 64) throw Error(TRITD_ERR_ARG, "solve with a finish: RP <= 64 only");
        f = *fin;
    }
    switch (RP) {
#define NS_CASE(RPV)                                                                            \
    case RPV:                                                                                   \
        hipLaunchKernelGGL(k_solve_ns<RPV>, dim3(1), dim3(RPV * 16), 0, st, P, Q, R, alpha, Ginv, \
                           flags, stop, f);                                                     \
        break;
        NS_CASE(16)
        NS_CASE(32)
        NS_CASE(48)
        NS_CASE(64)
#undef NS_CASE
        case 128:  // RP/16 workgroups
            hipLaunchKernelGGL(k_solve_mw<128>, dim3(128 / SB), dim3(MW_NT), 0, st, P, Q, R, alpha,
                               Ginv, flags, stop, mw_epoch());
            break;
        case 256:
            hipLaunchKernelGGL(k_solve_mw<256>, dim3(256 / SB), dim3(MW_NT), 0, st, P, Q, R, alpha,
                               Ginv, flags, stop, mw_epoch());
            break;
        default:
            throw Error(TRITD_ERR_UNSUPPORTED, "solve: RP not supported");
    }
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Y = M * Ginv (rows x RP), optional transposed copy YT[k*ldT + i]
// ---------------------------------------------------------------------------
template <int RP>
__global__ __launch_bounds__(64 * (RP / 16)) void k_apply(const double* __restrict__ M, int64_t rows,
                                                           const double* __restrict__ Ginv, double* Y,
                                                           double* YT, int64_t ldT, const int* stop,
                                                           int* flags) {
    // one wave per 16 x 16 tile of Y: rows r0..r0+15, columns 16*tn..;
    // v_mfma_f64_16x16x4_f64 over the RP/4 K-steps, every operand loaded
    // before the chain (A[m][k] = M(r0+m, 4s+k), B[k][n] = Ginv(4s+k, 16tn+n))
    if (stop && *stop) return;
    constexpr int KS = RP / 4, NT = 64 * (RP / 16), LDP = RP + 1;
    const int lane = threadIdx.x & 63, tn = threadIdx.x >> 6;
    const int m = lane & 15, kq = lane >> 4;
    const int64_t r0 = (int64_t)blockIdx.x * 16;
    const bool in = r0 + m < rows;
    const double* mp = M + (r0 + m) * RP + kq;
    const double* gp = Ginv + (int64_t)kq * RP + 16 * tn + m;
    double a[KS], b[KS];
    const double req = Ginv[ginv_req(RP)];  // the same word in every thread
    if (req != 0.0) {
        // the solve's pivots came near pinv's cutoff: every workgroup forms
        // pinv(saved Gram) in LDS (pinv.h) and multiplies by it instead
        __shared__ double pA[RP * LDP], pV[RP * LDP], rot[RP], red[NT / 64 + RP];
        __shared__ int pq[RP];
        for (int e = threadIdx.x; e < RP * RP; e += NT) {
            const int i = e / RP, j = e - (e / RP) * RP;
            pA[i * LDP + j] = Ginv[(int64_t)RP * RP + e];
        }
        __syncthreads();
        jacobi_pinv<RP, NT>(pA, pV, LDP, (int)req, pA, LDP, rot, pq, red, flags);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            a[s] = in ? mp[4 * s] : 0.0;
            b[s] = pA[(4 * s + kq) * LDP + 16 * tn + m];
        }
    } else {
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            a[s] = in ? mp[4 * s] : 0.0;
            b[s] = gp[(int64_t)4 * s * RP];
        }
    }
    d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = mfma4(a[s], b[s], acc);
    // C/D element r of lane l: Y(r0 + (l>>4) + 4r, 16tn + (l&15))
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = r0 + kq + 4 * r;
        if (i < rows) {
            Y[i * RP + 16 * tn + m] = acc[r];
            if (YT) YT[(int64_t)(16 * tn + m) * ldT + i] = acc[r];
        }
    }
}

void launch_apply(int RP, const double* M, int64_t rows, const double* Ginv, double* Y, double* YT,
                  int64_t ldT, const int* stop, int* flags, hipStream_t st) {
    const dim3 grid((unsigned)cdiv(rows, 16)), block(64 * (RP / 16));
#define APPLY_CASE(RPV) \
    case RPV: hipLaunchKernelGGL(k_apply<RPV>, grid, block, 0, st, M, rows, Ginv, Y, YT, ldT, stop, flags); break;
    switch (RP) {
        APPLY_CASE(16)
        APPLY_CASE(32)
        APPLY_CASE(48)
        APPLY_CASE(64)
        default: throw Error(TRITD_ERR_UNSUPPORTED, "apply: RP not supported");
    }
#undef APPLY_CASE
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Small problems: Y = M * Ginv and G = Y^T Y in ONE workgroup (one launch
// instead of k_apply + k_gram).  The ADMM iteration applies and Grams each
// factor back to back (update_A/B/C, triple_decomp_ADMM.m:77-81,86-88,93-95);
// at the sensor shape (config 2: 64 / 4 / 1152 rows, RP 32) each of those
// launches is a few microseconds of dispatch and ramp around a fraction of a
// microsecond of work.  Rows are taken in chunks of 64: the 4 waves form the
// chunk's 16 x 16 tiles of Y (f64 MFMA, Ginv staged in LDS), store Y / Y^T
// and the chunk to LDS, then accumulate their tiles of G over it.  The sums
// run over rows in chunk order, a fixed order (not k_gram's): results agree
// to rounding.  The pinv fallback (pinv.h) runs once, in this workgroup.
// ---------------------------------------------------------------------------
template <int RP>
__global__ __launch_bounds__(256) void k_apply_gram(const double* __restrict__ M, int64_t rows,
                                                    const double* __restrict__ Ginv, double* Y,
                                                    double* YT, int64_t ldT, double* G,
                                                    const int* stop, int* flags) {
    if (stop && *stop) return;
    constexpr int NT = 256, NCT = RP / 16, KS = RP / 4;
    constexpr int LD = ((RP + 31) / 32) * 32 + 16;  // = 16 mod 32: conflict-free operand reads
    constexpr int LDP = RP + 1;                     // jacobi_pinv's own stride
    constexpr int UN = (2 * RP * LDP > 64 * LD) ? 2 * RP * LDP : 64 * LD;
    __shared__ double Gl[RP * LD];
    __shared__ double un[UN];  // pA | pV of the pinv fallback, then the Y chunk
    __shared__ double rot[RP], red[NT / 64 + RP];
    __shared__ int pq[RP];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int m = lane & 15, kq = lane >> 4;
    const double req = Ginv[ginv_req(RP)];
    if (req != 0.0) {
        double* pA = un;
        double* pV = un + RP * LDP;
        for (int e = tid; e < RP * RP; e += NT) {
            const int i = e / RP, j = e - (e / RP) * RP;
            pA[i * LDP + j] = Ginv[(int64_t)RP * RP + e];
        }
        __syncthreads();
        jacobi_pinv<RP, NT>(pA, pV, LDP, (int)req, Gl, LD, rot, pq, red, flags);
    } else {
        for (int e = tid; e < RP * RP; e += NT) {
            const int i = e / RP, j = e - (e / RP) * RP;
            Gl[i * LD + j] = Ginv[e];
        }
    }
    __syncthreads();
    double* Ys = un;
    constexpr int GT = NCT * NCT, GPW = (GT + 3) / 4;  // Gram tiles, per wave
    d4 gacc[GPW];
#pragma unroll
    for (int q = 0; q < GPW; ++q) gacc[q] = d4{0.0, 0.0, 0.0, 0.0};
    for (int64_t c0 = 0; c0 < rows; c0 += 64) {
        // Y tiles (rt, ct) of this chunk, wave w takes ids w, w+4, ...
        for (int id = w; id < 4 * NCT; id += 4) {
            const int rt = id / NCT, ct = id - (id / NCT) * NCT;
            const int64_t r0 = c0 + 16 * rt;
            const bool in = r0 + m < rows;
            const double* mp = M + (in ? (r0 + m) * RP : 0) + kq;
            double a[KS];
#pragma unroll
            for (int s = 0; s < KS; ++s) a[s] = in ? mp[4 * s] : 0.0;
            d4 acc = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int s = 0; s < KS; ++s) acc = mfma4(a[s], Gl[(4 * s + kq) * LD + 16 * ct + m], acc);
            // C/D element r of lane l: Y(r0 + (l>>4) + 4r, 16ct + (l&15))
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int rl = 16 * rt + kq + 4 * r;
                const int64_t i = c0 + rl;
                Ys[rl * LD + 16 * ct + m] = acc[r];  // zero for rows past the end
                if (i < rows) {
                    Y[i * RP + 16 * ct + m] = acc[r];
                    if (YT) YT[(int64_t)(16 * ct + m) * ldT + i] = acc[r];
                }
            }
        }
        __syncthreads();
        // G(ta, tb) += sum over the chunk's 64 rows: 16 K-steps of 4 rows
#pragma unroll
        for (int q = 0; q < GPW; ++q) {
            const int id = w + 4 * q;
            if (id < GT) {
                const int ta = id / NCT, tb = id - (id / NCT) * NCT;
#pragma unroll
                for (int s = 0; s < 16; ++s)
                    gacc[q] = mfma4(Ys[(4 * s + kq) * LD + 16 * ta + m], Ys[(4 * s + kq) * LD + 16 * tb + m],
                                    gacc[q]);
            }
        }
        __syncthreads();  // the chunk buffer is rewritten next
    }
#pragma unroll
    for (int q = 0; q < GPW; ++q) {
        const int id = w + 4 * q;
        if (id < GT) {
            const int ta = id / NCT, tb = id - (id / NCT) * NCT;
#pragma unroll
            for (int r = 0; r < 4; ++r) G[(int64_t)(16 * ta + kq + 4 * r) * RP + 16 * tb + m] = gacc[q][r];
        }
    }
}

bool apply_gram_small(int RP, int64_t rows) {
    // one CU's f64 MFMA against two launches of a few us each: worth it while
    // rows * RP^2 stays under ~5 us of one CU (config 3's largest factor)
    return RP <= 64 && (double)rows * RP * RP <= 327680.0;
}

void launch_apply_gram(int RP, const double* M, int64_t rows, const double* Ginv, double* Y,
                       double* YT, int64_t ldT, double* G, const int* stop, int* flags,
                       hipStream_t st) {
    if (!apply_gram_small(RP, rows)) throw Error(TRITD_ERR_ARG, "apply+Gram: problem too large for one workgroup");
#define AG_CASE(RPV) \
    case RPV: hipLaunchKernelGGL(k_apply_gram<RPV>, dim3(1), dim3(256), 0, st, M, rows, Ginv, Y, YT, ldT, G, stop, flags); break;
    switch (RP) {
        AG_CASE(16)
        AG_CASE(32)
        AG_CASE(48)
        AG_CASE(64)
        default: throw Error(TRITD_ERR_UNSUPPORTED, "apply+Gram: RP not supported");
    }
#undef AG_CASE
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// The pinv fallback as a launch of its own (before the generic apply of the
// fp32 path and of RP > 64; pinv.h): one workgroup, returns at once unless
// the solve set the request word.  RP <= 64 works in LDS; 128 / 256 in the
// Ginv buffer's scratch (the saved Gram is rotated in place, V beside it).
// ---------------------------------------------------------------------------
// (256 threads at every RP: the launch follows the solve on the side stream,
// beside a K2 / K5 grid of 256-thread workgroups, and a 1024-thread one would
// wait for that grid to drain; the fallback itself is rare)
template <int RP>
__global__ __launch_bounds__(256) void k_pinv_fix(double* Ginv, const int* stop, int* flags) {
    if (*stop) return;
    const double req = Ginv[ginv_req(RP)];
    if (req == 0.0) return;
    constexpr int NT = 256;
    __shared__ double rot[RP], red[NT / 64 + RP];
    __shared__ int pq[RP];
    double* G = Ginv + (int64_t)RP * RP;
    if constexpr (RP <= 64) {
        constexpr int LDP = RP + 1;
        __shared__ double pA[RP * LDP], pV[RP * LDP];
        for (int e = threadIdx.x; e < RP * RP; e += NT) {
            const int i = e / RP, j = e - (e / RP) * RP;
            pA[i * LDP + j] = G[e];
        }
        __syncthreads();
        jacobi_pinv<RP, NT>(pA, pV, LDP, (int)req, Ginv, RP, rot, pq, red, flags);
    } else {
        jacobi_pinv<RP, NT>(G, G + (int64_t)RP * RP, RP, (int)req, Ginv, RP, rot, pq, red, flags);
    }
}

void launch_pinv_fix(int RP, double* Ginv, const int* stop, int* flags, hipStream_t st) {
#define FIX_CASE(RPV) \
    case RPV: hipLaunchKernelGGL(k_pinv_fix<RPV>, dim3(1), dim3(256), 0, st, Ginv, stop, flags); break;
    switch (RP) {
        FIX_CASE(16)
        FIX_CASE(32)
        FIX_CASE(48)
        FIX_CASE(64)
        FIX_CASE(128)
        FIX_CASE(256)
        default: throw Error(TRITD_ERR_UNSUPPORTED, "pinv fallback: RP not supported");
    }
#undef FIX_CASE
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
