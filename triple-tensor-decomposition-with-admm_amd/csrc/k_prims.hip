// Primitive kernels: the API-level L1 ops of fast_robust_triple_tensor/ and
// the reductions the solver needs outside the loop.
//   K0 unfold          unfold.m:1-13       (LDS-tiled batched transpose)
//   K6 soft_threshold  soft_threshold.m:2  (16 B/lane streaming)
//   triple_product     triple_product.m:6  (MFMA, same tile as K5's L)
//   buildF/G/H         buildF.m:17-21 etc. (design matrices, for parity only)
#include <cstdlib>

#include "kernels.h"

namespace tritd {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// sum of squares of a padded tensor (pads are zero) -> per-block partials
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_sumsq(const double* __restrict__ X, int64_t n,
                                               double* partial) {
    double s = 0.0;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
        s = fma(X[e], X[e], s);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    __shared__ double red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        partial[2 * blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
        partial[2 * blockIdx.x + 1] = 0.0;
    }
}

int sumsq_blocks(const Geom& g) {
    int64_t b = cdiv(g.Ntm, 256 * 8);
    return (int)(b < 2048 ? (b < 1 ? 1 : b) : 2048);
}

void launch_sumsq_padded(const Geom& g, const double* X, double* partial, int nblocks,
                         hipStream_t st) {
    hipLaunchKernelGGL(k_sumsq, dim3(nblocks), dim3(256), 0, st, X, g.Ntm, partial);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// triple product L(i,j,t) = sum_k Ah(i,k) Bh(j,k) Ch(t,k)  (triple_product.m:6)
// written to / compared against a strided tensor X(i,j,t) = X[i + ldj*j + ldt*t]
// (the caller's column-major array: ldj = n1, ldt = n1*n2; no padded copy).
// mode 0: write L; mode 1: per-block partials of sum (L-X)^2 and sum X^2
// (the driver's RRE, traffic_triple_comparison.m:62-63,194-199).
//
// K5's L half on its own: a wave owns one ij-tile (16 rows i of one fibre j,
// its Khatri-Rao row in registers) and walks the t-tiles; the workgroup's 8
// waves share the C^T slice of each t-tile, staged in LDS double-buffered
// (the slice of t-tile tt+1 is loaded into registers before tile tt's MFMAs
// and written after them: one barrier per t-tile).  Per t-tile a wave runs
// RP/4 f64 MFMAs and stores 4 x 128 B pieces of L (16 consecutive i at 4
// t-values per store).  Bound: f64 MFMA (2*N*R flops).
// Measured at 512^3 r = 8 (rocprofv3, tools/rounds/r4/round4_tpab.sh, round 4; box to
// box spread ~10 us): 8 waves 336.5-347.7 us, 4 waves 339-344; four slice
// buffers with a barrier every second t-tile 353.6; two MFMA accumulation
// chains 357.0 (the extra LDS and registers cost more occupancy than the
// barriers save); the factors read in their reference layouts (no pack
// kernel) 358.5; no LDS at all — one wave per workgroup loading its operands
// from L2 by buffer loads — 371.7, or 385.9 with the next t-tile's operands
// prefetched (122 VGPRs); s_setprio(1) around the MFMA chain 337.6 vs 334.0.
// Round 6: the two-tile form with each workgroup's t-chunk of C^T staged in LDS
// once and no barrier in the walk (chunks of 2 / 4 / 8 / 16 t-tiles) ran 0.784
// / 0.529 / 0.406 / 0.379 vs 0.342 ms, bitwise equal: the per-workgroup start
// (Khatri-Rao gather, LDS fill) is what a t-chunk pays again, not the barriers
// (profiles/round6/tp3_chunks_dropped.txt).  (Round 3's form staged 32 t-values per step
// without double buffering, two barriers each: 0.464 ms.)
// ---------------------------------------------------------------------------
#ifndef TP_WV
#define TP_WV 8
#endif
constexpr int TP_WAVES = TP_WV;

template <int RP, int MODE>
__global__ __launch_bounds__(64 * TP_WAVES) void k_tp(const double* __restrict__ Ah,
                                                      const double* __restrict__ Bh,
                                                      const double* __restrict__ ChT, double* L,
                                                      const double* __restrict__ X, double* partial,
                                                      int64_t n1p, int64_t n1l, int64_t n3,
                                                      int64_t n3p, int64_t tiles, int64_t ldj,
                                                      int64_t ldt, int64_t ahj, int64_t bhj) {
    constexpr int KS = RP / 4;
    constexpr int SK = 17;  // odd row stride of the [k][t] slice (K5's L operand layout)
    constexpr int NT = 64 * TP_WAVES;
    constexpr int SP = RP * 8;  // d2v pairs per slice (RP rows of 16 t)
    constexpr int NS = (SP + NT - 1) / NT;
    __shared__ double sct[2][RP * SK];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int il = lane & 15, tg = lane >> 4;
    const int64_t tile = (int64_t)blockIdx.x * TP_WAVES + wid;
    const bool active = tile < tiles;
    const int64_t qper = n1p >> 4;
    const int64_t j = active ? tile / qper : 0;
    const int64_t i = active ? ((tile - j * qper) << 4) + il : 0;
    const bool row_ok = active && i < n1l;
    double kr[KS];
    {
        // unconditional loads, all issued first (k_admm.hip: the KR gather)
        double av[KS], bv[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + tg;
            av[s] = Ah[j * ahj + i * RP + k];  // kernels.h: KR source
            bv[s] = Bh[j * bhj + k];
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) kr[s] = active ? av[s] * bv[s] : 0.0;
    }
    const int64_t ntt = n3p >> 4;
    d2v sv[NS];
    auto stage_load = [&](int64_t tt) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * NT;
            if (SP % NT == 0 || e < SP) {
                const int k = e >> 3, t = (e & 7) * 2;
                sv[q] = *reinterpret_cast<const d2v*>(ChT + (int64_t)k * n3p + tt * 16 + t);
            }
        }
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * NT;
            if (SP % NT == 0 || e < SP) {
                const int k = e >> 3, t = (e & 7) * 2;
                sct[buf][k * SK + t] = sv[q][0];
                sct[buf][k * SK + t + 1] = sv[q][1];
            }
        }
    };
    const int64_t obase = i + ldj * j;
    double sn = 0.0, sd = 0.0;
    stage_load(0);
    stage_store(0);
    __syncthreads();
    for (int64_t tt = 0; tt < ntt; ++tt) {
        const int buf = (int)(tt & 1);
        const bool more = tt + 1 < ntt;
        if (more) stage_load(tt + 1);
        const double* cT = sct[buf];
        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < KS; ++s)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(cT[(4 * s + tg) * SK + il], kr[s], acc, 0, 0, 0);
        // C/D element r of lane l: L(i, j, t = 16 tt + (l>>4) + 4r)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            const int64_t t = tt * 16 + tg + 4 * rr;
            if (!row_ok || t >= n3) continue;
            const int64_t off = obase + ldt * t;
            if (MODE == 0) {
                __builtin_nontemporal_store(acc[rr], L + off);
            } else {
                const double x = X[off];
                const double dlt = acc[rr] - x;
                sn = fma(dlt, dlt, sn);
                sd = fma(x, x, sd);
            }
        }
        if (more) stage_store(buf ^ 1);  // buf^1 was last read in t-tile tt-1
        __syncthreads();
    }
    if (MODE == 1) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            sn += __shfl_xor(sn, off);
            sd += __shfl_xor(sd, off);
        }
        __shared__ double red[2][TP_WAVES];
        if (lane == 0) {
            red[0][wid] = sn;
            red[1][wid] = sd;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double a = 0.0, b = 0.0;
            for (int w = 0; w < TP_WAVES; ++w) {
                a += red[0][w];
                b += red[1][w];
            }
            partial[2 * blockIdx.x] = a;
            partial[2 * blockIdx.x + 1] = b;
        }
    }
}

// The same with TWO ij-tiles per wave (32 consecutive i of one fibre j,
// mode 0, RP <= 64): both accumulate against the same C^T operand read, and
// before the stores v_permlane16_swap pairs their rows so that one store
// instruction writes two t-rows of 32 i = 2 x 256 B (the one-tile form stores
// 4 x 128 B pieces, one per t-row).  Needs qper even (both tiles in one j).
template <int RP>
__global__ __launch_bounds__(64 * TP_WAVES) void k_tp2(const double* __restrict__ Ah,
                                                       const double* __restrict__ Bh,
                                                       const double* __restrict__ ChT, double* L,
                                                       int64_t n1p, int64_t n1l, int64_t n3,
                                                       int64_t n3p, int64_t tiles, int64_t ldj,
                                                       int64_t ldt, int64_t ahj, int64_t bhj) {
    constexpr int KS = RP / 4;
    constexpr int SK = 17;
    constexpr int NT = 64 * TP_WAVES;
    constexpr int SP = RP * 8;
    constexpr int NS = (SP + NT - 1) / NT;
    __shared__ double sct[2][RP * SK];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int il = lane & 15, tg = lane >> 4;
    const int64_t tile0 = ((int64_t)blockIdx.x * TP_WAVES + wid) * 2;  // tiles tile0, tile0 + 1
    const bool active = tile0 < tiles;
    const int64_t qper = n1p >> 4;
    const int64_t j = active ? tile0 / qper : 0;
    const int64_t i0 = active ? (tile0 - j * qper) << 4 : 0;  // first i of the 32
    double kr0[KS], kr1[KS];
    {
        // unconditional loads, all issued first (k_admm.hip: the KR gather;
        // an inactive wave reads rows 0..31, in range since qper is even)
        double a0[KS], a1[KS], bv[KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + tg;
            bv[s] = Bh[j * bhj + k];
            a0[s] = Ah[j * ahj + (i0 + il) * RP + k];
            a1[s] = Ah[j * ahj + (i0 + 16 + il) * RP + k];
        }
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            kr0[s] = active ? a0[s] * bv[s] : 0.0;
            kr1[s] = active ? a1[s] * bv[s] : 0.0;
        }
    }
    const int64_t ntt = n3p >> 4;
    d2v sv[NS];
    auto stage_load = [&](int64_t tt) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * NT;
            if (SP % NT == 0 || e < SP) {
                const int k = e >> 3, t = (e & 7) * 2;
                sv[q] = *reinterpret_cast<const d2v*>(ChT + (int64_t)k * n3p + tt * 16 + t);
            }
        }
    };
    auto stage_store = [&](int buf) {
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int e = threadIdx.x + q * NT;
            if (SP % NT == 0 || e < SP) {
                const int k = e >> 3, t = (e & 7) * 2;
                sct[buf][k * SK + t] = sv[q][0];
                sct[buf][k * SK + t + 1] = sv[q][1];
            }
        }
    };
    // after the swap lane l holds i = i0 + (l & 31) at t-row 2 (l >> 5) (+1 in
    // the second register) of each group of four
    const int64_t irow = i0 + (lane & 31);
    const bool row_ok = active && irow < n1l;
    const int64_t obase = irow + ldj * j;
    const int th = 2 * (lane >> 5);
    auto swap = [](double x, double y, double& a, double& b) {
        const unsigned xl = __double2loint(x), xh = __double2hiint(x);
        const unsigned yl = __double2loint(y), yh = __double2hiint(y);
        const auto lo = __builtin_amdgcn_permlane16_swap(xl, yl, false, false);
        const auto hi = __builtin_amdgcn_permlane16_swap(xh, yh, false, false);
        a = __hiloint2double((int)hi[0], (int)lo[0]);
        b = __hiloint2double((int)hi[1], (int)lo[1]);
    };
    stage_load(0);
    stage_store(0);
    __syncthreads();
    for (int64_t tt = 0; tt < ntt; ++tt) {
        const int buf = (int)(tt & 1);
        const bool more = tt + 1 < ntt;
        if (more) stage_load(tt + 1);
        const double* cT = sct[buf];
        d4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const double c = cT[(4 * s + tg) * SK + il];
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(c, kr0[s], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(c, kr1[s], acc1, 0, 0, 0);
        }
        // C/D element r of lane l: t = 16 tt + (l>>4) + 4r, i = i0 (+16 in acc1) + (l&15)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            double a, b;
            swap(acc0[rr], acc1[rr], a, b);
            const int64_t t = tt * 16 + 4 * rr + th;
            if (row_ok && t < n3) __builtin_nontemporal_store(a, L + obase + ldt * t);
            if (row_ok && t + 1 < n3) __builtin_nontemporal_store(b, L + obase + ldt * (t + 1));
        }
        if (more) stage_store(buf ^ 1);
        __syncthreads();
    }
}

int tp_grid(const Geom& g) { return (int)cdiv(g.tiles, TP_WAVES); }
static bool tp2_ok(const Geom& g) { return g.RP <= 64 && ((g.n1p >> 4) & 1) == 0; }

void launch_tp(const Geom& g, const double* Ah, const double* Bh, const double* ChT, double* Lout,
               const double* X, double* partial, int mode, int64_t ldj, int64_t ldt,
               hipStream_t st, int64_t ahj, int64_t bhj) {
    if (bhj < 0) bhj = g.RP;
    if (g.n3p % 16) throw Error(TRITD_ERR_ARG, "triple_product: n3p must be a multiple of 16");
    const dim3 grid(tp_grid(g)), block(64 * TP_WAVES);
#ifndef TP_TWO
#define TP_TWO 1
#endif
    if (TP_TWO && mode == 0 && tp2_ok(g)) {
        const dim3 grid2((unsigned)cdiv(g.tiles, 2 * TP_WAVES));
#define TP2_CASE(RPV)                                                                                \
    case RPV:                                                                                        \
        hipLaunchKernelGGL((k_tp2<RPV>), grid2, block, 0, st, Ah, Bh, ChT, Lout, g.n1p, g.n1l, g.n3,   \
                           g.n3p, g.tiles, ldj, ldt, ahj, bhj);                                      \
        break;
        switch (g.RP) {
            TP2_CASE(16)
            TP2_CASE(32)
            TP2_CASE(48)
            TP2_CASE(64)
        }
#undef TP2_CASE
        TRITD_CHECK_LAUNCH();
        return;
    }
#define TP_CASE(RPV)                                                                                 \
    case RPV:                                                                                        \
        if (mode == 0)                                                                               \
            hipLaunchKernelGGL((k_tp<RPV, 0>), grid, block, 0, st, Ah, Bh, ChT, Lout, X,      \
                               partial, g.n1p, g.n1l, g.n3, g.n3p, g.tiles, ldj, ldt, ahj, bhj);      \
        else                                                                                         \
            hipLaunchKernelGGL((k_tp<RPV, 1>), grid, block, 0, st, Ah, Bh, ChT, Lout, X,      \
                               partial, g.n1p, g.n1l, g.n3, g.n3p, g.tiles, ldj, ldt, ahj, bhj);      \
        break;
    switch (g.RP) {
        TP_CASE(16)
        TP_CASE(32)
        TP_CASE(48)
        TP_CASE(64)
        TP_CASE(128)
        TP_CASE(256)
        default:
            throw Error(TRITD_ERR_UNSUPPORTED, "rank not supported by triple_product");
    }
#undef TP_CASE
    TRITD_CHECK_LAUNCH();
}

// Reference-layout factors (device) -> the CP factor layout of common.h:
// Ah[i*RP+k] = A(i,p,q), Bh[j*RP+k] = B(p,j,q), ChT[k*n3p+t] = C(p,q,t),
// k = p + r*q (zero for k >= R and for the padded rows)
__global__ __launch_bounds__(256) void k_pack_factors(const double* __restrict__ A,
                                                      const double* __restrict__ B,
                                                      const double* __restrict__ C, int64_t n1,
                                                      int64_t n2, int64_t n3, int r, int RP,
                                                      int64_t n1p, int64_t n3p, double* Ah,
                                                      double* Bh, double* ChT) {
    const int R = r * r;
    const int64_t na = n1p * RP, nb = n2 * RP, nc = (int64_t)RP * n3p;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < na + nb + nc;
         e += (int64_t)gridDim.x * 256) {
        if (e < na) {
            const int64_t i = e / RP;
            const int k = (int)(e % RP);
            Ah[e] = (i < n1 && k < R) ? A[i + n1 * k] : 0.0;
        } else if (e < na + nb) {
            const int64_t f = e - na, jj = f / RP;
            const int k = (int)(f % RP), p = k % r, q = k / r;
            Bh[f] = k < R ? B[p + (int64_t)r * jj + (int64_t)r * n2 * q] : 0.0;
        } else {
            const int64_t f = e - na - nb, t = f % n3p;
            const int k = (int)(f / n3p);
            ChT[f] = (k < R && t < n3) ? C[k + (int64_t)R * t] : 0.0;
        }
    }
}

void launch_pack_factors(const Geom& g, const double* A, const double* B, const double* C,
                         double* Ah, double* Bh, double* ChT, hipStream_t st) {
    const int64_t tot = g.n1p * g.RP + g.n2 * g.RP + (int64_t)g.RP * g.n3p;
    int64_t b = cdiv(tot, 256);
    if (b > 4096) b = 4096;
    hipLaunchKernelGGL(k_pack_factors, dim3((unsigned)b), dim3(256), 0, st, A, B, C, g.n1, g.n2,
                       g.n3, g.r, g.RP, g.n1p, g.n3p, Ah, Bh, ChT);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// K0: batched transpose in[b][c][r] (r fastest) -> out[b][r][c] (c fastest).
//   unfold mode 2 (permute [2 1 3]): rows n1, cols n2, batch n3
//   unfold mode 3 (permute [3 1 2]): rows n1*n2, cols n3, batch 1
// 64 x 64 tile through LDS, 16-byte global accesses on both sides, nontemporal
// (streamed once: round 5, tools/unfold3_probe.hip at 512^3, mode 2 0.352 ->
// 0.329 ms = 6.52 TB/s).
// ---------------------------------------------------------------------------
constexpr int TT = 64;
// FULL: every tile is whole and 16-B aligned (checked on the host), so the
// kernel carries no bounds logic and issues its eight loads back to back
// (the bounds-checked form ran mode 2 at 512^3 in 0.425 vs 0.342 ms).
template <bool FULL>
__global__ __launch_bounds__(256) void k_transpose(const double* __restrict__ in,
                                                   double* __restrict__ out, int64_t rows,
                                                   int64_t cols) {
    __shared__ double tile[TT][TT + 1];
    const int64_t b = blockIdx.z;
    const int64_t r0 = (int64_t)blockIdx.x * TT, c0 = (int64_t)blockIdx.y * TT;
    const double* src = in + b * rows * cols;
    double* dst = out + b * rows * cols;
    const int th = threadIdx.x;
    // load: thread -> (c = th/32 + 8m, r = 2*(th%32))
    {
        const int rr = 2 * (th & 31), cc = th >> 5;
        if constexpr (FULL) {
            d2v v[8];
#pragma unroll
            for (int m = 0; m < 8; ++m)
                v[m] = __builtin_nontemporal_load(reinterpret_cast<const d2v*>(src + (c0 + cc + 8 * m) * rows + r0 + rr));
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                tile[cc + 8 * m][rr] = v[m].x;
                tile[cc + 8 * m][rr + 1] = v[m].y;
            }
        } else {
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int c = cc + 8 * m;
                const int64_t gc = c0 + c, gr = r0 + rr;
                tile[c][rr] = (gc < cols && gr < rows) ? src[gc * rows + gr] : 0.0;
                tile[c][rr + 1] = (gc < cols && gr + 1 < rows) ? src[gc * rows + gr + 1] : 0.0;
            }
        }
    }
    __syncthreads();
    // store: thread -> (r = th/32 + 8m, c = 2*(th%32))
    {
        const int cc = 2 * (th & 31), rr = th >> 5;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int r = rr + 8 * m;
            const int64_t gr = r0 + r, gc = c0 + cc;
            if constexpr (FULL) {
                __builtin_nontemporal_store(d2v{tile[cc][r], tile[cc + 1][r]},
                                            reinterpret_cast<d2v*>(dst + gr * cols + gc));
            } else {
                if (gr < rows && gc < cols) dst[gr * cols + gc] = tile[cc][r];
                if (gr < rows && gc + 1 < cols) dst[gr * cols + gc + 1] = tile[cc + 1][r];
            }
        }
    }
}

// Tall single transpose (unfold mode 3: rows = n1*n2 >> cols = n3): TR x TC
// tiles with the column tile fastest in blockIdx.x, so the blocks resident
// together write whole output rows (cols doubles) instead of TC-wide slivers
// of rows spread over the whole output, and all global loads issue before
// the LDS stores.  Measured at 512^3 (tools/prim_stream.hip): 32 x 128 tiles
// 0.385 ms = 5.58 TB/s vs 0.41 ms for the 64 x 64 row-fastest kernel.
// Round 5 (tools/unfold3_probe.hip, one box): nontemporal loads and stores
// and 128 x 64 tiles (1 KB read runs per column) 0.337 ms = 6.38 TB/s; 32 x
// 128 nontemporal 0.347, plain 0.369.
template <int TR, int TC>
__global__ __launch_bounds__(256) void k_transpose_tall(const double* __restrict__ in,
                                                        double* __restrict__ out, int64_t rows,
                                                        int64_t cols, int64_t nct) {
    __shared__ double tile[TC][TR + 1];
    const int64_t ct = blockIdx.x % nct, rt = blockIdx.x / nct;
    const int64_t r0 = rt * TR, c0 = ct * TC;
    const int th = threadIdx.x;
    constexpr int PR = TR / 2, CPP = 256 / PR, ML = TC / CPP;  // loads: column pairs of rows
    d2v v[ML];
    const int rp = th % PR, cc = th / PR;
#pragma unroll
    for (int m = 0; m < ML; ++m)
        v[m] = __builtin_nontemporal_load(
            reinterpret_cast<const d2v*>(in + (c0 + cc + CPP * m) * rows + r0 + 2 * rp));
#pragma unroll
    for (int m = 0; m < ML; ++m) {
        tile[cc + CPP * m][2 * rp] = v[m].x;
        tile[cc + CPP * m][2 * rp + 1] = v[m].y;
    }
    __syncthreads();
    constexpr int PC = TC / 2, RPP = 256 / PC, MS = TR / RPP;  // stores: row pairs of columns
    const int cp = th % PC, rr = th / PC;
#pragma unroll
    for (int m = 0; m < MS; ++m) {
        const int r = rr + RPP * m;
        __builtin_nontemporal_store(d2v{tile[2 * cp][r], tile[2 * cp + 1][r]},
                                    reinterpret_cast<d2v*>(out + (r0 + r) * cols + c0 + 2 * cp));
    }
}

void launch_transpose_batched(const double* in, double* out, int64_t rows, int64_t cols,
                              int64_t batch, hipStream_t st) {
    if (batch > 65535) {  // grid z holds at most 65535: batches of matrices
        const int64_t mat = rows * cols;
        for (int64_t b0 = 0; b0 < batch; b0 += 65535)
            launch_transpose_batched(in + b0 * mat, out + b0 * mat, rows, cols,
                                     batch - b0 < 65535 ? batch - b0 : 65535, st);
        return;
    }
    if (cdiv(rows, TT) > INT32_MAX || cdiv(cols, TT) > 65535)
        throw Error(TRITD_ERR_ARG, "unfold: matrix too large for one transpose launch");
    constexpr int TR = 128, TC = 64;
    if (batch == 1 && rows % TR == 0 && cols % TC == 0 && rows >= 64 * cols &&
        (((uintptr_t)in | (uintptr_t)out) & 15) == 0 && (rows / TR) * (cols / TC) < (1LL << 31)) {
        const int64_t nct = cols / TC;
        hipLaunchKernelGGL((k_transpose_tall<TR, TC>), dim3((unsigned)((rows / TR) * nct)), dim3(256),
                           0, st, in, out, rows, cols, nct);
        TRITD_CHECK_LAUNCH();
        return;
    }
    const dim3 grid((unsigned)cdiv(rows, TT), (unsigned)cdiv(cols, TT), (unsigned)batch);
    const bool full = rows % TT == 0 && cols % TT == 0 && (((uintptr_t)in | (uintptr_t)out) & 15) == 0;
    if (full)
        hipLaunchKernelGGL(k_transpose<true>, grid, dim3(256), 0, st, in, out, rows, cols);
    else
        hipLaunchKernelGGL(k_transpose<false>, grid, dim3(256), 0, st, in, out, rows, cols);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// K6: soft_threshold.m:2  Y = sign(X).*max(abs(X)-lam, 0)
// ---------------------------------------------------------------------------
__device__ __forceinline__ double st1(double x, double lam) {
    const double s = x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : (x == 0.0 ? 0.0 : x));
    return s * fmax(fabs(x) - lam, 0.0);
}

// ST_U 16-B nontemporal loads per thread issued before the first store, a
// block owning ST_U * 256 consecutive pairs per step (tools/prim_stream.hip at
// 512^3: 0.339 ms = 6.33 TB/s, the plain-copy ceiling of the chip, vs 0.39-0.41 ms
// for one load per grid-stride step).  Round 5: on zeros four loads per thread
// timed 0.332 vs 0.337 ms (tools/st_probe.hip; sixteen 0.358, an XCD-major or
// 1 MB-strided block order 0.36-0.37), but on random data, interleaved in one
// process (tools/ab_st.py at commit eceb414, when ST_U was a knob), eight
// win: 0.3415 vs 0.3459 ms = 6.29 TB/s, the copy ceiling.
template <int ST_U>
__global__ __launch_bounds__(256) void k_soft_threshold(const double* __restrict__ X, int64_t n,
                                                        double lam, double* __restrict__ Y) {
    const int64_t n2 = n >> 1;
    const d2v* X2 = reinterpret_cast<const d2v*>(X);
    d2v* Y2 = reinterpret_cast<d2v*>(Y);
    for (int64_t base = (int64_t)blockIdx.x * ST_U * 256; base < n2;
         base += (int64_t)gridDim.x * ST_U * 256) {
        d2v v[ST_U];
#pragma unroll
        for (int u = 0; u < ST_U; ++u) {
            const int64_t e = base + u * 256 + threadIdx.x;
            v[u] = e < n2 ? __builtin_nontemporal_load(X2 + e) : d2v{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < ST_U; ++u) {
            const int64_t e = base + u * 256 + threadIdx.x;
            d2v o;
            o.x = st1(v[u].x, lam);
            o.y = st1(v[u].y, lam);
            if (e < n2) __builtin_nontemporal_store(o, Y2 + e);
        }
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) Y[n - 1] = st1(X[n - 1], lam);
}

void launch_soft_threshold(const double* X, int64_t n, double lam, double* Y, hipStream_t st) {
    if (((uintptr_t)X | (uintptr_t)Y) & 15) throw Error(TRITD_ERR_ARG, "soft_threshold: 16-B alignment");
    constexpr int U = 8;
    int64_t blocks = cdiv(n / 2, 256 * U);
    if (blocks > 65536) blocks = 65536;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(k_soft_threshold<U>, dim3((unsigned)blocks), dim3(256), 0, st, X, n, lam, Y);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// buildF/G/H: out(k, a + nA*b), k = p + r*q, reference layouts in, column-major out
//   'F': out(k, j + n2 t) = B(p,j,q) C(p,q,t)      (buildF.m:12)
//   'G': out(k, i + n1 t) = A(i,p,q) C(p,q,t)      (buildG.m:12)
//   'H': out(k, i + n1 j) = A(i,p,q) B(p,j,q)      (buildH.m:12)
// ---------------------------------------------------------------------------
template <char W>
__global__ __launch_bounds__(256) void k_design(const double* P, const double* Q, int64_t nP,
                                                int64_t nQ, int r, double* out) {
    const int R = r * r;
    const int64_t total = (int64_t)R * nP * nQ;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * 256) {
        const int k = (int)(e % R);
        const int64_t col = e / R;
        const int64_t a = col % nP, b = col / nP;
        const int p = k % r, q = k / r;
        double x, y;
        if (W == 'F') {  // P = B (r,nP=n2,r), Q = C (r,r,nQ=n3)
            x = P[p + (int64_t)r * (a + nP * q)];
            y = Q[k + (int64_t)R * b];
        } else if (W == 'G') {  // P = A (nP=n1,r,r), Q = C
            x = P[a + nP * k];
            y = Q[k + (int64_t)R * b];
        } else {  // 'H': P = A, Q = B (r,nQ=n2,r)
            x = P[a + nP * k];
            y = Q[p + (int64_t)r * (b + nQ * q)];
        }
        out[e] = x * y;
    }
}

void launch_design(char which, const double* P, const double* Q, int64_t nP, int64_t nQ, int r,
                   double* out, hipStream_t st) {
    const int64_t total = (int64_t)r * r * nP * nQ;
    int64_t blocks = cdiv(total, 256);
    if (blocks > 16384) blocks = 16384;
    if (blocks < 1) blocks = 1;
    const dim3 grid((unsigned)blocks), block(256);
    if (which == 'F')
        hipLaunchKernelGGL(k_design<'F'>, grid, block, 0, st, P, Q, nP, nQ, r, out);
    else if (which == 'G')
        hipLaunchKernelGGL(k_design<'G'>, grid, block, 0, st, P, Q, nP, nQ, r, out);
    else
        hipLaunchKernelGGL(k_design<'H'>, grid, block, 0, st, P, Q, nP, nQ, r, out);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// column-major shard <-> tile-major (common.h).  One-off per solve.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_to_tm(const double* __restrict__ src, int64_t ld,
                                               int64_t n1l, int64_t n2, int64_t n3, int64_t n1p,
                                               int64_t ntt, int64_t Np, double* __restrict__ dst) {
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < Np; e += (int64_t)gridDim.x * 256) {
        const int64_t blk = e >> 8;  // ((g/4)*ntt + tt)*4 + g%4
        const int64_t q4 = blk >> 2, grp = q4 / ntt, tt = q4 - grp * ntt;
        const int64_t g = grp * 4 + (blk & 3);
        const int w = (int)(e & 255);
        const int p = w >> 7, l = (w & 127) >> 1, q = w & 1;
        const int r = 2 * p + q;
        const int64_t t = 16 * tt + (l >> 4) + 4 * r;
        const int64_t row = 16 * g + (l & 15);
        const int64_t j = row / n1p, i = row - j * n1p;
        dst[e] = (i < n1l && j < n2 && t < n3) ? src[(t * n2 + j) * ld + i] : 0.0;
    }
}

__global__ __launch_bounds__(256) void k_from_tm(const double* __restrict__ src, int64_t n1l,
                                                 int64_t n2, int64_t n3, int64_t n1p, int64_t ntt,
                                                 double* __restrict__ dst, int64_t ld) {
    const int64_t total = n1l * n2 * n3;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * 256) {
        const int64_t i = e % n1l, jt = e / n1l;
        const int64_t j = jt % n2, t = jt / n2;
        dst[(t * n2 + j) * ld + i] = src[tm_offset(i, j, t, n1p, ntt)];
    }
}

static unsigned grid_for(int64_t n) {
    int64_t b = cdiv(n, 256);
    return (unsigned)(b > 16384 ? 16384 : (b < 1 ? 1 : b));
}

void launch_to_tm(const Geom& g, const double* src, int64_t ld, double* dst, hipStream_t st) {
    hipLaunchKernelGGL(k_to_tm, dim3(grid_for(g.Ntm)), dim3(256), 0, st, src, ld, g.n1l, g.n2, g.n3,
                       g.n1p, g.ntt, g.Ntm, dst);
    TRITD_CHECK_LAUNCH();
}

void launch_from_tm(const Geom& g, const double* src, double* dst, int64_t ld, hipStream_t st) {
    hipLaunchKernelGGL(k_from_tm, dim3(grid_for(g.n1l * g.n2 * g.n3)), dim3(256), 0, st, src,
                       g.n1l, g.n2, g.n3, g.n1p, g.ntt, dst, ld);
    TRITD_CHECK_LAUNCH();
}

}  // namespace tritd
