// Mode contractions of the fp32 data path (D of class single)
// and the RP-general apply.
//
// MATLAB evaluates X_k*F' with X_k single as a single GEMM: M1, M2, M3 are
// accumulated in single here (W and T are single); the factor operands
// (A^ o B^, B^, A^) are the double factors rounded to single, as MATLAB
// converts the double design matrix F/G/H when it meets a single X_k.
#include "kernels.h"
#include "finish.h"

namespace tritd {

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4 mfma32c(float a, float b, f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// M1(i,k) = sum_j W[k][j*n1p + i] * B^(j,k)   (single)
// ---------------------------------------------------------------------------
// 16-byte loads (a lane owns 4 consecutive i, a wave 1 KB of a j-row), U = 8
// rows in flight per wave; the 4 waves take every 4th j and are summed
// through LDS in fixed order.  W at config 5 is 4.3 GB (as big as the tensor)
// and is read by M1 and M2: 4-byte-load kernels read it at ~4 TB/s (1.06 /
// 1.24 ms per launch, round 3).
__global__ __launch_bounds__(256) void k_m1_32v(const float* __restrict__ Wk,
                                                const double* __restrict__ Bh, float* M1,
                                                int64_t n1p, int64_t n2, int64_t plane, int RP,
                                                const int* stop) {
    if (*stop) return;
    constexpr int U = 8;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * 256 + 4 * lane;
    const int k = blockIdx.y;
    const bool in = i < n1p;  // n1p % 16 == 0: i..i+3 all in range
    f4 acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const f4* wp = reinterpret_cast<const f4*>(Wk + (int64_t)k * plane + (in ? i : 0));
    const int64_t ld4 = n1p >> 2;
    const double* bp = Bh + k;
    int64_t j = w;
    for (; j + 4 * (U - 1) < n2; j += 4 * U) {
        f4 v[U];
        float b[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v[u] = in ? __builtin_nontemporal_load(wp + (j + 4 * u) * ld4) : f4{0.0f, 0.0f, 0.0f, 0.0f};
            b[u] = (float)bp[(j + 4 * u) * RP];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[u][c] = fmaf(v[u][c], b[u], acc[u][c]);
    }
    for (; j < n2; j += 4) {
        const f4 v = in ? wp[j * ld4] : f4{0.0f, 0.0f, 0.0f, 0.0f};
        const float b = (float)bp[j * RP];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[0][c] = fmaf(v[c], b, acc[0][c]);
    }
    f4 t = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    __shared__ f4 red[4][64];
    red[w][lane] = t;
    __syncthreads();
    if (w == 0 && in) {
        const f4 sum = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
#pragma unroll
        for (int c = 0; c < 4; ++c) M1[(i + c) * RP + k] = sum[c];
    }
}

void launch_m1_32(const Geom& g, const float* Wk, const double* Bh, float* M1, const int* stop,
                  hipStream_t st) {
    hipLaunchKernelGGL(k_m1_32v, dim3((unsigned)cdiv(g.n1p, 256), g.RP), dim3(256), 0, st, Wk, Bh,
                       M1, g.n1p, g.n2, g.plane, g.RP, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// M2(j,k) = sum_i W[k][j*n1p + i] * A^(i,k)   (single sum, stored as double)
// ---------------------------------------------------------------------------
// Shards taller than k_m2_32w takes (n1p > 2048): 16-byte loads, a lane 4
// consecutive i per step, four independent accumulators, every load of the
// row in flight before the sums.
__global__ __launch_bounds__(256) void k_m2_32v(const float* __restrict__ Wk,
                                                const double* __restrict__ AhT, double* M2,
                                                int64_t n1p, int64_t n2, int64_t plane, int RP,
                                                const int* stop) {
    if (*stop) return;
    constexpr int U = 8;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t j = blockIdx.x;
    const int k = blockIdx.y * 4 + w;
    if (k >= RP) return;
    const f4* wp = reinterpret_cast<const f4*>(Wk + (int64_t)k * plane + j * n1p);
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2* ap = reinterpret_cast<const d2*>(AhT + (int64_t)k * n1p);
    const int64_t n4 = n1p >> 2;  // float4 groups of the row
    f4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    for (int64_t g0 = lane; g0 < n4; g0 += 64 * U) {
        f4 v[U];
        d2 a0[U], a1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t g = g0 + 64 * u;
            const bool in = g < n4;
            v[u] = in ? __builtin_nontemporal_load(wp + g) : f4{0.0f, 0.0f, 0.0f, 0.0f};
            a0[u] = in ? ap[2 * g] : d2{0.0, 0.0};
            a1[u] = in ? ap[2 * g + 1] : d2{0.0, 0.0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            f4& ac = acc[u & 3];
            ac[0] = fmaf(v[u][0], (float)a0[u][0], ac[0]);
            ac[1] = fmaf(v[u][1], (float)a0[u][1], ac[1]);
            ac[2] = fmaf(v[u][2], (float)a1[u][0], ac[2]);
            ac[3] = fmaf(v[u][3], (float)a1[u][1], ac[3]);
        }
    }
    const f4 t4 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
    float acc1 = (t4[0] + t4[1]) + (t4[2] + t4[3]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc1 += __shfl_xor(acc1, off);
    if (lane == 0) M2[j * RP + k] = (double)acc1;
}

// The same with the A^ row in registers: a wave owns one k and JB rows j, so
// the row k of A^T (n1p doubles, rounded to single once) is loaded once per
// JB rows instead of once per row (k_m2_32v re-read all of A^T for every j:
// 8.6 GB of L2 traffic beside the 4.3 GB of W at config 5).  n1p <= 64*4*UG.
// fin.on: workgroup (0, 0) first runs the previous iteration's norm
// reduction and stop test (finish.h), then its own rows — here rather than
// in M1, whose 2 048 workgroups are one full round of the chip (an extra one
// there lengthened M1 by ~60 us, config 5), and inside a workgroup of M2's
// 13 rounds rather than an extra column of them (which lengthened M2 by
// ~40 us).  M1, apply A and Gram A before it write only scratch and this
// iteration's A^ parity buffer.
template <int UG, int JB>
__global__ __launch_bounds__(256) void k_m2_32w(const float* __restrict__ Wk,
                                                const double* __restrict__ AhT, double* M2,
                                                int64_t n1p, int64_t n2, int64_t plane, int RP,
                                                const int* stop, FinishArgs fin) {
    if (fin.on && blockIdx.x == 0 && blockIdx.y == 0) {
        reduce_finish_wg<256>(fin);
        __syncthreads();
    }
    if (*stop) return;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int k = blockIdx.y;
    const int64_t j0 = ((int64_t)blockIdx.x * 4 + w) * JB;
    if (j0 >= n2) return;  // wave-uniform
    const int64_t n4 = n1p >> 2;
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2* ap = reinterpret_cast<const d2*>(AhT + (int64_t)k * n1p);
    f4 a[UG];
#pragma unroll
    for (int u = 0; u < UG; ++u) {
        const int64_t gi = lane + 64 * u;
        if (gi < n4) {
            const d2 x = ap[2 * gi], y = ap[2 * gi + 1];
            a[u] = f4{(float)x[0], (float)x[1], (float)y[0], (float)y[1]};
        } else {
            a[u] = f4{0.0f, 0.0f, 0.0f, 0.0f};
        }
    }
    const f4* wk = reinterpret_cast<const f4*>(Wk + (int64_t)k * plane);
    for (int jj = 0; jj < JB; ++jj) {
        const int64_t j = j0 + jj;
        if (j >= n2) break;  // wave-uniform
        const f4* wp = wk + j * n4;
        f4 v[UG];
#pragma unroll
        for (int u = 0; u < UG; ++u) {
            const int64_t gi = lane + 64 * u;
            v[u] = gi < n4 ? __builtin_nontemporal_load(wp + gi) : f4{0.0f, 0.0f, 0.0f, 0.0f};
        }
        f4 acc[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] = f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int u = 0; u < UG; ++u)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[u & 3][c] = fmaf(v[u][c], a[u][c], acc[u & 3][c]);
        const f4 t4 = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        float s1 = (t4[0] + t4[1]) + (t4[2] + t4[3]);
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) s1 += __shfl_xor(s1, off);
        if (lane == 0) M2[j * RP + k] = (double)s1;
    }
}

void launch_m2_32(const Geom& g, const float* Wk, const double* AhT, double* M2, const int* stop,
                  hipStream_t st, const FinishArgs& fin) {
    constexpr int UG = 8, JB = 8;
    if (g.n1p <= 64 * 4 * UG) {
        hipLaunchKernelGGL((k_m2_32w<UG, JB>), dim3((unsigned)cdiv(g.n2, 4 * JB), (unsigned)g.RP),
                           dim3(256), 0, st, Wk, AhT, M2, g.n1p, g.n2, g.plane, g.RP, stop, fin);
        TRITD_CHECK_LAUNCH();
        return;
    }
    if (fin.on)  // (n1p > 2048: the finish as its own launch, ahead of the contraction)
        launch_reduce_finish(fin.p, fin.n, fin.normD, fin.k, fin.tol, fin.errHist, fin.errL, fin.errO,
                             fin.ctrl, fin.single != 0, st, fin.clear != 0);
    hipLaunchKernelGGL(k_m2_32v, dim3((unsigned)g.n2, (unsigned)cdiv(g.RP, 4)), dim3(256), 0, st, Wk,
                       AhT, M2, g.n1p, g.n2, g.plane, g.RP, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// K2 (fp32) — M3(t,k) = sum_ij T(ij,t) A^(i,k) B^(j,k), any RP <= 256.
// Workgroup = (t-group of 4 t-tiles, i-tile q, j-chunk); wave w owns t-tile
// 4*tgrp + w and ALL RP columns (RP/16 f32x4 accumulators).  Walking j with
// q fixed keeps the 16 A^ rows of the i-tile in registers; per j the
// workgroup forms KR(ij,k) = single(A^(i,k) B^(j,k)) for the 16 ij of the
// tile in LDS (double-buffered, one barrier per j) and each wave streams its
// T tile (TX order: one dwordx4 per lane) as the B operand.  Per-workgroup
// partials are summed in fixed order by k_m3_reduce32.
// ---------------------------------------------------------------------------
constexpr int M3W = 4;

static int64_t m3_jchunks(const Geom& g) {
    const int64_t ntg = cdiv(g.ntt, 4), qper = g.n1p >> 4;
    int64_t jc = 2048 / (ntg * qper);
    // (round 6, three workgroups per CU: 3 / 6 chunks instead of 4 measured
    // slower, profiles/round6/c5_k2_ab.txt)
    if (jc < 1) jc = 1;
    if (jc > g.n2) jc = g.n2;
    return jc;
}

int m3_parts32(const Geom& g) { return (int)((g.n1p >> 4) * m3_jchunks(g)); }

// V (RP >= 64, the default there): KR stored [ij][il][m] with a 4-float pad
// per (ij, il) row (pitch MT + 4: the 16 lanes of a quarter-wave start on
// distinct 4-bank groups), so one ds_read_b128 gives a lane the A operands of
// four consecutive k-tiles — 4x fewer LDS reads than one float per MFMA.
template <int RP, bool V>
__global__ __launch_bounds__(64 * M3W) void k_m3_32(const float* __restrict__ T,
                                                    const double* __restrict__ Ah,
                                                    const double* __restrict__ Bh, double* part,
                                                    int64_t n1p, int64_t n2, int64_t n3p,
                                                    int64_t ntt, int64_t jc, const int* stop) {
    if (*stop) return;
    constexpr int MT = RP / 16;
    constexpr int KP = RP + 4;  // LDS row stride of KR (bank spread of the 4 ij rows a read touches)
    constexpr int PER = 16 * RP / (64 * M3W);  // KR elements formed per thread per j
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int il = lane & 15, tg = lane >> 4;
    const int64_t qper = n1p >> 4;
    const int64_t tgrp = blockIdx.x / (qper * jc);
    const int64_t rem = blockIdx.x - tgrp * qper * jc;
    const int64_t q = rem / jc, c = rem - q * jc;
    const int64_t ja = n2 * c / jc, jb = n2 * (c + 1) / jc;
    const int64_t tt = tgrp * 4 + wid;
    const bool tact = tt < ntt;
    const int64_t ttl = tact ? tt : ntt - 1;  // inactive waves read a valid tile, store nothing

    constexpr int PITCH = MT + 4;  // V layout: [row][il][m], m fastest
    constexpr int KSZ = V ? 16 * 16 * PITCH : 16 * KP;
    __shared__ __attribute__((aligned(16))) float krs[2][KSZ];
    // this thread's KR elements: e = threadIdx.x + 256 u -> (row e / RP, col e % RP)
    // (RP == 64 M3W, config 5: element u of thread x is (row u, k = x): one
    // B^ value per j and the 16 LDS writes at immediate offsets from one
    // address — the general form kept 24 VGPRs of per-u addresses live: 176
    // -> 148 VGPRs, three workgroups per CU instead of two, K2 4.94 -> 4.60 ms,
    // profiles/round6/c5_k2_ab.txt)
    constexpr bool ONEK = 64 * M3W == RP;
    double ah[PER > 0 ? PER : 1];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
        const int e = threadIdx.x + 64 * M3W * u;
        ah[u] = ONEK ? Ah[(q * 16 + u) * RP + threadIdx.x] : Ah[(q * 16 + e / RP) * RP + e % RP];
    }
    auto form = [&](int64_t j, int buf) {
        if constexpr (ONEK) {
            const int k = threadIdx.x;
            const double bh = Bh[j * RP + k];
            float* dst = &krs[buf][V ? (k & 15) * PITCH + (k >> 4) : k];
#pragma unroll
            for (int u = 0; u < PER; ++u) dst[u * (V ? 16 * PITCH : KP)] = (float)(ah[u] * bh);
        } else {
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = threadIdx.x + 64 * M3W * u;
                const int row = e / RP, k = e % RP;
                const int at = V ? (row * 16 + (k & 15)) * PITCH + (k >> 4) : row * KP + k;
                krs[buf][at] = (float)(ah[u] * Bh[j * RP + k]);
            }
        }
    };
    f4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = f4{0.0f, 0.0f, 0.0f, 0.0f};
    const f4* T4 = reinterpret_cast<const f4*>(T);
    auto tload = [&](int64_t j) { return T4[(tm_tile_base(j * qper + q, ttl, ntt) >> 2) + lane]; };

    if (ja < jb) {
        form(ja, 0);
        f4 bnext = tload(ja);
        __syncthreads();
        for (int64_t j = ja; j < jb; ++j) {
            const int buf = (int)((j - ja) & 1);
            const f4 b = bnext;
            if (j + 1 < jb) {
                bnext = tload(j + 1);
                form(j + 1, buf ^ 1);
            }
            const float* kr = krs[buf];
            if constexpr (V) {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const f4* ar = reinterpret_cast<const f4*>(kr + ((4 * s + tg) * 16 + il) * PITCH);
#pragma unroll
                    for (int mq = 0; mq < MT / 4; ++mq) {
                        const f4 a4 = ar[mq];
#pragma unroll
                        for (int u = 0; u < 4; ++u) acc[4 * mq + u] = mfma32c(a4[u], b[s], acc[4 * mq + u]);
                    }
                }
            } else {
#pragma unroll
                for (int s = 0; s < 4; ++s)
#pragma unroll
                    for (int m = 0; m < MT; ++m)
                        acc[m] = mfma32c(kr[(4 * s + tg) * KP + 16 * m + il], b[s], acc[m]);
            }
            __syncthreads();
        }
    }
    if (tact) {
        // the slab in the accumulators' own order (f32, as summed: exact):
        // f4 (tt*MT + m)*64 + lane, one 1 KB piece per store (k_m3_reduce32
        // maps it back: C/D row k = 16m + 4(l>>4) + rr, col t = 16 tt + (l & 15))
        f4* out = reinterpret_cast<f4*>(reinterpret_cast<float*>(part) + (q * jc + c) * n3p * RP);
#pragma unroll
        for (int m = 0; m < MT; ++m) out[(tt * MT + m) * 64 + lane] = acc[m];
    }
}

// M3 = single(sum over parts in fixed order), stored as double.  The parts
// are f32 slabs in K2's accumulator order (element e: rr = e & 3, lane =
// (e >> 2) & 63, m = (e >> 8) % MT, t-tile = (e >> 8) / MT) — half the bytes
// of double slabs, written 1 KB per store instead of 64 scattered words
// (config 5: 268 -> 134 MB written by K2 and read here)
__global__ __launch_bounds__(256) void k_m3_reduce32(const float* __restrict__ part, double* M3,
                                                     int64_t count, int nparts, int RP, const int* stop) {
    if (*stop) return;
    // a lane sums four consecutive elements (16-byte loads: 1 KB per wave
    // instruction instead of 256 B), each in the same slab order as before
    const int lane = threadIdx.x & 63, qd = threadIdx.x >> 6;
    const int64_t e0 = ((int64_t)blockIdx.x * 64 + lane) * 4;  // count % 4 == 0
    const f4* p4 = reinterpret_cast<const f4*>(part);
    const int64_t c4 = count >> 2;
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    if (e0 < count)
        for (int y0 = qd; y0 < nparts; y0 += 64) {  // 16 loads in flight, then the in-order sums
            f4 v[16];
#pragma unroll
            for (int u = 0; u < 16; ++u) {
                const int y = y0 + 4 * u;
                v[u] = y < nparts ? p4[(int64_t)y * c4 + (e0 >> 2)] : f4{0.0f, 0.0f, 0.0f, 0.0f};
            }
#pragma unroll
            for (int u = 0; u < 16; ++u)
                if (y0 + 4 * u < nparts)
#pragma unroll
                    for (int c = 0; c < 4; ++c) s[c] += (double)v[u][c];
        }
    __shared__ double red[4][4][64];
#pragma unroll
    for (int c = 0; c < 4; ++c) red[qd][c][lane] = s[c];
    __syncthreads();
    if (qd == 0 && e0 < count) {
        const int MT = RP >> 4;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int64_t e = e0 + c;
            const int rr = (int)(e & 3), l = (int)((e >> 2) & 63);
            const int64_t mt = e >> 8;
            const int64_t m = mt % MT, ttl = mt / MT;
            const int64_t t = ttl * 16 + (l & 15), k = 16 * m + 4 * (l >> 4) + rr;
            M3[t * RP + k] =
                (double)(float)(((red[0][c][lane] + red[1][c][lane]) + red[2][c][lane]) + red[3][c][lane]);
        }
    }
}

void launch_m3_32(const Geom& g, const float* T, const double* Ah, const double* Bh, double* part,
                  double* M3, const int* stop, hipStream_t st) {
    const int64_t jc = m3_jchunks(g), qper = g.n1p >> 4, ntg = cdiv(g.ntt, 4);
    const dim3 grid((unsigned)(ntg * qper * jc)), block(64 * M3W);
#define M3F_CASE(RPV)                                                                              \
    case RPV:                                                                                      \
        if (RPV >= 64)                                                                             \
            hipLaunchKernelGGL((k_m3_32<RPV, (RPV >= 64)>), grid, block, 0, st, T, Ah, Bh, part,   \
                               g.n1p, g.n2, g.n3p, g.ntt, jc, stop);                               \
        else                                                                                       \
            hipLaunchKernelGGL((k_m3_32<RPV, false>), grid, block, 0, st, T, Ah, Bh, part, g.n1p,  \
                               g.n2, g.n3p, g.ntt, jc, stop);                                      \
        break;
    switch (g.RP) {
        M3F_CASE(16)
        M3F_CASE(32)
        M3F_CASE(48)
        M3F_CASE(64)
        M3F_CASE(128)
        M3F_CASE(256)
        default:
            throw Error(TRITD_ERR_UNSUPPORTED, "rank not supported by the fp32 K2");
    }
#undef M3F_CASE
    TRITD_CHECK_LAUNCH();
    const int64_t count = g.n3p * g.RP;
    hipLaunchKernelGGL(k_m3_reduce32, dim3((unsigned)cdiv(count, 256)), dim3(256), 0, st,
                       reinterpret_cast<const float*>(part), M3, count, (int)(qper * jc), g.RP, stop);
    TRITD_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------
// Y = M * Ginv for any RP (fp32 path, fp64 RP > 64) on f64 MFMA: one wave per 16 x 16 tile of Y,
// A[m][k] = M(r0+m, 4s+k), B[k][n] = Ginv(4s+k, 16ct+n), RP/4 K-steps whose
// operands are loaded in batches of 16 before their MFMAs (both inputs are
// L2-resident: M is rows x RP, Ginv RP x RP).  At config 5 (rows 2048,
// RP 256) k_apply_gen took 0.28 ms per apply, three per iteration on the
// critical path (128 workgroups of sequential dot products, round 3's
// k_apply_gen).
// ---------------------------------------------------------------------------
typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));

template <int RP, typename TM>
__global__ __launch_bounds__(256) void k_apply_mfma(const TM* __restrict__ M, int64_t rows,
                                                    const double* __restrict__ Ginv, double* Y,
                                                    double* YT, int64_t ldT, float* YF,
                                                    int round32, const int* stop) {
    if (stop && *stop) return;
    constexpr int NT = RP / 16, KS = RP / 4;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t tile = (int64_t)blockIdx.x * 4 + w;
    const int64_t rt = tile / NT;
    const int ct = (int)(tile - rt * NT);
    const int64_t r0 = rt * 16;
    if (r0 >= rows) return;  // wave-uniform
    const int m = lane & 15, kq = lane >> 4;
    const bool in = r0 + m < rows;
    // K-steps in groups of four consecutive k per lane: at K-step 4g + u lane
    // (m, kq) takes k = 16 g + 4 kq + u, so one 16-byte (float) or two
    // 16-byte (double) loads of M serve four K-steps (the word-per-step form
    // took 34 us per apply at config 5).  Any k order is a valid MFMA sum;
    // this one is fixed.
    const TM* mp = M + (in ? (r0 + m) * RP : 0) + 4 * kq;
    const double* gp = Ginv + (int64_t)(4 * kq) * RP + 16 * ct + m;
    constexpr int NG = KS / 4, GB = NG < 4 ? NG : 4;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int g0 = 0; g0 < NG; g0 += GB) {
        double a[GB][4], b[GB][4];
#pragma unroll
        for (int gb = 0; gb < GB; ++gb) {
            const int g = g0 + gb;
            if constexpr (sizeof(TM) == 4) {
                typedef float f4l __attribute__((ext_vector_type(4)));
                const f4l v = in ? *reinterpret_cast<const f4l*>(mp + 16 * g) : f4l{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int u = 0; u < 4; ++u) a[gb][u] = (double)v[u];
            } else {
                const d2v v0 = in ? *reinterpret_cast<const d2v*>(mp + 16 * g) : d2v{0.0, 0.0};
                const d2v v1 = in ? *reinterpret_cast<const d2v*>(mp + 16 * g + 2) : d2v{0.0, 0.0};
                a[gb][0] = v0[0];
                a[gb][1] = v0[1];
                a[gb][2] = v1[0];
                a[gb][3] = v1[1];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) b[gb][u] = gp[(int64_t)(16 * g + u) * RP];
        }
#pragma unroll
        for (int gb = 0; gb < GB; ++gb)
#pragma unroll
            for (int u = 0; u < 4; ++u)
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[gb][u], b[gb][u], acc, 0, 0, 0);
    }
    const int k = 16 * ct + m;
    // YT through a per-wave LDS tile: each lane then writes 16 consecutive i
    // of one k-row (128-byte pieces) instead of one word per row
    __shared__ double tl[4][16 * 17];
    double* tw = tl[w];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = r0 + kq + 4 * r;
        double v = acc[r];
        if (round32) v = (double)(float)v;
        tw[(kq + 4 * r) * 17 + m] = v;
        if (i >= rows) continue;
        Y[i * RP + k] = v;
        if (YF) YF[i * RP + k] = (float)v;
    }
    if (YT) {
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        const int64_t i = r0 + m;  // lane m: row i; kq + 4 r: the k-row
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int kk = kq + 4 * r;
            if (i < rows) YT[(int64_t)(16 * ct + kk) * ldT + i] = tw[m * 17 + kk];
        }
    }
}

void launch_apply_gen(int RP, const double* M, const float* Mf, int64_t rows, double* Ginv,
                      double* Y, double* YT, int64_t ldT, float* YF, bool round32, const int* stop,
                      int* flags, hipStream_t st, bool fix) {
    if (fix) launch_pinv_fix(RP, Ginv, stop, flags, st);
    {
        const int64_t tiles = cdiv(rows, 16) * (RP / 16);
        const dim3 grid((unsigned)cdiv(tiles, 4)), block(256);
#define APPLY_MF_CASE(RPV)                                                                          \
    case RPV:                                                                                       \
        if (Mf)                                                                                     \
            hipLaunchKernelGGL((k_apply_mfma<RPV, float>), grid, block, 0, st, Mf, rows, Ginv, Y, YT, \
                               ldT, YF, (int)round32, stop);                                        \
        else                                                                                        \
            hipLaunchKernelGGL((k_apply_mfma<RPV, double>), grid, block, 0, st, M, rows, Ginv, Y,   \
                               YT, ldT, YF, (int)round32, stop);                                    \
        break;
        switch (RP) {
            APPLY_MF_CASE(16)
            APPLY_MF_CASE(32)
            APPLY_MF_CASE(48)
            APPLY_MF_CASE(64)
            APPLY_MF_CASE(128)
            APPLY_MF_CASE(256)
            default: throw Error(TRITD_ERR_UNSUPPORTED, "apply: RP not supported");
        }
#undef APPLY_MF_CASE
        TRITD_CHECK_LAUNCH();
    }
}

}  // namespace tritd
