// Symmetric Gauss-Jordan sweep of an SPD R x R Gram (k_contract.hip:
// k_solve, k_solve_ns) and the one-workgroup "side solve" that K2 and K5
// run in an extra workgroup of their own grid, so the solves
// of update_C and of the next update_A need no second stream.
#pragma once

#include <utility>

#include "kernels.h"
#include "pinv.h"

namespace tritd {

// Sweep step P.  Row P was published (by every wave: its candidate of that
// local row) into buffer P&1 by the previous step.  All reads are issued
// first; the row of pivot P+1 is updated before the others and published
// into the other buffer at once, so the barrier only waits on that.
template <int RP, int RW, int P>
__device__ __forceinline__ void sweep_step(double (&a)[RW], double* rowbuf, double* pivs, int c,
                                           int w) {
    constexpr int NW = RP / RW, W = P / RW, L = P % RW;
    const double* row = rowbuf + (P & 1) * NW * 64 + W * 64;  // a_Pc == a_cP
    const double piv = row[P];
    const double rc = row[c];
    double f[RW];  // a_iP for this wave's rows
#pragma unroll
    for (int q = 0; q < RW; ++q) f[q] = row[RW * w + q];
    pivs[P] = piv;  // every thread, same value
    const double d = 1.0 / piv;
    const bool pc = (c == P);
    const double s = rc * d;  // a_Pc / D
    const double m = pc ? 0.0 : 1.0;
    const double t = pc ? -d : s;
    if constexpr (P + 1 < RP) {
        constexpr int L2 = (P + 1) % RW;
        a[L2] = m * a[L2] - f[L2] * t;
        if (L2 == L && w == W) a[L] = t;  // (RW == 1 only)
        rowbuf[((P + 1) & 1) * NW * 64 + w * 64 + c] = a[L2];
#pragma unroll
        for (int q = 0; q < RW; ++q)
            if (q != L2) a[q] = m * a[q] - f[q] * t;
    } else {
#pragma unroll
        for (int q = 0; q < RW; ++q) a[q] = m * a[q] - f[q] * t;
    }
    // row P itself: a_Pc <- a_Pc/D, a_PP <- -1/D
    if (w == W) a[L] = t;
    __syncthreads();
}

template <int RP, int RW, int... Ps>
__device__ __forceinline__ void sweep_all(double (&a)[RW], double* rowbuf, double* pivs, int c,
                                          int w, std::integer_sequence<int, Ps...>) {
    (sweep_step<RP, RW, Ps>(a, rowbuf, pivs, c, w), ...);
}

// inv(P o Q + alpha I) by the sweep in one workgroup of NW waves (the host
// kernel's block): RP/NW rows per lane, lane = column (k_solve's algorithm
// and rounding with another row split).  rowbuf: 2*NW*64 doubles, pivs: RP
// doubles of LDS.
// Ginv is written directly (R x R block, zero pad), with the pinv request of
// pinv.h (the consumer replaces the inverse by pinv when the pivots come near
// MATLAB's cutoff).
// G = X^T X (RP x RP) of a row-major [rows][RP] factor in one workgroup of
// NW waves: wave w takes the 16 x 16 tiles w, w + NW, ... of G, each over all
// K-steps of 4 rows on v_mfma_f64_16x16x4_f64 (A[m][k] = X(i+k, 16ta+m),
// B[k][n] = X(i+k, 16tb+n)), loads 8 K-steps ahead; rows past the end are zero
template <int RP, int NW>
__device__ __forceinline__ void side_gram(const double* __restrict__ X, int64_t rows, double* G) {
    typedef double g4 __attribute__((ext_vector_type(4)));
    constexpr int NT = RP / 16, U = 8;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int m = lane & 15, kq = lane >> 4;
    const int64_t steps = (rows + 3) >> 2;
    for (int t = w; t < NT * NT; t += NW) {
        const int ta = t / NT, tb = t - (t / NT) * NT;
        const double* xa = X + 16 * ta + m;
        const double* xb = X + 16 * tb + m;
        g4 acc = g4{0.0, 0.0, 0.0, 0.0};
        for (int64_t s0 = 0; s0 < steps; s0 += U) {
            double a[U], b[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = 4 * (s0 + u) + kq;
                const bool in = i < rows;
                a[u] = in ? xa[i * RP] : 0.0;
                b[u] = in ? xb[i * RP] : 0.0;
            }
#pragma unroll
            for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc, 0, 0, 0);
        }
        // C/D element r of lane l: G(16ta + (l>>4) + 4r, 16tb + (l&15))
#pragma unroll
        for (int r = 0; r < 4; ++r) G[(int64_t)(16 * ta + kq + 4 * r) * RP + 16 * tb + m] = acc[r];
    }
}

template <int RP, int NW = 4>
__device__ __forceinline__ void side_solve(const SideSolve& s, double* rowbuf, double* pivs) {
    // the host kernel's other workgroups share this CU's SIMDs: win issue
    __builtin_amdgcn_s_setprio(3);
    constexpr int RW = RP / NW;
    const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int cc = c < RP ? c : 0;  // lanes >= RP read a valid column, never written back
    const double* P = s.P;
    const double* Q = s.Q;
    if (s.gram_rows > 0) {
        side_gram<RP, NW>(s.gram_src, s.gram_rows, s.gram_to);
        if (!s.solve) return;
        __syncthreads();  // (workgroup scope: the Gram is read back below by other waves)
        if (s.gram_which == 0)
            P = s.gram_to;
        else
            Q = s.gram_to;
    }
    double a[RW];
#pragma unroll
    for (int q = 0; q < RW; ++q) {
        const int i = RW * w + q;
        const bool in = (i < s.R) && (c < s.R);
        const double pq = P[i * RP + cc] * Q[i * RP + cc];
        const double g = (i == c) ? pq + s.alpha : pq;
        a[q] = in ? g : ((i == c) ? 1.0 : 0.0);
    }
    rowbuf[w * 64 + c] = a[0];
    __syncthreads();
    sweep_all<RP, RW>(a, rowbuf, pivs, c, w, std::make_integer_sequence<int, RP>{});
    if (c < RP)
#pragma unroll
        for (int q = 0; q < RW; ++q) {
            const int i = RW * w + q;
            s.Ginv[i * RP + c] = (i < s.R && c < s.R) ? -a[q] : 0.0;
        }
    // pinv's cutoff near: save the Gram and request the fallback (pinv.h)
    pinv_request<64 * NW>(pivots_near_cutoff(pivs, s.R), P, Q, s.R, RP, s.alpha, s.Ginv);
}

}  // namespace tritd
