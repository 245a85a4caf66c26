// MATLAB pinv of a symmetric Gram on the device: the fallback behind the R x R
// solves (triple_decomp_ADMM.m:78,86,93 and triple_decomp_ALS.m:27,32,37 use
// pinv; the solves compute an inverse).
//
// A solve whose pivot test comes within 1e3x of pinv's cutoff (sweep.h,
// k_contract.hip) saves its Gram G = P o Q + alpha I next to the inverse and
// sets the slot's request word (ginv_req).  The consumer of the inverse (the
// apply kernel, or k_pinv_fix before the generic apply) then replaces it by
//   pinv(G) = sum over |lambda_i| > R eps(max |lambda|) of v_i v_i^T / lambda_i
// from a symmetric eigendecomposition (G is symmetric, so its singular values
// are |lambda| and its singular vectors the eigenvectors up to sign): MATLAB's
// pinv, tolerance max(size(G)) * eps(max sigma) with size(G) = R x R.  When a
// value is dropped the pinv-truncation flag is raised (TRITD_FLAG_PINV_TOL),
// so the flag reports what pinv actually did, on every schedule alike.
//
// Eigendecomposition: cyclic two-sided Jacobi with the round-robin (Brent-Luk)
// ordering, RP/2 disjoint rotations per round applied in parallel as J^T A J
// (rows, then columns and V, one barrier each), sweeps until the off-diagonal
// mass is below 1e-30 of the total — the oracle's criterion (tritd_ref.c
// pinv_sym).  The zero pad beyond R is never rotated (a_pq = 0 there) and has
// lambda = 0, so it drops out.  A and V may live in LDS (RP <= 64) or in global
// scratch that only this workgroup touches (RP = 128, 256: __syncthreads()
// orders workgroup-scope global accesses).
#pragma once

#include "kernels.h"

namespace tritd {

// player at seat `i` in round `rd` of the circle method (seat 0 fixed)
__device__ __forceinline__ int rr_player(int i, int rd, int n) {
    return i == 0 ? 0 : 1 + (i - 1 + rd) % (n - 1);
}

// Block-wide fixed-order sum of one value per thread (red: NT/64 doubles of
// LDS).  Every thread returns the same total.
template <int NT>
__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    __syncthreads();  // red may still be read from the previous call
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) s += red[w];
    return s;
}

// out (row stride ldo, RP x RP, zero outside R x R) = pinv(A), A symmetric
// RP x RP with row stride ld and a zero pad beyond R; A and V (row stride ld)
// are overwritten.  rot: 2*RP doubles, pq: RP ints, red: NT/64 + RP doubles
// (all LDS).  Every thread of the NT-thread workgroup calls it.
template <int RP, int NT>
__device__ void jacobi_pinv(double* A, double* V, int ld, int R, double* out, int ldo,
                            double* rot, int* pq, double* red, int* flags) {
    constexpr int NP = RP / 2;
    const int tid = threadIdx.x;
    for (int e = tid; e < RP * RP; e += NT) {
        const int i = e / RP, j = e - (e / RP) * RP;
        V[i * ld + j] = (i == j) ? 1.0 : 0.0;
    }
    for (int sweep = 0; sweep < 60; ++sweep) {
        double off = 0.0, tot = 0.0;
        for (int e = tid; e < RP * RP; e += NT) {
            const int i = e / RP, j = e - (e / RP) * RP;
            const double x = A[i * ld + j];
            tot = fma(x, x, tot);
            if (i != j) off = fma(x, x, off);
        }
        off = block_sum<NT>(off, red);
        tot = block_sum<NT>(tot, red);
        if (off == 0.0 || off <= 1e-30 * tot) break;
        for (int rd = 0; rd < RP - 1; ++rd) {
            if (tid < NP) {
                int p = rr_player(tid, rd, RP), q = rr_player(RP - 1 - tid, rd, RP);
                if (p > q) {
                    const int x = p;
                    p = q;
                    q = x;
                }
                const double apq = A[p * ld + q];
                double c = 1.0, s = 0.0;
                if (apq != 0.0) {
                    const double app = A[p * ld + p], aqq = A[q * ld + q];
                    const double th = (aqq - app) / (2.0 * apq);
                    const double t = (th >= 0.0 ? 1.0 : -1.0) / (fabs(th) + sqrt(th * th + 1.0));
                    c = 1.0 / sqrt(t * t + 1.0);
                    s = t * c;
                }
                rot[2 * tid] = c;
                rot[2 * tid + 1] = s;
                pq[2 * tid] = p;
                pq[2 * tid + 1] = q;
            }
            __syncthreads();
            // A <- J^T A: rows p, q of every pair
            for (int task = tid; task < NP * RP; task += NT) {
                const int k = task / RP, j = task - (task / RP) * RP;
                const int p = pq[2 * k], q = pq[2 * k + 1];
                const double c = rot[2 * k], s = rot[2 * k + 1];
                const double ap = A[p * ld + j], aq = A[q * ld + j];
                A[p * ld + j] = c * ap - s * aq;
                A[q * ld + j] = s * ap + c * aq;
            }
            __syncthreads();
            // A <- A J, V <- V J: columns p, q of every pair
            for (int task = tid; task < NP * RP; task += NT) {
                const int k = task / RP, i = task - (task / RP) * RP;
                const int p = pq[2 * k], q = pq[2 * k + 1];
                const double c = rot[2 * k], s = rot[2 * k + 1];
                const double ap = A[i * ld + p], aq = A[i * ld + q];
                A[i * ld + p] = c * ap - s * aq;
                A[i * ld + q] = s * ap + c * aq;
                const double vp = V[i * ld + p], vq = V[i * ld + q];
                V[i * ld + p] = c * vp - s * vq;
                V[i * ld + q] = s * vp + c * vq;
            }
            __syncthreads();
        }
    }
    // weights 1/lambda for the kept eigenvalues (every thread scans the
    // diagonal in the same order: same smax, same decisions)
    double* w = red + NT / 64;
    double smax = 0.0;
    for (int i = 0; i < R; ++i) smax = fmax(smax, fabs(A[i * ld + i]));
    const double tol = (double)R * (smax > 0.0 ? ldexp(1.0, ilogb(smax) - 52) : 0.0);
    bool dropped = false;
    for (int i = 0; i < R; ++i) dropped |= !(fabs(A[i * ld + i]) > tol);
    __syncthreads();  // w aliases red: block_sum readers are done
    for (int i = tid; i < RP; i += NT) {
        const double lam = A[i * ld + i];
        w[i] = (i < R && fabs(lam) > tol) ? 1.0 / lam : 0.0;
    }
    __syncthreads();
    for (int e = tid; e < RP * RP; e += NT) {
        const int i = e / RP, j = e - (e / RP) * RP;
        double x = 0.0;
        if (i < R && j < R)
            for (int k = 0; k < R; ++k) x = fma(V[i * ld + k] * w[k], V[j * ld + k], x);
        out[i * ldo + j] = x;
    }
    if (tid == 0 && dropped) atomicOr(flags, 1);
    __syncthreads();
}

// The solves' side of the protocol (every thread calls it after its pivot
// test; `near` must be the same in every thread): save G = P o Q + alpha I
// (same expression as the solves build it) and set or clear the request word.
template <int NT>
__device__ __forceinline__ void pinv_request(bool near, const double* P, const double* Q, int R,
                                             int RP, double alpha, double* Ginv) {
    if (near) {
        double* G = Ginv + (int64_t)RP * RP;
        for (int e = threadIdx.x; e < RP * RP; e += NT) {
            const int i = e / RP, c = e - (e / RP) * RP;
            double g = 0.0;
            if (i < R && c < R) {
                const double pq = P[i * RP + c] * Q[i * RP + c];
                g = (i == c) ? pq + alpha : pq;
            }
            G[e] = g;
        }
    }
    if (threadIdx.x == 0) Ginv[ginv_req(RP)] = near ? (double)R : 0.0;
}

// pivot test of the sweeps: the smallest LDL^T pivot within 1e3x of pinv's
// cutoff R*eps(max pivot) (every thread reads the same pivots)
__device__ __forceinline__ bool pivots_near_cutoff(const double* pivs, int R) {
    double minpiv = 1e308, maxpiv = 0.0;
    for (int p = 0; p < R; ++p) {
        minpiv = fmin(minpiv, pivs[p]);
        maxpiv = fmax(maxpiv, pivs[p]);
    }
    const double tol = (double)R * ldexp(1.0, ilogb(maxpiv) - 52);
    return !(minpiv > 1e3 * tol);
}

}  // namespace tritd
