// errHist bookkeeping and the stop test of triple_decomp_ADMM.m:59-63 on the
// device, from K5's per-workgroup [sum resL^2, sum resO^2] pairs: the
// standalone k_reduce_finish and the extra workgroup of the next iteration's
// M1 (k_contract.hip) both run reduce_finish_wg, so they sum in the same
// fixed order (bitwise the same errHist and stop decision).
#pragma once

#include "kernels.h"

namespace tritd {

// ctrl[0] = stop flag, ctrl[1] = iterations completed (k of :68)
__device__ __forceinline__ void finish_body(const double* ss, double normD, int k, double tol,
                                            double* errHist, double* errL, double* errO, int* ctrl,
                                            int single) {
    double eL = sqrt(ss[0]) / normD;  // norm(resL(:))/normD
    double eO = sqrt(ss[1]) / normD;  // norm(resO(:))/normD
    double e = eL + eO;               // :59
    if (single) {  // single residuals: single norms, single quotients and sum
        const float fL = (float)sqrt(ss[0]) / (float)normD;
        const float fO = (float)sqrt(ss[1]) / (float)normD;
        eL = fL;
        eO = fO;
        e = (double)(fL + fO);
    }
    errHist[k - 1] = e;
    errL[k - 1] = eL;
    errO[k - 1] = eO;
    ctrl[1] = k;
    if (k > 1 && fabs(e - errHist[k - 2]) < tol * errHist[k - 2]) ctrl[0] = 1;  // :63
}

// One workgroup of NT >= 256 threads: threads 0..255 sum the pairs t, t+256,
// ... in order, then a fixed tree; thread 0 finishes.  clear: zero the pairs
// after reading them (each thread clears the pairs it read).
template <int NT>
__device__ __forceinline__ void reduce_finish_wg(const FinishArgs& f) {
    static_assert(NT >= 256, "reduce_finish_wg: 256 threads at least");
    if (f.ctrl[0]) return;  // (uniform: every thread reads the same word)
    __shared__ double sx[256], sy[256];
    const int t = threadIdx.x;
    if (t < 256) {
        double x = 0.0, y = 0.0;
#pragma unroll 8  // loads batched; the sums keep their sequential order
        for (int b = t; b < f.n; b += 256) {
            x += f.p[2 * b];
            y += f.p[2 * b + 1];
        }
        if (f.clear)
            for (int b = t; b < f.n; b += 256) {
                f.p[2 * b] = 0.0;
                f.p[2 * b + 1] = 0.0;
            }
        sx[t] = x;
        sy[t] = y;
    }
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) {
            sx[t] += sx[t + w];
            sy[t] += sy[t + w];
        }
        __syncthreads();
    }
    if (t == 0) {
        const double ss[2] = {sx[0], sy[0]};
        finish_body(ss, f.normD, f.k, f.tol, f.errHist, f.errL, f.errO, f.ctrl, f.single);
    }
}

}  // namespace tritd
