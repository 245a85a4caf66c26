// Driver-side metrics of the reference experiments:
//   evaluate(X, gt, mask)      traffic_triple_comparison.m:194-202 (also in
//                              video_triple_comparison.m): rmse = norm(X(mask) - gt),
//                              nrmse = rmse / norm(gt)
//   quality_ybz(X1, X2)        other_methods/Low-rank-.../quality_ybz.m:1-33, the
//                              mean over frames of psnr_index (psnr_index.m:1-4,
//                              10*log10(255^2/mse(x-y))) and ssim_index
//                              (IPI_RTC_FCTN-main/lib/ssim_index.m, the copy the
//                              driver's genpath resolves first; Gaussian 11x11
//                              window, sigma 1.5, K = [0.01 0.03], L = 255,
//                              filter2 'valid', mean2 of the map)
// Both are HBM-bound streaming reductions with fixed-order (deterministic)
// partial sums; the masked evaluate pairs the k-th true mask position (column-
// major order, MATLAB's X(mask)) with gt(k) through a wave-count scan.
#include "kernels.h"

namespace tritd {

static constexpr int EV_THREADS = 256;
static constexpr int EV_ROUNDS = 16;  // 256-element rounds per block
static constexpr int64_t EV_CHUNK = (int64_t)EV_THREADS * EV_ROUNDS;

__device__ __forceinline__ double block_sum(double v, double* sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    double s = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += sh[w];
    return s;
}

// Masked pass layout: wave w owns the EV_CHUNK = 4096 consecutive positions
// [4096 w, 4096 w + 4096) as 4 rounds in which lane l holds the 16 positions
// 1024 q + 16 l + (0..15) (one 16-byte mask load).  A position's rank among
// the true ones is the wave's offset + the true positions of lower lanes
// (the lane counts' bits, ballot by ballot) + those before it in its group.
static constexpr int MG = 16;                    // positions per lane per round
static constexpr int MROUNDS = (int)(EV_CHUNK / (64 * MG));
static_assert(MROUNDS * 64 * MG == EV_CHUNK, "wave chunk");

// bit b set <=> mask[e + b] != 0, b < 16 (positions past n read as false)
__device__ __forceinline__ uint32_t mask_bits(const uint8_t* __restrict__ mask, int64_t e, int64_t n,
                                              bool al) {
    uint32_t bits = 0;
    if (al && e + MG <= n) {
        const uint4 v = *reinterpret_cast<const uint4*>(mask + e);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < MG; ++k) bits |= (((w[k >> 2] >> (8 * (k & 3))) & 0xffu) != 0u) << k;
    } else {
        for (int k = 0; k < MG; ++k)
            if (e + k < n && mask[e + k]) bits |= 1u << k;
    }
    return bits;
}

// exclusive prefix over the lanes of c (0 <= c <= 16) and the wave total
__device__ __forceinline__ void wave_scan16(int c, int& below, int& total) {
    below = 0;
    total = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const uint64_t bal = __ballot((c >> k) & 1);
        below += (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u)) << k;
        total += __builtin_popcountll(bal) << k;
    }
}

// pass 1: number of true mask entries per wave chunk
__global__ __launch_bounds__(EV_THREADS) void k_mask_count(const uint8_t* __restrict__ mask,
                                                           int64_t n, int nw, int al,
                                                           int64_t* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int gw = (int)blockIdx.x * (EV_THREADS / 64) + (int)(threadIdx.x >> 6);
    if (gw >= nw) return;
    const int64_t base = (int64_t)gw * EV_CHUNK;
    int c = 0;
    for (int q = 0; q < MROUNDS; ++q)
        c += __builtin_popcount(mask_bits(mask, base + q * 64 * MG + MG * lane, n, al != 0));
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if (lane == 0) cnt[gw] = c;
}

// pass 2: exclusive scan of the chunk counts in one block: thread t owns
// the contiguous run [t*per, (t+1)*per), sums it, one block scan of the 256
// run totals, then each run is rewritten with its offset (integers: exact)
__global__ __launch_bounds__(EV_THREADS) void k_scan_counts(int64_t* __restrict__ cnt, int nb,
                                                            int64_t* __restrict__ total) {
    __shared__ int64_t sh[EV_THREADS];
    const int per = (nb + EV_THREADS - 1) / EV_THREADS;
    const int b0 = (int)threadIdx.x * per, b1 = min(nb, b0 + per);
    int64_t run = 0;
#pragma unroll 16  // one block: batch the loads (latency-bound otherwise)
    for (int b = b0; b < b1; ++b) run += cnt[b];
    sh[threadIdx.x] = run;
    __syncthreads();
    for (int off = 1; off < EV_THREADS; off <<= 1) {  // Hillis-Steele inclusive
        const int64_t add = (int)threadIdx.x >= off ? sh[threadIdx.x - off] : 0;
        __syncthreads();
        sh[threadIdx.x] += add;
        __syncthreads();
    }
    int64_t acc = sh[threadIdx.x] - run;
#pragma unroll 16
    for (int b = b0; b < b1; ++b) {
        const int64_t v = cnt[b];
        cnt[b] = acc;
        acc += v;
    }
    if (threadIdx.x == EV_THREADS - 1) *total = sh[EV_THREADS - 1];
}

// pass 3 (mask): sum (X(p) - gt(k))^2 and gt(k)^2 over the true positions p,
// k = rank of p among them; only X at true positions is loaded
__global__ __launch_bounds__(EV_THREADS) void k_eval_mask(const double* __restrict__ X,
                                                          const double* __restrict__ gt, int64_t m,
                                                          const uint8_t* __restrict__ mask,
                                                          const int64_t* __restrict__ off,
                                                          int64_t n, int nw, int al,
                                                          double* __restrict__ part) {
    const int lane = threadIdx.x & 63;
    const int gw = (int)blockIdx.x * (EV_THREADS / 64) + (int)(threadIdx.x >> 6);
    double sd = 0.0, sg = 0.0;
    if (gw < nw) {
        const int64_t base = (int64_t)gw * EV_CHUNK;
        int64_t k0 = off[gw];
        for (int q = 0; q < MROUNDS; ++q) {
            const int64_t e = base + q * 64 * MG + MG * lane;
            const uint32_t bits = mask_bits(mask, e, n, al != 0);
            int below, tot;
            wave_scan16(__builtin_popcount(bits), below, tot);
            int64_t k = k0 + below;
#pragma unroll
            for (int b = 0; b < MG; ++b) {
                if ((bits >> b) & 1u) {
                    if (k < m) {
                        const double g = gt[k];
                        const double d = X[e + b] - g;
                        sd += d * d;
                        sg += g * g;
                    }
                    ++k;
                }
            }
            k0 += tot;
        }
    }
    __shared__ double sh[EV_THREADS / 64];
    const double a = block_sum(sd, sh);
    const double b = block_sum(sg, sh);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = b;
    }
}

// pass 3 (no mask): X and gt paired elementwise
__global__ __launch_bounds__(EV_THREADS) void k_eval_full(const double* __restrict__ X,
                                                          const double* __restrict__ gt,
                                                          int64_t n, double* __restrict__ part) {
    const int64_t base = (int64_t)blockIdx.x * EV_CHUNK;
    double sd = 0.0, sg = 0.0;
    const bool whole = base + EV_CHUNK <= n && (((uintptr_t)X | (uintptr_t)gt) & 15) == 0;
    if (whole) {
        // every block but the last: 16-byte nontemporal loads, all issued before
        // the arithmetic (round 5: the tensors are streamed once)
        typedef double d2 __attribute__((ext_vector_type(2)));
        constexpr int Q = EV_ROUNDS / 2;
        const d2* X2 = reinterpret_cast<const d2*>(X + base);
        const d2* G2 = reinterpret_cast<const d2*>(gt + base);
        d2 xv[Q], gv[Q];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            xv[q] = __builtin_nontemporal_load(X2 + q * EV_THREADS + threadIdx.x);
            gv[q] = __builtin_nontemporal_load(G2 + q * EV_THREADS + threadIdx.x);
        }
#pragma unroll
        for (int q = 0; q < Q; ++q) {
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const double d = xv[q][c] - gv[q][c];
                sd += d * d;
                sg += gv[q][c] * gv[q][c];
            }
        }
    } else {
        for (int q = 0; q < EV_ROUNDS; ++q) {
            const int64_t e = base + (int64_t)q * EV_THREADS + threadIdx.x;
            if (e < n) {
                const double g = gt[e];
                const double d = X[e] - g;
                sd += d * d;
                sg += g * g;
            }
        }
    }
    __shared__ double sh[EV_THREADS / 64];
    const double a = block_sum(sd, sh);
    const double b = block_sum(sg, sh);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = a;
        part[2 * blockIdx.x + 1] = b;
    }
}

int64_t evaluate_blocks(int64_t n) { return cdiv(n, EV_CHUNK); }

void launch_evaluate(const double* X, const double* gt, int64_t m, const uint8_t* mask, int64_t n,
                     int64_t* scratch_i64, double* part, double* out2, int64_t* total,
                     hipStream_t st) {
    const int64_t nb = evaluate_blocks(n);
    if (nb > (int64_t)INT32_MAX / 4) throw Error(TRITD_ERR_ARG, "tensor too large for evaluate");
    if (mask) {
        const int nw = (int)nb;  // one wave per EV_CHUNK positions
        const unsigned grid = (unsigned)cdiv(nb, EV_THREADS / 64);
        const int al = ((uintptr_t)mask & 15) == 0;
        hipLaunchKernelGGL(k_mask_count, dim3(grid), dim3(EV_THREADS), 0, st, mask, n, nw, al,
                           scratch_i64);
        TRITD_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(EV_THREADS), 0, st, scratch_i64, nw, total);
        TRITD_CHECK_LAUNCH();
        hipLaunchKernelGGL(k_eval_mask, dim3(grid), dim3(EV_THREADS), 0, st, X, gt, m, mask,
                           scratch_i64, n, nw, al, part);
        TRITD_CHECK_LAUNCH();
        launch_reduce_pairs(part, (int)grid, out2, nullptr, st);
    } else {
        hipLaunchKernelGGL(k_eval_full, dim3((unsigned)nb), dim3(EV_THREADS), 0, st, X, gt, n, part);
        TRITD_CHECK_LAUNCH();
        launch_reduce_pairs(part, (int)nb, out2, nullptr, st);
    }
}

// ---------------------------------------------------------------------------
// quality_ybz: per-frame PSNR and SSIM of two n1 x n2 x nf tensors
// ---------------------------------------------------------------------------
static constexpr int QT = 16;            // output tile edge of the SSIM map
static constexpr int QW = 11;            // window edge
static constexpr int QI = QT + QW - 1;   // input tile edge (26)

// SSIM map tiles: block (tx, ty, frame) computes a QT x QT tile of the
// (n1-10) x (n2-10) 'valid' map and its partial sum (filter2 is a
// correlation; the Gaussian window is symmetric).  The window of
// ssim_index.m is fspecial('gaussian',11,1.5) normalised, i.e. g g' up to
// rounding (no entry reaches fspecial's eps cut-off), so the five local
// moments are filtered separably: g(u) = win(u,c)/sqrt(win(c,c)), c = 5,
// first along j (26 x 16 partials in LDS), then along i -- 22 taps per
// moment instead of 121.  Rounding differs from the 2-D sum by a few ulps.
__global__ __launch_bounds__(QT* QT) void k_ssim_tiles(const double* __restrict__ X,
                                                       const double* __restrict__ Y, int64_t n1,
                                                       int64_t n2, const double* __restrict__ win,
                                                       double C1, double C2,
                                                       double* __restrict__ part) {
    __shared__ double sx[QI][QI + 1], sy[QI][QI + 1];   // [column offset][row offset]
    __shared__ double hm[5][QT][QI + 1];                // j-filtered moments [out column][row]
    __shared__ double g[QW];
    const int tx = threadIdx.x % QT, ty = threadIdx.x / QT;  // tx along rows i (fast)
    const int64_t f = blockIdx.z;
    const int64_t i0 = (int64_t)blockIdx.x * QT, j0 = (int64_t)blockIdx.y * QT;
    const double* Xf = X + f * n1 * n2;
    const double* Yf = Y + f * n1 * n2;
    constexpr int c = QW / 2;
    if (threadIdx.x < QW) g[threadIdx.x] = win[c * QW + threadIdx.x] / sqrt(win[c * QW + c]);
    for (int e = threadIdx.x; e < QI * QI; e += QT * QT) {
        const int a = e % QI, b = e / QI;  // a: row offset, b: column offset
        const int64_t i = i0 + a, j = j0 + b;
        const bool in = i < n1 && j < n2;
        sx[b][a] = in ? Xf[j * n1 + i] : 0.0;
        sy[b][a] = in ? Yf[j * n1 + i] : 0.0;
    }
    __syncthreads();
    for (int e = threadIdx.x; e < QT * QI; e += QT * QT) {
        const int a = e % QI, b = e / QI;  // row a of the input tile, output column b
        double m1 = 0.0, m2 = 0.0, s11 = 0.0, s22 = 0.0, s12 = 0.0;
#pragma unroll
        for (int v2 = 0; v2 < QW; ++v2) {
            const double wt = g[v2];
            const double x = sx[b + v2][a], y = sy[b + v2][a];
            m1 += wt * x;
            m2 += wt * y;
            s11 += wt * (x * x);
            s22 += wt * (y * y);
            s12 += wt * (x * y);
        }
        hm[0][b][a] = m1;
        hm[1][b][a] = m2;
        hm[2][b][a] = s11;
        hm[3][b][a] = s22;
        hm[4][b][a] = s12;
    }
    __syncthreads();
    const int64_t mi = n1 - (QW - 1), mj = n2 - (QW - 1);  // valid map size
    const int64_t oi = i0 + tx, oj = j0 + ty;
    double v = 0.0;
    if (oi < mi && oj < mj) {
        double m[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int u = 0; u < QW; ++u) {
            const double wt = g[u];
#pragma unroll
            for (int q = 0; q < 5; ++q) m[q] += wt * hm[q][ty][tx + u];
        }
        const double m1 = m[0], m2 = m[1];
        const double mu1_sq = m1 * m1, mu2_sq = m2 * m2, mu1_mu2 = m1 * m2;
        const double sigma1_sq = m[2] - mu1_sq, sigma2_sq = m[3] - mu2_sq, sigma12 = m[4] - mu1_mu2;
        v = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) /
            ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2));
    }
    __shared__ double sh[QT * QT / 64];
    const double s = block_sum(v, sh);
    if (threadIdx.x == 0)
        part[(f * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x] = s;
}

// per-frame sum of squared differences (psnr's mse numerator): block per
// (chunk, frame) partials
static constexpr int SQ_CHUNK = 4096;
__global__ __launch_bounds__(256) void k_frame_sqdiff(const double* __restrict__ X,
                                                      const double* __restrict__ Y, int64_t fsz,
                                                      double* __restrict__ part) {
    const int64_t f = blockIdx.y;
    const int64_t b0 = (int64_t)blockIdx.x * SQ_CHUNK;
    double s = 0.0;
    for (int64_t e = b0 + threadIdx.x; e < b0 + SQ_CHUNK && e < fsz; e += 256) {
        const double d = X[f * fsz + e] - Y[f * fsz + e];
        s += d * d;
    }
    __shared__ double sh[4];
    const double t = block_sum(s, sh);
    if (threadIdx.x == 0) part[f * gridDim.x + blockIdx.x] = t;
}

// per frame (one wave each; lane-strided partial sums, then a fixed xor
// tree: deterministic): psnr(f) = 10 log10(255^2 / (sqsum/npix));
// ssim(f) = mean2(map) (-Inf when the frame is smaller than the window,
// ssim_index.m nargin == 2)
__global__ __launch_bounds__(64) void k_quality_finish(const double* __restrict__ sqpart, int nsq,
                                                       const double* __restrict__ sspart, int nss,
                                                       double npix, double nmap, int small,
                                                       double* __restrict__ psnr,
                                                       double* __restrict__ ssim) {
    const int64_t f = blockIdx.x;
    const int lane = threadIdx.x;
    double a = 0.0, s = 0.0;
    for (int b = lane; b < nsq; b += 64) a += sqpart[f * nsq + b];
    for (int b = lane; b < nss; b += 64) s += sspart[f * nss + b];
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        s += __shfl_xor(s, off);
    }
    if (lane == 0) {
        psnr[f] = 10.0 * log10(255.0 * 255.0 / (a / npix));
        ssim[f] = small ? -INFINITY : s / nmap;
    }
}

void launch_quality(const double* X, const double* Y, int64_t n1, int64_t n2, int64_t nf,
                    const double* win, double C1, double C2, double* scratch, double* psnr,
                    double* ssim, hipStream_t st) {
    const int64_t fsz = n1 * n2;
    const int nsq = (int)cdiv(fsz, SQ_CHUNK);
    double* sqpart = scratch;
    double* sspart = scratch + (size_t)nsq * nf;
    const bool small = n1 < QW || n2 < QW;
    const unsigned gx = small ? 0u : (unsigned)cdiv(n1 - (QW - 1), QT);
    const unsigned gy = small ? 0u : (unsigned)cdiv(n2 - (QW - 1), QT);
    const int nss = (int)(gx * gy);
    const double nmap = small ? 1.0 : (double)((n1 - (QW - 1)) * (n2 - (QW - 1)));
    // frames run on grid y/z (at most 65535 per launch on gfx950): batches of
    // QF frames, each batch's pointers offset to its first frame
    constexpr int64_t QF = 65535;
    for (int64_t f0 = 0; f0 < nf; f0 += QF) {
        const int64_t nb = nf - f0 < QF ? nf - f0 : QF;
        const double* Xb = X + f0 * fsz;
        const double* Yb = Y + f0 * fsz;
        double* sqb = sqpart + (size_t)nsq * f0;
        double* ssb = sspart + (size_t)nss * f0;
        hipLaunchKernelGGL(k_frame_sqdiff, dim3(nsq, (unsigned)nb), dim3(256), 0, st, Xb, Yb, fsz,
                           sqb);
        TRITD_CHECK_LAUNCH();
        if (!small) {
            hipLaunchKernelGGL(k_ssim_tiles, dim3(gx, gy, (unsigned)nb), dim3(QT * QT), 0, st, Xb,
                               Yb, n1, n2, win, C1, C2, ssb);
            TRITD_CHECK_LAUNCH();
        }
        hipLaunchKernelGGL(k_quality_finish, dim3((unsigned)nb), dim3(64), 0, st, sqb, nsq, ssb,
                           nss, (double)fsz, nmap, (int)small, psnr + f0, ssim + f0);
        TRITD_CHECK_LAUNCH();
    }
}

size_t quality_scratch(int64_t n1, int64_t n2, int64_t nf) {
    const int64_t nsq = cdiv(n1 * n2, SQ_CHUNK);
    const int64_t nss = (n1 < QW || n2 < QW) ? 0 : cdiv(n1 - (QW - 1), QT) * cdiv(n2 - (QW - 1), QT);
    return (size_t)((nsq + nss) * nf);
}

}  // namespace tritd
