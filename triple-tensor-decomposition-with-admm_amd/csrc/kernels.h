// Kernel launchers (host side) for libtritd.  All launches are asynchronous
// on the given stream; every ADMM-loop kernel early-exits when *stop != 0 so
// that iterations enqueued past the stop test of triple_decomp_ADMM.m:63
// become no-ops without a host round trip.
#pragma once

#include "common.h"

namespace tritd {

// Dense-E tile statistics: one atomic per wave into one of DENSE_SLOTS
// counters (summed on the host), not one per tile on a single counter.
constexpr int DENSE_SLOTS = 64;

struct DevState;  // solver.cpp

// ---- K5: fused ADMM update (k_admm.hip) ----------------------------------
// One R x R solve run by an extra workgroup (blockIdx 0) of K2 or K5
// (sweep.h: side_solve): Ginv = inv(P o Q + alpha I).  on = 0: none.
struct SideSolve {
    const double* P = nullptr;
    const double* Q = nullptr;
    double alpha = 0.0;
    double* Ginv = nullptr;
    int* flags = nullptr;
    int R = 0;
    int on = 0;
    // gram_rows > 0: the side workgroup first forms one operand itself,
    // gram_to = X^T X of the row-major [gram_rows][RP] factor gram_src, which
    // then stands for P (gram_which = 0) or Q (1): the fused single-GPU
    // schedule's Grams ride in the side job instead of a launch of their own
    const double* gram_src = nullptr;
    double* gram_to = nullptr;
    int64_t gram_rows = 0;
    int gram_which = 0;
    // 0: the Gram only, no solve (a sharded session's A^T A, formed beside
    // M2 for the all-reduce that follows it)
    int solve = 1;
};

// The reduction + stop test of one iteration's K5 norm pairs, run by an
// extra workgroup of the next iteration's M1 (single GPU: one launch less per
// iteration; finish.h)
struct FinishArgs {
    double* p = nullptr;  // n [sum resL^2, sum resO^2] pairs
    int n = 0;
    double normD = 0.0;
    int k = 0;
    double tol = 0.0;
    double* errHist = nullptr;
    double* errL = nullptr;
    double* errO = nullptr;
    int* ctrl = nullptr;
    int single = 0;
    int clear = 0;
    int on = 0;
};

struct K5Args {
    const double* D;
    double* O;
    double* E;   // dense E: only tiles whose compact slot overflowed (common.h)
    double* CE;  // compact E: one 32-double slot per tile
    double* YL;
    double* T;
    double* Wk;
    const double* Ah;
    const double* Bh;
    const double* Ch;
    const double* ChT;
    double* partial;  // [grid][2] sums of resL^2, resO^2
    int64_t n1p, n2, n3p, plane, tiles, ntt;
    IterScalars s;
    const int* stop;
    unsigned long long* dense_tiles;  // DENSE_SLOTS running counts of E tiles stored densely
    // derived-Y_O mode (dy): Y_O is not stored; K5 of iteration k+1 rebuilds
    // Y_O^(k) = Y_L^(k) - muO_k (E^(k) - E^(k-1)) from E^(k) (CE/E) and
    // E^(k-1) (CEp/Ep) and writes E^(k+1) over E^(k-1) (k_admm.hip)
    double* CEp;
    double* Ep;
    // Khatri-Rao operand source: kr(ij,k) = Ah[j*ahj + i*RP + k] * Bh[j*bhj + k].
    // CP (the executed model): ahj = 0, bhj = RP.  Qi model (opts.model='qi'):
    // Ah = H (k_qi.hip, rows j*n1p+i), ahj = n1p*RP, Bh = ones, bhj = 0.
    int64_t ahj, bhj;
    SideSolve side;  // RP <= 64, CP model: solve A of the next iteration
    int tsplit = 1;  // chunks of the t-walk (set by launch_k5: k5_tsplit)
};
int k5_grid(const Geom& g);
// chunks of the fp64 K5's t-walk (1 unless the problem has few ij-tiles); K5
// then runs k5_grid * k5_tsplit workgroups and W needs k5_tsplit sets
int k5_tsplit(const Geom& g);
int k5_parts32(const Geom& g);  // fp32 K5's norm-partial count (its workgroups)
// dense_e: E kept densely for every tile (no compact slots; dy only, RP <= 64)
void launch_k5(const Geom& g, const K5Args& a, bool prologue, hipStream_t st,
               bool dense_e = false);
// O_k = (D + invL_next*Y_L) - T_{k+1} (O is not stored by K5)
void launch_pool_probe(const Geom& g, double* D, double* YL, double* T, double* CE,
                       hipStream_t st);
void launch_ce_expand(const Geom& g, const double* CE, double* E, hipStream_t st);
void launch_o_fixup(const Geom& g, const double* D, const double* YL, const double* T,
                    double invL_next, double* O, hipStream_t st);
// partial sums -> out[0..1] (fixed-order tree)
void launch_reduce_pairs(const double* partial, int n, double* out, const int* stop, hipStream_t st);
// both in one launch (single GPU: nothing to all-reduce in between)
// single: D is of class single, so errHist(k) = single(norm/normD + norm/normD)
// with the norms rounded to single (MATLAB class rules)
void launch_reduce_finish(double* partial, int n, double normD, int k, double tol,
                          double* errHist, double* errL, double* errO, int* ctrl, bool single,
                          hipStream_t st, bool clear = false);
// errHist bookkeeping + stop test (triple_decomp_ADMM.m:59,63)
void launch_finish(const double* ss, double normD, int k, double tol, double* errHist, double* errL,
                   double* errO, int* ctrl, bool single, hipStream_t st);

// ---- contractions and small linear algebra (k_contract.hip) ---------------
// fin.on: the previous iteration's norm reduction and stop test in an extra
// workgroup (finish.h)
void launch_m1(const Geom& g, const double* Wk, const double* Bh, double* M1, const int* stop,
               hipStream_t st, const FinishArgs& fin = FinishArgs{});
// side: update_B's R x R solve in an extra workgroup (RP <= 64)
void launch_m2(const Geom& g, const double* Wk, const double* AhT, double* M2, const int* stop,
               hipStream_t st, const SideSolve& side = SideSolve{});
int m3_split(const Geom& g);
int m3_parts(const Geom& g);  // partial slabs of n3p*RP written by K2
// kr(ij,k) = Ah[j*ahj + i*RP + k] * Bh[j*bhj + k] (K5Args::ahj; bhj < 0 means RP)
// side: an R x R solve in an extra workgroup of the CP kernel (RP <= 64)
void launch_m3(const Geom& g, const double* T, const double* Ah, const double* Bh, double* part,
               double* M3, const int* stop, hipStream_t st, int64_t ahj = 0, int64_t bhj = -1,
               const SideSolve& side = SideSolve{});
// G = X^T X over `rows` rows of a row-major [rows][RP] factor
void launch_gram(int RP, const double* X, int64_t rows, double* G, const int* stop, hipStream_t st,
                 bool side = false);
// Ginv buffers, one per Gram slot (pinv.h): [0, RP^2) the inverse, read by
// the apply; [RP^2, 2 RP^2) the Gram, saved by a solve whose pivot test came
// near pinv's cutoff; [2 RP^2, 3 RP^2) eigenvector scratch of the RP > 64
// fallback; the request word at ginv_req (a double: R = replace the inverse
// by pinv of the saved R x R Gram, 0 = none).
// Past the request word: RP pivots and RP/16 step words of the multi-workgroup
// solve (k_solve_mw, RP = 128 / 256; zero-initialised with the buffer).
__host__ __device__ inline int64_t ginv_req(int RP) { return 3 * (int64_t)RP * RP; }
__host__ __device__ inline int64_t ginv_piv(int RP) { return ginv_req(RP) + 8; }
__host__ __device__ inline int64_t ginv_sync(int RP) { return ginv_piv(RP) + RP; }
inline size_t ginv_count(int RP) { return (size_t)ginv_sync(RP) + 16; }
// Ginv = inv(P o Q + alpha I) on the leading R x R block (zero elsewhere),
// plus the pinv request of pinv.h.  flags is unused by the solves since the
// pinv fallback raises TRITD_FLAG_PINV_TOL itself (kept for the call shape).
// fin.on (RP <= 64): the same launch first runs the norm reduction + stop
// test of the previous iteration (finish.h) — a sharded session's finish and
// update_B's solve both follow the first all-reduce, one launch for the two.
void launch_solve(int RP, int R, const double* P, const double* Q, double alpha, double* Ginv,
                  int* flags, const int* stop, hipStream_t st, const FinishArgs* fin = nullptr);
// Y = M * Ginv ([rows][RP]); optional transposed copy YT[k*ldT + i].  A set
// request word makes every workgroup use pinv(saved Gram) instead (pinv.h);
// flags[0] is raised when that pinv drops a singular value.
// Y = M * Ginv and G = Y^T Y in one workgroup (small problems: apply_gram_small)
bool apply_gram_small(int RP, int64_t rows);
void launch_apply_gram(int RP, const double* M, int64_t rows, const double* Ginv, double* Y,
                       double* YT, int64_t ldT, double* G, const int* stop, int* flags,
                       hipStream_t st);
void launch_apply(int RP, const double* M, int64_t rows, const double* Ginv, double* Y, double* YT,
                  int64_t ldT, const int* stop, int* flags, hipStream_t st);
// ---- Qi model (opts.model='qi', k_qi.hip; origin_triple_tensor/build{F,G,H}.m) ----
// H[(j*n1p+i)*RP + p+r*q] = sum_s Ah(i, q+r*s) Bh(j, p+r*s)  (zero for k >= R)
void launch_qi_h(const Geom& g, int r, const double* Ah, const double* Bh, double* H,
                 const int* stop, hipStream_t st);
// M1(i, q+r*s) = sum_j sum_p W(ij, p+r*q) Bh(j, p+r*s)
void launch_m1_qi(const Geom& g, int r, const double* Wk, const double* Bh, double* M1,
                  const int* stop, hipStream_t st);
// M2(j, p+r*s) = sum_i sum_q W(ij, p+r*q) Ah(i, q+r*s)
void launch_m2_qi(const Geom& g, int r, const double* Wk, const double* AhT, double* M2,
                  const int* stop, hipStream_t st);
// F F' / G G' / H H' of the Qi design matrices from the factor Grams
// (mode 0: X=B^TB, Y=C^TC; 1: X=A^TA, Y=C^TC; 2: X=A^TA, Y=B^TB)
void launch_qi_gram(int RP, int r, int mode, const double* X, const double* Y, double* out,
                    const int* stop, hipStream_t st);
void launch_fill(double* x, int64_t n, double v, hipStream_t st);
// out = sum_p in[p] (fixed order), written back to every in[p]  (virtual shards)
void launch_vsum(double* const* bufs, int nbufs, int64_t count, hipStream_t st);

// ---- primitives (k_prims.hip) ---------------------------------------------
void launch_sumsq_padded(const Geom& g, const double* X, double* partial, int nblocks,
                         hipStream_t st);
int sumsq_blocks(const Geom& g);
// triple product of device factors (layout of common.h) into / against a
// strided tensor X(i,j,t) = X[i + ldj*j + ldt*t] of the shard's n1l x n2 x n3:
// mode 0 writes L; mode 1 writes RRE partials partial[2*b] = sum (L-X)^2,
// [2*b+1] = sum X^2 (traffic_triple_comparison.m:62-63,194-199)
int tp_grid(const Geom& g);
void launch_tp(const Geom& g, const double* Ah, const double* Bh, const double* ChT, double* Lout,
               const double* X, double* partial, int mode, int64_t ldj, int64_t ldt,
               hipStream_t st, int64_t ahj = 0, int64_t bhj = -1);
// reference-layout device factors A (n1,r,r), B (r,n2,r), C (r,r,n3) -> Ah, Bh, ChT
void launch_pack_factors(const Geom& g, const double* A, const double* B, const double* C,
                         double* Ah, double* Bh, double* ChT, hipStream_t st);
void launch_transpose_batched(const double* in, double* out, int64_t rows, int64_t cols,
                              int64_t batch, hipStream_t st);
// layout conversions of the big tensors: column-major shard (leading dim ld,
// n1l x n2 x n3) <-> tile-major (common.h)
void launch_to_tm(const Geom& g, const double* src, int64_t ld, double* dst, hipStream_t st);
void launch_from_tm(const Geom& g, const double* src, double* dst, int64_t ld, hipStream_t st);
void launch_soft_threshold(const double* X, int64_t n, double lam, double* Y, hipStream_t st);
void launch_design(char which, const double* P, const double* Q, int64_t nP, int64_t nQ, int r,
                   double* out, hipStream_t st);

// ---- ALS variant (k_als.hip; triple_decomp_ALS.m) --------------------------
struct AlsFitArgs {
    const double* X;   // tile-major data tensor
    double* Wk;        // W = X x3 C^ (planes of n1p*n2)
    const double* Ah;
    const double* Bh;
    const double* Ch;
    double* partial;   // [grid][2]: sum (X - Xhat)^2, 0
    int64_t n1p, n2, n3p, plane, tiles, ntt;
    const int* stop;
    // nonconvex variant (fast_robust_triple_tensor/test.m:35-48; ncvx != 0):
    // Y = ((X - O) + rho*(L + Lam/rho))/onep; O' = shrink((X - Y) + Gam/rho, tau);
    // Lam += rho*(L - Y); Gam += rho*((X - Y) - O'); partial = sum ((X - Y) - O')^2.
    // O is double-buffered (O_in of iteration k-1, O_out of k), tile-major.
    int ncvx;
    const double* O_in;
    double *O_out, *Lam, *Gam;
    double rho, tau, onep;
};
int als_fit_grid(const Geom& g);
void launch_als_fit(const Geom& g, const AlsFitArgs& a, hipStream_t st);
void launch_als_finish(const double* ss, double Xnorm, int k, double tol, double* errHist,
                       int* ctrl, hipStream_t st);
void launch_tm_to_tx(const Geom& g, const double* src, double* dst, hipStream_t st);
// test.m:82-92: A1 <- sign(A1).*max(|A1| - gamma*(1./((|A1|+eps).^expo)), 0), into Ah and AhT
void launch_ncvx_shrink(const Geom& g, double* Ah, double* AhT, double gamma, double eps,
                        double expo, const int* stop, hipStream_t st);

// ---- driver-side metrics (k_metrics.hip) ------------------------------------
// evaluate (traffic_triple_comparison.m:194-202): out2 = {sum (X(mask)-gt)^2,
// sum gt^2}; mask may be null (X and gt paired elementwise, m == n); gt is
// read only below m (a mask with more true entries than m is reported by the
// caller through *total).  scratch_i64:
// evaluate_blocks(n) + 1 entries; part: 2*evaluate_blocks(n) doubles; *total
// receives nnz(mask) (untouched without a mask)
int64_t evaluate_blocks(int64_t n);
void launch_evaluate(const double* X, const double* gt, int64_t m, const uint8_t* mask, int64_t n,
                     int64_t* scratch_i64, double* part, double* out2, int64_t* total,
                     hipStream_t st);
// quality_ybz: per-frame psnr/ssim of n1 x n2 x nf tensors; win = the
// normalised 11x11 Gaussian (column-major, device); scratch: quality_scratch() doubles
size_t quality_scratch(int64_t n1, int64_t n2, int64_t nf);
void launch_quality(const double* X, const double* Y, int64_t n1, int64_t n2, int64_t nf,
                    const double* win, double C1, double C2, double* scratch, double* psnr,
                    double* ssim, hipStream_t st);

// ---------------------------------------------------------------------------
// fp32 data path (D of class single): T, O, E, Y_L, Y_O, W and
// the mode contractions in fp32; factors, Grams and solves in fp64.
// RP in {16, 32, 48, 64, 128, 256}.
// ---------------------------------------------------------------------------
struct IterScalars32 {
    float muL, muO, invL, invO, thr, den, invL_next;  // MATLAB: double scalar -> single
    float rden;  // 1/den in single (K5's division, k_admm32.hip)
};
struct K5Args32 {
    const float* D;
    float* O;
    float* E;   // dense E: only tiles whose compact slot overflowed
    float* CE;  // compact E: one 64-float slot per tile (k_admm32.hip)
    float* YL;
    float* YO;
    float* T;
    float* Wk;
    const double* Ah;
    const double* Bh;
    const float* ChF;  // C^ (n3p x RP) in single (the values are single-rounded already)
    double* partial;   // [grid][2] sums of resL^2, resO^2
    int64_t n1p, n2, n3p, plane, tiles, ntt;
    IterScalars32 s;
    const int* stop;
    unsigned long long* dense_tiles;
    int64_t slots;  // workgroups resident at once (2 per CU): the pair roles alternate per round
};
constexpr int CE32_SLOT = 64;  // floats per compact-E slot (50 values, their position bytes, the count)
bool rp_supported32(int RP);
int padded_rank32(int R);
void launch_k5_32(const Geom& g, const K5Args32& a, bool prologue, hipStream_t st);
void launch_to_tm32(const Geom& g, const float* src, int64_t ld, float* dst, hipStream_t st);
void launch_from_tm32(const Geom& g, const float* src, float* dst, int64_t ld, hipStream_t st);
void launch_sumsq32(const Geom& g, const float* X, double* partial, int nblocks, hipStream_t st);
void launch_o_fixup32(const Geom& g, const float* D, const float* YL, const float* T,
                      float invL_next, float* O, hipStream_t st);
void launch_ce_expand32(const Geom& g, const float* CE, float* E, hipStream_t st);
void launch_pool_probe32(const Geom& g, float* D, float* YL, float* YO, float* T, float* CE,
                         hipStream_t st);
void launch_widen(const float* x, int64_t n, double* y, hipStream_t st);
void launch_m1_32(const Geom& g, const float* Wk, const double* Bh, float* M1, const int* stop,
                  hipStream_t st);
void launch_m2_32(const Geom& g, const float* Wk, const double* AhT, double* M2, const int* stop,
                  hipStream_t st, const FinishArgs& fin = FinishArgs());
int m3_parts32(const Geom& g);
void launch_m3_32(const Geom& g, const float* T, const double* Ah, const double* Bh, double* part,
                  double* M3, const int* stop, hipStream_t st);
// Y = M * Ginv for any RP; M double or single (Mf); round32: results rounded to
// single (then stored as double; MATLAB's (X*F')*pinv(G) is single for single
// data); YT transposed copy, YF single copy (either may be null)
// (fix: the pinv fallback runs first, in k_pinv_fix: a one-workgroup launch
// that returns at once unless the request word is set; false when the caller
// launched it behind the solve already)
void launch_apply_gen(int RP, const double* M, const float* Mf, int64_t rows, double* Ginv,
                      double* Y, double* YT, int64_t ldT, float* YF, bool round32, const int* stop,
                      int* flags, hipStream_t st, bool fix = true);
// the pinv fallback alone (pinv.h): Ginv[0, RP^2) <- pinv(saved Gram) if requested
void launch_pinv_fix(int RP, double* Ginv, const int* stop, int* flags, hipStream_t st);

}  // namespace tritd
