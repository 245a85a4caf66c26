/*
 * tritd.h — C ABI of libtritd.so, the MI355X-native TriTD-ADMM solver.
 *
 * Drop-in boundary for the reference call surface
 *     [A,B,C,O,errHist] = triple_decomp_ADMM(D, r, opts)
 * (fast_robust_triple_tensor/triple_decomp_ADMM.m:1, called at
 *  traffic_triple_comparison.m:55 and — as triple_decomp_ADMM_outlier — at
 *  video_triple_comparison.m:54), plus the L1 primitives the drivers and the
 * north star name (triple_product.m:1, unfold.m:1, soft_threshold.m:1,
 * buildF.m:1, buildG.m:1, buildH.m:1).
 *
 * Conventions
 *  - Plain pointers and sizes only; no framework types.
 *  - All host arrays are MATLAB column-major: X(i,j,t) at i + n1*(j + n2*t).
 *  - Factors use the reference shapes: A (n1,r,r), B (r,n2,r), C (r,r,n3).
 *  - Functions named tritd_dev_* take DEVICE pointers and a hipStream_t
 *    (passed as void*, NULL = default stream) and do not synchronise, except
 *    the metric forms, which return host scalars (evaluate, quality).
 *  - Every function returns a tritd_status; on error the message is available
 *    from tritd_last_error() (thread-local).
 *  - Inputs are never written (MATLAB shares mxArrays copy-on-write).
 */
#ifndef TRITD_H
#define TRITD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    TRITD_OK = 0,
    TRITD_ERR_ARG = 1,         /* bad shape / pointer / mode (unfold.m:12 'Mode must be 1, 2, or 3.') */
    TRITD_ERR_OPTS = 2,        /* missing opts field (triple_decomp_ADMM.m:16-20) */
    TRITD_ERR_HIP = 3,         /* HIP runtime error */
    TRITD_ERR_RCCL = 4,        /* RCCL error */
    TRITD_ERR_NOMEM = 5,       /* device allocation failed */
    TRITD_ERR_NODEV = 6,       /* no usable gfx950 device */
    TRITD_ERR_UNSUPPORTED = 7, /* rank / dtype outside the built kernels */
    TRITD_ERR_STATE = 8        /* call order / session state */
} tritd_status;

/* opts struct of triple_decomp_ADMM.m:16-20.  `present` is a bitmask of the
 * TRITD_OPT_* fields the caller actually set; a missing required field is
 * reported exactly like MATLAB's "Reference to non-existent field 'x'."
 * Extra reference-driver fields (alphaA, alphaB, origin —
 * traffic_triple_comparison.m:48-51) are ignored by the reference and have
 * no slot here. */
enum {
    TRITD_OPT_MU = 1u << 0,
    TRITD_OPT_RHO = 1u << 1,
    TRITD_OPT_LAMBDA = 1u << 2,
    TRITD_OPT_LAMBDA2 = 1u << 3,
    TRITD_OPT_MAXITER = 1u << 4,
    TRITD_OPT_TOL = 1u << 5,
    TRITD_OPT_DISP = 1u << 6,
    TRITD_OPT_ALL = 0x7fu
};

typedef struct {
    double mu;        /* opts.mu      (muL = muO = mu, :16-17) */
    double rho;       /* opts.rho     (rhoL = rhoO = rho) */
    double lambda;    /* opts.lambda  (E soft-threshold weight, :47) */
    double lambda2;   /* opts.lambda2 (ridge of update_A/update_B, :34-35) */
    double tol;       /* opts.tol     (relative-change stop, :63) */
    int32_t maxIter;  /* opts.maxIter */
    int32_t disp;     /* opts.disp    (print every 10 iterations, :60-62) */
    uint32_t present; /* TRITD_OPT_* bitmask */
    uint32_t model;   /* opts.model (not read by the reference): TRITD_MODEL_CP (0, the executed
                         rank-r^2 CP builders, fast_robust_triple_tensor/buildF.m) or TRITD_MODEL_QI
                         (1, Qi's 3-index triple product of origin_triple_tensor/buildF.m:2-6,
                         buildG.m:7-11, buildH.m:7-11; fp64, r <= 8; ADMM only) */
} tritd_opts;

enum { TRITD_MODEL_CP = 0, TRITD_MODEL_QI = 1 };

/* Line printer used for opts.disp ("Iter %d, errL=%.2e, errO=%.2e").
 * Default: stdout.  MEX gateways install mexPrintf here. */
typedef void (*tritd_print_fn)(const char* line, void* user);

/* Warning flags (bitmask).  Not errors: the call succeeded and its outputs
 * are valid, but they may differ from the reference's beyond rounding.
 * TRITD_FLAG_PINV_TOL: MATLAB's pinv (triple_decomp_ADMM.m:78,86,93;
 * triple_decomp_ALS.m:27,32,37) truncated an R x R ridge Gram here: a solve's
 * smallest pivot came within 1e3x of pinv's tolerance max(size)*eps(max sigma),
 * the device formed pinv of that Gram (Jacobi eigensolver with MATLAB's
 * tolerance) and it dropped at least one singular value. */
enum { TRITD_FLAG_PINV_TOL = 1u };

const char* tritd_version(void);
const char* tritd_last_error(void);
/* TRITD_FLAG_* of the last one-shot solve on this thread (tritd_admm_*,
 * tritd_admm_sharded_virtual_f64, tritd_als_*, tritd_ncvx_f64; OR over the
 * shards of a device set); 0 after a call that raised none, and after any
 * failed libtritd call. */
uint32_t tritd_last_flags(void);
void tritd_set_print_callback(tritd_print_fn fn, void* user);
/* Number of visible gfx950 devices (0 on a host without a GPU). */
tritd_status tritd_device_count(int32_t* count);

/* ---------------------------------------------------------------------------
 * One-shot drop-in solver.
 * Replaces fast_robust_triple_tensor/triple_decomp_ADMM.m:1-70.
 *   D       : n1*n2*n3 doubles (host)
 *   A0,B0,C0: initial factors in reference layout (the MATLAB wrapper draws
 *             them with randn in the order of :23 so the RNG stream matches)
 *   A,B,C   : outputs, reference layout
 *   O, E    : outputs, n1*n2*n3 (E is the 6th, extra output; either may be NULL, which also
 *             skips its device-to-host transfer)
 *   errHist : capacity maxIter; *iters receives k (errHist = errHist(1:k), :68)
 * Runs on `device`; device = -1 runs on the device set of tritd_set_devices
 * (the current device when none is set).
 * ------------------------------------------------------------------------- */
tritd_status tritd_admm_f64(const double* D, int64_t n1, int64_t n2, int64_t n3, int32_t r,
                            const tritd_opts* opts, const double* A0, const double* B0,
                            const double* C0, double* A, double* B, double* C, double* O,
                            double* E, double* errHist, int32_t* iters, int32_t device);
/* The same for D of MATLAB class single: O, E and
 * every array derived from D are single; A, B, C, errHist double (holding
 * the single-rounded values MATLAB's class rules produce).  r <= 16.
 * MATLAB: the wrapper passes single(D) here, mxSINGLE_CLASS outputs. */
tritd_status tritd_admm_f32(const float* D, int64_t n1, int64_t n2, int64_t n3, int32_t r,
                            const tritd_opts* opts, const double* A0, const double* B0,
                            const double* C0, double* A, double* B, double* C, float* O, float* E,
                            double* errHist, int32_t* iters, int32_t device);

/* ---------------------------------------------------------------------------
 * Sessions: the device-resident ADMM loop, steppable (bench), shardable
 * along mode 1 (multi-GPU).  A session owns a shard i in [i0, i1) of the
 * global n1 x n2 x n3 problem (i0 = 0, i1 = n1 for one GPU).
 * ------------------------------------------------------------------------- */
typedef struct tritd_session tritd_session;
typedef struct tritd_comm tritd_comm;

enum {
    TRITD_SESSION_D_ON_DEVICE = 1, /* D is a device pointer on `device` */
    TRITD_SESSION_F32 = 2,         /* D is float (class single): the fp32 data path */
    TRITD_SESSION_PROBE = 4        /* choose where the tensor pool lives by timing the fused
                                      update's access pattern on up to 16 candidate allocations
                                      (~5-10 % on that kernel; pays off over hundreds of
                                      iterations, so the one-shot calls never do it) */
};

/* D points at D(i0,0,0) (double, or float with TRITD_SESSION_F32); consecutive (j,t) fibres are ldD elements apart
 * (ldD = n1 for a full column-major tensor).  A0 is the FULL (n1,r,r)
 * initial A (rows i0..i1-1 are used); B0, C0 are full.  comm = NULL for a
 * single process/GPU. */
tritd_status tritd_session_create(tritd_session** out, int32_t device, const void* D, int64_t ldD,
                                  int64_t n1, int64_t n2, int64_t n3, int64_t i0, int64_t i1,
                                  int32_t r, const tritd_opts* opts, const double* A0,
                                  const double* B0, const double* C0, tritd_comm* comm,
                                  uint32_t flags);
/* Enqueue `iters` ADMM iterations (no host synchronisation unless opts.disp).
 * Iterations after the stop test of :63 fires, or beyond maxIter, are no-ops. */
tritd_status tritd_session_run(tritd_session* s, int32_t iters);
/* Wait for the enqueued work; report iterations completed and the stop flag. */
tritd_status tritd_session_sync(tritd_session* s, int32_t* iters_done, int32_t* stopped);
/* Copy results to the host.  A: full (n1,r,r) buffer, only rows i0..i1-1 are
 * written; B, C full; O, E: the shard, leading dimension ldOE (>= i1-i0);
 * errHist capacity maxIter.  Any pointer may be NULL. */
tritd_status tritd_session_get(tritd_session* s, double* A, double* B, double* C, double* O,
                               double* E, int64_t ldOE, double* errHist, int32_t* iters);
/* Driver RRE (traffic_triple_comparison.m:62-63,194-199) of the current
 * factors against a device-resident reference tensor X (same shard/ld as D):
 *   sum over the shard of (triple_product(A,B,C) - X)^2 and of X^2.
 * (Combine across ranks, then RRE = sqrt(num/den).) */
tritd_status tritd_session_rre_parts(tritd_session* s, const double* dX, int64_t ldX, double* num,
                                     double* den);
/* fp32 sessions (TRITD_SESSION_F32): O, E and the reference tensor are float. */
tritd_status tritd_session_get_f32(tritd_session* s, double* A, double* B, double* C, float* O,
                                   float* E, int64_t ldOE, double* errHist, int32_t* iters);
tritd_status tritd_session_rre_parts_f32(tritd_session* s, const float* dX, int64_t ldX,
                                         double* num, double* den);
/* Kernel-level timing of the dominant kernels over the last run (ms per
 * launch, HIP events on the session stream; 0 when timing is disabled). */
/* enable: 0 off; TRITD_TIMING_ALL (1): per-iteration events around the
 * iteration, K2 and K5; TRITD_TIMING_K5 (2): around K5 only (each event
 * record is a stream marker that widens the next kernel boundary by µs) */
enum { TRITD_TIMING_ALL = 1, TRITD_TIMING_K5 = 2 };
tritd_status tritd_session_set_timing(tritd_session* s, int32_t enable);
tritd_status tritd_session_kernel_ms(tritd_session* s, double* fused_update_ms, double* mode3_ms,
                                     double* iteration_ms, int32_t* samples);
/* All-reduce time of the timed iterations (TRITD_TIMING_ALL, a session with
 * a communicator): the mean ms per iteration spent between
 * issuing the iteration's all-reduces and their completion on the session
 * stream (waiting for the slowest rank included), and how many all-reduces
 * an iteration issued (0 without a communicator).  Per-rank breakdown of
 * bench.py's N > 1 line: iteration ms - all-reduce ms = compute. */
tritd_status tritd_session_comm_ms(tritd_session* s, double* allreduce_ms, int32_t* per_iteration);
/* Placement probe of the session's tensor pool: the probe
 * time (ms) of each candidate pool that was tried (up to cap entries) and
 * the index kept.  *n = 1 when probing was skipped. */
tritd_status tritd_session_probe(tritd_session* s, double* ms, int32_t cap, int32_t* n,
                                 int32_t* picked);
/* Compact-E counters: E tiles stored densely (more than 28
 * nonzeros of 256) summed over all fused-update launches so far, and the
 * number of tiles one launch covers. */
tritd_status tritd_session_counters(tritd_session* s, int64_t* dense_tiles_total,
                                    int64_t* tiles_per_launch);
/* Streaming profile of the session's fused update: dense
 * N-element streams per launch (6 = D, Y_L, Y_O read + Y_L, Y_O, T written;
 * 4 with the derived Y_O of the fp64 path) and compact-E slot accesses per
 * tile (2 = E read + written; 3 = E^(k), E^(k-1) read + E^(k+1) written). */
tritd_status tritd_session_k5_profile(tritd_session* s, int32_t* dense_streams,
                                      int32_t* slot_accesses);
/* TRITD_FLAG_* raised by this session's solves so far (read at each sync). */
tritd_status tritd_session_flags(tritd_session* s, uint32_t* flags);
void tritd_session_destroy(tritd_session* s);

/* ---------------------------------------------------------------------------
 * Multi-GPU: one process per GPU, RCCL over xGMI.  Rank 0 creates the id,
 * the host side broadcasts its 128 bytes (e.g. torch.distributed), every
 * rank calls tritd_comm_create.
 * ------------------------------------------------------------------------- */
tritd_status tritd_comm_unique_id(void* id128);
tritd_status tritd_comm_create(tritd_comm** out, const void* id128, int32_t nranks, int32_t rank,
                               int32_t device);
/* Host transport: every all-reduce of a session using this comm drains the
 * session's stream, copies the buffer to the host and calls fn(buf, count, op,
 * user) (op 0 = sum, 1 = max; return 0 on success), then copies it back.  For
 * hosts that own a collective layer already (MPI, gloo) and for running the
 * multi-rank schedule with several ranks on one GPU (RCCL refuses a GPU twice
 * in one communicator).  tritd_comm_create (RCCL, device-side, asynchronous)
 * is the fast path. */
typedef int32_t (*tritd_allreduce_fn)(double* buf, int64_t count, int32_t op, void* user);
tritd_status tritd_comm_create_host(tritd_comm** out, tritd_allreduce_fn fn, void* user,
                                    int32_t nranks, int32_t rank, int32_t device);
void tritd_comm_destroy(tritd_comm* c);
/* What the communicator itself reports: for RCCL, ncclCommCount /
 * ncclCommUserRank read back from the communicator (so a caller can prove
 * RCCL saw every rank); for the host transport, the values it was created
 * with.  transport: 0 = RCCL, 1 = host. */
tritd_status tritd_comm_info(tritd_comm* c, int32_t* nranks, int32_t* rank, int32_t* transport);

/* Device set of the one-shot entry points (the MEX host
 * calls from its one thread).  With n > 1, tritd_admm_{f64,f32} (device =
 * -1) shard D along mode 1 over the set: the library runs one
 * session per shard with a communicator, each stepped by a library-owned
 * host thread (shard 0 on the calling thread, so disp prints stay there)
 * through the same fused two-all-reduce schedule as one process per GPU.
 * Distinct devices all-reduce over RCCL (communicators from ncclCommInitAll,
 * cached until the set changes or tritd_shutdown); one device repeated n
 * times runs n shards on it with an in-process all-reduce.  TRITD_SHOV=0
 * selects the phase-serial order driven from the calling thread instead.
 * n = 0 clears the set.  Replaces the reference's single-process CPU call
 * (triple_decomp_ADMM.m:1) for data that exceeds one GPU. */
tritd_status tritd_set_devices(const int32_t* devices, int32_t n);
/* Frees the cached communicators and clears the device set (mexAtExit). */
void tritd_shutdown(void);

/* Single-GPU rehearsal of the sharded path: `nshards` sessions on one device
 * whose all-reduces are summed on the device in shard order (the device set
 * {device} x nshards).  Used by the parity tests on a 1-GPU box. */
tritd_status tritd_admm_sharded_virtual_f64(const double* D, int64_t n1, int64_t n2, int64_t n3,
                                            int32_t r, const tritd_opts* opts, const double* A0,
                                            const double* B0, const double* C0, int32_t nshards,
                                            double* A, double* B, double* C, double* O, double* E,
                                            double* errHist, int32_t* iters, int32_t device);

/* ---------------------------------------------------------------------------
 * ALS variant: [A,B,C,errHist] = triple_decomp_ALS(X, r, opts)
 * (fast_robust_triple_tensor/triple_decomp_ALS.m:1-40).
 * Only opts.maxIter and opts.tol are read (:2-3): TRITD_OPT_MAXITER and
 * TRITD_OPT_TOL must be present, a missing one fails like MATLAB.  errHist(k)
 * = ||X - triple_product(A,B,C)||/||X|| is taken before the update of
 * iteration k; the stop test (:20) returns the factors of that iteration
 * un-updated, errHist = errHist(1:k).  Every mode uses the ridge 1e-9.  The
 * progress line "Iteration %d, relative error = %.4e" goes to the print
 * callback every 5 iterations (:17-19).  fp64, r <= 8.  device = -1 runs on
 * the device set of tritd_set_devices (mode-1 shards).
 * ------------------------------------------------------------------------- */
tritd_status tritd_als_f64(const double* X, int64_t n1, int64_t n2, int64_t n3, int32_t r,
                           const tritd_opts* opts, const double* A0, const double* B0,
                           const double* C0, double* A, double* B, double* C, double* errHist,
                           int32_t* iters, int32_t device);
/* Steppable ALS session (bench, one process per GPU with comm; shard rows
 * [i0, i1) as for tritd_session_create; flags: TRITD_SESSION_D_ON_DEVICE).
 * quiet = 1 skips the every-5-iterations progress line (and its host
 * synchronisation). */
/* Nonconvex variant, fast_robust_triple_tensor/test.m:1-73 (the file's function
 * is named triple_decomp_ADMM_outlier(X, r, rho, lambda, gamma_A, epsilon, p, theta,
 * maxIter, tol)).  Outlier ADMM over Y = X - O with duals
 * Lambda, Gamma, while A, B, C follow an ALS on X (ridge 1e-12 + reweighted
 * shrink on A, 1e-9 on B, C).  errHist(k) = ||X - Y - O||/||X|| after the updates,
 * printed every iteration ("Iteration %d, relative error = %.4e"); on the stop
 * test errHist holds *iters entries and O is that of iteration *iters - 1
 * (the reference breaks before O = O_new).  X, O column-major n1 x n2 x n3;
 * factors as tritd_admm_f64; errHist capacity maxIter; fp64, r <= 8.
 * device < 0: the device set (tritd_set_devices) or the current device. */
tritd_status tritd_ncvx_f64(const double* X, int64_t n1, int64_t n2, int64_t n3, int32_t r,
                           double rho, double lambda, double gamma_A, double epsilon, double p,
                           double theta, int32_t maxIter, double tol, const double* A0,
                           const double* B0, const double* C0, double* A, double* B, double* C,
                           double* O, double* errHist, int32_t* iters, int32_t device);

typedef struct tritd_als_session tritd_als_session;
tritd_status tritd_als_session_create(tritd_als_session** out, int32_t device, const double* X,
                                      int64_t ldX, int64_t n1, int64_t n2, int64_t n3, int64_t i0,
                                      int64_t i1, int32_t r, const tritd_opts* opts,
                                      const double* A0, const double* B0, const double* C0,
                                      tritd_comm* comm, uint32_t flags, int32_t quiet);
tritd_status tritd_als_session_run(tritd_als_session* s, int32_t iters);
tritd_status tritd_als_session_sync(tritd_als_session* s, int32_t* iters_done, int32_t* stopped);
tritd_status tritd_als_session_get(tritd_als_session* s, double* A, double* B, double* C,
                                   double* errHist, int32_t* iters);
/* timing: fit kernel (fused triple product + error + W) and mode-3 MTTKRP ms per launch */
tritd_status tritd_als_session_set_timing(tritd_als_session* s, int32_t enable);
tritd_status tritd_als_session_kernel_ms(tritd_als_session* s, double* fit_ms, double* mode3_ms,
                                         double* iteration_ms, int32_t* samples);
tritd_status tritd_als_session_flags(tritd_als_session* s, uint32_t* flags);
void tritd_als_session_destroy(tritd_als_session* s);
/* Single-GPU rehearsal of the sharded ALS (virtual shards, as above). */
tritd_status tritd_als_sharded_virtual_f64(const double* X, int64_t n1, int64_t n2, int64_t n3,
                                           int32_t r, const tritd_opts* opts, const double* A0,
                                           const double* B0, const double* C0, int32_t nshards,
                                           double* A, double* B, double* C, double* errHist,
                                           int32_t* iters, int32_t device);

/* ---------------------------------------------------------------------------
 * Primitives (host pointers).  Each replaces the named reference file.
 * ------------------------------------------------------------------------- */
/* Qi-model triple product X(i,j,t) = sum_{p,q,s} A(i,q,s) B(p,j,s) C(p,q,t)
 * (origin_triple_tensor/triple_product.m:8-19 as intended; equals
 * reshape(unfold(A,1)*buildF(B,C)) with origin_triple_tensor/buildF.m:2-6).
 * Host and device (stream) forms; r <= 16. */
tritd_status tritd_triple_product_qi_f64(const double* A, const double* B, const double* C,
                                         int64_t n1, int64_t n2, int64_t n3, int32_t r, double* X);
tritd_status tritd_dev_triple_product_qi_f64(const double* A, const double* B, const double* C,
                                             int64_t n1, int64_t n2, int64_t n3, int32_t r,
                                             double* X, void* stream);
/* triple_product.m:1-7: X = reshape(unfold(A,1)*buildF(B,C), n1,n2,n3). */
tritd_status tritd_triple_product_f64(const double* A, const double* B, const double* C, int64_t n1,
                                      int64_t n2, int64_t n3, int32_t r, double* X);
/* unfold.m:1-13: mode 1 reshape, mode 2 permute [2 1 3], mode 3 permute [3 1 2]. */
tritd_status tritd_unfold_f64(const double* X, int64_t n1, int64_t n2, int64_t n3, int32_t mode,
                              double* Xn);
/* soft_threshold.m:1-2: sign(X).*max(abs(X)-lam,0), n elements. */
tritd_status tritd_soft_threshold_f64(const double* X, int64_t n, double lam, double* Y);
/* buildF.m / buildG.m / buildH.m.  which = 'F' (P=B (r,n2,r), Q=C (r,r,n3)),
 * 'G' (P=A (n1,r,r), Q=C), 'H' (P=A, Q=B (r,n2,r)).  out: r^2 x (nP*nQ). */
tritd_status tritd_build_design_f64(char which, const double* P, const double* Q, int64_t nP,
                                    int64_t nQ, int32_t r, double* out);

/* Driver metrics.
 * evaluate(X, gt, mask) of traffic_triple_comparison.m:194-202 (identical in
 * video_triple_comparison.m): rmse = norm(X(mask) - gt(:)), nrmse = rmse /
 * norm(gt(:)).  X has n elements; mask is n bytes (MATLAB logical, nonzero =
 * true) or NULL for true(size(X)); gt holds m = nnz(mask) elements in
 * column-major order of the true positions (m = n without a mask) — a
 * mismatch fails like MATLAB's "Arrays have incompatible sizes" (gt is never
 * read past m).  The device variant takes a mask at any byte alignment.  */
tritd_status tritd_evaluate_f64(const double* X, int64_t n, const double* gt, int64_t m,
                                const uint8_t* mask, double* rmse, double* nrmse);
/* quality_ybz(imagery1, imagery2) (other_methods/Low-rank-.../quality_ybz.m:1-33):
 * mean over the nf frames (n1 x n2 each; trailing dims folded into nf) of
 * psnr_index = 10*log10(255^2/mse(x-y)) and ssim_index (Gaussian 11x11
 * window, sigma 1.5, K = [0.01 0.03], L = 255, 'valid' map; -Inf for frames
 * smaller than 11x11).  psnr_frames / ssim_frames (nf each) may be NULL.
 * Any nf (launched in batches of 65535 frames). */
tritd_status tritd_quality_f64(const double* X1, const double* X2, int64_t n1, int64_t n2,
                               int64_t nf, double* psnr, double* ssim, double* psnr_frames,
                               double* ssim_frames);
tritd_status tritd_dev_evaluate_f64(const double* X, int64_t n, const double* gt, int64_t m,
                                    const uint8_t* mask, double* rmse, double* nrmse, void* stream);
tritd_status tritd_dev_quality_f64(const double* X1, const double* X2, int64_t n1, int64_t n2,
                                   int64_t nf, double* psnr, double* ssim, double* psnr_frames,
                                   double* ssim_frames, void* stream);

/* Device-pointer variants (for device-resident callers and the bench). */
tritd_status tritd_dev_unfold_f64(const double* X, int64_t n1, int64_t n2, int64_t n3, int32_t mode,
                                  double* Xn, void* stream);
tritd_status tritd_dev_soft_threshold_f64(const double* X, int64_t n, double lam, double* Y,
                                          void* stream);
tritd_status tritd_dev_triple_product_f64(const double* A, const double* B, const double* C,
                                          int64_t n1, int64_t n2, int64_t n3, int32_t r, double* X,
                                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* TRITD_H */
