// Device-resident ALS loop of fast_robust_triple_tensor/triple_decomp_ALS.m
// (SURVEY.md §8f rank 2): one mode-1 shard on one GPU, same factor layout
// and small kernels as the ADMM session (solver.h).
#pragma once

#include "solver.h"

namespace tritd {

// Parameters of the nonconvex solver of fast_robust_triple_tensor/test.m:1
// (positional in the reference: rho, lambda, gamma_A, epsilon, p, theta).
struct NcvxParams {
    double rho, lambda, gamma_A, epsilon, p, theta;
};

class AlsSession {
   public:
    // X: double, column-major shard rows [i0, i1) with leading dim ldX (host,
    // or device with TRITD_SESSION_D_ON_DEVICE).  maxIter, tol: the only
    // opts fields the reference reads (triple_decomp_ALS.m:2-3).
    AlsSession(int device, const double* X, int64_t ldX, int64_t n1, int64_t n2, int64_t n3,
               int64_t i0, int64_t i1, int r, int maxIter, double tol, const double* A0,
               const double* B0, const double* C0, tritd_comm* comm, uint32_t flags,
               hipStream_t shared_stream = nullptr, bool defer_norm = false);
    ~AlsSession();
    AlsSession(const AlsSession&) = delete;
    AlsSession& operator=(const AlsSession&) = delete;

    void run(int iters);
    void sync(int* done, int* stopped);
    // TRITD_FLAG_* raised by the device so far (read at every sync)
    uint32_t flags() const { return flags_; }
    void get(double* A, double* B, double* C, double* errHist, int* iters);
    // the progress line of :17-19 (every 5 iterations, unconditional in the
    // reference); quiet = no host synchronisation for it (benchmarks)
    void set_quiet(bool q) { quiet_ = q; }
    void set_timing(bool on);
    void kernel_ms(double* fit, double* m3, double* it, int* samples);
    // Switch this session to the nonconvex solver of test.m (before run):
    // same fit/M1/M2/K2 kernels over X, plus the O / Lambda / Gamma ADMM
    // chain fused into the fit kernel, ridge 1e-12 + reweighted shrink on A,
    // errHist/stop/print at the END of the iteration (test.m:62-68).
    void enable_ncvx(const NcvxParams& p);
    bool ncvx() const { return ncvx_; }
    // O returned by test.m: that of iteration k-1 when the stop test broke
    // the loop at k (:67 before :71), else the last one; column-major shard
    void get_O(double* O, int64_t ldO);

    // --- phase interface (device groups drive these; see api.cpp) -------
    int next_iter();
    void phaseFit(int k);  // fit kernel -> red0 (sum of squares)
    void phaseErr(int k);  // errHist(k), stop test
    void phaseA(int k);    // M1, solve A, apply A, A^TA partial, M2 partial -> red1
    void phaseB(int k);    // solve B, apply B, B^TB, M3 partial -> red2
    void phaseC(int k);    // solve C, apply C, C^TC
    void phaseEnd(int k);  // ncvx: errHist(k), stop test (after the updates, test.m:62-65)
    void maybe_print(int k);
    double* red0() { return red0_.p; }
    double* red1() { return red1_.p; }
    double* red2() { return red2_.p; }
    int64_t red1_count() const { return g_.n2 * g_.RP + (int64_t)g_.RP * g_.RP; }
    int64_t red2_count() const { return g_.n3p * g_.RP; }
    void set_norm_from_red0();
    hipStream_t stream() const { return st_; }
    int device() const { return device_; }
    const Geom& geom() const { return g_; }

   private:
    void allreduce(double* buf, int64_t count);
    int device_;
    hipStream_t st_ = nullptr;
    bool own_stream_ = false;
    Geom g_;
    int maxIter_;
    double tol_;
    tritd_comm* comm_;
    double Xnorm_ = 0.0;
    int k_enq_ = 0;
    bool quiet_ = false;
    DBuf X_, XT_, Wk_;  // X tile-major, X in TX order (K2), W = X x3 C^
    DBuf Ah_, AhT_, Bh_, Ch_, ChT_, M1_, GinvA_, GinvB_, GinvC_, BtB_, CtC_;
    DBuf red0_, red1_, red2_, fitpart_, m3part_, sqpart_, errHist_;
    uint32_t flags_ = 0;
    int* ctrl_ = nullptr;  // [0] stop, [1] errHist entries, [2] pinv-tolerance flag
    bool timing_ = false;
    std::vector<hipEvent_t> ev_;  // per timed iteration: 5 events
    double acc_fit_ = 0, acc_m3_ = 0, acc_it_ = 0;
    int acc_n_ = 0;
    void harvest_timing();
    bool ncvx_ = false;
    NcvxParams np_{};
    DBuf Oa_, Ob_, Lam_, Gam_;  // ncvx: O double buffer (iteration parity), duals (tile-major)
};

}  // namespace tritd
