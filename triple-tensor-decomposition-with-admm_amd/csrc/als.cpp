// Device-resident ALS loop of fast_robust_triple_tensor/triple_decomp_ALS.m:1-40.
//
// Iteration k (reference order):
//   fit    Xhat = triple_product(A,B,C), errHist(k) = ||X - Xhat||/Xnorm   :15-16
//          + W = X x3 C^ for the next two updates (k_als.hip)
//   print  every 5 iterations                                               :17-19
//   stop   k > 1 && |e_k - e_{k-1}| < tol e_{k-1}: truncate, return         :20-23
//          (device flag: the update kernels of k early-exit)
//   A      M1 = X1 F' from W, solve (B^TB o C^TC + 1e-9 I), apply          :25-28
//   B      M2 = X2 G' from W and the new A, solve (A^TA o C^TC + 1e-9 I)    :30-33
//   C      M3 = X3 H' (K2 over the TX copy of X), solve (A^TA o B^TB + 1e-9 I) :35-38
// Sharded along mode 1 like the ADMM: the fit sum, [M2 | A^TA]
// and M3 are the three reductions.
#include "als.h"

#include <cmath>
#include <cstdlib>

namespace tritd {

void emit_line(const char* line);  // api.cpp

AlsSession::AlsSession(int device, const double* X, int64_t ldX, int64_t n1, int64_t n2,
                       int64_t n3, int64_t i0, int64_t i1, int r, int maxIter, double tol,
                       const double* A0, const double* B0, const double* C0, tritd_comm* comm,
                       uint32_t flags, hipStream_t shared_stream, bool defer_norm)
    : device_(device), maxIter_(maxIter < 0 ? 0 : maxIter), tol_(tol), comm_(comm) {
    TRITD_HIP(hipSetDevice(device_));
    g_ = make_geom(n1, n2, n3, i0, i1, r);
    if (!rp_supported(g_.RP))
        throw Error(TRITD_ERR_UNSUPPORTED, "r must be in 1..8 for the fp64 ALS path");
    if (shared_stream) {
        st_ = shared_stream;
    } else {
        own_stream_ = true;
        TRITD_HIP(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    }
    const size_t Np = (size_t)g_.Ntm;
    X_.alloc(Np);
    XT_.alloc(Np);
    TRITD_HIP(hipMemsetAsync(X_.p, 0, Np * sizeof(double), st_));
    Wk_.alloc((size_t)g_.RP * g_.plane);
    TRITD_HIP(hipMemsetAsync(Wk_.p, 0, Wk_.bytes(), st_));
    Ah_.alloc(g_.n1p * g_.RP);
    AhT_.alloc((size_t)g_.RP * g_.n1p);
    Bh_.alloc(g_.n2 * g_.RP);
    Ch_.alloc(g_.n3p * g_.RP);
    ChT_.alloc((size_t)g_.RP * g_.n3p);
    M1_.alloc(g_.n1p * g_.RP);
    // one inverse per Gram slot, kept across iterations (k_solve_ns refines
    // the previous one); zero = no start
    for (DBuf* b : {&GinvA_, &GinvB_, &GinvC_}) {
        b->alloc(ginv_count(g_.RP));  // inverse + pinv fallback space (pinv.h)
        TRITD_HIP(hipMemsetAsync(b->p, 0, b->bytes(), st_));
    }
    BtB_.alloc((size_t)g_.RP * g_.RP);
    CtC_.alloc((size_t)g_.RP * g_.RP);
    red0_.alloc(2);
    red1_.alloc(red1_count());
    red2_.alloc(red2_count());
    fitpart_.alloc(2 * (size_t)als_fit_grid(g_));
    m3part_.alloc((size_t)m3_parts(g_) * g_.n3p * g_.RP);
    sqpart_.alloc(2 * (size_t)sumsq_blocks(g_));
    errHist_.alloc(maxIter_ > 0 ? (size_t)maxIter_ : 1);
    for (DBuf* b : {&errHist_, &red0_, &red1_, &red2_})
        TRITD_HIP(hipMemsetAsync(b->p, 0, b->n * sizeof(double), st_));
    TRITD_HIP(hipMalloc(&ctrl_, 4 * sizeof(int)));
    TRITD_HIP(hipMemsetAsync(ctrl_, 0, 4 * sizeof(int), st_));

    // X -> tile-major, and its TX copy for the mode-3 contraction (one-off)
    if (g_.n1l > 0) {
        if (flags & TRITD_SESSION_D_ON_DEVICE) {
            launch_to_tm(g_, X, ldX, X_.p, st_);
        } else {
            DBuf tmp;
            tmp.alloc((size_t)(g_.n1l * n2 * n3));
            if (ldX == g_.n1l)  // contiguous: one 1-D copy (the 2-D form is slower from pageable memory)
                TRITD_HIP(hipMemcpyAsync(tmp.p, X, (size_t)(g_.n1l * n2 * n3) * sizeof(double),
                                         hipMemcpyHostToDevice, st_));
            else
                TRITD_HIP(hipMemcpy2DAsync(tmp.p, g_.n1l * sizeof(double), X, ldX * sizeof(double),
                                           g_.n1l * sizeof(double), (size_t)(n2 * n3),
                                           hipMemcpyHostToDevice, st_));
            launch_to_tm(g_, tmp.p, g_.n1l, X_.p, st_);
            TRITD_HIP(hipStreamSynchronize(st_));
        }
    }
    launch_tm_to_tx(g_, X_.p, XT_.p, st_);

    std::vector<double> Ah, AhT, Bh, Ch, ChT;
    pack_A(g_, A0, Ah, AhT);
    pack_B(g_, B0, Bh);
    pack_C(g_, C0, Ch, ChT);
    TRITD_HIP(hipMemcpy(Ah_.p, Ah.data(), Ah.size() * sizeof(double), hipMemcpyHostToDevice));
    TRITD_HIP(hipMemcpy(AhT_.p, AhT.data(), AhT.size() * sizeof(double), hipMemcpyHostToDevice));
    TRITD_HIP(hipMemcpy(Bh_.p, Bh.data(), Bh.size() * sizeof(double), hipMemcpyHostToDevice));
    TRITD_HIP(hipMemcpy(Ch_.p, Ch.data(), Ch.size() * sizeof(double), hipMemcpyHostToDevice));
    TRITD_HIP(hipMemcpy(ChT_.p, ChT.data(), ChT.size() * sizeof(double), hipMemcpyHostToDevice));

    // Xnorm = norm(X(:))  (:6)
    const int nb = sumsq_blocks(g_);
    launch_sumsq_padded(g_, X_.p, sqpart_.p, nb, st_);
    launch_reduce_pairs(sqpart_.p, nb, red0_.p, nullptr, st_);
    if (!defer_norm) {
        allreduce(red0_.p, 2);
        set_norm_from_red0();
    }
    // Grams of the initial B, C (replicated)
    launch_gram(g_.RP, Bh_.p, g_.n2, BtB_.p, ctrl_, st_);
    launch_gram(g_.RP, Ch_.p, g_.n3p, CtC_.p, ctrl_, st_);
    TRITD_HIP(hipStreamSynchronize(st_));
}

AlsSession::~AlsSession() {
    hip_quiet(hipSetDevice(device_));
    if (st_) hip_quiet(hipStreamSynchronize(st_));
    for (auto e : ev_) hip_quiet(hipEventDestroy(e));
    if (ctrl_) hip_quiet(hipFree(ctrl_));
    if (own_stream_ && st_) hip_quiet(hipStreamDestroy(st_));
}

void AlsSession::set_norm_from_red0() {
    double ss[2];
    TRITD_HIP(hipMemcpyAsync(ss, red0_.p, 2 * sizeof(double), hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipStreamSynchronize(st_));
    Xnorm_ = std::sqrt(ss[0]);
}

void AlsSession::allreduce(double* buf, int64_t count) {
    if (!comm_ || !comm_->active()) return;
    comm_allreduce(comm_, buf, count, false, st_);
}

int AlsSession::next_iter() {
    if (k_enq_ >= maxIter_) return 0;
    return ++k_enq_;
}

void AlsSession::enable_ncvx(const NcvxParams& p) {
    TRITD_HIP(hipSetDevice(device_));
    ncvx_ = true;
    np_ = p;
    const size_t Np = (size_t)g_.Ntm;
    for (DBuf* b : {&Oa_, &Ob_, &Lam_, &Gam_}) {
        b->alloc(Np);
        TRITD_HIP(hipMemsetAsync(b->p, 0, Np * sizeof(double), st_));
    }
}

void AlsSession::phaseFit(int k) {
    AlsFitArgs a{};
    a.X = X_.p; a.Wk = Wk_.p; a.Ah = Ah_.p; a.Bh = Bh_.p; a.Ch = Ch_.p;
    a.partial = fitpart_.p;
    a.n1p = g_.n1p; a.n2 = g_.n2; a.n3p = g_.n3p; a.plane = g_.plane; a.tiles = g_.tiles;
    a.ntt = g_.ntt;
    a.stop = ctrl_;
    if (ncvx_) {  // test.m:35-48; O of iteration k-1 in buffer (k-1)&1, O of k into k&1
        a.ncvx = 1;
        a.O_in = ((k - 1) & 1) ? Ob_.p : Oa_.p;
        a.O_out = (k & 1) ? Ob_.p : Oa_.p;
        a.Lam = Lam_.p;
        a.Gam = Gam_.p;
        a.rho = np_.rho;
        a.tau = np_.lambda / np_.rho;  // lambda/rho (:44); tau.*W_O = tau (W_O = ones, :43)
        a.onep = 1.0 + np_.rho;        // (1 + rho) (:36)
    }
    if (timing_) TRITD_HIP(hipEventRecord(ev_[ev_.size() - 5], st_));
    launch_als_fit(g_, a, st_);
    if (timing_) TRITD_HIP(hipEventRecord(ev_[ev_.size() - 4], st_));
    launch_reduce_pairs(fitpart_.p, als_fit_grid(g_), red0_.p, ctrl_, st_);
}

void AlsSession::phaseErr(int k) {
    if (ncvx_) return;  // test.m takes errHist after the updates: phaseEnd
    launch_als_finish(red0_.p, Xnorm_, k, tol_, errHist_.p, ctrl_, st_);
}

void AlsSession::phaseEnd(int k) {
    if (!ncvx_) return;
    // errHist(k) = norm(X(:) - Y_new(:) - O_new(:))/Xnorm (:62); the stop flag
    // set here makes every kernel of k+1 exit (:65-67)
    launch_als_finish(red0_.p, Xnorm_, k, tol_, errHist_.p, ctrl_, st_);
}

void AlsSession::phaseA(int k) {
    (void)k;
    const int RP = g_.RP;
    double* M2 = red1_.p;
    double* AtA = red1_.p + g_.n2 * RP;
    launch_m1(g_, Wk_.p, Bh_.p, M1_.p, ctrl_, st_);
    // ALS :27 ridge 1e-9; test.m:82 ridge 1e-12, then the reweighted shrink :86-89
    launch_solve(RP, g_.R, BtB_.p, CtC_.p, ncvx_ ? 1e-12 : 1e-9, GinvA_.p, ctrl_ + 2, ctrl_, st_);
    launch_apply(RP, M1_.p, g_.n1p, GinvA_.p, Ah_.p, AhT_.p, g_.n1p, ctrl_, ctrl_ + 2, st_);
    if (ncvx_)
        launch_ncvx_shrink(g_, Ah_.p, AhT_.p, np_.gamma_A, np_.epsilon, np_.theta - np_.p, ctrl_,
                           st_);
    launch_gram(RP, Ah_.p, g_.n1p, AtA, ctrl_, st_);
    launch_m2(g_, Wk_.p, AhT_.p, M2, ctrl_, st_);
}

void AlsSession::phaseB(int k) {
    (void)k;
    const int RP = g_.RP;
    const double* M2 = red1_.p;
    const double* AtA = red1_.p + g_.n2 * RP;
    launch_solve(RP, g_.R, AtA, CtC_.p, 1e-9, GinvB_.p, ctrl_ + 2, ctrl_, st_);  // :32
    launch_apply(RP, M2, g_.n2, GinvB_.p, Bh_.p, nullptr, 0, ctrl_, ctrl_ + 2, st_);
    launch_gram(RP, Bh_.p, g_.n2, BtB_.p, ctrl_, st_);
    if (timing_) TRITD_HIP(hipEventRecord(ev_[ev_.size() - 3], st_));
    launch_m3(g_, XT_.p, Ah_.p, Bh_.p, m3part_.p, red2_.p, ctrl_, st_);
    if (timing_) TRITD_HIP(hipEventRecord(ev_[ev_.size() - 2], st_));
}

void AlsSession::phaseC(int k) {
    (void)k;
    const int RP = g_.RP;
    const double* AtA = red1_.p + g_.n2 * RP;
    launch_solve(RP, g_.R, AtA, BtB_.p, 1e-9, GinvC_.p, ctrl_ + 2, ctrl_, st_);  // :37
    launch_apply(RP, red2_.p, g_.n3p, GinvC_.p, Ch_.p, ChT_.p, g_.n3p, ctrl_, ctrl_ + 2, st_);
    launch_gram(RP, Ch_.p, g_.n3p, CtC_.p, ctrl_, st_);
}

void AlsSession::maybe_print(int k) {
    if (quiet_ || (!ncvx_ && k % 5 != 0)) return;  // ALS :17; test.m:63 prints every iteration
    if (comm_ && comm_->rank != 0) return;
    int ctrl[2];
    double e;
    TRITD_HIP(hipMemcpyAsync(ctrl, ctrl_, 2 * sizeof(int), hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipMemcpyAsync(&e, errHist_.p + (k - 1), sizeof(double), hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipStreamSynchronize(st_));
    if (ctrl[1] != k) return;  // the loop broke before iteration k
    char line[128];
    std::snprintf(line, sizeof line, "Iteration %d, relative error = %.4e", k, e);  // :18 (test.m:63)
    emit_line(line);
}

void AlsSession::run(int iters) {
    TRITD_HIP(hipSetDevice(device_));
    for (int it = 0; it < iters; ++it) {
        const int k = next_iter();
        if (!k) break;
        if (timing_) {
            for (int e = 0; e < 5; ++e) {
                hipEvent_t ev;
                TRITD_HIP(hipEventCreate(&ev));
                ev_.push_back(ev);
            }
        }
        phaseFit(k);
        allreduce(red0_.p, 2);
        phaseErr(k);
        if (!ncvx_) maybe_print(k);
        phaseA(k);
        allreduce(red1_.p, red1_count());
        phaseB(k);
        allreduce(red2_.p, red2_count());
        phaseC(k);
        phaseEnd(k);
        if (ncvx_) maybe_print(k);
        if (timing_) TRITD_HIP(hipEventRecord(ev_[ev_.size() - 1], st_));
    }
}

void AlsSession::harvest_timing() {
    // events per iteration: [0] fit start, [1] fit end, [2] M3 start, [3] M3 end, [4] end
    for (size_t b = 0; b + 5 <= ev_.size(); b += 5) {
        float it = 0, m3 = 0, fit = 0;
        TRITD_HIP(hipEventElapsedTime(&it, ev_[b], ev_[b + 4]));
        TRITD_HIP(hipEventElapsedTime(&fit, ev_[b], ev_[b + 1]));
        TRITD_HIP(hipEventElapsedTime(&m3, ev_[b + 2], ev_[b + 3]));
        acc_it_ += it;
        acc_fit_ += fit;
        acc_m3_ += m3;
        ++acc_n_;
    }
    for (auto e : ev_) hip_quiet(hipEventDestroy(e));
    ev_.clear();
}

void AlsSession::set_timing(bool on) {
    timing_ = on;
    acc_fit_ = acc_m3_ = acc_it_ = 0;
    acc_n_ = 0;
}

void AlsSession::kernel_ms(double* fit, double* m3, double* it, int* samples) {
    const double n = acc_n_ ? (double)acc_n_ : 1.0;
    if (fit) *fit = acc_fit_ / n;
    if (m3) *m3 = acc_m3_ / n;
    if (it) *it = acc_it_ / n;
    if (samples) *samples = acc_n_;
}

void AlsSession::sync(int* done, int* stopped) {
    TRITD_HIP(hipSetDevice(device_));
    TRITD_HIP(hipStreamSynchronize(st_));
    if (!ev_.empty()) harvest_timing();
    int ctrl[3];
    TRITD_HIP(hipMemcpy(ctrl, ctrl_, 3 * sizeof(int), hipMemcpyDeviceToHost));
    if (ctrl[2] & 1) flags_ |= TRITD_FLAG_PINV_TOL;  // the pinv fallback dropped a value
    if (done) *done = ctrl[1];
    if (stopped) *stopped = ctrl[0];
}

void AlsSession::get(double* A, double* B, double* C, double* errHist, int* iters) {
    int done = 0, stopped = 0;
    sync(&done, &stopped);
    if (A) {
        std::vector<double> h(Ah_.n);
        TRITD_HIP(hipMemcpy(h.data(), Ah_.p, h.size() * sizeof(double), hipMemcpyDeviceToHost));
        unpack_A(g_, h, A);
    }
    if (B) {
        std::vector<double> h(Bh_.n);
        TRITD_HIP(hipMemcpy(h.data(), Bh_.p, h.size() * sizeof(double), hipMemcpyDeviceToHost));
        unpack_B(g_, h, B);
    }
    if (C) {
        std::vector<double> h(Ch_.n);
        TRITD_HIP(hipMemcpy(h.data(), Ch_.p, h.size() * sizeof(double), hipMemcpyDeviceToHost));
        unpack_C(g_, h, C);
    }
    if (errHist && done > 0)
        TRITD_HIP(hipMemcpy(errHist, errHist_.p, (size_t)done * sizeof(double),
                            hipMemcpyDeviceToHost));
    if (iters) *iters = done;
}

void AlsSession::get_O(double* O, int64_t ldO) {
    int done = 0, stopped = 0;
    sync(&done, &stopped);
    if (!ncvx_) throw Error(TRITD_ERR_STATE, "get_O: not a nonconvex (test.m) session");
    // :67 breaks before O = O_new (:71): a stop at k returns O of k-1
    const int kk = stopped ? done - 1 : done;
    const double* src = (kk & 1) ? Ob_.p : Oa_.p;  // kk = 0: the zero initial O
    if (g_.n1l > 0) {
        DBuf tmp;
        tmp.alloc((size_t)(g_.n1l * g_.n2 * g_.n3));
        launch_from_tm(g_, src, tmp.p, g_.n1l, st_);
        if (ldO == g_.n1l) {
            const size_t nb = (size_t)(g_.n1l * g_.n2 * g_.n3) * sizeof(double);
            populate_output(O, nb);
            TRITD_HIP(hipMemcpyAsync(O, tmp.p, nb, hipMemcpyDeviceToHost, st_));
        } else
            TRITD_HIP(hipMemcpy2DAsync(O, ldO * sizeof(double), tmp.p, g_.n1l * sizeof(double),
                                       g_.n1l * sizeof(double), (size_t)(g_.n2 * g_.n3),
                                       hipMemcpyDeviceToHost, st_));
        TRITD_HIP(hipStreamSynchronize(st_));
    }
}

}  // namespace tritd
