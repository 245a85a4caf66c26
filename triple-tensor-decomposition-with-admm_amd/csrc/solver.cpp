// Device-resident ADMM loop of fast_robust_triple_tensor/triple_decomp_ADMM.m:31-66.
//
// One iteration = four phases separated by the three all-reduces of the
// mode-1 sharded schedule:
//   A  M1, solve A (update_A :73-81), A^TA partial, M2 partial     -> red1
//   B  solve B (update_B :83-88), B^TB, M3 partial (K2)             -> red2
//   C  solve C (update_C :90-95), C^TC, fused update K5 (:38-53,:33) -> red3
//   D  errHist, stop test (:59-65)
// With one GPU the all-reduces vanish; with RCCL they are ncclAllReduce on
// the session stream; virtual-shard groups (api.cpp) sum the red buffers of
// several sessions on one device instead.
#include "solver.h"
#include "group.h"

#include <rocprofiler-sdk-roctx/roctx.h>
#include <sys/mman.h>

#include <algorithm>
#include <functional>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <system_error>
#include <thread>

namespace tritd {

void emit_line(const char* line);  // api.cpp

// roctx range over a scope (rocprofv3 --marker-trace shows them beside the
// kernels).  The loop is asynchronous, so a range spans the host's enqueue
// of its phase: which kernels belong to which ADMM statement, not GPU time.
struct Range {
    explicit Range(const char* name) { roctxRangePush(name); }
    ~Range() { roctxRangePop(); }
    Range(const Range&) = delete;
    Range& operator=(const Range&) = delete;
};

// ---------------------------------------------------------------------------
// layout conversions (reference shapes <-> CP factor matrices)
// ---------------------------------------------------------------------------
void pack_A(const Geom& g, const double* A, std::vector<double>& Ah, std::vector<double>& AhT) {
    Ah.assign(g.n1p * g.RP, 0.0);
    AhT.assign((size_t)g.RP * g.n1p, 0.0);
    for (int64_t il = 0; il < g.n1l; ++il)
        for (int k = 0; k < g.R; ++k) {
            const double v = A[(g.i0 + il) + g.n1 * k];  // A(i,p,q) at i + n1*(p + r*q)
            Ah[il * g.RP + k] = v;
            AhT[(size_t)k * g.n1p + il] = v;
        }
}

void pack_B(const Geom& g, const double* B, std::vector<double>& Bh) {
    Bh.assign(g.n2 * g.RP, 0.0);
    const int r = g.r;
    for (int64_t j = 0; j < g.n2; ++j)
        for (int q = 0; q < r; ++q)
            for (int p = 0; p < r; ++p) Bh[j * g.RP + p + r * q] = B[p + r * (j + g.n2 * q)];
}

void pack_C(const Geom& g, const double* C, std::vector<double>& Ch, std::vector<double>& ChT) {
    Ch.assign(g.n3p * g.RP, 0.0);
    ChT.assign((size_t)g.RP * g.n3p, 0.0);
    for (int64_t t = 0; t < g.n3; ++t)
        for (int k = 0; k < g.R; ++k) {
            const double v = C[k + (int64_t)g.R * t];  // C(p,q,t) at p + r*q + R*t
            Ch[t * g.RP + k] = v;
            ChT[(size_t)k * g.n3p + t] = v;
        }
}

void unpack_A(const Geom& g, const std::vector<double>& Ah, double* A) {
    for (int64_t il = 0; il < g.n1l; ++il)
        for (int k = 0; k < g.R; ++k) A[(g.i0 + il) + g.n1 * k] = Ah[il * g.RP + k];
}

void unpack_B(const Geom& g, const std::vector<double>& Bh, double* B) {
    const int r = g.r;
    for (int64_t j = 0; j < g.n2; ++j)
        for (int q = 0; q < r; ++q)
            for (int p = 0; p < r; ++p) B[p + r * (j + g.n2 * q)] = Bh[j * g.RP + p + r * q];
}

void unpack_C(const Geom& g, const std::vector<double>& Ch, double* C) {
    for (int64_t t = 0; t < g.n3; ++t)
        for (int k = 0; k < g.R; ++k) C[k + (int64_t)g.R * t] = Ch[t * g.RP + k];
}

// ---------------------------------------------------------------------------
Session::Session(int device, const void* D, int64_t ldD, int64_t n1, int64_t n2, int64_t n3,
                 int64_t i0, int64_t i1, int r, const tritd_opts& o, const double* A0,
                 const double* B0, const double* C0, tritd_comm* comm, uint32_t flags,
                 hipStream_t shared_stream, bool defer_normD)
    : device_(device), o_(o), comm_(comm) {
    TRITD_HIP(hipSetDevice(device_));
    g_ = make_geom(n1, n2, n3, i0, i1, r);
    f32_ = (flags & TRITD_SESSION_F32) != 0;
    probe_ = (flags & TRITD_SESSION_PROBE) != 0;
    es_ = f32_ ? sizeof(float) : sizeof(double);
    // fp32 path and fp64 r = 9..16: padded ranks 16/32/48/64/128/256 (the
    // K5 / K2 instantiations; fp64 RP = 128/256 runs K5 at one wave per SIMD
    // and K2 as 64-column passes — functional, not the tuned r <= 8 path)
    if (f32_ || g_.R > 64) g_.RP = padded_rank32(g_.R);
    // K5's t-split is fixed here: W's partial sets, K5's norm partials and
    // red1_'s tail are all sized by it (fp64 K5 only)
    if (!f32_) g_.tsplit = k5_tsplit(g_);
    // Schedules: one GPU without a group stream runs the
    // single-stream fused iteration (fp64 CP, RP <= 64) or else the
    // overlapped one (side-stream Grams and solves); with a communicator the
    // fused iteration with its two all-reduces, or the sharded side-stream
    // one; device groups sharing a stream run the phase-serial order.
    overlap_ = (comm == nullptr) && (shared_stream == nullptr);
    dy_ = !f32_;  // derived Y_O (k_admm.hip): every fp64 session
    {
        const char* de = std::getenv("TRITD_DENSE_E");  // force the E storage form (tests)
        de_mode_ = de ? std::atoi(de) : -1;
        // TRITD_SHOV=0: a communicator session runs the phase-serial order
        const char* sh = std::getenv("TRITD_SHOV");
        shov_ = comm != nullptr && comm->active() && shared_stream == nullptr &&
                !(sh && std::atoi(sh) == 0);
    }
    create_streams(shared_stream);
    if (overlap_ || shov_) {
        for (hipEvent_t* e : {&evAtA_, &evBtB_, &evCtC_, &evSA_, &evSB_, &evSC_})
            TRITD_HIP(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    qi_ = o_.model == TRITD_MODEL_QI;
    de_ = de_mode_ == 1 && de_eligible();  // forced from the start (E starts at zero)
    if (o_.model != TRITD_MODEL_CP && o_.model != TRITD_MODEL_QI)
        throw Error(TRITD_ERR_ARG, "opts.model must be 'cp' or 'qi'");
    if (qi_ && f32_)
        throw Error(TRITD_ERR_UNSUPPORTED, "opts.model='qi' is implemented for a double D only");
    if (!rp_supported32(g_.RP))
        throw Error(TRITD_ERR_UNSUPPORTED, "r must be in 1..16");
    if (qi_ && g_.r > 8) throw Error(TRITD_ERR_UNSUPPORTED, "opts.model='qi': r <= 8");
    {
        // one stream, side solves inside K2 / K5 (the cross-stream event of
        // the side-stream schedules costs ~10 us per sync on the main stream,
        // tools/sync_bench.hip); TRITD_FUSED=0 keeps the side-stream schedules
        const char* fe = std::getenv("TRITD_FUSED");
        fused_ = (overlap_ || shov_) && !qi_ && !f32_ && g_.RP <= 64 && !(fe && std::atoi(fe) == 0);
    }

    // deterministic mu schedule (:16-17, :56-57); muL == muO at every k
    mu_.resize((size_t)o_.maxIter + 2);
    {
        double mu = o_.mu;
        const double mu_max = o_.mu * 1e6;
        for (auto& m : mu_) {
            m = mu;
            mu = std::fmin(mu * o_.rho, mu_max);
        }
    }

    const size_t Np = (size_t)g_.Ntm;  // tile-major tensors (incl. group padding)
    {
        // the six streamed tensors live in one pool; each base is staggered so
        // that equal offsets of concurrently streamed tensors do not map to
        // the same HBM channel
        // 256 B: measured best of 0..4096 (tools/stagger_sweep.py at commit
        // 4a7facc, when the stagger was a knob)
        constexpr size_t stagger = 256;
        const size_t slot = round_up((int64_t)(Np * es_ + 5 * stagger), 4096);
        const size_t pool_bytes = 6 * slot;
        // compact E: 256 B per tile in either data type (before probing: the probe streams it)
        CE_.alloc_bytes((size_t)(g_.Ntm / 256) * 256);
        if (dy_) CE2_.alloc_bytes((size_t)(g_.Ntm / 256) * 256);
        // a host D is copied into a column-major staging buffer while the
        // placement probe runs (its kernels and the copy engine overlap), then
        // converted into the chosen pool below
        std::function<void()> upload;
        if (!(flags & TRITD_SESSION_D_ON_DEVICE) && g_.n1l > 0 && n2 * n3 > 0) {
            upload = [&] {
                dstage_.alloc_bytes((size_t)(g_.n1l * n2 * n3) * es_);
                hipStream_t cs = nullptr;
                TRITD_HIP(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
                hipError_t e;
                if (ldD == g_.n1l)  // contiguous shard: one 1-D copy
                    e = hipMemcpyAsync(dstage_.p, D, (size_t)(g_.n1l * n2 * n3) * es_,
                                       hipMemcpyHostToDevice, cs);
                else
                    e = hipMemcpy2DAsync(dstage_.p, g_.n1l * es_, D, ldD * es_, g_.n1l * es_,
                                         (size_t)(n2 * n3), hipMemcpyHostToDevice, cs);
                if (e == hipSuccess) e = hipStreamSynchronize(cs);
                hip_quiet(hipStreamDestroy(cs));
                TRITD_HIP(e);
            };
        }
        pool_.p = probe_pool(pool_bytes, slot, stagger, upload);
        TRITD_HIP(hipMemsetAsync(CE_.p, 0, CE_.bytes(), st_));
        if (dy_) TRITD_HIP(hipMemsetAsync(CE2_.p, 0, CE2_.bytes(), st_));
        pool_.n = pool_bytes / sizeof(double);
        int q = 0;
        for (DBuf* b : {&D_, &O_, &E_, &YL_, &YO_, &T_}) {
            b->p = reinterpret_cast<double*>(reinterpret_cast<char*>(pool_.p) + q * slot + q * stagger);
            b->n = (Np * es_) / sizeof(double);
            b->owned = false;
            TRITD_HIP(hipMemsetAsync(b->p, 0, Np * es_, st_));
            ++q;
        }
    }
    // W, plus the partial sets of a t-split K5 walk (k5_tsplit; fp64)
    Wk_.alloc_bytes((size_t)g_.RP * g_.plane * es_ * (size_t)g_.tsplit);
    TRITD_HIP(hipMemsetAsync(Wk_.p, 0, Wk_.bytes(), st_));
    if (f32_) ChF_.alloc_bytes((size_t)g_.n3p * g_.RP * sizeof(float));
    for (int q = 0; q < 2; ++q) {
        AhB_[q].alloc(g_.n1p * g_.RP);
        AhTB_[q].alloc((size_t)g_.RP * g_.n1p);
        TRITD_HIP(hipMemsetAsync(AhB_[q].p, 0, AhB_[q].bytes(), st_));
        TRITD_HIP(hipMemsetAsync(AhTB_[q].p, 0, AhTB_[q].bytes(), st_));
    }
    Ah_.owned = AhT_.owned = false;
    set_ah(0);  // the initial factors go to parity 0 (k done = 0)
    Bh_.alloc(g_.n2 * g_.RP);
    Ch_.alloc(g_.n3p * g_.RP);
    ChT_.alloc((size_t)g_.RP * g_.n3p);
    M1_.alloc_bytes((size_t)g_.n1p * g_.RP * es_);
    // one inverse per Gram slot, kept across iterations: each solve refines
    // the previous inverse of its own slot (k_solve_ns); zero = no start
    for (DBuf* b : {&GinvA_, &GinvB_, &GinvC_}) {
        b->alloc(ginv_count(g_.RP));  // inverse + pinv fallback space (pinv.h)
        TRITD_HIP(hipMemsetAsync(b->p, 0, b->bytes(), st_));
    }
    BtB_.alloc((size_t)g_.RP * g_.RP);
    CtC_.alloc((size_t)g_.RP * g_.RP);
    if (qi_) {
        H_.alloc((size_t)(g_.n1p * g_.n2 * g_.RP));
        TRITD_HIP(hipMemsetAsync(H_.p, 0, H_.bytes(), st_));
        ones_.alloc((size_t)g_.RP * g_.RP);
        launch_fill(ones_.p, (int64_t)ones_.n, 1.0, st_);
        for (DBuf* b : {&GqA_, &GqB_, &GqC_}) b->alloc((size_t)g_.RP * g_.RP);
    }
    k5tail_ = k5n();
    if (comm_ && comm_->active()) agree_counts();
    red1_.alloc(red1_count() + 2 * (size_t)k5tail_);  // + the tail for K5's norm partials
    red2_.alloc(red2_count());
    red3_.alloc(2);
    k5part_.alloc(2 * (size_t)k5n());
    m3part_.alloc((size_t)(f32_ ? m3_parts32(g_) : m3_parts(g_)) * g_.n3p * g_.RP);
    sqpart_.alloc(2 * (size_t)sumsq_blocks(g_));
    const size_t mi = o_.maxIter > 0 ? (size_t)o_.maxIter : 1;
    errHist_.alloc(mi);
    errL_.alloc(mi);
    errO_.alloc(mi);
    for (DBuf* b : {&errHist_, &errL_, &errO_, &red1_, &red2_, &red3_})
        TRITD_HIP(hipMemsetAsync(b->p, 0, b->n * sizeof(double), st_));
    const size_t ctrl_bytes = 4 * sizeof(int) + DENSE_SLOTS * sizeof(unsigned long long);
    TRITD_HIP(hipMalloc(&ctrl_, ctrl_bytes));
    TRITD_HIP(hipMemsetAsync(ctrl_, 0, ctrl_bytes, st_));

    // D -> tile-major device layout (one-off)
    if (g_.n1l > 0 && n2 * n3 > 0) {
        auto to_tm = [&](const void* src, int64_t ld) {
            if (f32_)
                launch_to_tm32(g_, static_cast<const float*>(src), ld, D_.f(), st_);
            else
                launch_to_tm(g_, static_cast<const double*>(src), ld, D_.p, st_);
        };
        if (flags & TRITD_SESSION_D_ON_DEVICE) {
            to_tm(D, ldD);
        } else {  // staged during the placement probe (above)
            to_tm(dstage_.p, g_.n1l);
            TRITD_HIP(hipStreamSynchronize(st_));
            dstage_.release();
        }
    }
    upload_factors(A0, B0, C0);

    // normD = norm(D(:))  (:28)
    const int nb = sumsq_blocks(g_);
    if (f32_)
        launch_sumsq32(g_, D_.f(), sqpart_.p, nb, st_);
    else
        launch_sumsq_padded(g_, D_.p, sqpart_.p, nb, st_);
    launch_reduce_pairs(sqpart_.p, nb, red3_.p, nullptr, st_);
    if (!defer_normD) {
        allreduce(red3_.p, 2);
        set_normD_from_red3();
    }

    // Grams of the initial B, C (replicated factors: no reduction needed)
    launch_gram(g_.RP, Bh_.p, g_.n2, BtB_.p, ctrl_, st_);
    launch_gram(g_.RP, Ch_.p, g_.n3p, CtC_.p, ctrl_, st_);

    // T of iteration 1 (:33) and W = T x3 C0 for update_A/update_B
    if (o_.maxIter > 0) launch_k5_any(1, /*prologue=*/true);
    if (fused_) {
        solve(0, BtB_.p, CtC_.p, o_.lambda2, GinvA_.p, st_);  // solve A of iteration 1
    } else if (overlap_ || shov_) {  // solve A of iteration 1 (needs the initial B^TB, C^TC)
        TRITD_HIP(hipEventRecord(evCtC_, st_));
        TRITD_HIP(hipStreamWaitEvent(side_, evCtC_, 0));
        solve(0, BtB_.p, CtC_.p, o_.lambda2, GinvA_.p, side_);
        TRITD_HIP(hipEventRecord(evSA_, side_));
        TRITD_HIP(hipStreamSynchronize(side_));
    }
    TRITD_HIP(hipStreamSynchronize(st_));
}

// Streams.  The side stream (Grams and R x R solves beside K5 / M3) is
// created at high priority: HIP maps streams of one priority onto a few
// hardware queues, and a same-priority side stream was measured sharing the
// main stream's queue (everything serialised, only the event waits added);
// the high-priority pool is separate.  Side kernels still wait for free CU
// slots while K5 / M3 occupy every SIMD; reserving CUs for them with
// CU-masked streams (hipExtStreamCreateWithCUMask, 8 of 256 CUs) slowed K5
// from 1.19 to 1.52 ms and M3 from 0.36 to 0.65 ms, so it is not used.
void Session::create_streams(hipStream_t shared_stream) {
    if (shared_stream) {
        st_ = shared_stream;
        return;
    }
    own_stream_ = true;
    TRITD_HIP(hipStreamCreateWithFlags(&st_, hipStreamNonBlocking));
    if (overlap_ || shov_) {
        int lo = 0, hi = 0;
        TRITD_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
        TRITD_HIP(hipStreamCreateWithPriority(&side_, hipStreamNonBlocking, hi));
    }
}

Session::~Session() {
    hip_quiet(hipSetDevice(device_));
    if (st_) hip_quiet(hipStreamSynchronize(st_));
    if (side_) {
        hip_quiet(hipStreamSynchronize(side_));
        hip_quiet(hipStreamDestroy(side_));
    }
    for (hipEvent_t e : {evAtA_, evBtB_, evCtC_, evSA_, evSB_, evSC_})
        if (e) hip_quiet(hipEventDestroy(e));
    for (auto e : ev_) hip_quiet(hipEventDestroy(e));
    if (ctrl_) hip_quiet(hipFree(ctrl_));
    if (own_stream_ && st_) hip_quiet(hipStreamDestroy(st_));
}

void Session::set_normD_from_red3() {
    double ss[2];
    TRITD_HIP(hipMemcpyAsync(ss, red3_.p, 2 * sizeof(double), hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipStreamSynchronize(st_));
    normD_ = std::sqrt(ss[0]);
    if (f32_) normD_ = (double)(float)normD_;  // norm of a single array is single
}

void Session::upload_factors(const double* A0, const double* B0, const double* C0) {
    std::vector<double> Ah, AhT, Bh, Ch, ChT;
    pack_A(g_, A0, Ah, AhT);
    pack_B(g_, B0, Bh);
    pack_C(g_, C0, Ch, ChT);
    TRITD_HIP(hipMemcpy(Ah_.p, Ah.data(), Ah.size() * sizeof(double), hipMemcpyHostToDevice));
    TRITD_HIP(hipMemcpy(AhT_.p, AhT.data(), AhT.size() * sizeof(double), hipMemcpyHostToDevice));
    TRITD_HIP(hipMemcpy(Bh_.p, Bh.data(), Bh.size() * sizeof(double), hipMemcpyHostToDevice));
    TRITD_HIP(hipMemcpy(Ch_.p, Ch.data(), Ch.size() * sizeof(double), hipMemcpyHostToDevice));
    TRITD_HIP(hipMemcpy(ChT_.p, ChT.data(), ChT.size() * sizeof(double), hipMemcpyHostToDevice));
    if (f32_) {
        std::vector<float> cf(Ch.size());
        for (size_t e = 0; e < Ch.size(); ++e) cf[e] = (float)Ch[e];
        TRITD_HIP(hipMemcpy(ChF_.p, cf.data(), cf.size() * sizeof(float), hipMemcpyHostToDevice));
    }
}

IterScalars Session::scalars(int k) const {
    IterScalars s;
    s.muL = mu_[(size_t)k - 1];
    s.muO = mu_[(size_t)k - 1];
    s.invL = 1.0 / s.muL;
    s.invO = 1.0 / s.muO;
    s.thr = o_.lambda / s.muO;
    s.den = s.muL + s.muO;
    s.rden = 1.0 / s.den;
    s.invL_next = 1.0 / mu_[(size_t)k];
    s.muO_prev = k >= 2 ? mu_[(size_t)k - 2] : 0.0;  // E^(0) = E^(-1) = 0: any value
    s.cprev = s.invO * s.muO_prev;
    return s;
}

IterScalars32 Session::scalars32(int k) const {
    // MATLAB: a double scalar meeting a single array is converted to single
    const IterScalars d = scalars(k);
    IterScalars32 s;
    s.muL = (float)d.muL;
    s.muO = (float)d.muO;
    s.invL = (float)d.invL;
    s.invO = (float)d.invO;
    s.thr = (float)d.thr;
    s.den = (float)d.den;
    s.rden = 1.0f / s.den;
    s.invL_next = (float)d.invL_next;
    return s;
}

void Session::do_m1() {
    if (qi_)
        launch_m1_qi(g_, g_.r, Wk_.p, Bh_.p, M1_.p, ctrl_, st_);
    else if (f32_)  // (its finish rides in M2: do_m2)
        launch_m1_32(g_, Wk_.f(), Bh_.p, M1_.f(), ctrl_, st_);
    else  // the previous K5's norm reduction and stop test in an extra workgroup (finish.h)
        launch_m1(g_, Wk_.p, Bh_.p, M1_.p, ctrl_, st_, take_finish());
}

// The pending norm reduction + stop test of the previous iteration (single
// GPU: K5's own partials), for an extra workgroup of the next M1 / M2
FinishArgs Session::take_finish() {
    FinishArgs f;
    if (norms_pending_ && !(comm_ && comm_->active())) {
        f.p = k5part_.p; f.n = k5n(); f.normD = normD_; f.k = pend_k_; f.tol = o_.tol;
        f.errHist = errHist_.p; f.errL = errL_.p; f.errO = errO_.p; f.ctrl = ctrl_;
        f.single = (int)f32_; f.on = 1;
        norms_pending_ = false;
    }
    return f;
}

void Session::do_m2(double* M2) {
    if (qi_)
        launch_m2_qi(g_, g_.r, Wk_.p, AhT_.p, M2, ctrl_, st_);
    else if (f32_)
        launch_m2_32(g_, Wk_.f(), AhT_.p, M2, ctrl_, st_, take_finish());
    else
        launch_m2(g_, Wk_.p, AhT_.p, M2, ctrl_, st_);
}

void Session::do_m3() {
    if (qi_)
        do_m3_qi();
    else if (f32_)
        launch_m3_32(g_, T_.f(), Ah_.p, Bh_.p, m3part_.p, red2_.p, ctrl_, st_);
    else
        launch_m3(g_, T_.p, Ah_.p, Bh_.p, m3part_.p, red2_.p, ctrl_, st_);
}

// Qi: H from the fresh A^, B^ (after update_B); read by K2 and by the K5 that follows
void Session::do_m3_qi() {
    launch_qi_h(g_, g_.r, Ah_.p, Bh_.p, H_.p, ctrl_, st_);
    launch_m3(g_, T_.p, H_.p, ones_.p, m3part_.p, red2_.p, ctrl_, st_, g_.n1p * g_.RP, 0);
}

void Session::solve(int mode, const double* P, const double* Q, double alpha, double* out,
                    hipStream_t s, const FinishArgs* fin) {
    if (!qi_) {
        launch_solve(g_.RP, g_.R, P, Q, alpha, out, ctrl_ + 2, ctrl_, s, fin);
    } else {
        if (fin) throw Error(TRITD_ERR_ARG, "solve with a finish: CP model only");
        double* G = (mode == 0 ? GqA_ : mode == 1 ? GqB_ : GqC_).p;
        launch_qi_gram(g_.RP, g_.r, mode, P, Q, G, ctrl_, s);
        launch_solve(g_.RP, g_.R, G, ones_.p, alpha, out, ctrl_ + 2, ctrl_, s);
    }
    // the generic apply's pinv fallback, on the solve's stream (a side-stream
    // solve then hands over a finished Ginv: one launch fewer on the main one).
    // Not for mode 0: solve A of iteration k+1 runs beside K5 of k, before k's
    // stop test, and a fallback there could raise TRITD_FLAG_PINV_TOL for an
    // update_A that MATLAB never performs when the loop stops at k (ADVICE
    // r5); apply A runs the fallback itself, after the stop test (do_apply_A)
    if (gen_apply() && mode != 0) launch_pinv_fix(g_.RP, out, ctrl_, ctrl_ + 2, s);
}

// (X*F')*pinv(G): fp64 path through the MFMA apply (RP <= 64); fp32
// path single in, single-rounded out (MATLAB single * double = single)
void Session::do_apply_A(double* Ginv) {
    // (fix = true: the pinv fallback of solve A runs here, after the stop test)
    if (f32_)
        launch_apply_gen(g_.RP, nullptr, M1_.f(), g_.n1p, Ginv, Ah_.p, AhT_.p, g_.n1p, nullptr,
                         true, ctrl_, ctrl_ + 2, st_, true);
    else if (g_.RP > 64)  // fp64 r = 9..16
        launch_apply_gen(g_.RP, M1_.p, nullptr, g_.n1p, Ginv, Ah_.p, AhT_.p, g_.n1p, nullptr,
                         false, ctrl_, ctrl_ + 2, st_, true);
    else
        launch_apply(g_.RP, M1_.p, g_.n1p, Ginv, Ah_.p, AhT_.p, g_.n1p, ctrl_, ctrl_ + 2, st_);
}

void Session::do_apply_B(const double* M2, double* Ginv) {
    if (f32_)
        launch_apply_gen(g_.RP, M2, nullptr, g_.n2, Ginv, Bh_.p, nullptr, 0, nullptr, true, ctrl_, ctrl_ + 2,
                         st_, false);
    else if (g_.RP > 64)  // fp64 r = 9..16
        launch_apply_gen(g_.RP, M2, nullptr, g_.n2, Ginv, Bh_.p, nullptr, 0, nullptr, false, ctrl_, ctrl_ + 2,
                         st_, false);
    else
        launch_apply(g_.RP, M2, g_.n2, Ginv, Bh_.p, nullptr, 0, ctrl_, ctrl_ + 2, st_);
}

void Session::do_apply_C(double* Ginv) {
    if (f32_)
        launch_apply_gen(g_.RP, red2_.p, nullptr, g_.n3p, Ginv, Ch_.p, ChT_.p, g_.n3p, ChF_.f(),
                         true, ctrl_, ctrl_ + 2, st_, false);
    else if (g_.RP > 64)  // fp64 r = 9..16
        launch_apply_gen(g_.RP, red2_.p, nullptr, g_.n3p, Ginv, Ch_.p, ChT_.p, g_.n3p, nullptr,
                         false, ctrl_, ctrl_ + 2, st_, false);
    else
        launch_apply(g_.RP, red2_.p, g_.n3p, Ginv, Ch_.p, ChT_.p, g_.n3p, ctrl_, ctrl_ + 2, st_);
}

// apply + Gram of one factor (update_A/B/C, :77-81,86-88,93-95): one launch
// for small fp64 problems (k_apply_gram), else k_apply then k_gram
bool Session::small_ag(int64_t rows) const {
    return !f32_ && !qi_ && g_.RP <= 64 && apply_gram_small(g_.RP, rows);
}

// Small factors (rows*RP^2 <= 327 680): with defer (the fused single-GPU
// schedule, side_gram_ok) the apply alone, the Gram left to the side solve
// that next reads it (SideSolve::gram_rows), else apply + Gram in one
// single-workgroup launch.  Larger factors: an apply and a Gram launch (a
// side-job Gram of 512 x 64 outlasts M2: config 4 1.34 -> 1.41 ms; beside
// K2 / K5 of a 64-row shard it doubled both, round 5, while at config 4 it
// moved nothing beyond box noise: profiles/round5/shard8_deferred_grams.txt).
// Returns whether the Gram was left to the side solve.
bool Session::apply_gram_A(double* AtA, bool defer) {
    if (defer && small_ag(g_.n1p)) {
        do_apply_A(GinvA_.p);
        return true;
    }
    if (small_ag(g_.n1p)) {
        launch_apply_gram(g_.RP, M1_.p, g_.n1p, GinvA_.p, Ah_.p, AhT_.p, g_.n1p, AtA, ctrl_, ctrl_ + 2, st_);
        return false;
    }
    do_apply_A(GinvA_.p);
    launch_gram(g_.RP, Ah_.p, g_.n1p, AtA, ctrl_, st_);
    return false;
}

bool Session::apply_gram_B(const double* M2, bool defer) {
    if (defer && small_ag(g_.n2)) {  // the Gram rides beside K2 (side solve C)
        do_apply_B(M2, GinvB_.p);
        return true;
    }
    if (small_ag(g_.n2)) {
        launch_apply_gram(g_.RP, M2, g_.n2, GinvB_.p, Bh_.p, nullptr, 0, BtB_.p, ctrl_, ctrl_ + 2, st_);
        return false;
    }
    do_apply_B(M2, GinvB_.p);
    launch_gram(g_.RP, Bh_.p, g_.n2, BtB_.p, ctrl_, st_);
    return false;
}

bool Session::apply_gram_C(bool defer) {
    if (defer && small_ag(g_.n3p)) {  // the Gram rides beside K5 (side solve A of k+1)
        do_apply_C(GinvC_.p);
        return true;
    }
    if (small_ag(g_.n3p)) {
        launch_apply_gram(g_.RP, red2_.p, g_.n3p, GinvC_.p, Ch_.p, ChT_.p, g_.n3p, CtC_.p, ctrl_, ctrl_ + 2,
                          st_);
        return false;
    }
    do_apply_C(GinvC_.p);
    launch_gram(g_.RP, Ch_.p, g_.n3p, CtC_.p, ctrl_, st_);
    return false;
}

// the Grams can ride in side solves on the fused schedule: A's on one GPU
// only (with a communicator A^TA is all-reduced with M2 before update_B's
// solve: it is formed by a gram-only side job of M2 instead), B's and C's in
// either case (replicated factors)
bool Session::side_gram_ok() const {
    return side_gram_bc_ok() && !(comm_ && comm_->active());
}

bool Session::side_gram_bc_ok() const { return !f32_ && !qi_ && g_.RP <= 64; }

// a sharded session's A^T A as a gram-only side job of M2: shards of up to
// 64 rows (16 K-steps of the side Gram, which then ends inside M2's time;
// its load round trips make 128+ rows outlast M2)
bool Session::gram_a_in_m2() const {
    return side_gram_bc_ok() && comm_ && comm_->active() && g_.n1p <= 64;
}

// side solve `s` first forms operand `which` (0 = P, 1 = Q) as X^T X into `to`
static void with_gram(SideSolve& s, const double* X, int64_t rows, double* to, int which) {
    s.gram_src = X;
    s.gram_rows = rows;
    s.gram_to = to;
    s.gram_which = which;
}

void Session::launch_k5_any(int k, bool prologue) {
    if (f32_) {
        K5Args32 a{};
        a.D = D_.f(); a.O = O_.f(); a.E = E_.f(); a.CE = CE_.f(); a.YL = YL_.f(); a.YO = YO_.f();
        a.T = T_.f(); a.Wk = Wk_.f();
        a.Ah = Ah_.p; a.Bh = Bh_.p; a.ChF = ChF_.f(); a.partial = k5part_.p;
        a.n1p = g_.n1p; a.n2 = g_.n2; a.n3p = g_.n3p; a.plane = g_.plane; a.tiles = g_.tiles;
        a.ntt = g_.ntt;
        a.s = scalars32(k);
        a.stop = ctrl_;
        a.dense_tiles = dense_tiles();
        launch_k5_32(g_, a, prologue, st_);
        return;
    }
    K5Args a{};
    a.D = D_.p; a.O = O_.p; a.YL = YL_.p; a.T = T_.p; a.Wk = Wk_.p;
    // E^(k-1) and E^(k-2) are read (Y_O is derived from them), E^(k) is
    // written over E^(k-2)
    a.E = e_buf(k - 1); a.CE = ce_buf(k - 1);
    a.Ep = e_buf(k); a.CEp = ce_buf(k);
    a.Ah = Ah_.p; a.Bh = Bh_.p; a.Ch = Ch_.p; a.ChT = ChT_.p;
    a.partial = (k5part_to_ && !prologue) ? k5part_to_ : k5part_.p;
    a.ahj = 0; a.bhj = g_.RP;
    if (qi_) {  // L = H Ch^T (H built before K2 of this iteration)
        a.Ah = H_.p; a.Bh = ones_.p;
        a.ahj = g_.n1p * g_.RP; a.bhj = 0;
    }
    a.n1p = g_.n1p; a.n2 = g_.n2; a.n3p = g_.n3p; a.plane = g_.plane; a.tiles = g_.tiles;
    a.ntt = g_.ntt;
    a.s = scalars(k);
    a.stop = ctrl_;
    a.dense_tiles = dense_tiles();
    if (!prologue) {
        a.side = k5side_;
        k5side_ = SideSolve{};
    }
    launch_k5(g_, a, prologue, st_, de_ && !prologue);
}

// Dense-E mode switch (once per solve).  On data whose outliers are not
// sparse (video: every compact-E tile overflows after a few iterations) the
// compact slots are pure overhead, so after iterations 8 and 24 the dense
// tiles of the launches since the last check are counted (one host sync) and,
// at half of all tiles or more, the compact tiles of E^(k) and E^(k-1) are
// expanded into the dense buffers and K5 runs in its dense-E form from k+1 on.
// Storage only: the values are the same either way.
void Session::maybe_dense_e(int k) {
    if (de_ || de_mode_ != -1 || !de_eligible() || (k != 8 && k != 24)) return;
    int64_t total = 0, per = 0;
    counters(&total, &per);
    const int launches = k - de_prev_k_;
    const double frac = (launches > 0 && per > 0) ? (double)(total - de_prev_) / ((double)launches * per) : 0.0;
    de_prev_ = total;
    de_prev_k_ = k;
    if (frac < 0.5) return;
    launch_ce_expand(g_, ce_buf(k), e_buf(k), st_);
    launch_ce_expand(g_, ce_buf(k - 1), e_buf(k - 1), st_);
    de_ = true;
}

void populate_output(void* p, size_t bytes) { populate_output_threads(p, bytes, 16); }

OutputPrefault::OutputPrefault(void* O, void* E, size_t bytes) {
    if (!O && !E) return;
    try {  // an optimisation only: no thread, no prefault (get() faults the pages in)
        t_ = std::thread([O, E, bytes] {
            if (O) populate_output_threads(O, bytes, 8);
            if (E) populate_output_threads(E, bytes, 8);
        });
    } catch (const std::system_error&) {
    }
}

void OutputPrefault::join() {
    if (t_.joinable()) t_.join();
}

void populate_output_threads(void* p, size_t bytes, unsigned max_threads) {
    if (!p || bytes < ((size_t)64 << 20)) return;
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23  // Linux 5.14
#endif
    constexpr uintptr_t PG = 4096, GR = (uintptr_t)2 << 20;
    const uintptr_t a = ((uintptr_t)p + PG - 1) & ~(PG - 1);
    const uintptr_t e = ((uintptr_t)p + bytes) & ~(PG - 1);
    if (e <= a) return;
    // transparent huge pages where the kernel offers them on request
    // (THP "madvise" mode): 512x fewer faults, the zeroing in 2 MB pieces
    // (host test: 1.12 s -> 0.16 s to populate 1 GB on one thread)
    {
        const uintptr_t ha = (a + GR - 1) & ~(GR - 1), he = e & ~(GR - 1);
        if (he > ha) (void)madvise((void*)ha, (size_t)(he - ha), MADV_HUGEPAGE);
    }
    const unsigned hc = std::thread::hardware_concurrency();
    const uintptr_t nt = std::min<uintptr_t>(max_threads ? max_threads : 1, hc ? hc : 1);
    const uintptr_t chunk = (((e - a) / nt) + GR - 1) & ~(GR - 1);
    std::vector<std::thread> th;
    th.reserve((size_t)((e - a + chunk - 1) / chunk));
    for (uintptr_t s = a; s < e; s += chunk) {
        const size_t len = (size_t)std::min(chunk, e - s);
        try {
            th.emplace_back([s, len] { (void)madvise((void*)s, len, MADV_POPULATE_WRITE); });
        } catch (const std::system_error&) {  // no thread to spare: this piece on the caller's
            (void)madvise((void*)s, len, MADV_POPULATE_WRITE);
        }
    }
    for (auto& t : th) t.join();
}

// ncclResult_t as GroupAbort::enqueue reads it: 0 done, 1 in progress, else
// 100 + the error
int nccl_state(ncclResult_t r) {
    return r == ncclSuccess ? 0 : r == ncclInProgress ? 1 : 100 + (int)r;
}

void comm_allreduce(tritd_comm* c, double* buf, int64_t count, bool max, hipStream_t st) {
    if (c->group) {  // a device-group shard: the communicator only under the abort protocol
        const int s = c->group->enqueue(
            c->rank,
            [&] {
                return nccl_state(ncclAllReduce(buf, buf, (size_t)count, ncclFloat64,
                                                max ? ncclMax : ncclSum, c->comm, st));
            },
            [&] {
                ncclResult_t a = ncclSuccess;
                const ncclResult_t q = ncclCommGetAsyncError(c->comm, &a);
                return nccl_state(q != ncclSuccess ? q : a);
            });
        if (s < 0)
            throw Error(TRITD_ERR_RCCL, "all-reduce not issued: another shard of the device group failed");
        if (s != 0)
            throw Error(TRITD_ERR_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString((ncclResult_t)(s - 100)));
        return;
    }
    if (c->comm) {
        const ncclResult_t r = ncclAllReduce(buf, buf, (size_t)count, ncclFloat64,
                                             max ? ncclMax : ncclSum, c->comm, st);
        if (r != ncclSuccess) throw Error(TRITD_ERR_RCCL, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
        return;
    }
    std::vector<double> h((size_t)count);
    TRITD_HIP(hipMemcpyAsync(h.data(), buf, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
    TRITD_HIP(hipStreamSynchronize(st));
    if (c->host_fn(h.data(), count, max ? 1 : 0, c->host_user) != 0)
        throw Error(TRITD_ERR_RCCL, "host all-reduce callback failed");
    TRITD_HIP(hipMemcpyAsync(buf, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, st));
    TRITD_HIP(hipStreamSynchronize(st));
}

void Session::allreduce(double* buf, int64_t count) {
    if (!comm_ || !comm_->active()) return;
    const int a = ar_in_iter_++;
    if (a < EV_AR) mark(6 + 2 * a);
    comm_allreduce(comm_, buf, count, false, st_);
    if (a < EV_AR) mark(7 + 2 * a);
}

// Every rank must issue each all-reduce with the same count.  red1 and red2
// are fixed by (n2, n3, r); the norm-partial tail of red1 follows the shard
// height (K5's grid), so it is sized to the largest shard's and the pairs past
// this rank's own stay zero (k_reduce_finish clears what it consumed).  The
// schedule itself (maxIter, disp: the print flushes the pending norms) must
// agree too.  One max-all-reduce of (x, -x) pairs at creation: every rank
// sees the same result, so a mismatch fails on all of them alike instead of
// hanging the first collective that differs.
void Session::agree_counts() {
    const double c[5] = {(double)k5n(), (double)red1_count(), (double)red2_count(),
                         (double)o_.maxIter, (double)(o_.disp != 0)};
    double h[10];
    for (int q = 0; q < 5; ++q) {
        h[2 * q] = c[q];
        h[2 * q + 1] = -c[q];
    }
    DBuf v;
    v.alloc(10);
    TRITD_HIP(hipMemcpyAsync(v.p, h, sizeof h, hipMemcpyHostToDevice, st_));
    comm_allreduce(comm_, v.p, 10, /*max=*/true, st_);
    TRITD_HIP(hipMemcpyAsync(h, v.p, sizeof h, hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipStreamSynchronize(st_));
    k5tail_ = (int)h[0];
    static const char* what[5] = {"", "n2 or r", "n3 or r", "opts.maxIter", "opts.disp"};
    for (int q = 1; q < 5; ++q)
        if (h[2 * q] != -h[2 * q + 1])
            throw Error(TRITD_ERR_ARG, std::string("ranks disagree on ") + what[q] +
                                           " (every rank must create its session with the same "
                                           "n1, n2, n3, r and opts)");
}

int Session::next_iter() {
    if (k_enq_ >= o_.maxIter) return 0;
    ++k_enq_;
    set_ah(k_enq_);
    return k_enq_;
}

void Session::set_ah(int k) {
    Ah_.p = AhB_[k & 1].p;
    Ah_.n = AhB_[k & 1].n;
    AhT_.p = AhTB_[k & 1].p;
    AhT_.n = AhTB_[k & 1].n;
}

void Session::flush_norms() {
    if (!norms_pending_) return;
    if (!(comm_ && comm_->active())) {  // single GPU: K5's own partials
        launch_reduce_finish(k5part_.p, k5n(), normD_, pend_k_, o_.tol, errHist_.p, errL_.p, errO_.p,
                             ctrl_, f32_, st_);
        norms_pending_ = false;
        return;
    }
    double* parts = red1_.p + red1_count();
    allreduce(parts, 2 * (int64_t)k5tail_);
    launch_reduce_finish(parts, k5tail_, normD_, pend_k_, o_.tol, errHist_.p, errL_.p, errO_.p,
                         ctrl_, f32_, st_, /*clear=*/true);
    norms_pending_ = false;
}

void Session::phaseA(int k) {
    (void)k;
    const int RP = g_.RP;
    double* M2 = red1_.p;
    double* AtA = red1_.p + g_.n2 * RP;
    do_m1();
    solve(0, BtB_.p, CtC_.p, o_.lambda2, GinvA_.p, st_);
    apply_gram_A(AtA);
    do_m2(M2);
}

void Session::phaseB(int k) {
    (void)k;
    const int RP = g_.RP;
    const double* M2 = red1_.p;
    const double* AtA = red1_.p + g_.n2 * RP;
    solve(1, AtA, CtC_.p, o_.lambda2, GinvB_.p, st_);
    apply_gram_B(M2);
    mark(1);
    do_m3();
    mark(2);
}

void Session::phaseC(int k) {
    const int RP = g_.RP;
    const double* AtA = red1_.p + g_.n2 * RP;
    solve(2, AtA, BtB_.p, 1e-9, GinvC_.p, st_);  // :93 ridge
    apply_gram_C();
    launch_k5_full(k, /*fused_finish=*/false);
}

// Placement probing.  K5 is HBM-bound and its bandwidth depends on where the
// pool lands physically: per allocation it is stable, across allocations it
// is not (measured 5.1-5.2 vs 5.7-6.05 TB/s for the same pattern, about one
// allocation in three fast; tools/aos_pattern.hip).  With room to spare,
// allocate up to TRITD_PROBE (default 8) candidate pools at once, time K5's
// access pattern on each and keep the fastest.  Results do not depend on the choice (addresses never enter the
// arithmetic).  Small problems skip it.  Only sessions created with
// TRITD_SESSION_PROBE probe: the one-shot calls (the MATLAB drop-in) do not,
// since a 100-iteration solve loses more to the probe than K5 gains
// (bench.py end_to_end: +17 ms at config 4, +5.7 s at config 5, round 5).
// TRITD_PROBE=n overrides either way (1 = off).
double* Session::probe_pool(size_t pool_bytes, size_t slot, size_t stagger,
                            std::function<void()> overlap) {
    const char* pe = std::getenv("TRITD_PROBE");
    // a session asked to probe (TRITD_SESSION_PROBE) tries 8 candidates, with
    // a host D copied in while the probe kernels run (`overlap`); without the
    // flag the first allocation is kept: for a one-shot 100-iteration solve
    // the candidate pools' allocation costs more than a fast placement saves
    // (config 4: 250 vs 212 ms end to end, profiles/round5/bench_line.json;
    // DESIGN.md §3)
    int want = pe ? std::atoi(pe) : (probe_ ? 8 : 1);
    // (small pools too: a mode-1 shard of 64 rows at 512^3 is a 0.8 GB pool, and
    // the slowest of P ranks sets the sharded iteration)
    if (pool_bytes < ((size_t)128 << 20)) want = 1;
    // rounds of `want` candidates until both placement classes have shown up
    // (fastest below 0.92 x slowest: the classes differ by ~10 %), so the one
    // kept is a fast one; a box whose first eight all landed in one class
    // (bench line 707 it/s with eight slow pools, vs 730-737) gets one more
    // round (a second one-class round is taken as that box's only class: with
    // one third of the pools fast, sixteen slow ones in a row are rare).
    // Earlier rounds stay allocated while the next one is drawn, so it gets
    // new pages.  Why a placement matters and why no layout removes it:
    // DESIGN.md §3 (profiles/round5/placement_strategies.txt).
    constexpr int rounds = 2;
    // keep room for the chosen pool, the other session buffers and 4 GiB
    const size_t reserve = pool_bytes / 2 + ((size_t)4 << 30);
    std::vector<double*> cand;
    auto alloc_round = [&](int n) {
        size_t fr = 0, tot = 0;
        TRITD_HIP(hipMemGetInfo(&fr, &tot));
        const size_t room = fr > reserve ? (fr - reserve) / pool_bytes : 0;
        if ((size_t)n > room) n = (int)room;
        if (cand.empty() && n < 1) n = 1;  // the pool itself
        // (hipDeviceMallocContiguous pools probe no differently:
        // tools/contig_probe.py at commit 4a7facc)
        for (int c = 0; c < n; ++c) {
            void* p = nullptr;
            if (hipMalloc(&p, pool_bytes) != hipSuccess) {
                (void)hipGetLastError();
                break;
            }
            cand.push_back(static_cast<double*>(p));
        }
    };
    alloc_round(want);
    if (cand.empty()) throw Error(TRITD_ERR_NOMEM, "hipMalloc of the tensor pool failed");
    probe_ms_.clear();
    size_t best = 0;
    if (want > 1 && cand.size() > 1) {
        // candidate c: a warm launch, then REPS launches each between events
        constexpr int REPS = 2;
        std::vector<hipEvent_t> ev;
        auto probe_on = [&](size_t c) {
            char* f[6];
            for (int q = 0; q < 6; ++q) f[q] = reinterpret_cast<char*>(cand[c]) + q * slot + q * stagger;
            // pool order: D, O, E, YL, YO, T
            if (f32_)
                launch_pool_probe32(g_, (float*)f[0], (float*)f[3], (float*)f[4], (float*)f[5], CE_.f(), st_);
            else
                launch_pool_probe(g_, (double*)f[0], (double*)f[3], (double*)f[5], CE_.p, st_);
        };
        // enqueue every candidate of [from, end) without waiting
        auto enqueue_from = [&](size_t from) {
            for (size_t c = from; c < cand.size(); ++c) {
                probe_on(c);  // warm
                for (int r = 0; r < REPS; ++r) {
                    hipEvent_t e0, e1;
                    TRITD_HIP(hipEventCreate(&e0));
                    TRITD_HIP(hipEventCreate(&e1));
                    ev.push_back(e0);
                    ev.push_back(e1);
                    TRITD_HIP(hipEventRecord(e0, st_));
                    probe_on(c);
                    TRITD_HIP(hipEventRecord(e1, st_));
                }
            }
        };
        auto collect_from = [&](size_t from) {
            for (size_t c = from; c < cand.size(); ++c) {
                float ms = 1e30f;
                for (int r = 0; r < REPS; ++r) {
                    const size_t q = 2 * (c * REPS + r);
                    TRITD_HIP(hipEventSynchronize(ev[q + 1]));
                    float x = 0.f;
                    TRITD_HIP(hipEventElapsedTime(&x, ev[q], ev[q + 1]));
                    ms = std::fmin(ms, x);
                }
                probe_ms_.push_back(ms);
                if (ms < probe_ms_[best]) best = c;
            }
        };
        // both placement classes seen: the fastest candidate is a fast one
        auto clearly_fast = [&] {
            const auto mm = std::minmax_element(probe_ms_.begin(), probe_ms_.end());
            return *mm.first < 0.92 * *mm.second;
        };
        enqueue_from(0);
        if (overlap) {  // the host copy of D runs while the probes do
            overlap();
            overlap = nullptr;
        }
        collect_from(0);
        for (int r = 1; r < rounds && !clearly_fast(); ++r) {
            const size_t from = cand.size();
            alloc_round(want);
            if (cand.size() == from) break;
            enqueue_from(from);
            collect_from(from);
        }
        for (hipEvent_t e : ev) hip_quiet(hipEventDestroy(e));
    } else {
        probe_ms_.assign(cand.size(), 0.0);
    }
    if (overlap) overlap();  // (no probe ran)
    for (size_t c = 0; c < cand.size(); ++c)
        if (c != best) hip_quiet(hipFree(cand[c]));
    probe_pick_ = (int)best;
    return cand[best];
}

void Session::launch_k5_full(int k, bool fused_finish) {
    mark(3);
    launch_k5_any(k, /*prologue=*/false);
    mark(4);
    if (fused_finish)  // single GPU: no all-reduce between the norm sums and the stop test
        launch_reduce_finish(k5part_.p, k5n(), normD_, k, o_.tol, errHist_.p, errL_.p,
                             errO_.p, ctrl_, f32_, st_);
    else
        launch_reduce_pairs(k5part_.p, k5n(), red3_.p, ctrl_, st_);
}

// Single-GPU iteration.  Same kernels and data flow as phases A-D, but each
// R x R solve runs on the side stream as soon as its Grams exist:
//   solve B (A^TA, C^TC) || M2        solve C (A^TA, B^TB) || M3
//   solve A of k+1 (B^TB, C^TC) || K5
// Every buffer a side kernel reads is next written on the main stream only
// after an event the side stream records behind that kernel.
void Session::iterate_overlapped(int k) {
    const int RP = g_.RP;
    double* M2 = red1_.p;
    double* AtA = red1_.p + g_.n2 * RP;
    // main: M1 -> apply A -> Gram A -> solve B -> M2 -> apply B -> K2 -> apply C -> K5 -> finish
    // side: Gram B -> solve C (|| K2) | Gram C -> solve A(k+1) (|| K5)
    // Gram A^TA and solve B are on the critical path (M2 beside them is only
    // ~20 us): on the main stream they cost their own time, on the side stream
    // that plus two cross-stream waits (each widens a kernel boundary by ~6 us)
    do_m1();
    TRITD_HIP(hipStreamWaitEvent(st_, evSA_, 0));
    do_apply_A(GinvA_.p);
    launch_gram(RP, Ah_.p, g_.n1p, AtA, ctrl_, st_);
    if (RP >= 128) {
        // padded ranks 128 / 256 (config 5): solve B (~0.15 ms, k_solve_mw)
        // on the high-priority side stream, issued before M2 (~0.65 ms there)
        // so that its workgroups are dispatched first and run beside it
        TRITD_HIP(hipEventRecord(evAtA_, st_));
        TRITD_HIP(hipStreamWaitEvent(side_, evAtA_, 0));
        solve(1, AtA, CtC_.p, o_.lambda2, GinvB_.p, side_);
        TRITD_HIP(hipEventRecord(evSB_, side_));
        do_m2(M2);
        TRITD_HIP(hipStreamWaitEvent(st_, evSB_, 0));
    } else {
        solve(1, AtA, CtC_.p, o_.lambda2, GinvB_.p, st_);
        do_m2(M2);
    }
    do_apply_B(M2, GinvB_.p);
    TRITD_HIP(hipEventRecord(evBtB_, st_));
    TRITD_HIP(hipStreamWaitEvent(side_, evBtB_, 0));
    launch_gram(RP, Bh_.p, g_.n2, BtB_.p, ctrl_, side_, true);
    solve(2, AtA, BtB_.p, 1e-9, GinvC_.p, side_);  // :93 ridge
    TRITD_HIP(hipEventRecord(evSC_, side_));
    mark(1);
    do_m3();
    mark(2);
    TRITD_HIP(hipStreamWaitEvent(st_, evSC_, 0));
    do_apply_C(GinvC_.p);
    TRITD_HIP(hipEventRecord(evCtC_, st_));
    TRITD_HIP(hipStreamWaitEvent(side_, evCtC_, 0));
    launch_gram(RP, Ch_.p, g_.n3p, CtC_.p, ctrl_, side_, true);
    solve(0, BtB_.p, CtC_.p, o_.lambda2, GinvA_.p, side_);
    TRITD_HIP(hipEventRecord(evSA_, side_));
    if (qi_) {
        launch_k5_full(k, /*fused_finish=*/true);
        return;
    }
    // the norm reduction and stop test of k ride in the next M1 (do_m1; fp32:
    // M2, do_m2), or flush_norms when the loop ends first
    mark(3);
    launch_k5_any(k, /*prologue=*/false);
    mark(4);
    norms_pending_ = true;
    pend_k_ = k;
}

// Single-stream iteration (fused_): every kernel on the main stream in
// dependency order, the R x R solves inside the launches they run beside
//   M1 -> apply A -> Gram A -> M2 (+ solve B) -> apply B -> Gram B ->
//   K2 (+ solve C) -> apply C -> Gram C -> K5 (+ solve A of k+1) -> norms
// One process per GPU: M2 -> AR(M2 | A^TA) -> solve B (k_solve_ns, main),
// AR(M3) after K2, AR(norms) after K5.
void Session::iterate_fused(int k) {
    const int RP = g_.RP;
    double* M2 = red1_.p;
    double* AtA = red1_.p + g_.n2 * RP;
    std::unique_ptr<Range> ph(new Range("update_A (:73-81)"));
    const bool defer = side_gram_ok(), defer_bc = side_gram_bc_ok();
    const bool ga_m2 = gram_a_in_m2();
    do_m1();
    const bool gA = ga_m2 ? (do_apply_A(GinvA_.p), false) : apply_gram_A(AtA, defer);
    ph.reset(new Range("update_B (:83-88)"));
    if (comm_ && comm_->active()) {
        if (ga_m2) {  // A^T A beside M2, for the all-reduce below
            SideSolve sg;
            sg.on = 1;
            sg.solve = 0;
            sg.R = g_.R;
            with_gram(sg, Ah_.p, g_.n1p, AtA, 0);
            launch_m2(g_, Wk_.p, AhT_.p, M2, ctrl_, st_, sg);
        } else {
            do_m2(M2);
        }
        // M1 .. M2 above ran before the stop test of iteration k-1: they
        // write only scratch and this iteration's A^ parity buffer.  The
        // all-reduce carries K5(k-1)'s norm partials; the finish of k-1
        // follows it, and every kernel after that checks its stop flag.
        const bool pend = norms_pending_;
        allreduce(red1_.p, red1_count() + (pend ? 2 * (int64_t)k5tail_ : 0));
        // the finish of k-1 and update_B's solve in one launch (the finish
        // runs first; the apply of B after it sees its stop flag)
        FinishArgs f;
        if (pend) {
            f.p = red1_.p + red1_count(); f.n = k5tail_; f.normD = normD_; f.k = pend_k_;
            f.tol = o_.tol; f.errHist = errHist_.p; f.errL = errL_.p; f.errO = errO_.p;
            f.ctrl = ctrl_; f.single = (int)f32_; f.clear = 1; f.on = 1;
            norms_pending_ = false;
        }
        solve(1, AtA, CtC_.p, o_.lambda2, GinvB_.p, st_, pend ? &f : nullptr);
    } else {
        // update_B's solve (A^TA of this iteration, C^TC) beside M2
        SideSolve sb;
        sb.P = AtA; sb.Q = CtC_.p; sb.alpha = o_.lambda2; sb.Ginv = GinvB_.p; sb.flags = ctrl_ + 2;
        sb.R = g_.R; sb.on = 1;
        if (gA) with_gram(sb, Ah_.p, g_.n1p, AtA, 0);
        launch_m2(g_, Wk_.p, AhT_.p, M2, ctrl_, st_, sb);
    }
    const bool gB = apply_gram_B(M2, defer_bc);
    ph.reset(new Range("update_C (:90-95)"));
    mark(1);
    SideSolve sc;  // update_C's solve (:93 ridge) beside K2
    sc.P = AtA; sc.Q = BtB_.p; sc.alpha = 1e-9; sc.Ginv = GinvC_.p; sc.flags = ctrl_ + 2;
    sc.R = g_.R; sc.on = 1;
    if (gB) with_gram(sc, Bh_.p, g_.n2, BtB_.p, 1);
    launch_m3(g_, T_.p, Ah_.p, Bh_.p, m3part_.p, red2_.p, ctrl_, st_, 0, -1, sc);
    mark(2);
    allreduce(red2_.p, red2_count());
    const bool gC = apply_gram_C(defer_bc);
    // the next update_A's solve (B^TB, C^TC of this iteration) beside K5
    ph.reset(new Range("fused update K5 (:38-59, :33)"));
    k5side_.P = BtB_.p; k5side_.Q = CtC_.p; k5side_.alpha = o_.lambda2; k5side_.Ginv = GinvA_.p;
    k5side_.flags = ctrl_ + 2; k5side_.R = g_.R; k5side_.on = 1;
    if (gC) with_gram(k5side_, Ch_.p, g_.n3p, CtC_.p, 1);
    if (comm_ && comm_->active()) {
        // the norm partials stay per workgroup in red1_'s tail: all-reduced
        // with the next iteration's M2 | A^TA (or by flush_norms)
        k5part_to_ = red1_.p + red1_count();
        mark(3);
        launch_k5_any(k, /*prologue=*/false);
        mark(4);
        k5part_to_ = nullptr;
        norms_pending_ = true;
        pend_k_ = k;
    } else {
        // the norm reduction and stop test of k ride in the next M1 (do_m1),
        // or flush_norms when the loop ends first
        mark(3);
        launch_k5_any(k, /*prologue=*/false);
        mark(4);
        norms_pending_ = true;
        pend_k_ = k;
    }
}

// Sharded iteration (one process per GPU).  The all-reduce
// of M2 + A^TA gates solve B, which stays on the critical path; the other two
// solves and the two replicated Grams run on the side stream:
//   main: M1 -> apply A -> Gram A -> M2 -> AR(M2, A^TA) -> solve B -> apply B
//         -> M3 -> AR(M3) -> apply C -> K5 -> AR(norms) -> finish
//   side: Gram B -> solve C (|| M3 + its AR) | Gram C -> solve A(k+1) (|| K5)
// Hazards as in iterate_overlapped: every buffer a side kernel reads is next
// written on the main stream only after an event recorded behind it.
void Session::iterate_sharded(int k) {
    const int RP = g_.RP;
    double* M2 = red1_.p;
    double* AtA = red1_.p + g_.n2 * RP;
    do_m1();
    TRITD_HIP(hipStreamWaitEvent(st_, evSA_, 0));
    do_apply_A(GinvA_.p);
    launch_gram(RP, Ah_.p, g_.n1p, AtA, ctrl_, st_);
    do_m2(M2);
    allreduce(red1_.p, red1_count());
    solve(1, AtA, CtC_.p, o_.lambda2, GinvB_.p, st_);
    do_apply_B(M2, GinvB_.p);
    TRITD_HIP(hipEventRecord(evBtB_, st_));
    TRITD_HIP(hipStreamWaitEvent(side_, evBtB_, 0));
    launch_gram(RP, Bh_.p, g_.n2, BtB_.p, ctrl_, side_, true);
    solve(2, AtA, BtB_.p, 1e-9, GinvC_.p, side_);  // :93 ridge
    TRITD_HIP(hipEventRecord(evSC_, side_));
    mark(1);
    do_m3();
    mark(2);
    allreduce(red2_.p, red2_count());
    TRITD_HIP(hipStreamWaitEvent(st_, evSC_, 0));
    do_apply_C(GinvC_.p);
    TRITD_HIP(hipEventRecord(evCtC_, st_));
    TRITD_HIP(hipStreamWaitEvent(side_, evCtC_, 0));
    launch_gram(RP, Ch_.p, g_.n3p, CtC_.p, ctrl_, side_, true);
    solve(0, BtB_.p, CtC_.p, o_.lambda2, GinvA_.p, side_);
    TRITD_HIP(hipEventRecord(evSA_, side_));
    launch_k5_full(k, /*fused_finish=*/false);
    allreduce(red3_.p, 2);
    phaseD(k);
}

void Session::phaseD(int k) {
    launch_finish(red3_.p, normD_, k, o_.tol, errHist_.p, errL_.p, errO_.p, ctrl_, f32_, st_);
}

void Session::maybe_print(int k) {
    if (!o_.disp || k % 10 != 0) return;
    flush_norms();
    if (comm_ && comm_->rank != 0) return;
    int ctrl[2];
    double eL, eO;
    TRITD_HIP(hipMemcpyAsync(ctrl, ctrl_, 2 * sizeof(int), hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipMemcpyAsync(&eL, errL_.p + (k - 1), sizeof(double), hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipMemcpyAsync(&eO, errO_.p + (k - 1), sizeof(double), hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipStreamSynchronize(st_));
    if (ctrl[1] != k) return;  // stopped earlier: MATLAB never reached iteration k
    char line[128];
    std::snprintf(line, sizeof line, "Iter %d, errL=%.2e, errO=%.2e", k, eL, eO);  // :61
    emit_line(line);
}

void Session::run(int iters) {
    TRITD_HIP(hipSetDevice(device_));
    for (int it = 0; it < iters; ++it) {
        const int k = next_iter();
        if (!k) break;
        if (timing_) {
            // slots: 0 iteration start, 1/2 K2, 3/4 K5, 5 iteration end; at
            // TRITD_TIMING_K5 only 3/4 exist (each record is a stream marker
            // that widens the gap to the next kernel by several us)
            const bool ar = comm_ && comm_->active();
            for (int e = 0; e < EV_SLOTS; ++e) {
                hipEvent_t ev = nullptr;
                if ((timing_ == TRITD_TIMING_ALL && (e < 6 || ar)) || e == 3 || e == 4)
                    TRITD_HIP(hipEventCreate(&ev));
                ev_.push_back(ev);
            }
            ev_iter_.push_back(k);
            mark(0);
        }
        ar_in_iter_ = 0;
        Range it_range("tritd:iteration");
        if (fused_) {
            iterate_fused(k);
        } else if (overlap_) {
            iterate_overlapped(k);
        } else if (shov_) {
            iterate_sharded(k);
        } else {
            phaseA(k);
            allreduce(red1_.p, red1_count());
            phaseB(k);
            allreduce(red2_.p, red2_count());
            phaseC(k);
            allreduce(red3_.p, 2);
            phaseD(k);
        }
        mark(5);
        ar_in_iter_ = EV_AR;  // all-reduces outside the iteration (a flush) are not timed
        maybe_print(k);
        maybe_dense_e(k);
    }
    flush_norms();  // the last iteration's stop test (errHist complete after every run)
}

void Session::harvest_timing() {
    for (size_t b = 0; b + EV_SLOTS <= ev_.size(); b += EV_SLOTS) {
        float it = 0, m3 = 0, k5 = 0;
        if (ev_[b]) TRITD_HIP(hipEventElapsedTime(&it, ev_[b], ev_[b + 5]));
        if (ev_[b + 1]) TRITD_HIP(hipEventElapsedTime(&m3, ev_[b + 1], ev_[b + 2]));
        TRITD_HIP(hipEventElapsedTime(&k5, ev_[b + 3], ev_[b + 4]));
        int nar = 0;
        for (int a = 0; a < EV_AR; ++a) {
            hipEvent_t e0 = ev_[b + 6 + 2 * a], e1 = ev_[b + 7 + 2 * a];
            if (!e0 || !e1 || hipEventQuery(e1) != hipSuccess) continue;  // not recorded this iteration
            float ms = 0;
            if (hipEventElapsedTime(&ms, e0, e1) == hipSuccess) {
                acc_ar_ += ms;
                ++nar;
            }
        }
        (void)hipGetLastError();  // an unrecorded pair is not an error
        if (nar > ar_per_iter_) ar_per_iter_ = nar;
        acc_it_ += it;
        acc_m3_ += m3;
        acc_k5_ += k5;
        ++acc_n_;
    }
    for (auto e : ev_)
        if (e) hip_quiet(hipEventDestroy(e));
    ev_.clear();
    ev_iter_.clear();
}

void Session::sync(int* done, int* stopped) {
    TRITD_HIP(hipSetDevice(device_));
    if (side_) TRITD_HIP(hipStreamSynchronize(side_));
    TRITD_HIP(hipStreamSynchronize(st_));
    if (!ev_.empty()) harvest_timing();
    int ctrl[3];
    TRITD_HIP(hipMemcpy(ctrl, ctrl_, 3 * sizeof(int), hipMemcpyDeviceToHost));
    if (ctrl[2] & 1) flags_ |= TRITD_FLAG_PINV_TOL;  // the pinv fallback dropped a value
    if (ctrl[2] & 2)  // k_solve_mw: a workgroup gave up waiting for a peer (never expected)
        throw Error(TRITD_ERR_HIP, "multi-workgroup R x R solve: a peer workgroup never arrived");
    if (done) *done = ctrl[1];
    if (stopped) *stopped = ctrl[0];
}

void Session::mark(int slot) {
    if (!timing_) return;
    hipEvent_t e = ev_[ev_.size() - EV_SLOTS + slot];
    if (e) TRITD_HIP(hipEventRecord(e, st_));
}

void Session::set_timing(int level) {
    timing_ = level;
    acc_k5_ = acc_m3_ = acc_it_ = acc_ar_ = 0;
    acc_n_ = ar_per_iter_ = 0;
}

void Session::comm_ms(double* allreduce_ms, int* per_iter) {
    const double n = acc_n_ ? (double)acc_n_ : 1.0;
    if (allreduce_ms) *allreduce_ms = acc_ar_ / n;
    if (per_iter) *per_iter = ar_per_iter_;
}

void Session::kernel_ms(double* k5, double* m3, double* it, int* samples) {
    const double n = acc_n_ ? (double)acc_n_ : 1.0;
    if (k5) *k5 = acc_k5_ / n;
    if (m3) *m3 = acc_m3_ / n;
    if (it) *it = acc_it_ / n;
    if (samples) *samples = acc_n_;
}

void Session::get(double* A, double* B, double* C, void* O, void* E, int64_t ldOE,
                  double* errHist, int* iters, bool populated) {
    int done = 0, stopped = 0;
    sync(&done, &stopped);
    if (A) {  // the A of the last finished iteration (its parity buffer)
        std::vector<double> h(AhB_[done & 1].n);
        TRITD_HIP(hipMemcpy(h.data(), finished_ah(done), h.size() * sizeof(double),
                            hipMemcpyDeviceToHost));
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
    if (O && g_.n1l > 0 && done > 0) {  // O of iteration `done` from D, Y_L, T (K5 does not store it)
        if (f32_)
            launch_o_fixup32(g_, D_.f(), YL_.f(), T_.f(), (float)(1.0 / mu_[(size_t)done]), O_.f(),
                             st_);
        else
            launch_o_fixup(g_, D_.p, YL_.p, T_.p, 1.0 / mu_[(size_t)done], O_.p, st_);
    }
    if (E && g_.n1l > 0) {  // E lives in compact form
        if (f32_)
            launch_ce_expand32(g_, CE_.f(), E_.f(), st_);
        else if (!de_)  // (dense-E mode: E^(done) is dense already)
            launch_ce_expand(g_, ce_buf(done), e_buf(done), st_);
    }
    if ((O || E) && g_.n1l > 0) {
        // Round 6 (the drop-in's one-shot call): the host
        // pages of both outputs are populated on two threads while the device
        // rebuilds O, expands E and converts both to column-major, each into
        // a buffer of its own; the D2H copies (PCIe, ~30 GB/s on the boxes
        // measured: profiles/round6/pcie_probe.txt) then run back to back
        // into pages that no longer fault.  (Fresh pages cost the copy a
        // factor 2.5: 12.3 vs 30.2 GB/s.)
        const size_t nb = (size_t)(g_.n1l * g_.n2 * g_.n3) * es_;
        const bool whole = ldOE == g_.n1l;  // a whole tensor (one-shot calls): contiguous copies
        std::vector<std::thread> pop;
        pop.reserve(2);
        struct Join {
            std::vector<std::thread>& t;
            ~Join() {
                for (auto& x : t)
                    if (x.joinable()) x.join();
            }
        } join{pop};
        if (whole && !populated)
            for (void* dst : {O, E})
                if (dst) {
                    try {  // (an optimisation: without the thread the copy faults the pages in)
                        pop.emplace_back([dst, nb] { populate_output_threads(dst, nb, 8); });
                    } catch (const std::system_error&) {
                    }
                }
        DBuf tmp[2];
        int q = 0;
        for (auto pr : {std::make_pair(O, O_.p), std::make_pair(E, e_buf(done))}) {
            if (!pr.first) continue;
            tmp[q].alloc_bytes(nb);
            if (f32_)
                launch_from_tm32(g_, reinterpret_cast<float*>(pr.second), tmp[q].f(), g_.n1l, st_);
            else
                launch_from_tm(g_, pr.second, tmp[q].p, g_.n1l, st_);
            ++q;
        }
        for (auto& x : pop) x.join();
        q = 0;
        for (void* dst : {O, E}) {
            if (!dst) continue;
            if (whole)
                TRITD_HIP(hipMemcpyAsync(dst, tmp[q].p, nb, hipMemcpyDeviceToHost, st_));
            else
                TRITD_HIP(hipMemcpy2DAsync(dst, ldOE * es_, tmp[q].p, g_.n1l * es_, g_.n1l * es_,
                                           (size_t)(g_.n2 * g_.n3), hipMemcpyDeviceToHost, st_));
            ++q;
        }
        TRITD_HIP(hipStreamSynchronize(st_));
    }
    if (errHist && done > 0)
        TRITD_HIP(hipMemcpy(errHist, errHist_.p, (size_t)done * sizeof(double), hipMemcpyDeviceToHost));
    if (iters) *iters = done;
}

void Session::counters(int64_t* dense_tiles_total, int64_t* tiles_per_launch) {
    TRITD_HIP(hipSetDevice(device_));
    unsigned long long h[DENSE_SLOTS] = {};
    TRITD_HIP(hipStreamSynchronize(st_));
    TRITD_HIP(hipMemcpy(h, dense_tiles(), sizeof h, hipMemcpyDeviceToHost));
    unsigned long long t = 0;
    for (unsigned long long x : h) t += x;
    if (dense_tiles_total) *dense_tiles_total = (int64_t)t;
    if (tiles_per_launch) *tiles_per_launch = g_.Ntm / 256;
}

void Session::rre_parts(const void* dX, int64_t ldX, double* num, double* den) {
    TRITD_HIP(hipSetDevice(device_));
    DBuf Xd, part, out;
    const double* src = static_cast<const double*>(dX);
    if (f32_) {  // the reference tensor in single: widen (exactly) to double
        const int64_t cnt = (g_.n2 * g_.n3 - 1) * ldX + g_.n1l;
        Xd.alloc((size_t)cnt);
        launch_widen(static_cast<const float*>(dX), cnt, Xd.p, st_);
        src = Xd.p;
    }
    const int grid = tp_grid(g_);
    part.alloc(2 * (size_t)grid);
    out.alloc(2);
    int done = 0;
    sync(&done, nullptr);
    const double* ah = finished_ah(done);
    // X(i,j,t) of the shard at src[i + ldX*(j + n2*t)]
    if (qi_) {
        launch_qi_h(g_, g_.r, ah, Bh_.p, H_.p, nullptr, st_);
        launch_tp(g_, H_.p, ones_.p, ChT_.p, nullptr, src, part.p, 1, ldX, ldX * g_.n2, st_,
                  g_.n1p * g_.RP, 0);
    } else {
        launch_tp(g_, ah, Bh_.p, ChT_.p, nullptr, src, part.p, 1, ldX, ldX * g_.n2, st_);
    }
    launch_reduce_pairs(part.p, grid, out.p, nullptr, st_);
    double h[2];
    TRITD_HIP(hipMemcpyAsync(h, out.p, sizeof h, hipMemcpyDeviceToHost, st_));
    TRITD_HIP(hipStreamSynchronize(st_));
    *num = h[0];
    *den = h[1];
}

}  // namespace tritd
