// Device-resident TriTD-ADMM session (one mode-1 shard on one GPU).
#pragma once

#include <rccl/rccl.h>

#include <functional>
#include <thread>
#include <vector>

#include "kernels.h"

namespace tritd {
class GroupAbort;
}

struct tritd_comm {
    ncclComm_t comm = nullptr;             // RCCL (tritd_comm_create; group_comms)
    tritd_allreduce_fn host_fn = nullptr;  // or a host transport (tritd_comm_create_host)
    void* host_user = nullptr;
    int nranks = 1, rank = 0, device = 0;
    // a shard of a device group driven by run_threaded: its non-blocking RCCL
    // communicator is used only through the group's abort protocol (group.h)
    tritd::GroupAbort* group = nullptr;
    bool active() const { return comm != nullptr || host_fn != nullptr || group != nullptr; }
};

namespace tritd {

// Host output buffers of a device-to-host copy: populate their pages in
// parallel first (MADV_HUGEPAGE, then MADV_POPULATE_WRITE on up to 16
// threads; content unchanged).
// A fresh array (numpy zeros, mxCreate*) is mapped lazily, and the copy into
// it then runs at the single-threaded page-fault rate (~16 GB/s measured
// against ~55 GB/s into populated memory).  No-op below 64 MB.
void populate_output(void* p, size_t bytes);
void populate_output_threads(void* p, size_t bytes, unsigned max_threads);

// The one-shot calls' outputs O and E (whole tensors in the caller's memory)
// faulted in on a background thread while the iterations run on the device:
// a D2H copy into pages that fault runs at 12.6 instead of 30 GB/s
// (profiles/round6/pcie_probe.txt), and populating them in get() took as long
// as the copies.  join() before Session::get(..., populated = true).
class OutputPrefault {
public:
    OutputPrefault(void* O, void* E, size_t bytes);
    ~OutputPrefault() { join(); }
    void join();

private:
    std::thread t_;
};

// In-place all-reduce (sum, or max) of `count` doubles over the comm's ranks,
// ordered on stream st: ncclAllReduce, or the host transport (drains st).
void comm_allreduce(tritd_comm* c, double* buf, int64_t count, bool max, hipStream_t st);

// A device buffer of doubles; freed on destruction.
struct DBuf {
    double* p = nullptr;
    size_t n = 0;
    bool owned = true;  // false: a view into another DBuf
    DBuf() = default;
    DBuf(const DBuf&) = delete;
    DBuf& operator=(const DBuf&) = delete;
    ~DBuf() {
        if (p && owned) hip_quiet(hipFree(p));
    }
    void alloc(size_t count) {
        n = count;
        TRITD_HIP(hipMalloc(&p, (count ? count : 1) * sizeof(double)));
    }
    void alloc_bytes(size_t bytes) { alloc((bytes + sizeof(double) - 1) / sizeof(double)); }
    void release() {
        if (p && owned) hip_quiet(hipFree(p));
        p = nullptr;
        n = 0;
    }
    float* f() const { return reinterpret_cast<float*>(p); }
    size_t bytes() const { return n * sizeof(double); }
};

// Host-side layout conversions between the reference shapes and the device
// factor layout (common.h / DESIGN.md §3).
void pack_A(const Geom& g, const double* A, std::vector<double>& Ah, std::vector<double>& AhT);
void pack_B(const Geom& g, const double* B, std::vector<double>& Bh);
void pack_C(const Geom& g, const double* C, std::vector<double>& Ch, std::vector<double>& ChT);
void unpack_A(const Geom& g, const std::vector<double>& Ah, double* A);
void unpack_B(const Geom& g, const std::vector<double>& Bh, double* B);
void unpack_C(const Geom& g, const std::vector<double>& Ch, double* C);

class Session {
   public:
    // D: double, or float when flags has TRITD_SESSION_F32 (the fp32 data path)
    Session(int device, const void* D, int64_t ldD, int64_t n1, int64_t n2, int64_t n3, int64_t i0,
            int64_t i1, int r, const tritd_opts& o, const double* A0, const double* B0,
            const double* C0, tritd_comm* comm, uint32_t flags, hipStream_t shared_stream = nullptr,
            bool defer_normD = false);
    ~Session();

    // Enqueue iterations (full collective schedule; used without a virtual group)
    void run(int iters);
    void sync(int* done, int* stopped);
    // TRITD_FLAG_* raised by the device so far (read at every sync)
    uint32_t flags() const { return flags_; }
    // O, E: double, or float for an fp32 session.  populated: the caller has
    // already faulted in the pages of whole-tensor O and E (OutputPrefault)
    void get(double* A, double* B, double* C, void* O, void* E, int64_t ldOE, double* errHist,
             int* iters, bool populated = false);
    // dX: device tensor of the session's data type
    void rre_parts(const void* dX, int64_t ldX, double* num, double* den);
    bool is_f32() const { return f32_; }
    void counters(int64_t* dense_tiles_total, int64_t* tiles_per_launch);
    void k5_profile(int* dense_streams, int* slot_accesses) const {
        // dense-E mode: E^(k), E^(k-1) read and E^(k+1) written densely, no slots
        *dense_streams = de_ ? 7 : (dy_ ? 4 : 6);  // (fp32: 6, Y_O stored)
        *slot_accesses = de_ ? 0 : (dy_ ? 3 : 2);
    }
    bool dense_e() const { return de_; }
    void set_timing(int level);  // 0 off, TRITD_TIMING_ALL, TRITD_TIMING_K5
    void kernel_ms(double* k5, double* m3, double* it, int* samples);
    // per timed iteration (TRITD_TIMING_ALL, with a communicator): ms inside
    // the iteration's all-reduces (issue to completion on the session stream,
    // so it includes waiting for the slowest rank) and their count
    void comm_ms(double* allreduce_ms, int* per_iter);
    const std::vector<double>& probe_ms() const { return probe_ms_; }
    int probe_pick() const { return probe_pick_; }

    // --- phase interface (virtual shard groups drive these directly) ------
    // Returns false when iteration k is beyond maxIter (nothing enqueued).
    int next_iter();  // reserves the next iteration number (or 0)
    void phaseA(int k);  // M1, solve A, A^TA partial, M2 partial -> red1
    void phaseB(int k);  // solve B, B^TB, M3 partial -> red2
    void phaseC(int k);  // solve C, C^TC, K5, norm partial -> red3
    void phaseD(int k);  // errHist / stop test
    double* red1() { return red1_.p; }
    double* red2() { return red2_.p; }
    double* red3() { return red3_.p; }
    int64_t red1_count() const { return g_.n2 * g_.RP + (int64_t)g_.RP * g_.RP; }
    int64_t red2_count() const { return g_.n3p * g_.RP; }
    hipStream_t stream() const { return st_; }
    // normD support for groups: local sum of squares in red3[0]
    void set_normD_from_red3();
    void maybe_print(int k);
    const Geom& geom() const { return g_; }
    int device() const { return device_; }

   private:
    void allreduce(double* buf, int64_t count);
    // single-GPU schedule: the three R x R solves run on a side stream, each
    // overlapped with the big kernel that precedes its consumer
    void iterate_overlapped(int k);
    // one process per GPU with RCCL: the phase order with the Grams of B, C
    // and the solves of C, A(k+1) on the side stream
    void iterate_sharded(int k);
    // single stream, no events (default for the fp64 CP model at RP <= 64):
    // the solves of update_C and of the next update_A run in an extra
    // workgroup of K2 / K5 (sweep.h), solve B on the main stream; with a
    // communicator the same order with its three all-reduces
    void iterate_fused(int k);
    bool fused_ = false;
    // K5's norm-partial count (its workgroups; the fp32 rank-split K5 has more)
    int k5n() const { return f32_ ? k5_parts32(g_) : k5_grid(g_) * g_.tsplit; }
    // pairs in red1_'s norm-partial tail: the largest k5n() over the ranks
    // (shards of different heights launch different K5 grids, and every rank
    // must all-reduce the same count); set by agree_counts()
    int k5tail_ = 0;
    void agree_counts();
    SideSolve k5side_;  // the side solve of the next K5 launch
    // communicator: K5's norm partials of iteration pend_k_ wait in red1_'s
    // tail for the next iteration's first all-reduce (one all-reduce fewer
    // per iteration); flush_norms() all-reduces and finishes them alone
    bool norms_pending_ = false;
    int pend_k_ = 0;
    double* k5part_to_ = nullptr;  // where the next K5 writes its partials (null: k5part_)
    void flush_norms();
    bool shov_ = false;
    void create_streams(hipStream_t shared_stream);
    void launch_k5_full(int k, bool fused_finish);
    bool small_ag(int64_t rows) const;
    bool apply_gram_A(double* AtA, bool defer = false);
    bool apply_gram_B(const double* M2, bool defer = false);
    bool apply_gram_C(bool defer = false);
    bool side_gram_ok() const;
    bool side_gram_bc_ok() const;
    bool gram_a_in_m2() const;
    // the applies take the generic kernel (launch_apply_gen): fp32, or RP > 64
    bool gen_apply() const { return f32_ || g_.RP > 64; }
    FinishArgs take_finish();
    bool overlap_ = false;
    hipStream_t side_ = nullptr;
    hipEvent_t evAtA_ = nullptr, evBtB_ = nullptr, evCtC_ = nullptr;
    hipEvent_t evSA_ = nullptr, evSB_ = nullptr, evSC_ = nullptr;
    DBuf GinvA_, GinvB_, GinvC_;
    // candidate pools timed with K5's access pattern; `overlap` (the host
    // copy of D) runs while the probe kernels do
    double* probe_pool(size_t pool_bytes, size_t slot, size_t stagger,
                       std::function<void()> overlap);
    DBuf dstage_;  // column-major staging of a host D (creation only)
    std::vector<double> probe_ms_;  // probe time of each candidate pool (ms)
    int probe_pick_ = 0;
    void upload_factors(const double* A0, const double* B0, const double* C0);
    IterScalars scalars(int k) const;
    IterScalars32 scalars32(int k) const;
    // data-type dispatch of the per-iteration kernels
    void do_m1();
    void do_m2(double* M2);
    void do_m3();
    void do_m3_qi();
    void do_apply_A(double* Ginv);
    void do_apply_B(const double* M2, double* Ginv);
    void do_apply_C(double* Ginv);
    void launch_k5_any(int k, bool prologue);
    bool f32_ = false;
    size_t es_ = sizeof(double);  // bytes per element of D, O, E, Y_L, Y_O, T, W, M1
    DBuf ChF_;                    // C^ in single (fp32 path)

    int device_;
    hipStream_t st_ = nullptr;
    bool own_stream_ = false;
    Geom g_;
    tritd_opts o_;
    tritd_comm* comm_;
    std::vector<double> mu_;  // mu_[k-1] = muL = muO of iteration k
    double normD_ = 0.0;
    int k_enq_ = 0;

    DBuf pool_;  // declared first: destroyed after the views into it
    DBuf D_, O_, E_, YL_, YO_, T_, Wk_;
    DBuf CE_;  // compact E slots (common.h)
    // derived Y_O (k_admm.hip, fp64 default, TRITD_DY=0 disables): E^(k) lives
    // in compact buffer k % 2 (CE_, CE2_) and dense buffer k % 2 (E_, and the
    // pool slot of Y_O, which is not stored in this mode)
    bool dy_ = false;
    // dense-E mode of K5 (k_admm.hip DE): de_mode_ -1 automatic (switch once E
    // has turned dense: checked after iterations 8 and 24), 0 never, 1 from the
    // start (TRITD_DENSE_E); de_prev_* = the dense-tile count at the last check
    bool de_ = false;
    int de_mode_ = -1;
    int64_t de_prev_ = 0;
    int de_prev_k_ = 0;
    bool de_eligible() const { return dy_ && !f32_ && !qi_ && g_.RP <= 64; }
    void maybe_dense_e(int k);
    DBuf CE2_;
    double* ce_buf(int k) const { return (dy_ && (k & 1)) ? CE2_.p : CE_.p; }
    double* e_buf(int k) const { return (dy_ && (k & 1)) ? YO_.p : E_.p; }
    // A^ (and its transpose) by iteration parity: iteration k writes
    // AhB_[k&1], so the A of the last finished iteration survives a next
    // iteration that has already started (the speculative start of
    // iterate_fused with a communicator); Ah_/AhT_ are views of the current one
    DBuf AhB_[2], AhTB_[2];
    // Ah_/AhT_ are valid only while iterations are being enqueued: after a
    // run they point at the parity of the last ENQUEUED iteration, which after
    // a stop (or a speculative iteration of the comm schedule) holds a newer
    // or partial A.  Readers after run() use finished_ah().
    DBuf Ah_, AhT_, Bh_, Ch_, ChT_, M1_, BtB_, CtC_;
    void set_ah(int k);
    // A^ of the last finished iteration `done` (as returned by sync)
    const double* finished_ah(int done) const { return AhB_[done & 1].p; }
    // Qi model (opts.model = TRITD_MODEL_QI, k_qi.hip): H = the Qi mode-3 design
    // matrix by rows ij (K2/K5 Khatri-Rao operand), an all-ones RP x RP block
    // (the Hadamard factor of the solve and the B operand of the KR product),
    // and the design Grams of the three solves
    bool qi_ = false;
    DBuf H_, ones_, GqA_, GqB_, GqC_;
    // inv(design Gram + alpha I) of update_A (mode 0), _B (1), _C (2)
    void solve(int mode, const double* P, const double* Q, double alpha, double* out,
               hipStream_t s, const FinishArgs* fin = nullptr);
    DBuf red1_, red2_, red3_;
    DBuf k5part_, m3part_, sqpart_;
    DBuf errHist_, errL_, errO_;
    uint32_t flags_ = 0;
    bool probe_ = false;  // TRITD_SESSION_PROBE: time candidate pools at creation
    int* ctrl_ = nullptr;  // [0] stop, [1] k done, [2] pinv-tolerance flag, then DENSE_SLOTS u64 dense-E counters
    unsigned long long* dense_tiles() const {
        return reinterpret_cast<unsigned long long*>(ctrl_ + 4);
    }

    int timing_ = 0;
    void mark(int slot);  // record timing event `slot` of this iteration (if it exists)
    // per timed iteration: EV_SLOTS events — 0 start, 1/2 K2, 3/4 K5, 5 end,
    // then a (before, after) pair per all-reduce of the iteration
    static constexpr int EV_AR = 4;  // all-reduce pairs timed per iteration
    static constexpr int EV_SLOTS = 6 + 2 * EV_AR;
    std::vector<hipEvent_t> ev_;
    std::vector<int> ev_iter_;
    int ar_in_iter_ = 0;  // all-reduces issued so far in the current iteration
    double acc_k5_ = 0, acc_m3_ = 0, acc_it_ = 0, acc_ar_ = 0;
    int acc_n_ = 0, ar_per_iter_ = 0;
    void harvest_timing();
};

}  // namespace tritd
