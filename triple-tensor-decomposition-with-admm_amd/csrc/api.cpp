// C ABI of libtritd.so (include/tritd.h).  Every entry point validates its
// arguments the way the reference fails (missing opts field, bad unfold
// mode, >3-D data), converts exceptions into tritd_status + a thread-local
// message, and never writes its inputs.
#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "als.h"
#include "group.h"
#include "solver.h"

using namespace tritd;

namespace {
thread_local std::string g_last_error;
thread_local uint32_t g_last_flags = 0;  // TRITD_FLAG_* of the last one-shot solve
tritd_print_fn g_print = nullptr;
void* g_print_user = nullptr;
std::mutex g_mutex;  // calls are not re-entrant (SURVEY.md §8b Threading)

tritd_status fail(tritd_status s, const std::string& m) {
    g_last_error = m;
    g_last_flags = 0;
    return s;
}

// set once this library has touched the HIP runtime (pick_device): before
// that, an entry point does not call into HIP at all, so a host-only call
// (tritd_version, a host-transport tritd_comm_info, ...) leaves the process
// without a HIP runtime initialised
std::atomic<bool> g_hip_used{false};

template <class F>
tritd_status guarded(F&& f) {
    try {
        // hipGetLastError (TRITD_CHECK_LAUNCH) reports the thread's last error
        // from any caller: one left by an earlier, unrelated call (the host
        // program's, or an ignored failure in a destructor) is not this call's
        if (g_hip_used.load(std::memory_order_relaxed)) (void)hipGetLastError();
        f();
        g_last_error.clear();
        return TRITD_OK;
    } catch (const Error& e) {
        return fail(e.code, e.what());
    } catch (const std::bad_alloc&) {
        return fail(TRITD_ERR_NOMEM, "host allocation failed");
    } catch (const std::exception& e) {
        return fail(TRITD_ERR_HIP, e.what());
    }
}

void check_opts(const tritd_opts* o) {
    if (!o) throw Error(TRITD_ERR_OPTS, "opts is NULL");
    // triple_decomp_ADMM.m:16-20 reads the fields in this order
    static const struct {
        uint32_t bit;
        const char* name;
    } fields[] = {{TRITD_OPT_MU, "mu"},         {TRITD_OPT_RHO, "rho"},   {TRITD_OPT_LAMBDA, "lambda"},
                  {TRITD_OPT_LAMBDA2, "lambda2"}, {TRITD_OPT_MAXITER, "maxIter"},
                  {TRITD_OPT_TOL, "tol"},       {TRITD_OPT_DISP, "disp"}};
    for (const auto& f : fields)
        if (!(o->present & f.bit))
            throw Error(TRITD_ERR_OPTS, std::string("Reference to non-existent field '") + f.name + "'.");
}

// triple_decomp_ALS.m:2-3 reads only these two, in this order
void check_als_opts(const tritd_opts* o) {
    if (!o) throw Error(TRITD_ERR_OPTS, "opts is NULL");
    if (!(o->present & TRITD_OPT_MAXITER))
        throw Error(TRITD_ERR_OPTS, "Reference to non-existent field 'maxIter'.");
    if (!(o->present & TRITD_OPT_TOL))
        throw Error(TRITD_ERR_OPTS, "Reference to non-existent field 'tol'.");
}

tritd_opts normalized(const tritd_opts* o) {
    tritd_opts c = *o;
    if (c.maxIter < 0) c.maxIter = 0;  // for k = 1:maxIter runs zero times
    return c;
}

void check_dims(int64_t n1, int64_t n2, int64_t n3, int32_t r, bool f32 = false) {
    if (n1 <= 0 || n2 <= 0 || n3 <= 0) throw Error(TRITD_ERR_ARG, "tensor dimensions must be positive");
    if (r <= 0) throw Error(TRITD_ERR_ARG, "rank r must be positive");
    // wide = the ADMM paths (fp32 and fp64 r <= 16); ALS / test.m solver kernels stop at r = 8
    if (!f32 && r > 8) throw Error(TRITD_ERR_UNSUPPORTED, "this path supports r <= 8 (R = r^2 <= 64)");
    if (f32 && r > 16) throw Error(TRITD_ERR_UNSUPPORTED, "r <= 16 (R = r^2 <= 256)");
}

void need(const void* p, const char* what) {
    if (!p) throw Error(TRITD_ERR_ARG, std::string(what) + " is NULL");
}

// first HIP use of an entry point: from here on guarded() clears the
// thread's stale HIP error before each call; this call's is cleared now
void hip_entry() {
    if (!g_hip_used.exchange(true, std::memory_order_relaxed)) (void)hipGetLastError();
}

int pick_device(int32_t device) {
    hip_entry();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        throw Error(TRITD_ERR_NODEV, "no HIP device visible (libtritd has no CPU fallback)");
    int d = device;
    if (d < 0) TRITD_HIP(hipGetDevice(&d));
    if (d >= n) throw Error(TRITD_ERR_NODEV, "device index out of range");
    hipDeviceProp_t prop;
    TRITD_HIP(hipGetDeviceProperties(&prop, d));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        throw Error(TRITD_ERR_NODEV, std::string("libtritd is built for gfx950, device is ") + prop.gcnArchName);
    TRITD_HIP(hipSetDevice(d));
    return d;
}

hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Device set of the one-shot entry points (tritd_set_devices), and the RCCL
// communicators of a set of distinct devices (group_comms): created on
// first use, kept in this process-global context until the set changes or
// tritd_shutdown (SURVEY.md §8b Ownership).
std::vector<int> g_devices;
std::vector<int> g_comm_devs;
std::vector<ncclComm_t> g_comms;

// Scratch of the device-form products (packed factor copies), kept per
// (device, stream) and grown on demand, so that a call returns without
// waiting for its kernels (tritd.h: device forms do not synchronise): calls on
// one stream are ordered by it and reuse its buffers.  Heap-held and never
// destroyed at exit (the HIP runtime may be gone by then); tritd_shutdown
// frees it.  (Stream-ordered hipMallocAsync scratch on the null stream read
// back as zeros on a repeated call on ROCm 7.2: tools/rounds/r4/iso_tp.sh, round 4.)
// The entry's `done` event marks the end of the last call's kernels: a call
// makes its stream wait on it (device side) before overwriting the buffers,
// which orders it after that call even when a destroyed stream's handle is
// reused.
//
// The host never waits on `done` (hipEventSynchronize / hipEventQuery): the
// stream it was last recorded on may be one the caller has destroyed since,
// and on ROCm 7.2 both calls read the event's stream object without checking
// that it is alive — if the freed memory holds "capture active" in the
// stream's capture-status word, they write "invalidated" into it and return
// hipErrorCapturedEvent ("operation not permitted on an event last recorded
// in a capturing stream"; libamdhip64 7.2.70200, hipEventSynchronize at
// 0x9a552..0x9ac90, hipEventQuery at 0x99b2c..0x99cd0).  That is round 5's
// intermittent failure (profiles/round5/gpu_tests_null_stream_wait_failure.
// log.txt): test_gpu_devprod.py left 16 entries of 24 destroyed streams; the
// next null-stream product evicted one with an unchecked
// hipEventSynchronize(victim->done), whose error stayed in the thread's last
// error and failed the following launch check.  hipStreamWaitEvent checks the
// recording stream's handle before using it, so the device-side wait is
// safe.  Host-side waits are now hipStreamSynchronize on the caller's (live)
// stream after that wait, or hipDeviceSynchronize where no stream of the
// entry is known (eviction, tritd_shutdown).  DESIGN.md §6.
// Bounded: at most SCRATCH_CAP entries; a new (device, stream)
// beyond that evicts the least recently used entry after the device has
// drained.  Each entry has its own lock, held over one call's enqueue (two
// host threads on one stream would otherwise interleave their packs and
// products); the map's lock is held only to find, insert or evict an entry,
// so calls on different streams do not serialise.
struct ScratchSet {
    std::array<DBuf, 5> buf;
    hipEvent_t done = nullptr;
    std::mutex m;
    uint64_t used = 0;  // LRU stamp (under g_scratch_mutex)
    int busy = 0;       // calls holding or waiting for m (under g_scratch_mutex)
    ~ScratchSet() {
        // (a destructor cannot report; a failure must not stay behind as the
        // thread's last error either, or the next launch check would report it)
        if (done && hipEventDestroy(done) != hipSuccess) (void)hipGetLastError();
    }
};
constexpr size_t SCRATCH_CAP = 16;
std::mutex g_scratch_mutex;
std::map<std::pair<int, hipStream_t>, std::unique_ptr<ScratchSet>>* g_scratch = nullptr;
uint64_t g_scratch_clock = 0;

// One call's hold on the (device, stream) entry: its lock for the enqueue.
class ScratchLease {
public:
    explicit ScratchLease(hipStream_t st) : st_(st) {
        int dev = 0;
        TRITD_HIP(hipGetDevice(&dev));
        {
            std::lock_guard<std::mutex> lk(g_scratch_mutex);
            if (!g_scratch) g_scratch = new std::map<std::pair<int, hipStream_t>, std::unique_ptr<ScratchSet>>();
            auto& slot = (*g_scratch)[{dev, st}];
            if (!slot) {
                evict_locked();
                slot.reset(new ScratchSet());
            }
            s_ = slot.get();
            s_->used = ++g_scratch_clock;
            ++s_->busy;
        }
        // from here on the destructor owns the busy count: a HIP call below
        // that throws must not leave the entry busy for good
        try {
            lk_ = std::unique_lock<std::mutex>(s_->m);
            if (!s_->done) TRITD_HIP(hipEventCreateWithFlags(&s_->done, hipEventDisableTiming));
            else TRITD_HIP(hipStreamWaitEvent(st, s_->done, 0));
        } catch (...) {
            release();
            throw;
        }
    }
    ~ScratchLease() { release(); }
    ScratchSet& set() { return *s_; }
    hipStream_t stream() const { return st_; }

private:
    void release() {
        if (!s_) return;
        if (lk_.owns_lock()) lk_.unlock();
        std::lock_guard<std::mutex> lk(g_scratch_mutex);
        --s_->busy;
        s_ = nullptr;
    }
    // the least recently used idle entry leaves once the map is full; its
    // last product may still read the buffers (and its stream may be gone):
    // drain the device, then free
    static void evict_locked() {
        if (g_scratch->size() < SCRATCH_CAP) return;
        auto victim = g_scratch->end();
        for (auto it = g_scratch->begin(); it != g_scratch->end(); ++it)
            if (it->second && it->second->busy == 0 &&
                (victim == g_scratch->end() || it->second->used < victim->second->used))
                victim = it;
        if (victim == g_scratch->end()) return;  // all in use: grow past the cap
        TRITD_HIP(hipDeviceSynchronize());
        g_scratch->erase(victim);
    }
    hipStream_t st_ = nullptr;
    ScratchSet* s_ = nullptr;
    std::unique_lock<std::mutex> lk_;
};

// buffer `slot` of the lease's entry, grown on demand: the stream already
// waits for the entry's last call (the lease), so once the stream has drained
// no kernel reads the old buffer
double* scratch(ScratchLease& lease, int slot, size_t count) {
    DBuf& b = lease.set().buf[slot];
    if (b.p && b.n < count) {
        TRITD_HIP(hipStreamSynchronize(lease.stream()));
        double* old = b.p;
        b.p = nullptr;
        b.n = 0;
        TRITD_HIP(hipFree(old));
    }
    if (!b.p) b.alloc(count);
    return b.p;
}

void drop_scratch() {
    std::lock_guard<std::mutex> lk(g_scratch_mutex);
    if (!g_scratch || g_scratch->empty()) return;
    // the last product on each stream may still read the buffers, and the
    // streams may be gone: drain the device once
    if (hipDeviceSynchronize() != hipSuccess) (void)hipGetLastError();
    for (auto it = g_scratch->begin(); it != g_scratch->end();) {
        if (it->second && it->second->busy) {  // a call on another thread holds it
            ++it;
            continue;
        }
        it = g_scratch->erase(it);
    }
}

// Wait out a non-blocking communicator's "in progress" state (its
// initialisation, an enqueue, a finalize); any other state is returned.
ncclResult_t nccl_settle(ncclComm_t c) {
    ncclResult_t a = ncclInProgress;
    while (a == ncclInProgress) {
        const ncclResult_t q = ncclCommGetAsyncError(c, &a);
        if (q != ncclSuccess) return q;
        if (a == ncclInProgress) std::this_thread::yield();
    }
    return a;
}

void drop_comms() {
    for (ncclComm_t c : g_comms)
        if (c) {
            const ncclResult_t f = ncclCommFinalize(c);
            if (f == ncclSuccess || f == ncclInProgress) (void)nccl_settle(c);
            (void)ncclCommDestroy(c);
        }
    g_comms.clear();
    g_comm_devs.clear();
}

// The communicators of a set of distinct devices: what ncclCommInitAll
// builds, but NON-BLOCKING (config.blocking = 0), so that no call of a shard
// thread waits inside RCCL for a peer — the device group's abort protocol
// (group.h: GroupAbort) relies on it.  Created from this thread in one group.
void group_comms(const std::vector<int>& devs) {
    if (g_comm_devs == devs && !g_comms.empty()) return;
    drop_comms();
    const int P = (int)devs.size();
    ncclUniqueId id;
    ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) throw Error(TRITD_ERR_RCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
    std::vector<ncclComm_t> cs((size_t)P, nullptr);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    // nothing inside the group throws: a failure is recorded, the
    // group is always closed, and the communicators it started are aborted
    hipError_t he = hipSuccess;
    r = ncclGroupStart();
    for (int p = 0; p < P && (r == ncclSuccess || r == ncclInProgress); ++p) {
        he = hipSetDevice(devs[p]);
        if (he != hipSuccess) {
            (void)hipGetLastError();
            break;
        }
        r = ncclCommInitRankConfig(&cs[p], P, id, p, &cfg);
    }
    const ncclResult_t re = ncclGroupEnd();
    if (r == ncclInProgress) r = ncclSuccess;
    if (r == ncclSuccess && re != ncclInProgress) r = re;
    for (int p = 0; p < P && r == ncclSuccess && he == hipSuccess; ++p)
        if (cs[p]) r = nccl_settle(cs[p]);
    if (r != ncclSuccess || he != hipSuccess) {
        for (ncclComm_t c : cs)
            if (c) (void)ncclCommAbort(c);
        if (he != hipSuccess)
            throw Error(TRITD_ERR_HIP, std::string("hipSetDevice (device group): ") + hipGetErrorString(he));
        throw Error(TRITD_ERR_RCCL, std::string("ncclCommInitRankConfig (device group): ") + ncclGetErrorString(r));
    }
    g_comms = cs;
    g_comm_devs = devs;
}

// A device set driven from the calling thread (SURVEY.md §8b Threading):
// distinct devices reduce with one grouped ncclAllReduce per buffer over the
// shards' streams; one device repeated (virtual shards: the sharded schedule
// on one GPU) sums the shards' buffers on a shared stream instead.
struct DeviceGroup {
    std::vector<int> devs;
    bool same = true;
    hipStream_t vst = nullptr;  // shared stream of virtual shards
    DeviceGroup(const std::vector<int>& d, int64_t n1) : devs(d) {
        const int P = (int)devs.size();
        if (P < 1 || P > 16) throw Error(TRITD_ERR_ARG, "a device set holds 1..16 devices");
        if (P > n1) throw Error(TRITD_ERR_ARG, "more shards than mode-1 rows");
        bool distinct = true;
        for (int p = 0; p < P; ++p) {
            if (devs[p] != devs[0]) same = false;
            for (int q = 0; q < p; ++q)
                if (devs[p] == devs[q]) distinct = false;
        }
        if (!same && !distinct)
            throw Error(TRITD_ERR_ARG, "a device set is distinct devices or one device repeated");
        for (int dv : devs) pick_device(dv);
        if (distinct && P > 1) group_comms(devs);
        if (same && P > 1) {
            TRITD_HIP(hipSetDevice(devs[0]));
            TRITD_HIP(hipStreamCreateWithFlags(&vst, hipStreamNonBlocking));
        }
    }
    ~DeviceGroup() {
        if (vst) hip_quiet(hipStreamDestroy(vst));
    }
    int size() const { return (int)devs.size(); }
    // balanced rows: every shard non-empty
    std::pair<int64_t, int64_t> rows(int p, int64_t n1) const {
        return {n1 * p / size(), n1 * (p + 1) / size()};
    }
    // in-place sum of buf[p] (count doubles on device p, stream st[p]) over p
    void reduce(const std::vector<double*>& buf, const std::vector<hipStream_t>& st,
                int64_t count) const {
        const int P = size();
        if (P == 1) return;
        if (same) {
            launch_vsum(const_cast<double* const*>(buf.data()), P, count, vst);
            return;
        }
        // a hipSetDevice failure inside the group is recorded, not thrown, so
        // that the group is always closed (as in group_comms)
        hipError_t he = hipSuccess;
        ncclResult_t rr = ncclGroupStart();
        for (int p = 0; p < P && rr == ncclSuccess; ++p) {
            he = hipSetDevice(devs[p]);
            if (he != hipSuccess) {
                (void)hipGetLastError();
                break;
            }
            rr = ncclAllReduce(buf[p], buf[p], (size_t)count, ncclFloat64, ncclSum, g_comms[p], st[p]);
        }
        ncclResult_t re = ncclGroupEnd();
        if (he != hipSuccess)
            throw Error(TRITD_ERR_HIP, std::string("hipSetDevice (grouped all-reduce): ") + hipGetErrorString(he));
        if (rr == ncclInProgress) rr = ncclSuccess;  // non-blocking communicators (group_comms)
        if (re == ncclInProgress) re = ncclSuccess;
        for (int p = 0; p < P && rr == ncclSuccess && re == ncclSuccess; ++p) re = nccl_settle(g_comms[p]);
        if (rr != ncclSuccess || re != ncclSuccess)
            throw Error(TRITD_ERR_RCCL, std::string("grouped ncclAllReduce: ") +
                                            ncclGetErrorString(rr != ncclSuccess ? rr : re));
    }
    // reduce a per-session buffer (member function `get`) over all shards
    template <class S>
    void reduce(std::vector<std::unique_ptr<S>>& ss, double* (S::*get)(), int64_t count) const {
        std::vector<double*> b;
        std::vector<hipStream_t> st;
        for (auto& s : ss) {
            b.push_back(((*s).*get)());
            st.push_back(s->stream());
        }
        reduce(b, st, count);
    }
    template <class S, class F>
    static void each(std::vector<std::unique_ptr<S>>& ss, F&& f) {
        for (auto& s : ss) {
            TRITD_HIP(hipSetDevice(s->device()));
            f(*s);
        }
    }
};

// Drive one session per shard of a device group, each on its own host thread
// (group.h: run_shard_threads; shard 0 on the calling thread), all through a
// communicator: the group's non-blocking RCCL communicators (group_comms) for
// distinct devices, the in-process ThreadReducer for one device repeated.
// shard(p, comm) builds, runs and reads back shard p and returns its
// TRITD_FLAG_* bits.  A shard that throws aborts the group: the ThreadReducer
// wakes its waiters; the RCCL communicators are aborted under the group's
// abort protocol (GroupAbort), after which no shard touches them again — a
// shard blocked on its stream is released by the abort and fails at its next
// all-reduce.  The aborted communicators leave the cache once every thread
// has joined.  The first error is rethrown.
template <class F>
void run_threaded(DeviceGroup& grp, F&& shard) {
    const int P = grp.size();
    std::unique_ptr<ThreadReducer> red;
    std::unique_ptr<GroupAbort> ga;
    if (grp.same) red.reset(new ThreadReducer(P));
    else ga.reset(new GroupAbort(P));
    std::vector<tritd_comm> comms((size_t)P);
    for (int p = 0; p < P; ++p) {
        comms[p].nranks = P;
        comms[p].rank = p;
        comms[p].device = grp.devs[p];
        if (grp.same) {
            comms[p].host_fn = &ThreadReducer::allreduce;
            comms[p].host_user = &red->ranks[p];
        } else {
            comms[p].comm = g_comms[p];  // owned by the cache (group_comms)
            comms[p].group = ga.get();
        }
    }
    std::vector<uint32_t> fl((size_t)P, 0);
    auto abort_all = [&] {
        if (red) {
            red->abort();
            return;
        }
        ga->abort([&](int p) {
            if (comms[p].comm) (void)ncclCommAbort(comms[p].comm);  // frees it
            comms[p].comm = nullptr;
        });
    };
    try {
        run_shard_threads(
            P,
            [&](int p) {
                TRITD_HIP(hipSetDevice(grp.devs[p]));
                fl[p] = shard(p, &comms[p]);
            },
            abort_all);
    } catch (...) {
        if (ga && ga->aborted()) {  // every thread has joined: forget the freed communicators
            g_comms.clear();
            g_comm_devs.clear();
        }
        throw;
    }
    for (int p = 0; p < P; ++p) g_last_flags |= fl[p];
}

// One ADMM problem sharded along mode 1 over `devs`, driven
// the way one process per GPU drives it: each shard is a Session with a
// communicator, stepped by its own host thread through the same schedule
// bench.py and the multi-rank tests run (the fused single-stream iteration
// with two all-reduces per iteration, or its side-stream form for fp32 / Qi /
// r > 8).  Distinct devices all-reduce over RCCL (communicators from
// group_comms, cached); one device repeated uses the in-process
// ThreadReducer.  Shard 0 runs on the calling thread, so `disp` prints (the
// MEX's mexPrintf) stay on the host's own thread.  D, O, E are column-major
// n1 x n2 x n3 host arrays of es-byte elements.
void run_group_serial(const std::vector<int>& devs, const void* D, size_t es, uint32_t flags,
                      int64_t n1, int64_t n2, int64_t n3, int32_t r, const tritd_opts& o,
                      const double* A0, const double* B0, const double* C0, double* A, double* B,
                      double* C, void* O, void* E, double* errHist, int32_t* iters);

void run_group(const std::vector<int>& devs, const void* D, size_t es, uint32_t flags, int64_t n1,
               int64_t n2, int64_t n3, int32_t r, const tritd_opts& o, const double* A0,
               const double* B0, const double* C0, double* A, double* B, double* C, void* O,
               void* E, double* errHist, int32_t* iters) {
    {
        // TRITD_SHOV=0: the phase-serial order of round 1 (one host thread
        // enqueues every shard's phases, three reductions per iteration)
        const char* sh = std::getenv("TRITD_SHOV");
        if (sh && std::atoi(sh) == 0) {
            run_group_serial(devs, D, es, flags, n1, n2, n3, r, o, A0, B0, C0, A, B, C, O, E,
                             errHist, iters);
            return;
        }
    }
    DeviceGroup grp(devs, n1);
    const int P = grp.size();
    if (P == 1) {
        Session s(devs[0], D, n1, n1, n2, n3, 0, n1, r, o, A0, B0, C0, nullptr, flags);
        OutputPrefault pf(O, E, (size_t)(n1 * n2 * n3) * es);
        s.run(o.maxIter);
        pf.join();
        int k = 0;
        s.get(A, B, C, O, E, n1, errHist, &k, true);
        g_last_flags |= s.flags();
        if (iters) *iters = k;
        return;
    }
    run_threaded(grp, [&](int p, tritd_comm* comm) {
        const auto [i0, i1] = grp.rows(p, n1);
        Session s(devs[p], static_cast<const char*>(D) + i0 * es, n1, n1, n2, n3, i0, i1, r, o, A0,
                  B0, C0, comm, flags);
        s.run(o.maxIter);
        int k = 0;
        s.get(A, p == 0 ? B : nullptr, p == 0 ? C : nullptr,
              O ? static_cast<char*>(O) + i0 * es : nullptr,
              E ? static_cast<char*>(E) + i0 * es : nullptr, n1, p == 0 ? errHist : nullptr, &k);
        if (p == 0 && iters) *iters = k;
        return s.flags();
    });
}

// The phase-serial schedule (TRITD_SHOV=0): every iteration runs the four
// phases of solver.cpp on each shard with the three reductions between them.  D, O, E are column-major n1 x n2 x n3 host arrays
// of es-byte elements.
void run_group_serial(const std::vector<int>& devs, const void* D, size_t es, uint32_t flags,
                      int64_t n1, int64_t n2, int64_t n3, int32_t r, const tritd_opts& o,
                      const double* A0, const double* B0, const double* C0, double* A, double* B,
                      double* C, void* O, void* E, double* errHist, int32_t* iters) {
    DeviceGroup grp(devs, n1);
    const int P = grp.size();
    std::vector<std::unique_ptr<Session>> ss;
    for (int p = 0; p < P; ++p) {
        const auto [i0, i1] = grp.rows(p, n1);
        TRITD_HIP(hipSetDevice(devs[p]));
        ss.emplace_back(new Session(devs[p], static_cast<const char*>(D) + i0 * es, n1, n1, n2, n3,
                                    i0, i1, r, o, A0, B0, C0, nullptr, flags, grp.vst,
                                    /*defer_normD=*/true));
    }
    auto each = [&](auto&& f) { DeviceGroup::each(ss, f); };
    grp.reduce(ss, &Session::red3, 2);
    each([](Session& s) { s.set_normD_from_red3(); });
    for (int it = 0; it < o.maxIter; ++it) {
        int k = 0;
        each([&](Session& s) { k = s.next_iter(); });
        if (!k) break;
        each([&](Session& s) { s.phaseA(k); });
        grp.reduce(ss, &Session::red1, ss[0]->red1_count());
        each([&](Session& s) { s.phaseB(k); });
        grp.reduce(ss, &Session::red2, ss[0]->red2_count());
        each([&](Session& s) { s.phaseC(k); });
        grp.reduce(ss, &Session::red3, 2);
        each([&](Session& s) { s.phaseD(k); });
        TRITD_HIP(hipSetDevice(devs[0]));
        ss[0]->maybe_print(k);
    }
    int k = 0;
    for (int p = 0; p < P; ++p) {
        const int64_t i0 = ss[p]->geom().i0;
        TRITD_HIP(hipSetDevice(devs[p]));
        ss[p]->get(A, p == 0 ? B : nullptr, p == 0 ? C : nullptr,
                   O ? static_cast<char*>(O) + i0 * es : nullptr,
                   E ? static_cast<char*>(E) + i0 * es : nullptr, n1, p == 0 ? errHist : nullptr, &k);
        g_last_flags |= ss[p]->flags();
    }
    if (iters) *iters = k;
}

// triple_decomp_ALS over a device set: the ALS phases (als.cpp) with the
// fit sum, [M2 | A^TA] and M3 reduced between them.
void run_als_group_serial(const std::vector<int>& devs, const double* X, int64_t n1, int64_t n2,
                          int64_t n3, int32_t r, int maxIter, double tol, const double* A0,
                          const double* B0, const double* C0, double* A, double* B, double* C,
                          double* errHist, int32_t* iters, const NcvxParams* ncvx, double* O);

// triple_decomp_ALS / the test.m solver over a device set: one AlsSession
// per shard with a communicator (its run() carries the fit-sum, [M2 | A^TA]
// and M3 all-reduces), one host thread per shard (run_threaded);
// TRITD_SHOV=0 keeps the phase-serial order (run_als_group_serial).
void run_als_group(const std::vector<int>& devs, const double* X, int64_t n1, int64_t n2,
                   int64_t n3, int32_t r, int maxIter, double tol, const double* A0,
                   const double* B0, const double* C0, double* A, double* B, double* C,
                   double* errHist, int32_t* iters, const NcvxParams* ncvx = nullptr,
                   double* O = nullptr) {
    {
        const char* sh = std::getenv("TRITD_SHOV");
        if (sh && std::atoi(sh) == 0) {
            run_als_group_serial(devs, X, n1, n2, n3, r, maxIter, tol, A0, B0, C0, A, B, C, errHist,
                                 iters, ncvx, O);
            return;
        }
    }
    DeviceGroup grp(devs, n1);
    run_threaded(grp, [&](int p, tritd_comm* comm) {
        const auto [i0, i1] = grp.rows(p, n1);
        AlsSession s(devs[p], X + i0, n1, n1, n2, n3, i0, i1, r, maxIter, tol, A0, B0, C0,
                     grp.size() > 1 ? comm : nullptr, 0);
        if (ncvx) s.enable_ncvx(*ncvx);
        s.run(maxIter);
        int k = 0;
        s.get(A, p == 0 ? B : nullptr, p == 0 ? C : nullptr, p == 0 ? errHist : nullptr, &k);
        if (ncvx && O) s.get_O(O + s.geom().i0, n1);
        if (p == 0 && iters) *iters = k;
        return s.flags();
    });
}

void run_als_group_serial(const std::vector<int>& devs, const double* X, int64_t n1, int64_t n2,
                          int64_t n3, int32_t r, int maxIter, double tol, const double* A0,
                          const double* B0, const double* C0, double* A, double* B, double* C,
                          double* errHist, int32_t* iters, const NcvxParams* ncvx, double* O) {
    DeviceGroup grp(devs, n1);
    const int P = grp.size();
    std::vector<std::unique_ptr<AlsSession>> ss;
    for (int p = 0; p < P; ++p) {
        const auto [i0, i1] = grp.rows(p, n1);
        TRITD_HIP(hipSetDevice(devs[p]));
        ss.emplace_back(new AlsSession(devs[p], X + i0, n1, n1, n2, n3, i0, i1, r, maxIter, tol, A0,
                                       B0, C0, nullptr, 0, grp.vst, /*defer_norm=*/true));
        if (ncvx) ss.back()->enable_ncvx(*ncvx);
    }
    auto each = [&](auto&& f) { DeviceGroup::each(ss, f); };
    grp.reduce(ss, &AlsSession::red0, 2);
    each([](AlsSession& s) { s.set_norm_from_red0(); });
    for (int it = 0; it < maxIter; ++it) {
        int k = 0;
        each([&](AlsSession& s) { k = s.next_iter(); });
        if (!k) break;
        each([&](AlsSession& s) { s.phaseFit(k); });
        grp.reduce(ss, &AlsSession::red0, 2);
        each([&](AlsSession& s) { s.phaseErr(k); });
        TRITD_HIP(hipSetDevice(devs[0]));
        if (!ncvx) ss[0]->maybe_print(k);
        each([&](AlsSession& s) { s.phaseA(k); });
        grp.reduce(ss, &AlsSession::red1, ss[0]->red1_count());
        each([&](AlsSession& s) { s.phaseB(k); });
        grp.reduce(ss, &AlsSession::red2, ss[0]->red2_count());
        each([&](AlsSession& s) { s.phaseC(k); });
        each([&](AlsSession& s) { s.phaseEnd(k); });  // ncvx: errHist / stop after the updates
        if (ncvx) {
            TRITD_HIP(hipSetDevice(devs[0]));
            ss[0]->maybe_print(k);
        }
    }
    int k = 0;
    for (int p = 0; p < P; ++p) {
        TRITD_HIP(hipSetDevice(devs[p]));
        ss[p]->get(A, p == 0 ? B : nullptr, p == 0 ? C : nullptr, p == 0 ? errHist : nullptr, &k);
        if (ncvx && O) ss[p]->get_O(O + ss[p]->geom().i0, n1);
        g_last_flags |= ss[p]->flags();
    }
    if (iters) *iters = k;
}
// fspecial('gaussian', 11, 1.5), then ssim_index's window/sum(sum(window));
// column-major (the window is symmetric)
std::vector<double> ssim_window() {
    const int siz = 5;
    const double sd = 1.5;
    std::vector<double> h(121);
    double mx = 0.0;
    for (int c = 0; c < 11; ++c)
        for (int r = 0; r < 11; ++r) {
            const double x = c - siz, y = r - siz;  // [x,y] = meshgrid(-siz:siz)
            const double v = std::exp(-(x * x + y * y) / (2 * sd * sd));
            h[c * 11 + r] = v;
            mx = std::max(mx, v);
        }
    for (double& v : h)
        if (v < 2.220446049250313e-16 * mx) v = 0.0;  // h(h < eps*max(h(:))) = 0
    for (int pass = 0; pass < 2; ++pass) {  // fspecial's h/sum(h(:)), then ssim_index's sum(sum())
        double tot = 0.0;
        if (pass == 0) {
            for (double v : h) tot += v;
        } else {
            for (int c = 0; c < 11; ++c) {
                double col = 0.0;
                for (int r = 0; r < 11; ++r) col += h[c * 11 + r];
                tot += col;
            }
        }
        if (tot != 0.0)
            for (double& v : h) v /= tot;
    }
    return h;
}
}  // namespace

namespace tritd {
void emit_line(const char* line) {
    if (g_print) {
        g_print(line, g_print_user);
    } else {
        std::printf("%s\n", line);
        std::fflush(stdout);
    }
}
}  // namespace tritd

extern "C" {

const char* tritd_version(void) { return "tritd-mi355x 0.2.0 (gfx950, fp64 r<=8, fp32 r<=16)"; }
const char* tritd_last_error(void) { return g_last_error.c_str(); }
uint32_t tritd_last_flags(void) { return g_last_flags; }

void tritd_set_print_callback(tritd_print_fn fn, void* user) {
    g_print = fn;
    g_print_user = user;
}

tritd_status tritd_device_count(int32_t* count) {
    return guarded([&] {
        need(count, "count");
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
        *count = n;
    });
}

tritd_status tritd_admm_f64(const double* D, int64_t n1, int64_t n2, int64_t n3, int32_t r,
                            const tritd_opts* opts, const double* A0, const double* B0,
                            const double* C0, double* A, double* B, double* C, double* O,
                            double* E, double* errHist, int32_t* iters, int32_t device) {
    std::lock_guard<std::mutex> lk(g_mutex);
    g_last_flags = 0;
    return guarded([&] {
        check_opts(opts);
        check_dims(n1, n2, n3, r, true);  // fp64 ADMM: r <= 16 (r > 8 untuned)
        need(D, "D"); need(A0, "A0"); need(B0, "B0"); need(C0, "C0");
        const tritd_opts o = normalized(opts);
        if (device < 0 && g_devices.size() > 1) {
            run_group(g_devices, D, sizeof(double), 0, n1, n2, n3, r, o, A0, B0, C0, A, B, C, O, E,
                      errHist, iters);
            return;
        }
        const int dev = pick_device(device < 0 && !g_devices.empty() ? g_devices[0] : device);
        Session s(dev, D, n1, n1, n2, n3, 0, n1, r, o, A0, B0, C0, nullptr, 0);
        OutputPrefault pf(O, E, (size_t)(n1 * n2 * n3) * sizeof(double));
        s.run(o.maxIter);
        pf.join();
        int k = 0;
        s.get(A, B, C, O, E, n1, errHist, &k, true);
        g_last_flags |= s.flags();
        if (iters) *iters = k;
    });
}

tritd_status tritd_admm_f32(const float* D, int64_t n1, int64_t n2, int64_t n3, int32_t r,
                            const tritd_opts* opts, const double* A0, const double* B0,
                            const double* C0, double* A, double* B, double* C, float* O, float* E,
                            double* errHist, int32_t* iters, int32_t device) {
    std::lock_guard<std::mutex> lk(g_mutex);
    g_last_flags = 0;
    return guarded([&] {
        check_opts(opts);
        check_dims(n1, n2, n3, r, true);
        need(D, "D"); need(A0, "A0"); need(B0, "B0"); need(C0, "C0");
        const tritd_opts o = normalized(opts);
        if (device < 0 && g_devices.size() > 1) {
            run_group(g_devices, D, sizeof(float), TRITD_SESSION_F32, n1, n2, n3, r, o, A0, B0, C0,
                      A, B, C, O, E, errHist, iters);
            return;
        }
        const int dev = pick_device(device < 0 && !g_devices.empty() ? g_devices[0] : device);
        Session s(dev, D, n1, n1, n2, n3, 0, n1, r, o, A0, B0, C0, nullptr, TRITD_SESSION_F32);
        OutputPrefault pf(O, E, (size_t)(n1 * n2 * n3) * sizeof(float));
        s.run(o.maxIter);
        pf.join();
        int k = 0;
        s.get(A, B, C, O, E, n1, errHist, &k, true);
        g_last_flags |= s.flags();
        if (iters) *iters = k;
    });
}

tritd_status tritd_session_create(tritd_session** out, int32_t device, const void* D, int64_t ldD,
                                  int64_t n1, int64_t n2, int64_t n3, int64_t i0, int64_t i1,
                                  int32_t r, const tritd_opts* opts, const double* A0,
                                  const double* B0, const double* C0, tritd_comm* comm,
                                  uint32_t flags) {
    return guarded([&] {
        need(out, "out");
        *out = nullptr;
        check_opts(opts);
        check_dims(n1, n2, n3, r, true);  // ADMM, fp64 or fp32: r <= 16
        need(D, "D"); need(A0, "A0"); need(B0, "B0"); need(C0, "C0");
        if (i0 < 0 || i1 > n1 || i0 >= i1) throw Error(TRITD_ERR_ARG, "bad shard range");
        if (ldD < i1 - i0) throw Error(TRITD_ERR_ARG, "ldD smaller than the shard");
        const int dev = pick_device(device);
        auto* s = new Session(dev, D, ldD, n1, n2, n3, i0, i1, r, normalized(opts), A0, B0, C0,
                              comm, flags);
        *out = reinterpret_cast<tritd_session*>(s);
    });
}

tritd_status tritd_session_run(tritd_session* s, int32_t iters) {
    return guarded([&] {
        need(s, "session");
        reinterpret_cast<Session*>(s)->run(iters);
    });
}

tritd_status tritd_session_sync(tritd_session* s, int32_t* iters_done, int32_t* stopped) {
    return guarded([&] {
        need(s, "session");
        int d = 0, st = 0;
        reinterpret_cast<Session*>(s)->sync(&d, &st);
        if (iters_done) *iters_done = d;
        if (stopped) *stopped = st;
    });
}

tritd_status tritd_session_get(tritd_session* s, double* A, double* B, double* C, double* O,
                               double* E, int64_t ldOE, double* errHist, int32_t* iters) {
    return guarded([&] {
        need(s, "session");
        auto* S = reinterpret_cast<Session*>(s);
        if (S->is_f32()) throw Error(TRITD_ERR_ARG, "fp32 session: use tritd_session_get_f32");
        if ((O || E) && ldOE < S->geom().n1l) throw Error(TRITD_ERR_ARG, "ldOE smaller than the shard");
        int k = 0;
        S->get(A, B, C, O, E, ldOE, errHist, &k);
        if (iters) *iters = k;
    });
}

tritd_status tritd_session_get_f32(tritd_session* s, double* A, double* B, double* C, float* O,
                                   float* E, int64_t ldOE, double* errHist, int32_t* iters) {
    return guarded([&] {
        need(s, "session");
        auto* S = reinterpret_cast<Session*>(s);
        if (!S->is_f32()) throw Error(TRITD_ERR_ARG, "fp64 session: use tritd_session_get");
        if ((O || E) && ldOE < S->geom().n1l) throw Error(TRITD_ERR_ARG, "ldOE smaller than the shard");
        int k = 0;
        S->get(A, B, C, O, E, ldOE, errHist, &k);
        if (iters) *iters = k;
    });
}

tritd_status tritd_session_rre_parts(tritd_session* s, const double* dX, int64_t ldX, double* num,
                                     double* den) {
    return guarded([&] {
        need(s, "session"); need(dX, "X"); need(num, "num"); need(den, "den");
        auto* S = reinterpret_cast<Session*>(s);
        if (S->is_f32()) throw Error(TRITD_ERR_ARG, "fp32 session: use tritd_session_rre_parts_f32");
        S->rre_parts(dX, ldX, num, den);
    });
}

tritd_status tritd_session_rre_parts_f32(tritd_session* s, const float* dX, int64_t ldX,
                                         double* num, double* den) {
    return guarded([&] {
        need(s, "session"); need(dX, "X"); need(num, "num"); need(den, "den");
        auto* S = reinterpret_cast<Session*>(s);
        if (!S->is_f32()) throw Error(TRITD_ERR_ARG, "fp64 session: use tritd_session_rre_parts");
        S->rre_parts(dX, ldX, num, den);
    });
}

tritd_status tritd_session_set_timing(tritd_session* s, int32_t enable) {
    return guarded([&] {
        need(s, "session");
        if (enable < 0 || enable > TRITD_TIMING_K5) throw Error(TRITD_ERR_ARG, "timing level 0..2");
        reinterpret_cast<Session*>(s)->set_timing(enable);
    });
}

tritd_status tritd_session_kernel_ms(tritd_session* s, double* fused_update_ms, double* mode3_ms,
                                     double* iteration_ms, int32_t* samples) {
    return guarded([&] {
        need(s, "session");
        int n = 0;
        reinterpret_cast<Session*>(s)->kernel_ms(fused_update_ms, mode3_ms, iteration_ms, &n);
        if (samples) *samples = n;
    });
}

tritd_status tritd_session_comm_ms(tritd_session* s, double* allreduce_ms, int32_t* per_iteration) {
    return guarded([&] {
        need(s, "session");
        int n = 0;
        reinterpret_cast<Session*>(s)->comm_ms(allreduce_ms, &n);
        if (per_iteration) *per_iteration = n;
    });
}

tritd_status tritd_session_probe(tritd_session* s, double* ms, int32_t cap, int32_t* n,
                                 int32_t* picked) {
    return guarded([&] {
        need(s, "session");
        const Session* q = reinterpret_cast<Session*>(s);
        const std::vector<double>& v = q->probe_ms();
        for (int32_t c = 0; ms && c < cap && c < (int32_t)v.size(); ++c) ms[c] = v[c];
        if (n) *n = (int32_t)v.size();
        if (picked) *picked = q->probe_pick();
    });
}

tritd_status tritd_session_counters(tritd_session* s, int64_t* dense_tiles_total,
                                    int64_t* tiles_per_launch) {
    return guarded([&] {
        need(s, "session");
        reinterpret_cast<Session*>(s)->counters(dense_tiles_total, tiles_per_launch);
    });
}

tritd_status tritd_session_k5_profile(tritd_session* s, int32_t* dense_streams,
                                      int32_t* slot_accesses) {
    return guarded([&] {
        need(s, "session"); need(dense_streams, "dense_streams"); need(slot_accesses, "slot_accesses");
        int a = 0, b = 0;
        reinterpret_cast<Session*>(s)->k5_profile(&a, &b);
        *dense_streams = a;
        *slot_accesses = b;
    });
}

tritd_status tritd_session_flags(tritd_session* s, uint32_t* flags) {
    return guarded([&] {
        need(s, "session");
        need(flags, "flags");
        *flags = reinterpret_cast<Session*>(s)->flags();
    });
}

void tritd_session_destroy(tritd_session* s) { delete reinterpret_cast<Session*>(s); }

tritd_status tritd_comm_unique_id(void* id128) {
    return guarded([&] {
        need(id128, "id");
        ncclUniqueId id;
        const ncclResult_t r = ncclGetUniqueId(&id);
        if (r != ncclSuccess) throw Error(TRITD_ERR_RCCL, ncclGetErrorString(r));
        std::memcpy(id128, &id, sizeof id);
    });
}

tritd_status tritd_comm_create(tritd_comm** out, const void* id128, int32_t nranks, int32_t rank,
                               int32_t device) {
    return guarded([&] {
        need(out, "out"); need(id128, "id");
        *out = nullptr;
        if (nranks < 1 || rank < 0 || rank >= nranks) throw Error(TRITD_ERR_ARG, "bad rank/nranks");
        const int dev = pick_device(device);
        auto c = std::make_unique<tritd_comm>();
        c->nranks = nranks;
        c->rank = rank;
        c->device = dev;
        ncclUniqueId id;
        std::memcpy(&id, id128, sizeof id);
        const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
        if (r != ncclSuccess) throw Error(TRITD_ERR_RCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
        *out = c.release();
    });
}

tritd_status tritd_comm_create_host(tritd_comm** out, tritd_allreduce_fn fn, void* user,
                                    int32_t nranks, int32_t rank, int32_t device) {
    return guarded([&] {
        need(out, "out");
        *out = nullptr;
        if (!fn) throw Error(TRITD_ERR_ARG, "fn is NULL");
        if (nranks < 1 || rank < 0 || rank >= nranks) throw Error(TRITD_ERR_ARG, "bad rank/nranks");
        auto c = std::make_unique<tritd_comm>();
        c->nranks = nranks;
        c->rank = rank;
        c->device = pick_device(device);
        c->host_fn = fn;
        c->host_user = user;
        *out = c.release();
    });
}

void tritd_comm_destroy(tritd_comm* c) {
    if (!c) return;
    if (c->comm) (void)ncclCommDestroy(c->comm);
    delete c;
}

tritd_status tritd_comm_info(tritd_comm* c, int32_t* nranks, int32_t* rank, int32_t* transport) {
    return guarded([&] {
        need(c, "comm");
        int n = c->nranks, me = c->rank;
        if (c->comm) {
            ncclResult_t r = ncclCommCount(c->comm, &n);
            if (r == ncclSuccess) r = ncclCommUserRank(c->comm, &me);
            if (r != ncclSuccess) throw Error(TRITD_ERR_RCCL, std::string("ncclCommCount: ") + ncclGetErrorString(r));
        }
        if (nranks) *nranks = n;
        if (rank) *rank = me;
        if (transport) *transport = c->comm ? 0 : 1;
    });
}

tritd_status tritd_admm_sharded_virtual_f64(const double* D, int64_t n1, int64_t n2, int64_t n3,
                                            int32_t r, const tritd_opts* opts, const double* A0,
                                            const double* B0, const double* C0, int32_t nshards,
                                            double* A, double* B, double* C, double* O, double* E,
                                            double* errHist, int32_t* iters, int32_t device) {
    std::lock_guard<std::mutex> lk(g_mutex);
    g_last_flags = 0;
    return guarded([&] {
        check_opts(opts);
        check_dims(n1, n2, n3, r, true);  // fp64 ADMM: r <= 16 (r > 8 untuned)
        need(D, "D"); need(A0, "A0"); need(B0, "B0"); need(C0, "C0");
        if (nshards < 1 || nshards > 16 || nshards > n1) throw Error(TRITD_ERR_ARG, "nshards must be in 1..min(16,n1)");
        const int dev = pick_device(device);
        run_group(std::vector<int>(nshards, dev), D, sizeof(double), 0, n1, n2, n3, r,
                  normalized(opts), A0, B0, C0, A, B, C, O, E, errHist, iters);
    });
}

tritd_status tritd_set_devices(const int32_t* devices, int32_t n) {
    std::lock_guard<std::mutex> lk(g_mutex);
    return guarded([&] {
        if (n < 0 || n > 16) throw Error(TRITD_ERR_ARG, "a device set holds 0..16 devices");
        if (n > 0) need(devices, "devices");
        std::vector<int> d(devices, devices + n);
        int count = 0;
        if (hipGetDeviceCount(&count) != hipSuccess) count = 0;
        for (int x : d)
            if (x < 0 || x >= count) throw Error(TRITD_ERR_NODEV, "device index out of range");
        if (d != g_comm_devs) drop_comms();
        g_devices = d;
    });
}

void tritd_shutdown(void) {
    std::lock_guard<std::mutex> lk(g_mutex);
    drop_comms();
    g_devices.clear();
    drop_scratch();
}

// ---------------------------------------------------------------------------
// ALS variant (triple_decomp_ALS.m)
// ---------------------------------------------------------------------------
tritd_status tritd_als_f64(const double* X, int64_t n1, int64_t n2, int64_t n3, int32_t r,
                           const tritd_opts* opts, const double* A0, const double* B0,
                           const double* C0, double* A, double* B, double* C, double* errHist,
                           int32_t* iters, int32_t device) {
    std::lock_guard<std::mutex> lk(g_mutex);
    g_last_flags = 0;
    return guarded([&] {
        check_als_opts(opts);
        check_dims(n1, n2, n3, r);
        need(X, "X"); need(A0, "A0"); need(B0, "B0"); need(C0, "C0");
        const int maxIter = opts->maxIter < 0 ? 0 : opts->maxIter;
        if (device < 0 && g_devices.size() > 1) {
            run_als_group(g_devices, X, n1, n2, n3, r, maxIter, opts->tol, A0, B0, C0, A, B, C,
                          errHist, iters);
            return;
        }
        const int dev = pick_device(device < 0 && !g_devices.empty() ? g_devices[0] : device);
        AlsSession s(dev, X, n1, n1, n2, n3, 0, n1, r, maxIter, opts->tol, A0, B0, C0, nullptr, 0);
        s.run(maxIter);
        int k = 0;
        s.get(A, B, C, errHist, &k);
        g_last_flags |= s.flags();
        if (iters) *iters = k;
    });
}

tritd_status tritd_als_sharded_virtual_f64(const double* X, int64_t n1, int64_t n2, int64_t n3,
                                           int32_t r, const tritd_opts* opts, const double* A0,
                                           const double* B0, const double* C0, int32_t nshards,
                                           double* A, double* B, double* C, double* errHist,
                                           int32_t* iters, int32_t device) {
    std::lock_guard<std::mutex> lk(g_mutex);
    g_last_flags = 0;
    return guarded([&] {
        check_als_opts(opts);
        check_dims(n1, n2, n3, r);
        need(X, "X"); need(A0, "A0"); need(B0, "B0"); need(C0, "C0");
        if (nshards < 1 || nshards > 16 || nshards > n1)
            throw Error(TRITD_ERR_ARG, "nshards must be in 1..min(16,n1)");
        const int dev = pick_device(device);
        run_als_group(std::vector<int>(nshards, dev), X, n1, n2, n3, r,
                      opts->maxIter < 0 ? 0 : opts->maxIter, opts->tol, A0, B0, C0, A, B, C,
                      errHist, iters);
    });
}

tritd_status tritd_ncvx_f64(const double* X, int64_t n1, int64_t n2, int64_t n3, int32_t r,
                           double rho, double lambda, double gamma_A, double epsilon, double p,
                           double theta, int32_t maxIter, double tol, const double* A0,
                           const double* B0, const double* C0, double* A, double* B, double* C,
                           double* O, double* errHist, int32_t* iters, int32_t device) {
    std::lock_guard<std::mutex> lk(g_mutex);
    g_last_flags = 0;
    return guarded([&] {
        check_dims(n1, n2, n3, r);
        need(X, "X"); need(A0, "A0"); need(B0, "B0"); need(C0, "C0");
        need(A, "A"); need(B, "B"); need(C, "C"); need(O, "O"); need(errHist, "errHist");
        if (!(rho != 0.0)) throw Error(TRITD_ERR_ARG, "rho must be non-zero");
        const NcvxParams np{rho, lambda, gamma_A, epsilon, p, theta};
        const int mi = maxIter < 0 ? 0 : maxIter;
        if (device < 0 && g_devices.size() > 1) {
            run_als_group(g_devices, X, n1, n2, n3, r, mi, tol, A0, B0, C0, A, B, C, errHist, iters,
                          &np, O);
            return;
        }
        const int dev = pick_device(device < 0 && !g_devices.empty() ? g_devices[0] : device);
        AlsSession s(dev, X, n1, n1, n2, n3, 0, n1, r, mi, tol, A0, B0, C0, nullptr, 0);
        s.enable_ncvx(np);
        s.run(mi);
        int k = 0;
        s.get(A, B, C, errHist, &k);
        s.get_O(O, n1);
        g_last_flags |= s.flags();
        if (iters) *iters = k;
    });
}

tritd_status tritd_als_session_create(tritd_als_session** out, int32_t device, const double* X,
                                      int64_t ldX, int64_t n1, int64_t n2, int64_t n3, int64_t i0,
                                      int64_t i1, int32_t r, const tritd_opts* opts,
                                      const double* A0, const double* B0, const double* C0,
                                      tritd_comm* comm, uint32_t flags, int32_t quiet) {
    return guarded([&] {
        need(out, "out");
        *out = nullptr;
        check_als_opts(opts);
        check_dims(n1, n2, n3, r);
        need(X, "X"); need(A0, "A0"); need(B0, "B0"); need(C0, "C0");
        if (flags & ~(uint32_t)TRITD_SESSION_D_ON_DEVICE)
            throw Error(TRITD_ERR_UNSUPPORTED, "ALS sessions are fp64 (flags: D_ON_DEVICE only)");
        if (i0 < 0 || i1 > n1 || i0 >= i1) throw Error(TRITD_ERR_ARG, "bad shard range");
        if (ldX < i1 - i0) throw Error(TRITD_ERR_ARG, "ldX smaller than the shard");
        const int dev = pick_device(device);
        auto* s = new AlsSession(dev, X, ldX, n1, n2, n3, i0, i1, r,
                                 opts->maxIter < 0 ? 0 : opts->maxIter, opts->tol, A0, B0, C0,
                                 comm, flags);
        s->set_quiet(quiet != 0);
        *out = reinterpret_cast<tritd_als_session*>(s);
    });
}

tritd_status tritd_als_session_run(tritd_als_session* s, int32_t iters) {
    return guarded([&] {
        need(s, "session");
        reinterpret_cast<AlsSession*>(s)->run(iters);
    });
}

tritd_status tritd_als_session_sync(tritd_als_session* s, int32_t* iters_done, int32_t* stopped) {
    return guarded([&] {
        need(s, "session");
        int d = 0, st = 0;
        reinterpret_cast<AlsSession*>(s)->sync(&d, &st);
        if (iters_done) *iters_done = d;
        if (stopped) *stopped = st;
    });
}

tritd_status tritd_als_session_get(tritd_als_session* s, double* A, double* B, double* C,
                                   double* errHist, int32_t* iters) {
    return guarded([&] {
        need(s, "session");
        int k = 0;
        reinterpret_cast<AlsSession*>(s)->get(A, B, C, errHist, &k);
        if (iters) *iters = k;
    });
}

tritd_status tritd_als_session_set_timing(tritd_als_session* s, int32_t enable) {
    return guarded([&] {
        need(s, "session");
        reinterpret_cast<AlsSession*>(s)->set_timing(enable != 0);
    });
}

tritd_status tritd_als_session_kernel_ms(tritd_als_session* s, double* fit_ms, double* mode3_ms,
                                         double* iteration_ms, int32_t* samples) {
    return guarded([&] {
        need(s, "session");
        int n = 0;
        reinterpret_cast<AlsSession*>(s)->kernel_ms(fit_ms, mode3_ms, iteration_ms, &n);
        if (samples) *samples = n;
    });
}

tritd_status tritd_als_session_flags(tritd_als_session* s, uint32_t* flags) {
    return guarded([&] {
        need(s, "session");
        need(flags, "flags");
        *flags = reinterpret_cast<AlsSession*>(s)->flags();
    });
}

void tritd_als_session_destroy(tritd_als_session* s) { delete reinterpret_cast<AlsSession*>(s); }

// ---------------------------------------------------------------------------
// primitives
// ---------------------------------------------------------------------------
tritd_status tritd_dev_triple_product_f64(const double* A, const double* B, const double* C,
                                          int64_t n1, int64_t n2, int64_t n3, int32_t r, double* X,
                                          void* stream) {
    return guarded([&] {
        hip_entry();  // device pointers from the caller: HIP is in use
        check_dims(n1, n2, n3, r, true);
        need(A, "A"); need(B, "B"); need(C, "C"); need(X, "X");
        hipStream_t st = as_stream(stream);
        Geom g = make_geom(n1, n2, n3, 0, n1, r);
        g.RP = padded_rank32(g.R);  // 16..256: the kernel is instantiated for every padded rank
        ScratchLease lease(st);
        ScratchSet& ss = lease.set();
        double* Ah = scratch(lease, 0, (size_t)(g.n1p * g.RP));
        double* Bh = scratch(lease, 1, (size_t)(n2 * g.RP));
        double* ChT = scratch(lease, 2, (size_t)g.RP * g.n3p);
        launch_pack_factors(g, A, B, C, Ah, Bh, ChT, st);
        launch_tp(g, Ah, Bh, ChT, X, nullptr, nullptr, 0, n1, n1 * n2, st);
        TRITD_HIP(hipEventRecord(ss.done, st));
    });
}

// Qi model: H (k_qi.hip) is the Khatri-Rao operand of the same kernel
tritd_status tritd_dev_triple_product_qi_f64(const double* A, const double* B, const double* C,
                                             int64_t n1, int64_t n2, int64_t n3, int32_t r,
                                             double* X, void* stream) {
    return guarded([&] {
        hip_entry();  // device pointers from the caller: HIP is in use
        check_dims(n1, n2, n3, r, true);
        need(A, "A"); need(B, "B"); need(C, "C"); need(X, "X");
        hipStream_t st = as_stream(stream);
        Geom g = make_geom(n1, n2, n3, 0, n1, r);
        g.RP = padded_rank32(g.R);
        ScratchLease lease(st);
        ScratchSet& ss = lease.set();
        double* Ah = scratch(lease, 0, (size_t)(g.n1p * g.RP));
        double* Bh = scratch(lease, 1, (size_t)(n2 * g.RP));
        double* ChT = scratch(lease, 2, (size_t)g.RP * g.n3p);
        double* H = scratch(lease, 3, (size_t)(g.n1p * n2 * g.RP));
        double* ones = scratch(lease, 4, (size_t)g.RP);
        launch_pack_factors(g, A, B, C, Ah, Bh, ChT, st);
        launch_fill(ones, g.RP, 1.0, st);
        launch_qi_h(g, r, Ah, Bh, H, nullptr, st);
        launch_tp(g, H, ones, ChT, X, nullptr, nullptr, 0, n1, n1 * n2, st, g.n1p * g.RP, 0);
        TRITD_HIP(hipEventRecord(ss.done, st));
    });
}

tritd_status tritd_triple_product_qi_f64(const double* A, const double* B, const double* C,
                                         int64_t n1, int64_t n2, int64_t n3, int32_t r, double* X) {
    return guarded([&] {
        check_dims(n1, n2, n3, r, true);
        need(A, "A"); need(B, "B"); need(C, "C"); need(X, "X");
        pick_device(-1);
        const int64_t R = (int64_t)r * r;
        DBuf dA, dB, dC, dX;
        dA.alloc(n1 * R); dB.alloc(R * n2); dC.alloc(R * n3); dX.alloc((size_t)(n1 * n2 * n3));
        TRITD_HIP(hipMemcpy(dA.p, A, dA.n * 8, hipMemcpyHostToDevice));
        TRITD_HIP(hipMemcpy(dB.p, B, dB.n * 8, hipMemcpyHostToDevice));
        TRITD_HIP(hipMemcpy(dC.p, C, dC.n * 8, hipMemcpyHostToDevice));
        const tritd_status s =
            tritd_dev_triple_product_qi_f64(dA.p, dB.p, dC.p, n1, n2, n3, r, dX.p, nullptr);
        if (s != TRITD_OK) throw Error(s, g_last_error);
        populate_output(X, dX.n * 8);
        TRITD_HIP(hipMemcpy(X, dX.p, dX.n * 8, hipMemcpyDeviceToHost));
    });
}

tritd_status tritd_triple_product_f64(const double* A, const double* B, const double* C, int64_t n1,
                                      int64_t n2, int64_t n3, int32_t r, double* X) {
    return guarded([&] {
        check_dims(n1, n2, n3, r, true);  // r <= 16
        need(A, "A"); need(B, "B"); need(C, "C"); need(X, "X");
        pick_device(-1);
        const int64_t R = (int64_t)r * r;
        DBuf dA, dB, dC, dX;
        dA.alloc(n1 * R); dB.alloc(R * n2); dC.alloc(R * n3); dX.alloc((size_t)(n1 * n2 * n3));
        TRITD_HIP(hipMemcpy(dA.p, A, dA.n * 8, hipMemcpyHostToDevice));
        TRITD_HIP(hipMemcpy(dB.p, B, dB.n * 8, hipMemcpyHostToDevice));
        TRITD_HIP(hipMemcpy(dC.p, C, dC.n * 8, hipMemcpyHostToDevice));
        const tritd_status s = tritd_dev_triple_product_f64(dA.p, dB.p, dC.p, n1, n2, n3, r, dX.p, nullptr);
        if (s != TRITD_OK) throw Error(s, g_last_error);
        populate_output(X, dX.n * 8);
        TRITD_HIP(hipMemcpy(X, dX.p, dX.n * 8, hipMemcpyDeviceToHost));
    });
}

tritd_status tritd_dev_unfold_f64(const double* X, int64_t n1, int64_t n2, int64_t n3, int32_t mode,
                                  double* Xn, void* stream) {
    return guarded([&] {
        hip_entry();  // device pointers from the caller: HIP is in use
        if (mode < 1 || mode > 3) throw Error(TRITD_ERR_ARG, "Mode must be 1, 2, or 3.");  // unfold.m:12
        if (n1 <= 0 || n2 <= 0 || n3 <= 0) throw Error(TRITD_ERR_ARG, "tensor dimensions must be positive");
        need(X, "X"); need(Xn, "Xn");
        hipStream_t st = as_stream(stream);
        if (mode == 1)
            TRITD_HIP(hipMemcpyAsync(Xn, X, (size_t)(n1 * n2 * n3) * 8, hipMemcpyDeviceToDevice, st));
        else if (mode == 2)
            launch_transpose_batched(X, Xn, n1, n2, n3, st);
        else
            launch_transpose_batched(X, Xn, n1 * n2, n3, 1, st);
    });
}

tritd_status tritd_unfold_f64(const double* X, int64_t n1, int64_t n2, int64_t n3, int32_t mode,
                              double* Xn) {
    return guarded([&] {
        if (mode < 1 || mode > 3) throw Error(TRITD_ERR_ARG, "Mode must be 1, 2, or 3.");
        if (n1 <= 0 || n2 <= 0 || n3 <= 0) throw Error(TRITD_ERR_ARG, "tensor dimensions must be positive");
        need(X, "X"); need(Xn, "Xn");
        pick_device(-1);
        const size_t n = (size_t)(n1 * n2 * n3);
        DBuf a, b;
        a.alloc(n); b.alloc(n);
        TRITD_HIP(hipMemcpy(a.p, X, n * 8, hipMemcpyHostToDevice));
        const tritd_status s = tritd_dev_unfold_f64(a.p, n1, n2, n3, mode, b.p, nullptr);
        if (s != TRITD_OK) throw Error(s, g_last_error);
        populate_output(Xn, n * 8);
        TRITD_HIP(hipMemcpy(Xn, b.p, n * 8, hipMemcpyDeviceToHost));
    });
}

tritd_status tritd_dev_soft_threshold_f64(const double* X, int64_t n, double lam, double* Y,
                                          void* stream) {
    return guarded([&] {
        hip_entry();  // device pointers from the caller: HIP is in use
        if (n < 0) throw Error(TRITD_ERR_ARG, "n must be >= 0");
        if (n == 0) return;
        need(X, "X"); need(Y, "Y");
        launch_soft_threshold(X, n, lam, Y, as_stream(stream));
    });
}

tritd_status tritd_soft_threshold_f64(const double* X, int64_t n, double lam, double* Y) {
    return guarded([&] {
        if (n < 0) throw Error(TRITD_ERR_ARG, "n must be >= 0");
        if (n == 0) return;
        need(X, "X"); need(Y, "Y");
        pick_device(-1);
        DBuf a, b;
        a.alloc(n); b.alloc(n);
        TRITD_HIP(hipMemcpy(a.p, X, n * 8, hipMemcpyHostToDevice));
        launch_soft_threshold(a.p, n, lam, b.p, nullptr);
        populate_output(Y, n * 8);
        TRITD_HIP(hipMemcpy(Y, b.p, n * 8, hipMemcpyDeviceToHost));
    });
}

tritd_status tritd_build_design_f64(char which, const double* P, const double* Q, int64_t nP,
                                    int64_t nQ, int32_t r, double* out) {
    return guarded([&] {
        if (which != 'F' && which != 'G' && which != 'H') throw Error(TRITD_ERR_ARG, "which must be 'F', 'G' or 'H'");
        if (nP <= 0 || nQ <= 0 || r <= 0) throw Error(TRITD_ERR_ARG, "sizes must be positive");
        need(P, "P"); need(Q, "Q"); need(out, "out");
        pick_device(-1);
        const int64_t R = (int64_t)r * r;
        // P: 'F' -> B (r,nP,r); 'G','H' -> A (nP,r,r).  Q: 'F','G' -> C (r,r,nQ); 'H' -> B (r,nQ,r)
        DBuf dP, dQ, dO;
        dP.alloc(nP * R); dQ.alloc(nQ * R); dO.alloc(R * nP * nQ);
        TRITD_HIP(hipMemcpy(dP.p, P, dP.n * 8, hipMemcpyHostToDevice));
        TRITD_HIP(hipMemcpy(dQ.p, Q, dQ.n * 8, hipMemcpyHostToDevice));
        launch_design(which, dP.p, dQ.p, nP, nQ, r, dO.p, nullptr);
        populate_output(out, dO.n * 8);
        TRITD_HIP(hipMemcpy(out, dO.p, dO.n * 8, hipMemcpyDeviceToHost));
    });
}

// ---------------------------------------------------------------------------
// driver metrics
// ---------------------------------------------------------------------------
tritd_status tritd_dev_evaluate_f64(const double* X, int64_t n, const double* gt, int64_t m,
                                    const uint8_t* mask, double* rmse, double* nrmse,
                                    void* stream) {
    return guarded([&] {
        hip_entry();  // device pointers from the caller: HIP is in use
        if (n < 0 || m < 0) throw Error(TRITD_ERR_ARG, "sizes must be >= 0");
        need(rmse, "rmse"); need(nrmse, "nrmse");
        if (!mask && m != n) throw Error(TRITD_ERR_ARG, "Arrays have incompatible sizes for this operation.");
        if (n > 0) { need(X, "X"); }
        if (m > 0) { need(gt, "gt"); }
        hipStream_t st = as_stream(stream);
        double h[2] = {0.0, 0.0};
        if (n > 0) {
            const int64_t nb = evaluate_blocks(n);
            DBuf part, out;
            part.alloc(2 * (size_t)nb);
            out.alloc(2);
            int64_t* sc = nullptr;
            TRITD_HIP(hipMalloc(&sc, (size_t)(nb + 1) * sizeof(int64_t)));
            struct Free { int64_t* p; ~Free() { hip_quiet(hipFree(p)); } } fr{sc};
            launch_evaluate(X, gt, m, mask, n, sc, part.p, out.p, sc + nb, st);
            int64_t total = n;
            if (mask)
                TRITD_HIP(hipMemcpyAsync(&total, sc + nb, sizeof total, hipMemcpyDeviceToHost, st));
            TRITD_HIP(hipMemcpyAsync(h, out.p, sizeof h, hipMemcpyDeviceToHost, st));
            TRITD_HIP(hipStreamSynchronize(st));
            // X(mask)-gt(:) with numel(X(mask)) ~= numel(gt) fails in MATLAB
            // (the kernels read gt only below m; the sums are unused then)
            if (total != m) throw Error(TRITD_ERR_ARG, "Arrays have incompatible sizes for this operation.");
        } else if (m != 0) {
            throw Error(TRITD_ERR_ARG, "Arrays have incompatible sizes for this operation.");
        }
        *rmse = std::sqrt(h[0]);
        *nrmse = *rmse / std::sqrt(h[1]);
    });
}

tritd_status tritd_evaluate_f64(const double* X, int64_t n, const double* gt, int64_t m,
                                const uint8_t* mask, double* rmse, double* nrmse) {
    return guarded([&] {
        if (n < 0 || m < 0) throw Error(TRITD_ERR_ARG, "sizes must be >= 0");
        need(rmse, "rmse"); need(nrmse, "nrmse");
        if (n > 0) { need(X, "X"); }
        if (m > 0) { need(gt, "gt"); }
        pick_device(-1);
        DBuf dX, dg, dm;
        dX.alloc((size_t)n);
        dg.alloc((size_t)m);
        if (n > 0) TRITD_HIP(hipMemcpy(dX.p, X, (size_t)n * 8, hipMemcpyHostToDevice));
        if (m > 0) TRITD_HIP(hipMemcpy(dg.p, gt, (size_t)m * 8, hipMemcpyHostToDevice));
        const uint8_t* dmask = nullptr;
        if (mask) {
            dm.alloc_bytes((size_t)n);
            if (n > 0) TRITD_HIP(hipMemcpy(dm.p, mask, (size_t)n, hipMemcpyHostToDevice));
            dmask = reinterpret_cast<const uint8_t*>(dm.p);
        }
        const tritd_status s = tritd_dev_evaluate_f64(dX.p, n, dg.p, m, dmask, rmse, nrmse, nullptr);
        if (s != TRITD_OK) throw Error(s, g_last_error);
    });
}


tritd_status tritd_dev_quality_f64(const double* X1, const double* X2, int64_t n1, int64_t n2,
                                   int64_t nf, double* psnr, double* ssim, double* psnr_frames,
                                   double* ssim_frames, void* stream) {
    return guarded([&] {
        hip_entry();  // device pointers from the caller: HIP is in use
        if (n1 <= 0 || n2 <= 0 || nf <= 0) throw Error(TRITD_ERR_ARG, "sizes must be positive");
        need(X1, "X1"); need(X2, "X2"); need(psnr, "psnr"); need(ssim, "ssim");
        hipStream_t st = as_stream(stream);
        const std::vector<double> w = ssim_window();
        DBuf dw, scratch, pf, sf;
        dw.alloc(w.size());
        TRITD_HIP(hipMemcpyAsync(dw.p, w.data(), w.size() * 8, hipMemcpyHostToDevice, st));
        scratch.alloc(quality_scratch(n1, n2, nf));
        pf.alloc((size_t)nf);
        sf.alloc((size_t)nf);
        const double C1 = (0.01 * 255) * (0.01 * 255), C2 = (0.03 * 255) * (0.03 * 255);
        launch_quality(X1, X2, n1, n2, nf, dw.p, C1, C2, scratch.p, pf.p, sf.p, st);
        std::vector<double> hp((size_t)nf), hs((size_t)nf);
        TRITD_HIP(hipMemcpyAsync(hp.data(), pf.p, (size_t)nf * 8, hipMemcpyDeviceToHost, st));
        TRITD_HIP(hipMemcpyAsync(hs.data(), sf.p, (size_t)nf * 8, hipMemcpyDeviceToHost, st));
        TRITD_HIP(hipStreamSynchronize(st));
        double mp = 0.0, ms = 0.0;  // mean(): sequential sum / count
        for (int64_t f = 0; f < nf; ++f) {
            mp += hp[(size_t)f];
            ms += hs[(size_t)f];
        }
        *psnr = mp / (double)nf;
        *ssim = ms / (double)nf;
        if (psnr_frames) std::copy(hp.begin(), hp.end(), psnr_frames);
        if (ssim_frames) std::copy(hs.begin(), hs.end(), ssim_frames);
    });
}

tritd_status tritd_quality_f64(const double* X1, const double* X2, int64_t n1, int64_t n2,
                               int64_t nf, double* psnr, double* ssim, double* psnr_frames,
                               double* ssim_frames) {
    return guarded([&] {
        if (n1 <= 0 || n2 <= 0 || nf <= 0) throw Error(TRITD_ERR_ARG, "sizes must be positive");
        need(X1, "X1"); need(X2, "X2"); need(psnr, "psnr"); need(ssim, "ssim");
        pick_device(-1);
        const size_t n = (size_t)(n1 * n2 * nf);
        DBuf a, b;
        a.alloc(n);
        b.alloc(n);
        TRITD_HIP(hipMemcpy(a.p, X1, n * 8, hipMemcpyHostToDevice));
        TRITD_HIP(hipMemcpy(b.p, X2, n * 8, hipMemcpyHostToDevice));
        const tritd_status s = tritd_dev_quality_f64(a.p, b.p, n1, n2, nf, psnr, ssim, psnr_frames,
                                                     ssim_frames, nullptr);
        if (s != TRITD_OK) throw Error(s, g_last_error);
    });
}

}  // extern "C"
