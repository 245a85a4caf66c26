// Host-side driver of a device group: one host thread per mode-1 shard
// (SURVEY.md §8e), the in-process all-reduce of shards that share a GPU, and
// the abort protocol that keeps a failing shard from leaving the others
// blocked — or touching a communicator that the abort has freed.
//
// No HIP or RCCL here: the communicator operations come in as callables, so
// tests/test_group_tsan.py builds this file into a ThreadSanitizer harness
// (tests/group_harness.cpp) on the CPU with the same code the library runs.
#pragma once

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <exception>
#include <mutex>
#include <thread>
#include <vector>

namespace tritd {

// In-process all-reduce of a device group whose shards share a GPU (one
// device repeated: RCCL refuses a GPU twice in one communicator): each
// shard's host transport lands here, on that shard's host thread.  Sums run
// in shard order (s = b0; s += b1; ...), like the device-side virtual-shard
// sum.  abort() wakes every waiter with a failure, so a shard that throws
// never leaves the others blocked in a collective.
struct ThreadReducer {
    struct Rank {
        ThreadReducer* r;
        int rank;
    };
    int P;
    std::vector<Rank> ranks;
    std::vector<double*> bufs;
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    bool aborted = false;
    explicit ThreadReducer(int p) : P(p), bufs(p, nullptr) {
        for (int q = 0; q < p; ++q) ranks.push_back({this, q});
    }
    bool barrier() {
        std::unique_lock<std::mutex> lk(m);
        if (aborted) return false;
        const uint64_t g = gen;
        if (++arrived == P) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g || aborted; });
        }
        return !aborted;
    }
    void abort() {
        std::lock_guard<std::mutex> lk(m);
        aborted = true;
        cv.notify_all();
    }
    // tritd_allreduce_fn: (buf, count, op 0 sum / 1 max, user) -> 0 on success
    static int32_t allreduce(double* buf, int64_t count, int32_t op, void* user) {
        Rank* rk = static_cast<Rank*>(user);
        ThreadReducer* r = rk->r;
        {
            std::lock_guard<std::mutex> lk(r->m);
            r->bufs[rk->rank] = buf;
        }
        if (!r->barrier()) return 1;
        if (rk->rank == 0) {  // the others wait at the next barrier
            for (int64_t e = 0; e < count; ++e) {
                double v = r->bufs[0][e];
                for (int q = 1; q < r->P; ++q) v = op ? (v < r->bufs[q][e] ? r->bufs[q][e] : v) : v + r->bufs[q][e];
                for (int q = 0; q < r->P; ++q) r->bufs[q][e] = v;
            }
        }
        return r->barrier() ? 0 : 1;
    }
};

// Abort state of the communicators of one device group (one per shard).
// Every use of shard p's communicator — an enqueue, a completion poll, the
// abort itself — runs under lock(p) and only while !aborted, so once abort()
// has run no thread touches a communicator again.  The communicators are
// non-blocking (api.cpp: group_comms), so no call holds a lock while it
// waits for a peer: a shard whose peer has failed sees the abort at its next
// poll instead of waiting forever inside the library.
class GroupAbort {
public:
    explicit GroupAbort(int p) : locks_(p) {}
    bool aborted() const { return aborted_.load(std::memory_order_acquire); }
    // Run op() on shard p's communicator unless the group has been aborted
    // (false: aborted, op not run).
    template <class Op>
    bool use(int p, Op&& op) {
        std::lock_guard<std::mutex> lk(locks_[p]);
        if (aborted()) return false;
        op();
        return true;
    }
    // Enqueue on shard p, then poll the communicator until the enqueue has
    // completed (non-blocking communicators return "in progress" while they
    // connect): enqueue() and poll() return 0 done, 1 in progress, or an
    // error code, which is returned.  -1: the group was aborted.
    template <class Enq, class Poll>
    int enqueue(int p, Enq&& enq, Poll&& poll) {
        int s = 0;
        if (!use(p, [&] { s = enq(); })) return -1;
        while (s == 1) {
            std::this_thread::yield();
            if (!use(p, [&] { s = poll(); })) return -1;
        }
        return s;
    }
    // First caller: mark the group aborted, then abort_comm(p) for every
    // shard under its lock (waits for an enqueue or poll in progress to
    // return, which it does without waiting for peers).  Later callers
    // return at once.  Returns whether this call aborted.
    template <class AbortComm>
    bool abort(AbortComm&& abort_comm) {
        if (aborted_.exchange(true, std::memory_order_acq_rel)) return false;
        for (size_t p = 0; p < locks_.size(); ++p) {
            std::lock_guard<std::mutex> lk(locks_[p]);
            abort_comm((int)p);
        }
        return true;
    }

private:
    std::atomic<bool> aborted_{false};
    std::vector<std::mutex> locks_;
};

// Run body(p) for p = 0..P-1, shard 0 on the calling thread (a host print
// callback such as mexPrintf stays on the host's own thread), the others on
// threads of their own.  A shard that throws calls abort_all() — which must
// release every other shard from its collectives — and the first error (in
// shard order) is rethrown once every thread has joined.
template <class Body, class AbortAll>
void run_shard_threads(int P, Body&& body, AbortAll&& abort_all) {
    std::vector<std::exception_ptr> err((size_t)P);
    auto run = [&](int p) {
        try {
            body(p);
        } catch (...) {
            err[(size_t)p] = std::current_exception();
            abort_all();
        }
    };
    std::vector<std::thread> th;
    th.reserve(P > 1 ? (size_t)(P - 1) : 0);
    // a thread that cannot be started fails the call: the shards already
    // running are released from their collectives and joined first
    std::exception_ptr spawn_err;
    for (int p = 1; p < P && !spawn_err; ++p) {
        try {
            th.emplace_back(run, p);
        } catch (...) {
            spawn_err = std::current_exception();
            abort_all();
        }
    }
    if (!spawn_err) run(0);
    for (auto& t : th) t.join();
    if (spawn_err) std::rethrow_exception(spawn_err);
    for (int p = 0; p < P; ++p)
        if (err[(size_t)p]) std::rethrow_exception(err[(size_t)p]);
}

}  // namespace tritd
