// ThreadSanitizer harness of the device-group host logic (csrc/group.h):
// the code libtritd runs, with the GPU and RCCL replaced by host models.
//   1. ThreadReducer: P shard threads all-reduce (sum / max) many rounds of
//      different lengths; results equal the shard-order sums.
//   2. ThreadReducer abort: a shard throws mid-run; every other shard is
//      released from its barrier, and the first error is rethrown.
//   3. GroupAbort over a model of non-blocking RCCL communicators: an
//      all-reduce stays "in progress" until every peer has enqueued it (a
//      failed peer never does).  A shard throws mid-run; the abort frees the
//      communicators; the others must see the abort at their next poll and
//      never touch a freed communicator (counted), and nothing may hang.
// Built by tests/test_group_tsan.py with -fsanitize=thread.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <vector>

#include "group.h"

using tritd::GroupAbort;
using tritd::run_shard_threads;
using tritd::ThreadReducer;

static int fails = 0;
#define EXPECT(c)                                                           \
    do {                                                                    \
        if (!(c)) {                                                         \
            std::fprintf(stderr, "%s:%d: expected %s\n", __FILE__, __LINE__, #c); \
            ++fails;                                                        \
        }                                                                   \
    } while (0)

static void reducer_sums(int P, int rounds) {
    ThreadReducer red(P);
    std::vector<int> bad(P, 0);
    run_shard_threads(
        P,
        [&](int p) {
            std::vector<double> buf;
            for (int k = 0; k < rounds; ++k) {
                const int n = 1 + (k * 7) % 13;
                const int op = k % 3 == 2;  // every third round a max
                buf.assign(n, 0.0);
                for (int e = 0; e < n; ++e) buf[e] = (double)(p + 1) * (k + 1) + e;
                if (ThreadReducer::allreduce(buf.data(), n, op, &red.ranks[p]) != 0) {
                    ++bad[p];
                    return;
                }
                for (int e = 0; e < n; ++e) {
                    double want = 0.0;
                    for (int q = 0; q < P; ++q) {
                        const double v = (double)(q + 1) * (k + 1) + e;
                        want = op ? (q == 0 || v > want ? v : want) : (q == 0 ? v : want + v);
                    }
                    if (buf[e] != want) ++bad[p];
                }
            }
        },
        [&] { red.abort(); });
    for (int p = 0; p < P; ++p) EXPECT(bad[p] == 0);
}

static void reducer_abort(int P, int thrower, int at) {
    ThreadReducer red(P);
    std::atomic<int> released{0};
    std::string what;
    try {
        run_shard_threads(
            P,
            [&](int p) {
                double x = 1.0;
                for (int k = 0;; ++k) {
                    if (p == thrower && k == at) throw std::runtime_error("shard failed");
                    if (ThreadReducer::allreduce(&x, 1, 0, &red.ranks[p]) != 0) {
                        released.fetch_add(1);
                        throw std::runtime_error("released");
                    }
                    x = 1.0;
                }
            },
            [&] { red.abort(); });
    } catch (const std::exception& e) {
        what = e.what();
    }
    EXPECT(released.load() == P - 1);
    // the first error in shard order: a released shard below the thrower, or
    // the thrower itself when it is shard 0
    EXPECT(what == (thrower == 0 ? "shard failed" : "released"));
}

// Non-blocking communicator model: all-reduce round k completes once all P
// shards have enqueued it; until then its poll says "in progress".
struct Net {
    explicit Net(int P) : P(P), enq((size_t)P), freed((size_t)P) {
        for (auto& e : enq) e.store(0);
        for (auto& f : freed) f.store(false);
    }
    int P;
    std::vector<std::atomic<int>> enq;     // rounds enqueued per shard
    std::vector<std::atomic<bool>> freed;  // the abort freed this communicator
    std::atomic<int> use_after_free{0};
    int enqueue(int p, int k) {
        if (freed[p].load()) use_after_free.fetch_add(1);
        enq[p].store(k + 1);
        return poll(p, k);
    }
    int poll(int p, int k) {
        if (freed[p].load()) use_after_free.fetch_add(1);
        for (int q = 0; q < P; ++q)
            if (enq[q].load() < k + 1) return 1;  // a peer has not arrived: in progress
        return 0;
    }
};

static void group_abort(int P, int thrower, int at) {
    Net net(P);
    GroupAbort ga(P);
    std::atomic<int> aborted_seen{0}, completed{0};
    std::string what;
    try {
        run_shard_threads(
            P,
            [&](int p) {
                for (int k = 0; k < 1000; ++k) {
                    if (p == thrower && k == at) throw std::runtime_error("shard failed");
                    const int s = ga.enqueue(p, [&] { return net.enqueue(p, k); },
                                             [&] { return net.poll(p, k); });
                    if (s < 0) {
                        aborted_seen.fetch_add(1);
                        throw std::runtime_error("aborted");
                    }
                    EXPECT(s == 0);
                    completed.fetch_add(1);
                }
            },
            [&] {
                ga.abort([&](int p) { net.freed[p].store(true); });
            });
    } catch (const std::exception& e) {
        what = e.what();
    }
    EXPECT(net.use_after_free.load() == 0);
    EXPECT(aborted_seen.load() == P - 1);
    EXPECT(ga.aborted());
    EXPECT(what == (thrower == 0 ? "shard failed" : "aborted"));
    // a second abort is a no-op
    EXPECT(!ga.abort([&](int) { EXPECT(false); }));
}

static void group_clean(int P) {
    Net net(P);
    GroupAbort ga(P);
    run_shard_threads(
        P,
        [&](int p) {
            for (int k = 0; k < 300; ++k) {
                const int s = ga.enqueue(p, [&] { return net.enqueue(p, k); },
                                         [&] { return net.poll(p, k); });
                EXPECT(s == 0);
            }
        },
        [&] { ga.abort([&](int p) { net.freed[p].store(true); }); });
    EXPECT(!ga.aborted());
    EXPECT(net.use_after_free.load() == 0);
}

int main() {
    for (int P : {2, 3, 4, 8}) reducer_sums(P, 400);
    for (int P : {2, 4}) {
        reducer_abort(P, 0, 5);
        reducer_abort(P, P - 1, 37);
        group_clean(P);
        group_abort(P, 0, 0);
        group_abort(P, 1, 50);
        group_abort(P, P - 1, 123);
    }
    group_abort(8, 5, 17);
    if (fails) {
        std::fprintf(stderr, "%d expectations failed\n", fails);
        return 1;
    }
    std::printf("group harness ok\n");
    return 0;
}
