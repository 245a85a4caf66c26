"""Per-rank time of the mode-1 sharded schedule on ONE GPU (SURVEY.md §8e;
VERDICT r4 next 4): a session over rows [0, n1/P) of the config-4 problem
with a one-rank RCCL communicator runs exactly the kernels and the two
all-reduces of one rank of a P-GPU run (the all-reduces are trivially one
rank).  Prints the events breakdown (iteration, K5, K2, all-reduce ms) and
the untimed wall rate.  Run under rocprofv3 --kernel-trace --stats for the
per-kernel chain.

    python tools/shard_timing.py [P ...]        (default 8)
    SHARD_MODES=rccl,none   none: no communicator (the single-GPU schedule)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import tritd  # noqa: E402
from tritd import synth  # noqa: E402

n, r = 512, 8
Ps = [int(x) for x in sys.argv[1:]] or [8]
rows_max = n // min(Ps)
d = synth.low_rank_plus_outliers(rows_max, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=400, tol=0.0)
modes = os.environ.get("SHARD_MODES", "rccl").split(",")
A0 = np.asfortranarray(np.random.default_rng(123).standard_normal((n, r, r)))
for P in Ps:
    i1 = n // P
    for mode in modes:
        comm = tritd.Comm(tritd.Comm.unique_id(), 1, 0, 0) if mode == "rccl" else None
        s = tritd.Session(r, opts, A0, d["B0"], d["C0"], n1=n, n2=n, n3=n, i0=0, i1=i1,
                          D=np.asfortranarray(d["D"][:i1]), device=0, comm=comm)
        s.run(20)
        s.sync()
        t0 = time.perf_counter()
        s.run(100)
        tq = time.perf_counter()  # the host's enqueue of 100 iterations (run returns unsynchronised)
        s.sync()
        wall = (time.perf_counter() - t0) * 10
        enq = (tq - t0) * 10
        s.set_timing(True)
        s.run(50)
        s.sync()
        km = s.kernel_ms()
        ar, nar = s.comm_ms()
        print("P=%d rows=%d %-5s: wall %.4f ms/it (host enqueue %.4f) | events: iteration %.4f  "
              "K5 %.4f  K2 %.4f  all-reduce %.4f (%d per it)"
              % (P, i1, mode, wall, enq, km["iteration"], km["fused_update"], km["mode3"], ar, nar),
              flush=True)
        s.close()
        if comm is not None:
            comm.close()
