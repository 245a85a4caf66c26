"""Dev helper: per-rank compute time of the mode-1 sharded schedule, without
communication.  A session over rows [0, n1/P) of the config-4 problem with no
communicator runs a rank's kernels; TRITD_OVERLAP=0 forces the phase-serial
schedule the sharded path uses, 3 the overlapped single-GPU schedule.
usage: python tools/shard_timing.py [P ...]"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import synth

n, r = 512, 8
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=200, tol=0.0)
Ps = [int(x) for x in sys.argv[1:]] or [1, 2, 4, 8]
# modes: serial phase order / overlapped single-GPU order (no communicator);
# rccl-serial / rccl-sharded: a one-rank RCCL communicator (the all-reduces
# run, trivially) with TRITD_SHOV=0 / 1
modes = os.environ.get("SHARD_MODES", "serial,overlap,rccl-serial,rccl-sharded").split(",")
for P in Ps:
    i1 = n // P
    for mode in modes:
        os.environ["TRITD_OVERLAP"] = "3" if mode == "overlap" else "0"
        os.environ["TRITD_SHOV"] = "1" if mode == "rccl-sharded" else "0"
        comm = tritd.Comm(tritd.Comm.unique_id(), 1, 0, 0) if mode.startswith("rccl") else None
        s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, i0=0, i1=i1,
                          D=np.asfortranarray(d["D"][:i1]), device=0, comm=comm)
        import time
        s.run(10); s.sync()
        t0 = time.perf_counter(); s.run(40); t1 = time.perf_counter(); s.sync(); t2 = time.perf_counter()
        s.set_timing(True); s.run(40); s.sync()
        km = s.kernel_ms()
        print("P=%d rows=%d %-13s: iteration %.4f ms  k5 %.4f  m3 %.4f | untimed: enqueue %.4f ms/it, wall %.4f ms/it" %
              (P, i1, mode, km["iteration"], km["fused_update"], km["mode3"], (t1 - t0) * 25, (t2 - t0) * 25), flush=True)
        s.close()
        if comm is not None:
            comm.close()
