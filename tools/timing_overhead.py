"""Dev helper: wall-clock per ADMM iteration at 512^3 r=8 (the bench workload)
with the per-kernel timing events on / off, and for the side-stream modes
(TRITD_OVERLAP = 3: Grams + solves on the side stream, 2: solves only, 0: one stream)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import torch
import tritd
from tritd import synth

n, r, K = 512, 8, 40
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=200, tol=0.0)
for ov in os.environ.get("OVS", "3,2,0").split(","):
    os.environ["TRITD_OVERLAP"] = ov
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, D=d["D"], device=0)
    s.run(5); s.sync()
    for timing in (False, True, False):
        s.set_timing(timing)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        s.run(K); s.sync()
        dt = (time.perf_counter() - t0) / K * 1e3
        km = s.kernel_ms() if timing else {}
        print("overlap=%s timing=%d  %.4f ms/it  %s" % (ov, timing, dt,
              {k: round(v, 4) for k, v in km.items()} if km else ""), flush=True)
    s.close()
