"""Host enqueue cost per ADMM iteration vs the GPU's own time per iteration
(configs 2, 3, 4): if enqueueing takes as long as running, the host bounds it."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import tritd  # noqa: E402
from tritd import synth  # noqa: E402

cases = {
    2: (lambda: synth.sensor_like(54, 4, 1152, 5, missing=0.10, seed=0, init_seed=123), synth.TRAFFIC_OPTS, 5),
    3: (lambda: synth.video_like(240, 320, 300, 5, seed=0, init_seed=123), synth.VIDEO_OPTS, 5),
    4: (lambda: synth.low_rank_plus_outliers(512, 512, 512, 8, p_out=0.05, seed=0, init_seed=123),
        synth.TRAFFIC_OPTS, 8),
}
for c, (mk, o, r) in cases.items():
    d = mk()
    D = d["D"]
    n1, n2, n3 = D.shape
    opts = dict(o, maxIter=400, tol=0.0)
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n1, n2=n2, n3=n3, D=D, device=0, probe=False)
    s.run(20)
    s.sync()
    K = 200 if c != 4 else 60
    t0 = time.perf_counter()
    s.run(K)
    t1 = time.perf_counter()
    s.sync()
    t2 = time.perf_counter()
    print("config %d: enqueue %.1f us/it, total %.1f us/it" % (c, (t1 - t0) / K * 1e6, (t2 - t0) / K * 1e6),
          flush=True)
    s.close()
