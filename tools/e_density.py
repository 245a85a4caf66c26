"""Dev helper: fraction of nonzero E (and per-16x16-tile max count) per iteration
of the bench workload, stepping one session.  usage: python tools/e_density.py [n]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import synth
n = int(sys.argv[1]) if len(sys.argv) > 1 else 512
r = 8
data = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=100)
s = tritd.Session(r, opts, data["A0"], data["B0"], data["C0"], n1=n, n2=n, n3=n, D=data["D"], device=0)
for k in range(1, 101):
    s.run(1)
    if k % 5 and k > 12:
        continue
    E = s.get()["E"]
    nz = E != 0
    # per 16 (i) x 16 (t) tile counts for fixed j
    t = nz.reshape(n // 16, 16, n, n // 16, 16).sum(axis=(1, 4))
    print("k %3d  nnz %.4f  tile max %3d  p99 %5.1f  tiles>32 %.4f" % (
        k, nz.mean(), t.max(), np.percentile(t, 99), (t > 32).mean()), flush=True)
s.close()
