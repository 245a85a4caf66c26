"""Dev helper: compact-E dense-tile fraction and errHist of a standalone
n1 x 512 x 512 r=8 solve (rows [0, n1) of the config-4 tensor, its own
problem) versus the one-rank shard emulation of tools/shard_timing.py.
usage: python tools/dense_check.py n1 [n1 ...]"""
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
for n1 in [int(x) for x in sys.argv[1:]]:
    for kind in ("standalone", "shard-of-512"):
        big = kind != "standalone"
        s = tritd.Session(r, opts, d["A0"][:n1] if not big else d["A0"], d["B0"], d["C0"],
                          n1=(n if big else n1), n2=n, n3=n, i0=0, i1=n1,
                          D=np.asfortranarray(d["D"][:n1]), device=0)
        out = []
        for it in (10, 40, 40):
            d0, tpl = s.counters()
            s.run(it); s.sync()
            d1, _ = s.counters()
            out.append("%.2f%%" % (100.0 * (d1 - d0) / it / tpl))
        eh = s.get()["errHist"] if hasattr(s, "get") else None
        print("n1=%d %-12s dense E tiles per window %s  errHist[-1] %s" %
              (n1, kind, out, None if eh is None else "%.3e" % eh[-1]), flush=True)
        s.close()
