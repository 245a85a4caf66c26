"""Dev helper: sweep the pool stagger (TRITD_STAGGER) in one process."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import synth
n, r = 512, 8
rng = np.random.default_rng(0)
D = np.asfortranarray(rng.standard_normal((n, n, n)))
A0, B0, C0 = synth.random_factors(n, n, n, r, 123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=100)
vals = [int(v) for v in sys.argv[1].split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
for rep in range(reps):
    for st in vals:
        os.environ["TRITD_STAGGER"] = str(st)
        s = tritd.Session(r, opts, A0, B0, C0, n1=n, n2=n, n3=n, D=D, device=0)
        s.run(2); s.sync(); s.set_timing(True); s.run(10); s.sync()
        km = s.kernel_ms()
        print("stagger %8d rep %d: k5 %.3f ms m3 %.3f it %.3f" % (st, rep, km["fused_update"], km["mode3"], km["iteration"]), flush=True)
        s.close()
