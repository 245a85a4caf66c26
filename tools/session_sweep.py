"""Dev helper: several sessions in one process (fresh allocations each) to
expose placement-dependent bandwidth of the fused update."""
import os, sys, time
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
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    s = tritd.Session(r, opts, A0, B0, C0, n1=n, n2=n, n3=n, D=D, device=0)
    s.run(3); s.sync(); s.set_timing(True); s.run(20); s.sync()
    km = s.kernel_ms()
    print("stagger=%s rep %d: k5 %.3f ms  m3 %.3f  it %.3f" % (os.environ.get("TRITD_STAGGER", "0"), rep, km["fused_update"], km["mode3"], km["iteration"]), flush=True)
    s.close()
