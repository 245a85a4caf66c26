"""Dev helper: K5 / K2 time per element for several mode-1 shard heights
(rows of one session, no communicator) at n2 = n3 = 512, r = 8."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import synth

r = 8
d = synth.low_rank_plus_outliers(512, 512, 512, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=200, tol=0.0)
cases = [(0, 512), (0, 256), (256, 512), (0, 384), (0, 192), (0, 128), (0, 320)]
for i0, i1 in cases:
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=512, n2=512, n3=512, i0=i0, i1=i1,
                      D=np.asfortranarray(d["D"][i0:i1]), device=0)
    s.run(10); s.sync(); s.set_timing(True); s.run(30); s.sync()
    km = s.kernel_ms()
    rows = i1 - i0
    print("rows [%3d,%3d) k5 %.4f ms (%.3f us/row)  m3 %.4f ms (%.3f us/row)  it %.4f" % (
        i0, i1, km["fused_update"], km["fused_update"] * 1e3 / rows, km["mode3"], km["mode3"] * 1e3 / rows,
        km["iteration"]), flush=True)
    s.close()
