"""Dev helper: K5 time of a shard vs a standalone problem of the same rows.
usage: python tools/shape_k5.py"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import synth

r = 8
opts = dict(synth.TRAFFIC_OPTS, maxIter=200, tol=0.0)
d = synth.low_rank_plus_outliers(512, 512, 512, r, p_out=0.05, seed=0, init_seed=123)


def run(label, n1, i1, D, A0):
    s = tritd.Session(r, opts, A0, d["B0"], d["C0"], n1=n1, n2=512, n3=512, i0=0, i1=i1,
                      D=np.asfortranarray(D), device=0)
    s.run(5); s.sync(); s.set_timing(True); s.run(20); s.sync()
    km = s.kernel_ms()
    ms, pick = s.probe()
    print("%-34s it %.4f k5 %.4f m3 %.4f probe %s pick %d" % (label, km["iteration"], km["fused_update"],
          km["mode3"], [round(x, 3) for x in ms], pick), flush=True)
    s.close()


run("shard 0..256 of 512", 512, 256, d["D"][:256], d["A0"])
run("standalone 256x512x512", 256, 256, d["D"][:256], d["A0"][:256])
os.environ["TRITD_PROBE"] = "1"
run("shard 0..256, no probe", 512, 256, d["D"][:256], d["A0"])
del os.environ["TRITD_PROBE"]
run("shard 0..384 of 512", 512, 384, d["D"][:384], d["A0"])
run("shard 0..192 of 512", 512, 192, d["D"][:192], d["A0"])
run("full 512", 512, 512, d["D"], d["A0"])
