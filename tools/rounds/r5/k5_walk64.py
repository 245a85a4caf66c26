"""fp64 K5 (config 4's r = 8) vs walk length at equal N = 2^27: n3 = 256 / 512
/ 1024 gives 16 / 32 / 64 t-tiles per wave walk.  A falling per-element time
with the walk length prices K5's per-workgroup fixed costs (prologue loads,
Khatri-Rao gather, W epilogue, turnover).  python tools/rounds/r5/k5_walk64.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import tritd  # noqa: E402
from tritd import synth  # noqa: E402

r = 8
for (n1, n2, n3) in [(512, 1024, 256), (512, 512, 512), (512, 256, 1024)]:
    d = synth.low_rank_plus_outliers(n1, n2, n3, r, p_out=0.05, seed=0, init_seed=123)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=60, tol=0.0)
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n1, n2=n2, n3=n3, D=d["D"], device=0)
    del d
    s.run(10)
    s.sync()
    s.set_timing(True)
    s.run(20)
    s.sync()
    km = s.kernel_ms()
    print("%dx%dx%d (t-tiles per walk %d): K5 %.4f ms  K2 %.4f ms  iteration %.4f ms"
          % (n1, n2, n3, n3 // 16, km["fused_update"], km["mode3"], km["iteration"]), flush=True)
    s.close()
