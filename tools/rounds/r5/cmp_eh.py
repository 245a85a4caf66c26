"""errHist of two libtritd builds on the same fp32 problem (256^3 r=16, 100
iterations: config 5's rank), side by side, plus the max |L| difference of
one K5 step.  usage: python tools/rounds/r5/cmp_eh.py libA.so libB.so"""
import ctypes as C
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import _lib, api, synth
libs = []
for p in sys.argv[1:3]:
    l = C.CDLL(os.path.abspath(p))
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(l, name):
            fn = getattr(l, name); fn.restype = res; fn.argtypes = args
    libs.append(l)
n, r = 256, 16
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
D = d["D"].astype(np.float32, order="F")
opts = dict(synth.TRAFFIC_OPTS, maxIter=int(os.environ.get("ITERS", "100")))
out = []
for l in libs:
    api.lib = _lib.lib = l
    A, B, Cc, O, eh, E, k = tritd.triple_decomp_ADMM(D, r, opts, d["A0"], d["B0"], d["C0"],
                                                     return_E=True, return_iters=True)
    out.append((A, B, Cc, O, eh, E, k))
    print(sys.argv[1 + len(out) - 1], "k", k, flush=True)
ea, eb = out[0][4], out[1][4]
m = min(len(ea), len(eb))
for i in range(m):
    print("%3d %.9e %.9e rel %.2e" % (i + 1, ea[i], eb[i], abs(ea[i] - eb[i]) / ea[i]))
for key, q in (("A", 0), ("B", 1), ("C", 2), ("O", 3), ("E", 5)):
    x, y = out[0][q].astype(np.float64), out[1][q].astype(np.float64)
    print(key, "rel diff", np.linalg.norm(x - y) / max(np.linalg.norm(x), 1e-300))
