"""Dev helper: do A/B builds of libtritd.so give bitwise-identical solves?
usage: python tools/ab_same.py lib1.so,lib2.so [n] [r] [iters]
Runs the same session (synthetic n^3, rank r) with each library and compares
errHist, A, B, C, O, E with the first library's, bitwise."""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import tritd  # noqa: E402
from tritd import _lib, api, synth  # noqa: E402
paths = sys.argv[1].split(",")
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
r = int(sys.argv[3]) if len(sys.argv) > 3 else 8
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 12
n1 = n2 = n3 = n
if os.environ.get("AB_CFG", "4") == "5":  # 2048x2048x256 r=16 fp32 (bench.py --config 5)
    n1, n2, n3, r = 2048, 2048, 256, 16
    d = synth.low_rank_plus_outliers_f32(n1, n2, n3, r, p_out=0.05, seed=0, init_seed=123)
else:
    d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=iters)
ref = None
for p in paths:
    l = C.CDLL(os.path.abspath(p))
    for name, (res, args) in _lib.SIGNATURES.items():
        if hasattr(l, name):
            fn = getattr(l, name); fn.restype = res; fn.argtypes = args
    api.lib = _lib.lib = l
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n1, n2=n2, n3=n3, D=d["D"], device=0,
                      probe=False)
    s.run(iters); s.sync()
    out = s.get()
    s.close()
    if ref is None:
        ref = out
        print("%s: reference (k=%d, errHist[-1]=%.6e)" % (p, out["k"], out["errHist"][-1]))
        continue
    same = {k: bool(np.array_equal(np.asarray(out[k]), np.asarray(ref[k])))
            for k in ("errHist", "A", "B", "C", "O", "E")}
    print("%s: bitwise %s" % (p, same), flush=True)
