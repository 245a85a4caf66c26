"""Dev helper: interleaved in-process A/B of two (or more) builds of libtritd.so.
usage: python tools/ab_lib.py lib1.so,lib2.so reps [iters]"""
import ctypes as C
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import _lib, api, synth
paths, reps = sys.argv[1].split(","), int(sys.argv[2])
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
libs = {}
for p in paths:
    l = C.CDLL(os.path.abspath(p))
    for name, (res, args) in _lib.SIGNATURES.items():
        if not hasattr(l, name):
            continue
        fn = getattr(l, name); fn.restype = res; fn.argtypes = args
    libs[p] = l
n, r = 512, int(os.environ.get("AB_R", "8"))
n1 = n2 = n3 = n
cfg5 = os.environ.get("AB_CFG", "4") == "5"
if cfg5:  # 2048x2048x256 r=16 fp32 (bench.py --config 5)
    n1, n2, n3, r = 2048, 2048, 256, 16
    dd = synth.low_rank_plus_outliers_f32(n1, n2, n3, r, p_out=0.05, seed=0, init_seed=123)
    D, A0, B0, C0 = dd["D"], dd["A0"], dd["B0"], dd["C0"]
    del dd
elif os.environ.get("AB_DATA", "bench") == "noise":  # E dense everywhere (worst case for CE)
    rng = np.random.default_rng(0)
    D = np.asfortranarray(rng.standard_normal((n, n, n)))
    A0, B0, C0 = synth.random_factors(n, n, n, r, 123)
else:  # the bench workload (low rank + 5 % outliers)
    dd = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
    D, A0, B0, C0 = dd["D"], dd["A0"], dd["B0"], dd["C0"]
warm = int(os.environ.get("AB_WARM", "15"))
opts = dict(synth.TRAFFIC_OPTS, maxIter=100, tol=float(os.environ.get("AB_TOL", "1e-5")))
res = {p: [] for p in paths}
for rep in range(reps):
    for p in paths:
        api.lib = _lib.lib = libs[p]
        s = tritd.Session(r, opts, A0, B0, C0, n1=n1, n2=n2, n3=n3, D=D, device=0)
        s.run(warm); s.sync(); s.set_timing(True); s.run(iters); s.sync()
        km = s.kernel_ms()
        pr = s.probe() if hasattr(libs[p], "tritd_session_probe") else None
        res[p].append((km["iteration"], km["fused_update"], km["mode3"]))
        print("%s rep %d: it %.3f k5 %.3f m3 %.3f probe %s" % (p, rep, km["iteration"], km["fused_update"], km["mode3"], pr), flush=True)
        s.close()
for p in paths:
    a = np.array(res[p])
    print("%s median it %.3f k5 %.3f m3 %.3f | min it %.3f" % (p, *np.median(a, 0), a[:, 0].min()))
