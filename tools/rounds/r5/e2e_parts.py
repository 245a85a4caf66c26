"""Where the one-shot triple_decomp_ADMM's host-to-host time goes at config 4
(512^3 r=8 fp64, 100 iterations): the call itself, a Session doing the same
steps (create = upload + layout, run, get = downloads), and 1 GB host<->device
copies from pageable memory (fresh np.zeros / touched) and from memory
registered with hipHostRegister (registration timed).
python tools/rounds/r5/e2e_parts.py"""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import tritd  # noqa: E402
from tritd import hip, synth  # noqa: E402

n, r = 512, 8
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=100)
for rep in range(3):
    t = time.perf_counter()
    tritd.triple_decomp_ADMM(d["D"], r, opts, d["A0"], d["B0"], d["C0"], return_E=True)
    print("one-shot call: %.1f ms" % ((time.perf_counter() - t) * 1e3), flush=True)
for rep in range(2):
    t0 = time.perf_counter()
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, D=d["D"], device=0)
    s.sync()
    t1 = time.perf_counter()
    s.run(100)
    s.sync()
    t2 = time.perf_counter()
    res = s.get()
    t3 = time.perf_counter()
    s.close()
    print("session: create %.1f ms  run(100) %.1f ms  get %.1f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3), flush=True)
rt = hip.rt
rt.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
rt.hipHostRegister.restype = C.c_int
rt.hipHostUnregister.argtypes = [C.c_void_p]
rt.hipHostUnregister.restype = C.c_int
nb = n * n * n * 8
dev = hip.DeviceArray(nb)
def copy_h2d(a):
    t = time.perf_counter(); hip.check(rt.hipMemcpy(C.c_void_p(dev.ptr), C.c_void_p(a.ctypes.data), nb, 1), "h2d"); return (time.perf_counter() - t) * 1e3
def copy_d2h(a):
    t = time.perf_counter(); hip.check(rt.hipMemcpy(C.c_void_p(a.ctypes.data), C.c_void_p(dev.ptr), nb, 2), "d2h"); return (time.perf_counter() - t) * 1e3
a = np.zeros(n * n * n)
print("D2H into fresh np.zeros: %.1f ms" % copy_d2h(a))
print("D2H again (touched): %.1f ms" % copy_d2h(a))
print("H2D from touched: %.1f ms" % copy_h2d(a))
b = np.zeros(n * n * n)
t = time.perf_counter(); e = rt.hipHostRegister(C.c_void_p(b.ctypes.data), nb, 0); treg = (time.perf_counter() - t) * 1e3
print("hipHostRegister fresh 1 GB: rc %d, %.1f ms" % (e, treg))
print("D2H registered: %.1f ms" % copy_d2h(b))
print("H2D registered: %.1f ms" % copy_h2d(b))
t = time.perf_counter(); rt.hipHostUnregister(C.c_void_p(b.ctypes.data)); print("unregister: %.1f ms" % ((time.perf_counter() - t) * 1e3))
c = np.ones(n * n * n)
t = time.perf_counter(); e = rt.hipHostRegister(C.c_void_p(c.ctypes.data), nb, 0); treg = (time.perf_counter() - t) * 1e3
print("hipHostRegister touched 1 GB: rc %d, %.1f ms" % (e, treg))
print("H2D registered: %.1f ms" % copy_h2d(c))
rt.hipHostUnregister(C.c_void_p(c.ctypes.data))
