"""Timing experiment: K5's t-walk phase clocks (s_memtime) from a K5_PROF=1
build, on the bench workload.
usage: TRITD_LIB=ab/prof.so python tools/rounds/r4/k5_prof.py"""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import tritd
from tritd import _lib, synth

lib = _lib.lib
lib.tritd_k5prof.argtypes = [C.POINTER(C.c_ulonglong)]
n, r = 512, 8
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=100, tol=0.0)
s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, D=d["D"], device=0)
s.run(15); s.sync()
buf = (C.c_ulonglong * 16)()
lib.tritd_k5prof(buf)  # clear
s.set_timing(True); s.run(10); s.sync()
km = s.kernel_ms()
lib.tritd_k5prof(buf)
steps = buf[8]
names = ["prefetch issue", "decode E, E^(k-1)", "L MFMAs", "elementwise + Y_L stores", "encode E",
         "T transpose + store", "W MFMAs", "staging + barrier"]
tot = sum(buf[q] for q in range(8))
print("K5 %.4f ms, %d wave-steps; clocks per wave-step (s_memtime):" % (km["fused_update"], steps))
for q in range(8):
    print("  %-26s %8.1f  (%4.1f %%)" % (names[q], buf[q] / steps, 100.0 * buf[q] / tot))
print("  %-26s %8.1f" % ("total", tot / steps))
s.close()
