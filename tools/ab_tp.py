"""Dev helper: interleaved in-process A/B of the device-form triple product on
512^3 r=8 (bench.py's primitive), with an env knob read at each launch.
usage: python tools/ab_tp.py VAR v1,v2 reps"""
import ctypes as C
import os
import statistics
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
from tritd import hip  # noqa: E402
from tritd._lib import check, lib  # noqa: E402
var, vals, reps = sys.argv[1], sys.argv[2].split(","), int(sys.argv[3])
n, r = 512, 8
N, R = n ** 3, r * r
rng = np.random.default_rng(0)
hip.set_device(0)
A = hip.DeviceArray.from_host(rng.standard_normal(n * R))
B = hip.DeviceArray.from_host(rng.standard_normal(R * n))
Cc = hip.DeviceArray.from_host(rng.standard_normal(R * n))
Y = hip.DeviceArray(N * 8)
p = lambda t: C.c_void_p(t.ptr)  # noqa: E731
ev = hip.EventTimer(None)
res = {v: [] for v in vals}
outs = {}
for rep in range(reps):
    for v in vals:
        if v == "-":
            os.environ.pop(var, None)
        else:
            os.environ[var] = v
        fn = lambda: check(lib.tritd_dev_triple_product_f64(p(A), p(B), p(Cc), n, n, n, r, p(Y),  # noqa: E731
                                                            C.c_void_p(0)))
        for _ in range(3):
            fn()
        hip.synchronize()
        ev.start()
        for _ in range(20):
            fn()
        ms = ev.stop() / 20
        res[v].append(ms)
        if rep == 0:
            h = np.empty(N)
            Y.to_host(h)
            outs[v] = h
for v in vals:
    ms = statistics.median(res[v])
    print("%s=%s median %.4f ms  %.3f of f64 MFMA" % (var, v, ms, 2.0 * N * R / (ms * 1e-3) / 78.6e12))
ref = outs[vals[0]]
for v in vals[1:]:
    print("%s bitwise equal to %s: %s" % (v, vals[0], bool(np.array_equal(outs[v], ref))))
