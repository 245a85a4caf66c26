"""Host <-> device copy rates on this box (round 6, the one-shot call's get):
D2H of 1 GB into fresh pageable pages, into prefaulted pageable pages, into
pinned memory (hipHostMalloc), and a chunked D2H through two pinned 64 MB
buffers with the host copy-out on T threads overlapping the next DMA."""
import ctypes as C
import os
import sys
import threading
import time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import tritd  # noqa: E402,F401
from tritd import hip  # noqa: E402

rt = hip.rt
rt.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
rt.hipHostFree.argtypes = [C.c_void_p]
rt.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
rt.hipMemcpyAsync.restype = C.c_int
N = 1 << 30
src = hip.DeviceArray(N)
rt.hipMemset(C.c_void_p(src.ptr), 1, N)
hip.synchronize()


def rate(f, label, reps=3):
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        best = min(best, time.perf_counter() - t0)
    print("%-44s %6.1f GB/s  (%.1f ms)" % (label, N / best / 1e9, best * 1e3), flush=True)


def fresh():
    a = np.empty(N // 8)
    src.to_host(a)
rate(fresh, "D2H into fresh pageable pages")
buf = np.ones(N // 8)
rate(lambda: src.to_host(buf), "D2H into prefaulted pageable pages")
pin = C.c_void_p()
assert rt.hipHostMalloc(C.byref(pin), N, 0) == 0
rate(lambda: rt.hipMemcpy(pin, C.c_void_p(src.ptr), N, 2), "D2H into pinned (hipHostMalloc)")
rate(lambda: rt.hipMemcpy(C.c_void_p(src.ptr), pin, N, 1), "H2D from pinned")
rate(lambda: rt.hipMemcpy(C.c_void_p(src.ptr), C.c_void_p(buf.ctypes.data), N, 1), "H2D from pageable")
pinv = np.ctypeslib.as_array(C.cast(pin, C.POINTER(C.c_double)), shape=(N // 8,))
for T in (1, 4, 8, 16):
    def par_copy():
        n = N // 8
        ths = []
        for q in range(T):
            a, b = n * q // T, n * (q + 1) // T
            th = threading.Thread(target=np.copyto, args=(buf[a:b], pinv[a:b]))
            th.start()
            ths.append(th)
        for th in ths:
            th.join()
    rate(par_copy, "host memcpy pinned -> pageable, %d threads" % T)
rt.hipHostFree(pin)
