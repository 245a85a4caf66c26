"""Timing experiment: per-wave start/end clocks of K5 and K2 (one launch each)
from a -DTRITD_WTRACE=1 build (csrc/wtrace.h), on the bench workload.
    bash tools/build_k5_variants.sh wt="-DTRITD_WTRACE=1"
    TRITD_LIB=ab/wt.so python tools/wtrace.py
Reports the launch span, the shader clock (s_memtime ticks per s_memrealtime
tick x 100 MHz), wave lifetimes and how the span splits into ramp, body and
tail (when the first/last waves start and end)."""
import ctypes as C
import os
import sys
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import tritd  # noqa: E402
from tritd import _lib, synth  # noqa: E402

lib = _lib.lib
n, r = 512, 8
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=100, tol=0.0)
s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, D=d["D"], device=0)
s.run(20)
s.sync()


def report(name, nw):
    f = getattr(lib, name + "_read")
    f.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    buf = (C.c_ulonglong * (5 * nw))()
    assert f(buf, nw) == 0
    a = np.frombuffer(buf, dtype=np.uint64).reshape(nw, 5).astype(np.float64)
    a = a[a[:, 0] > 0]
    r0, r1, c0, c1 = a[:, 0], a[:, 1], a[:, 2], a[:, 3]
    t0 = r0.min()
    us = lambda x: (x - t0) / 100.0  # realtime ticks at 100 MHz -> us
    life = (r1 - r0) / 100.0
    clk = (c1 - c0) / np.maximum(r1 - r0, 1) * 100.0  # MHz
    hw = a[:, 4].astype(np.uint64)
    xcc = (hw >> np.uint64(32)) & np.uint64(0xF)
    print("== %s: %d waves" % (name, len(a)))
    print("  span %.1f us (first start -> last end)" % us(r1.max()))
    print("  starts: p0 %.1f p50 %.1f p99 %.1f max %.1f us" % tuple(np.percentile(us(r0), [0, 50, 99, 100])))
    print("  ends:   min %.1f p1 %.1f p50 %.1f max %.1f us" % tuple(np.percentile(us(r1), [0, 1, 50, 100])))
    print("  lifetime: min %.1f p50 %.1f max %.1f us" % tuple(np.percentile(life, [0, 50, 100])))
    print("  shader clock: p1 %.0f p50 %.0f p99 %.0f MHz" % tuple(np.percentile(clk, [1, 50, 99])))
    for x in range(8):
        m = xcc == x
        if m.any():
            print("    xcc %d: %5d waves, end p50 %.1f max %.1f us, life p50 %.1f" %
                  (x, m.sum(), np.median(us(r1[m])), us(r1[m]).max(), np.median(life[m])))
    # waves sharing a SIMD (HW_ID: simd [5:4], cu [11:8], sh [12], se [15:13])
    hw32 = hw & np.uint64(0xFFFFFFFF)
    key = (xcc << np.uint64(16)) | (((hw32 >> np.uint64(13)) & np.uint64(7)) << np.uint64(8)) | \
          (((hw32 >> np.uint64(12)) & np.uint64(1)) << np.uint64(7)) | \
          (((hw32 >> np.uint64(8)) & np.uint64(15)) << np.uint64(2)) | ((hw32 >> np.uint64(4)) & np.uint64(3))
    ks = np.unique(key)
    per = [np.sort(us(r1[key == k])) for k in ks]
    cnt = np.array([len(p) for p in per])
    last = np.array([p[-1] for p in per])
    first = np.array([p[0] for p in per])
    print("  SIMDs %d, waves per SIMD min %d max %d; SIMD end (last wave) p1 %.1f p50 %.1f max %.1f us; "
          "first wave end p50 %.1f" % (len(ks), cnt.min(), cnt.max(), *np.percentile(last, [1, 50, 100]),
                                       np.median(first)))
    np.savez(os.path.join(ROOT, "gpurun_out", name + ".npz"), a=a)
    return a


report("g_wt_k5", 16384)
report("g_wt_k2", 2048)
s.close()
