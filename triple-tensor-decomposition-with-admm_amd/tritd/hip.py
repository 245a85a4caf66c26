"""Device memory, streams and events through the HIP runtime libtritd itself
is bound to — for hosts that hand libtritd device pointers without a
framework (bench.py, the GPU tests): no second HIP runtime in the process.

    from tritd import hip
    x = hip.DeviceArray.from_host(np.ascontiguousarray(X))   # upload
    y = hip.DeviceArray.empty(x.nbytes)
    ev = hip.EventTimer(stream=None); ev.start(); ...; ms = ev.stop()
    y.to_host(out)

The runtime is the copy of libamdhip64 that the dynamic loader bound for
libtritd.so (tritd._lib: /opt/rocm's unless torch was imported first), opened
with RTLD_NOLOAD so this module never loads another one.
"""
from __future__ import annotations

import ctypes as C
import os

from . import _lib

_H2D, _D2H, _D2D = 1, 2, 3


def _open_runtime():
    try:
        return C.CDLL("libamdhip64.so.7", mode=os.RTLD_NOLOAD | os.RTLD_GLOBAL)
    except OSError as e:  # libtritd.so is loaded, so its runtime is too
        raise ImportError(f"no HIP runtime mapped beside libtritd.so: {e}") from e


rt = _open_runtime()
vp = C.c_void_p
for _name, _args in {
    "hipMalloc": [C.POINTER(vp), C.c_size_t],
    "hipFree": [vp],
    "hipMemcpy": [vp, vp, C.c_size_t, C.c_int],
    "hipMemset": [vp, C.c_int, C.c_size_t],
    "hipDeviceSynchronize": [],
    "hipSetDevice": [C.c_int],
    "hipStreamCreate": [C.POINTER(vp)],
    "hipStreamDestroy": [vp],
    "hipStreamSynchronize": [vp],
    "hipEventCreate": [C.POINTER(vp)],
    "hipEventDestroy": [vp],
    "hipEventRecord": [vp, vp],
    "hipEventSynchronize": [vp],
    "hipEventElapsedTime": [C.POINTER(C.c_float), vp, vp],
    "hipGetErrorString": [C.c_int],
}.items():
    _fn = getattr(rt, _name)
    _fn.argtypes = _args
    _fn.restype = C.c_char_p if _name == "hipGetErrorString" else C.c_int


def check(err, what):
    if err != 0:
        raise _lib.TritdError(3, f"{what}: {rt.hipGetErrorString(err).decode(errors='replace')}")


def set_device(d):
    check(rt.hipSetDevice(int(d)), "hipSetDevice")


def synchronize():
    check(rt.hipDeviceSynchronize(), "hipDeviceSynchronize")


class DeviceArray:
    """`nbytes` of device memory (hipMalloc), freed by free() / on collection."""

    def __init__(self, nbytes):
        self.nbytes = int(nbytes)
        p = vp()
        check(rt.hipMalloc(C.byref(p), max(self.nbytes, 1)), "hipMalloc")
        self.ptr = p.value

    @classmethod
    def empty(cls, nbytes):
        return cls(nbytes)

    @classmethod
    def from_host(cls, a):
        """Upload a C- or F-contiguous numpy array (its memory order)."""
        if not (a.flags.c_contiguous or a.flags.f_contiguous):
            raise ValueError("from_host: contiguous array expected")
        d = cls(a.nbytes)
        check(rt.hipMemcpy(vp(d.ptr), vp(a.ctypes.data), a.nbytes, _H2D), "hipMemcpy H2D")
        return d

    def to_host(self, a):
        """Download into a contiguous numpy array of the same byte size."""
        if a.nbytes != self.nbytes or not (a.flags.c_contiguous or a.flags.f_contiguous):
            raise ValueError("to_host: contiguous array of %d bytes expected" % self.nbytes)
        check(rt.hipMemcpy(vp(a.ctypes.data), vp(self.ptr), a.nbytes, _D2H), "hipMemcpy D2H")
        return a

    def zero(self):
        check(rt.hipMemset(vp(self.ptr), 0, self.nbytes), "hipMemset")

    def free(self):
        if self.ptr:
            rt.hipFree(vp(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Stream:
    def __init__(self):
        s = vp()
        check(rt.hipStreamCreate(C.byref(s)), "hipStreamCreate")
        self.handle = s.value

    def synchronize(self):
        check(rt.hipStreamSynchronize(vp(self.handle)), "hipStreamSynchronize")

    def close(self):
        if self.handle:
            rt.hipStreamDestroy(vp(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class EventTimer:
    """Milliseconds between start() and stop() on one stream (None: the null
    stream), from HIP events recorded on that stream."""

    def __init__(self, stream=None):
        self.st = vp(stream.handle if isinstance(stream, Stream) else stream)
        self.e = [vp(), vp()]
        for e in self.e:
            check(rt.hipEventCreate(C.byref(e)), "hipEventCreate")

    def start(self):
        check(rt.hipEventRecord(self.e[0], self.st), "hipEventRecord")

    def stop(self):
        check(rt.hipEventRecord(self.e[1], self.st), "hipEventRecord")
        check(rt.hipEventSynchronize(self.e[1]), "hipEventSynchronize")
        ms = C.c_float()
        check(rt.hipEventElapsedTime(C.byref(ms), self.e[0], self.e[1]), "hipEventElapsedTime")
        return float(ms.value)

    def __del__(self):
        try:
            for e in self.e:
                if e:
                    rt.hipEventDestroy(e)
        except Exception:
            pass
