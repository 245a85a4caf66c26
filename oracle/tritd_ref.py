"""ctypes loader for the C restatement (oracle/tritd_ref.c) — TEST
INFRASTRUCTURE ONLY (tests/, __graft_entry__.smoke(), bench.py cpu_baseline)."""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PATH = os.path.join(HERE, "build", "libtritd_ref.so")
vp = C.c_void_p
i64 = C.c_int64


def load():
    if not os.path.exists(PATH):
        raise ImportError("oracle/build/libtritd_ref.so missing: run `make -C oracle`")
    lib = C.CDLL(PATH)
    lib.tritd_ref_admm.restype = C.c_int
    lib.tritd_ref_admm.argtypes = [vp, i64, i64, i64, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                   vp, C.c_int]
    lib.tritd_ref_admm_f32.restype = C.c_int
    lib.tritd_ref_admm_f32.argtypes = lib.tritd_ref_admm.argtypes
    lib.tritd_ref_triple_product.argtypes = [vp, vp, vp, i64, i64, i64, C.c_int, vp]
    lib.tritd_ref_unfold.argtypes = [vp, i64, i64, i64, C.c_int, vp]
    lib.tritd_ref_build.argtypes = [C.c_char, vp, vp, i64, i64, C.c_int, vp]
    lib.tritd_ref_threads.restype = C.c_int
    lib.tritd_ref_set_threads.argtypes = [C.c_int]
    return lib


def _p(a):
    return C.c_void_p(a.ctypes.data)


def admm(lib, D, r, opts, A0, B0, C0, max_iters=0):
    """C restatement; D of dtype float32 selects the MATLAB-single path."""
    single = np.asarray(D).dtype == np.float32
    D = np.asfortranarray(D, dtype=np.float32 if single else np.float64)
    n1, n2, n3 = D.shape
    o = np.array([opts["mu"], opts["rho"], opts["lambda"], opts["lambda2"], opts["maxIter"],
                  opts["tol"], opts["disp"]], dtype=np.float64)
    A = np.zeros((n1, r, r), order="F")
    B = np.zeros((r, n2, r), order="F")
    Cc = np.zeros((r, r, n3), order="F")
    dt = np.float32 if single else np.float64
    O = np.zeros((n1, n2, n3), order="F", dtype=dt)
    E = np.zeros((n1, n2, n3), order="F", dtype=dt)
    eh = np.zeros(max(int(opts["maxIter"]), 1))
    A0, B0, C0 = (np.asfortranarray(x, dtype=np.float64) for x in (A0, B0, C0))
    fn = lib.tritd_ref_admm_f32 if single else lib.tritd_ref_admm
    k = fn(_p(D), n1, n2, n3, r, _p(o), _p(A0), _p(B0), _p(C0), _p(A), _p(B),
                           _p(Cc), _p(O), _p(E), _p(eh), int(max_iters))
    return A, B, Cc, O, eh[:k].copy(), E, k
