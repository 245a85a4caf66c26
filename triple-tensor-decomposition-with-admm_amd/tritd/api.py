"""Reference-mirroring host API (the MATLAB call surface, in Python).

Every function here keeps the name, argument meaning and failure behaviour of
the MATLAB file it replaces and runs on the GPU through libtritd.so:

    triple_decomp_ADMM(D, r, opts)          fast_robust_triple_tensor/triple_decomp_ADMM.m:1
    triple_decomp_ADMM_outlier(D, r, opts)  alias expected at video_triple_comparison.m:54
    triple_decomp_ADMM_outlier(X, r, rho, lambda, gamma_A, epsilon, p, theta, maxIter, tol)
                                            fast_robust_triple_tensor/test.m:1 (nonconvex variant)
    triple_decomp_ALS(X, r, opts)           fast_robust_triple_tensor/triple_decomp_ALS.m:1
    triple_product(A, B, C[, model])        triple_product.m:1 (model='qi': origin_triple_tensor/)
    unfold(X, mode)                         unfold.m:1
    soft_threshold(X, lam)                  soft_threshold.m:1
    buildF(B, C) / buildG(A, C) / buildH(A, B)   buildF.m:1 / buildG.m:1 / buildH.m:1
    evaluate(X, gt, mask)                   traffic_triple_comparison.m:194-202
    quality_ybz(X1, X2)                     other_methods/Low-rank-.../quality_ybz.m:1

Arrays are numpy, MATLAB (column-major) semantics.  `opts` is a dict (or any
object with attributes) holding the fields the reference reads
(mu, rho, lambda, lambda2, maxIter, tol, disp); a missing one raises
``KeyError("Reference to non-existent field 'x'.")`` like MATLAB, extras
(alphaA, alphaB, origin, ...) are ignored.  One optional field is this
build's own: ``opts.model`` = 'cp' (default: the executed rank-r^2 CP builders)
or 'qi' (Qi's 3-index triple product, origin_triple_tensor/build{F,G,H}.m;
SURVEY.md §8f rank 4).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import PinvToleranceWarning, TritdError, check, check_flags, lib

REQUIRED = ("mu", "rho", "lambda", "lambda2", "maxIter", "tol", "disp")


def _get(opts, name):
    if isinstance(opts, dict):
        return opts[name] if name in opts else None
    return getattr(opts, name, None)


def make_opts(opts):
    """dict/struct -> tritd_opts; raises like MATLAB on a missing field."""
    o = _lib.Opts()
    present = 0
    for name in REQUIRED:
        v = _get(opts, name)
        if v is None:
            raise KeyError(f"Reference to non-existent field '{name}'.")
        present |= _lib.OPT_BITS[name]
    o.mu = float(_get(opts, "mu"))
    o.rho = float(_get(opts, "rho"))
    o.lambda_ = float(_get(opts, "lambda"))
    o.lambda2 = float(_get(opts, "lambda2"))
    o.tol = float(_get(opts, "tol"))
    o.maxIter = int(_get(opts, "maxIter"))
    o.disp = int(bool(_get(opts, "disp")))
    o.present = present
    o.model = model_code(_get(opts, "model"))
    return o


def model_code(m):
    """opts.model -> TRITD_MODEL_*: absent/'cp' -> 0, 'qi' -> 1."""
    if m is None:
        return 0
    key = str(m).lower()
    if key not in _lib.MODELS:
        raise ValueError("opts.model must be 'cp' or 'qi'")
    return _lib.MODELS[key]


def _f64(X):
    return np.asarray(X, dtype=np.float64)


def _fortran(X):
    return np.asfortranarray(_f64(X))


def _size3(X):
    if X.ndim > 3:
        raise ValueError("D must have at most 3 dimensions")
    s = tuple(X.shape) + (1, 1, 1)
    return int(s[0]), int(s[1]), int(s[2])


def _ptr(a):
    return C.c_void_p(a.ctypes.data) if a is not None else None


def initial_factors(n1, n2, n3, r, opts=None, rng=None):
    """A0, B0, C0 in the order of triple_decomp_ADMM.m:23.  Explicit
    opts['A0'/'B0'/'C0'] win (MATLAB's Ziggurat randn is not reproducible
    outside MATLAB, so callers that need parity pass them in)."""
    A0 = _get(opts, "A0") if opts is not None else None
    B0 = _get(opts, "B0") if opts is not None else None
    C0 = _get(opts, "C0") if opts is not None else None
    rng = rng if rng is not None else np.random.default_rng()
    if A0 is None:
        A0 = rng.standard_normal((n1, r, r))
    if B0 is None:
        B0 = rng.standard_normal((r, n2, r))
    if C0 is None:
        C0 = rng.standard_normal((r, r, n3))
    A0 = _fortran(A0).reshape((n1, r, r), order="F")
    B0 = _fortran(B0).reshape((r, n2, r), order="F")
    C0 = _fortran(C0).reshape((r, r, n3), order="F")
    return A0, B0, C0


def triple_decomp_ADMM(D, r, opts, A0=None, B0=None, C0=None, *, device=-1, return_E=False,
                       return_iters=False, virtual_shards=0):
    """[A,B,C,O,errHist] = triple_decomp_ADMM(D, r, opts) on the GPU.

    Extra outputs beyond the reference signature: E (``return_E``) and the
    iteration count (``return_iters``).  ``virtual_shards=P`` runs the mode-1
    sharded schedule as P shards on one device (rehearsal of the multi-GPU
    path).  A float32 D runs the single-class path (MATLAB semantics of a
    `single` D: O, E float32; A, B, C, errHist float64), r <= 16."""
    o = make_opts(opts)
    if np.asarray(D).dtype == np.float32:
        return _admm_f32(D, r, o, opts, A0, B0, C0, device, return_E, return_iters)
    D = _fortran(D)
    n1, n2, n3 = _size3(D)
    r = int(r)
    if A0 is None or B0 is None or C0 is None:
        A0, B0, C0 = initial_factors(n1, n2, n3, r, opts)
    else:
        A0, B0, C0 = initial_factors(n1, n2, n3, r, dict(A0=A0, B0=B0, C0=C0))
    A = np.zeros((n1, r, r), order="F")
    B = np.zeros((r, n2, r), order="F")
    Cf = np.zeros((r, r, n3), order="F")
    O = np.zeros((n1, n2, n3), order="F")
    # E only when asked for (a full tensor more to bring back from the device)
    E = np.zeros((n1, n2, n3), order="F") if return_E else None
    errHist = np.zeros(max(o.maxIter, 1))
    k = _lib.i32(0)
    if virtual_shards and virtual_shards > 1:
        check_flags(lib.tritd_admm_sharded_virtual_f64(_ptr(D), n1, n2, n3, r, C.byref(o), _ptr(A0),
                                                 _ptr(B0), _ptr(C0), int(virtual_shards), _ptr(A),
                                                 _ptr(B), _ptr(Cf), _ptr(O), _ptr(E),
                                                 _ptr(errHist), C.byref(k), int(device)), "triple_decomp_ADMM")
    else:
        check_flags(lib.tritd_admm_f64(_ptr(D), n1, n2, n3, r, C.byref(o), _ptr(A0), _ptr(B0), _ptr(C0),
                                 _ptr(A), _ptr(B), _ptr(Cf), _ptr(O), _ptr(E), _ptr(errHist),
                                 C.byref(k), int(device)), "triple_decomp_ADMM")
    errHist = errHist[: k.value].copy()  # :68 errHist = errHist(1:k)
    out = [A, B, Cf, O, errHist]
    if return_E:
        out.append(E)
    if return_iters:
        out.append(k.value)
    return tuple(out)


def _admm_f32(D, r, o, opts, A0, B0, C0, device, return_E, return_iters):
    D = np.asfortranarray(D, dtype=np.float32)
    n1, n2, n3 = _size3(D)
    r = int(r)
    if A0 is None or B0 is None or C0 is None:
        A0, B0, C0 = initial_factors(n1, n2, n3, r, opts)
    else:
        A0, B0, C0 = initial_factors(n1, n2, n3, r, dict(A0=A0, B0=B0, C0=C0))
    A = np.zeros((n1, r, r), order="F")
    B = np.zeros((r, n2, r), order="F")
    Cf = np.zeros((r, r, n3), order="F")
    O = np.zeros((n1, n2, n3), order="F", dtype=np.float32)
    E = np.zeros((n1, n2, n3), order="F", dtype=np.float32) if return_E else None
    errHist = np.zeros(max(o.maxIter, 1))
    k = _lib.i32(0)
    check_flags(lib.tritd_admm_f32(_ptr(D), n1, n2, n3, r, C.byref(o), _ptr(A0), _ptr(B0), _ptr(C0),
                             _ptr(A), _ptr(B), _ptr(Cf), _ptr(O), _ptr(E), _ptr(errHist),
                             C.byref(k), int(device)), "triple_decomp_ADMM")
    out = [A, B, Cf, O, errHist[: k.value].copy()]
    if return_E:
        out.append(E)
    if return_iters:
        out.append(k.value)
    return tuple(out)


# the name video_triple_comparison.m:54 calls (unresolvable in the reference)
def triple_decomp_ncvx(X, r, rho, lam, gamma_A, epsilon, p, theta, maxIter, tol, A0=None,
                       B0=None, C0=None, *, device=-1, return_iters=False):
    """[A,B,C,O,errHist] of fast_robust_triple_tensor/test.m:1-73 on the GPU
    (the nonconvex variant): outlier ADMM over
    Y = X - O with duals Lambda/Gamma fused into the ALS fit kernel, the
    factors an ALS on X with ridge 1e-12 and the reweighted shrink
    sign(A1).*max(|A1| - gamma_A./(|A1|+epsilon).^(theta-p), 0) on A (:77-92).
    The progress line of :63 goes to the printer every iteration.  On the stop
    test (:65-67) errHist is truncated and O is that of the previous iteration
    (the reference breaks before O = O_new, :71).  fp64, r <= 8."""
    X = _fortran(X)
    n1, n2, n3 = _size3(X)
    r = int(r)
    maxIter = int(maxIter)
    if A0 is None or B0 is None or C0 is None:
        A0, B0, C0 = initial_factors(n1, n2, n3, r)
    else:
        A0, B0, C0 = initial_factors(n1, n2, n3, r, dict(A0=A0, B0=B0, C0=C0))
    A = np.zeros((n1, r, r), order="F")
    B = np.zeros((r, n2, r), order="F")
    Cf = np.zeros((r, r, n3), order="F")
    O = np.zeros((n1, n2, n3), order="F")
    errHist = np.zeros(max(maxIter, 1))
    k = _lib.i32(0)
    check_flags(lib.tritd_ncvx_f64(_ptr(X), n1, n2, n3, r, float(rho), float(lam), float(gamma_A),
                             float(epsilon), float(p), float(theta), maxIter, float(tol), _ptr(A0),
                             _ptr(B0), _ptr(C0), _ptr(A), _ptr(B), _ptr(Cf), _ptr(O), _ptr(errHist),
                             C.byref(k), int(device)), "triple_decomp_ADMM_outlier")
    out = [A, B, Cf, O, errHist[: k.value].copy()]
    if return_iters:
        out.append(k.value)
    return tuple(out)


def triple_decomp_ADMM_outlier(*args, **kw):
    """The name the video driver calls (video_triple_comparison.m:54).  In the
    reference it resolves to two different files' internal names: with
    (D, r, opts) it is the ADMM solver (origin_triple_tensor/triple_decomp_ADMM.m:1,
    same maths as the fast one), with the 10 positional arguments of
    fast_robust_triple_tensor/test.m:1 it is the nonconvex variant."""
    if len(args) >= 10:
        return triple_decomp_ncvx(*args, **kw)
    return triple_decomp_ADMM(*args, **kw)


def make_als_opts(opts):
    """opts of triple_decomp_ALS.m:2-3 (only maxIter and tol are read, in
    that order; a missing one raises like MATLAB, everything else is ignored)."""
    o = _lib.Opts()
    for name in ("maxIter", "tol"):
        if _get(opts, name) is None:
            raise KeyError(f"Reference to non-existent field '{name}'.")
    o.maxIter = int(_get(opts, "maxIter"))
    o.tol = float(_get(opts, "tol"))
    o.present = _lib.OPT_MAXITER | _lib.OPT_TOL
    return o


def triple_decomp_ALS(X, r, opts, A0=None, B0=None, C0=None, *, device=-1, return_iters=False,
                      virtual_shards=0):
    """[A,B,C,errHist] = triple_decomp_ALS(X, r, opts) on the GPU
    (fast_robust_triple_tensor/triple_decomp_ALS.m:1-40).

    The initial factors are drawn here in the order of :8-10 unless given
    (MATLAB's randn is not reproducible outside MATLAB).  The progress line of
    :17-19 goes to the printer (``tritd.set_printer``; stdout by default).
    ``return_iters`` adds k; ``virtual_shards=P`` runs the mode-1 sharded
    schedule as P shards on one device.  fp64, r <= 8."""
    o = make_als_opts(opts)
    X = _fortran(X)
    n1, n2, n3 = _size3(X)
    r = int(r)
    if A0 is None or B0 is None or C0 is None:
        A0, B0, C0 = initial_factors(n1, n2, n3, r, opts)
    else:
        A0, B0, C0 = initial_factors(n1, n2, n3, r, dict(A0=A0, B0=B0, C0=C0))
    A = np.zeros((n1, r, r), order="F")
    B = np.zeros((r, n2, r), order="F")
    Cf = np.zeros((r, r, n3), order="F")
    errHist = np.zeros(max(o.maxIter, 1))
    k = _lib.i32(0)
    if virtual_shards and virtual_shards > 1:
        check_flags(lib.tritd_als_sharded_virtual_f64(_ptr(X), n1, n2, n3, r, C.byref(o), _ptr(A0),
                                                _ptr(B0), _ptr(C0), int(virtual_shards), _ptr(A),
                                                _ptr(B), _ptr(Cf), _ptr(errHist), C.byref(k),
                                                int(device)), "triple_decomp_ALS")
    else:
        check_flags(lib.tritd_als_f64(_ptr(X), n1, n2, n3, r, C.byref(o), _ptr(A0), _ptr(B0), _ptr(C0),
                                _ptr(A), _ptr(B), _ptr(Cf), _ptr(errHist), C.byref(k),
                                int(device)), "triple_decomp_ALS")
    out = [A, B, Cf, errHist[: k.value].copy()]  # :21 errHist = errHist(1:k)
    if return_iters:
        out.append(k.value)
    return tuple(out)


def triple_product(A, B, C_, model="cp"):
    """Xhat = triple_product(A, B, C)  (triple_product.m:1-7).  model='qi': Qi's
    3-index product sum_{p,q,s} A(i,q,s)B(p,j,s)C(p,q,t)
    (origin_triple_tensor/triple_product.m:8-19, buildF.m:2-6)."""
    A = _fortran(A)
    B = _fortran(B)
    C_ = _fortran(C_)
    n1, r, _ = _size3(A)
    n2 = _size3(B)[1]
    n3 = _size3(C_)[2]
    X = np.zeros((n1, n2, n3), order="F")
    fn = lib.tritd_triple_product_qi_f64 if model_code(model) else lib.tritd_triple_product_f64
    check(fn(_ptr(A), _ptr(B), _ptr(C_), n1, n2, n3, r, _ptr(X)))
    return X


def unfold(X, mode):
    """Xn = unfold(X, mode)  (unfold.m:1-13)."""
    X = _fortran(X)
    n1, n2, n3 = _size3(X)
    shapes = {1: (n1, n2 * n3), 2: (n2, n1 * n3), 3: (n3, n1 * n2)}
    out = np.zeros(shapes.get(int(mode), (1,)), order="F")
    check(lib.tritd_unfold_f64(_ptr(X), n1, n2, n3, int(mode), _ptr(out)))
    return out


def soft_threshold(X, lam):
    """O = soft_threshold(X, lam)  (soft_threshold.m:1-2)."""
    X = _fortran(X)
    Y = np.zeros_like(X, order="F")
    check(lib.tritd_soft_threshold_f64(_ptr(X), X.size, float(lam), _ptr(Y)))
    return Y


def evaluate(X, gt, mask=None):
    """[rmse, nrmse] = evaluate(X, gt, mask)  (traffic_triple_comparison.m:194-202):
    rmse = norm(X(mask) - gt(:)), nrmse = rmse / norm(gt(:)); mask None means
    true(size(X)).  gt holds the masked entries in column-major order."""
    X = _fortran(X)
    gt = _fortran(gt)
    m = None
    if mask is not None:
        mk = np.asarray(mask)
        if mk.shape != X.shape:
            raise ValueError("Index exceeds the number of array elements (mask shape differs).")
        m = np.asfortranarray(mk != 0).view(np.uint8)
    rmse, nrmse = C.c_double(0), C.c_double(0)
    check(lib.tritd_evaluate_f64(_ptr(X), X.size, _ptr(gt), gt.size, _ptr(m) if m is not None else None,
                                 C.byref(rmse), C.byref(nrmse)))
    return rmse.value, nrmse.value


def quality_ybz(imagery1, imagery2, per_frame=False):
    """[psnr, ssim] = quality_ybz(imagery1, imagery2): mean over the frames
    (dims 3.. folded) of psnr_index and ssim_index (dynamic range [0, 255])."""
    X1 = _fortran(imagery1)
    X2 = _fortran(imagery2)
    if X1.shape != X2.shape:
        raise ValueError("imagery1 and imagery2 must have the same size")
    n1 = X1.shape[0]
    n2 = X1.shape[1] if X1.ndim > 1 else 1
    nf = max(X1.size // max(n1 * n2, 1), 1)
    p, s = C.c_double(0), C.c_double(0)
    pf = np.zeros(nf)
    sf = np.zeros(nf)
    check(lib.tritd_quality_f64(_ptr(X1), _ptr(X2), n1, n2, nf, C.byref(p), C.byref(s), _ptr(pf),
                                _ptr(sf)))
    if per_frame:
        return p.value, s.value, pf, sf
    return p.value, s.value


def _design(which, P, Q, nP, nQ, r):
    out = np.zeros((r * r, nP * nQ), order="F")
    check(lib.tritd_build_design_f64(which.encode(), _ptr(P), _ptr(Q), nP, nQ, r, _ptr(out)))
    return out


def buildF(B, C_):
    """F = buildF(B, C)  (buildF.m:1-22)."""
    B = _fortran(B)
    C_ = _fortran(C_)
    r, n2, _ = _size3(B)
    return _design("F", B, C_, n2, _size3(C_)[2], r)


def buildG(A, C_):
    """G = buildG(A, C)  (buildG.m:1-22)."""
    A = _fortran(A)
    C_ = _fortran(C_)
    n1, r, _ = _size3(A)
    return _design("G", A, C_, n1, _size3(C_)[2], r)


def buildH(A, B):
    """H = buildH(A, B)  (buildH.m:1-22)."""
    A = _fortran(A)
    B = _fortran(B)
    n1, r, _ = _size3(A)
    return _design("H", A, B, n1, _size3(B)[1], r)


# ---------------------------------------------------------------------------
# Sessions: device-resident loop (bench, multi-GPU)
# ---------------------------------------------------------------------------
class Session:
    """One mode-1 shard [i0, i1) of an n1 x n2 x n3 problem on one GPU.

    D is either a host numpy array holding the shard (column-major, leading
    dimension ldD) or, with ``d_device_ptr``, a device pointer.  ``dtype``
    float32 (or a float32 D) selects the single-class path.  ``probe``
    (default True) times candidate placements of the tensor pool at creation
    and keeps the fastest (TRITD_SESSION_PROBE): worth it for a session that
    runs hundreds of iterations, not for one solve."""

    def __init__(self, r, opts, A0, B0, C0, *, n1, n2, n3, i0=0, i1=None, D=None,
                 d_device_ptr=None, ldD=None, device=0, comm=None, dtype=None, probe=True):
        self._s = C.c_void_p()
        o = make_opts(opts)
        i1 = n1 if i1 is None else i1
        A0 = _fortran(A0)
        B0 = _fortran(B0)
        C0 = _fortran(C0)
        if dtype is None:
            dtype = np.asarray(D).dtype if D is not None else np.float64
        self.f32 = np.dtype(dtype) == np.float32
        flags = _lib.SESSION_F32 if self.f32 else 0
        if probe:
            flags |= _lib.SESSION_PROBE
        if d_device_ptr is not None:
            _lib.check_one_runtime("Session(d_device_ptr=...)")
            dptr = C.c_void_p(int(d_device_ptr))
            flags |= _lib.SESSION_D_ON_DEVICE
            ldD = ldD if ldD is not None else (i1 - i0)
        else:
            D = np.asfortranarray(D, dtype=np.float32 if self.f32 else np.float64)
            dptr = _ptr(D)
            ldD = ldD if ldD is not None else D.shape[0]
        self.n1, self.n2, self.n3, self.i0, self.i1, self.r = n1, n2, n3, i0, i1, r
        self.maxIter = o.maxIter
        check(lib.tritd_session_create(C.byref(self._s), int(device), dptr, int(ldD), n1, n2, n3,
                                       i0, i1, r, C.byref(o), _ptr(A0), _ptr(B0), _ptr(C0),
                                       comm.handle if comm is not None else None, flags))

    def run(self, iters):
        check(lib.tritd_session_run(self._s, int(iters)))

    def sync(self):
        d, s = _lib.i32(0), _lib.i32(0)
        check(lib.tritd_session_sync(self._s, C.byref(d), C.byref(s)))
        return d.value, bool(s.value)

    def flags(self):
        """TRITD_FLAG_* raised so far (read at each sync)."""
        f = C.c_uint32(0)
        check(lib.tritd_session_flags(self._s, C.byref(f)))
        return f.value

    def get(self):
        r, n1, n2, n3 = self.r, self.n1, self.n2, self.n3
        nl = self.i1 - self.i0
        A = np.zeros((n1, r, r), order="F")
        B = np.zeros((r, n2, r), order="F")
        Cf = np.zeros((r, r, n3), order="F")
        dt = np.float32 if self.f32 else np.float64
        O = np.zeros((nl, n2, n3), order="F", dtype=dt)
        E = np.zeros((nl, n2, n3), order="F", dtype=dt)
        eh = np.zeros(max(self.maxIter, 1))
        k = _lib.i32(0)
        fn = lib.tritd_session_get_f32 if self.f32 else lib.tritd_session_get
        check(fn(self._s, _ptr(A), _ptr(B), _ptr(Cf), _ptr(O), _ptr(E), nl, _ptr(eh), C.byref(k)))
        _lib.warn_flags(self.flags(), "Session")
        return dict(A=A, B=B, C=Cf, O=O, E=E, errHist=eh[: k.value].copy(), k=k.value)

    def rre_parts(self, dX_ptr, ldX):
        _lib.check_one_runtime("Session.rre_parts")
        num, den = C.c_double(0), C.c_double(0)
        fn = lib.tritd_session_rre_parts_f32 if self.f32 else lib.tritd_session_rre_parts
        check(fn(self._s, C.c_void_p(int(dX_ptr)), int(ldX), C.byref(num), C.byref(den)))
        return num.value, den.value

    def comm_ms(self):
        """(mean all-reduce ms per timed iteration, all-reduces per iteration)
        — set_timing(True) with a communicator (tritd_session_comm_ms)."""
        ms, n = C.c_double(0), _lib.i32(0)
        check(lib.tritd_session_comm_ms(self._s, C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def probe(self):
        """(probe ms of each candidate tensor pool, index kept)"""
        cap = 64  # up to three rounds of candidates (solver.cpp probe_pool)
        ms = (C.c_double * cap)()
        n, k = _lib.i32(0), _lib.i32(0)
        check(lib.tritd_session_probe(self._s, ms, cap, C.byref(n), C.byref(k)))
        return [ms[i] for i in range(min(n.value, cap))], k.value

    def counters(self):
        """(E tiles stored densely over all fused-update launches, tiles per launch)"""
        a, b = _lib.i64(0), _lib.i64(0)
        check(lib.tritd_session_counters(self._s, C.byref(a), C.byref(b)))
        return a.value, b.value

    def k5_profile(self):
        """(dense N-streams per fused-update launch, compact-E slot accesses per tile)"""
        a, b = _lib.i32(0), _lib.i32(0)
        check(lib.tritd_session_k5_profile(self._s, C.byref(a), C.byref(b)))
        return a.value, b.value

    def set_timing(self, on=True):
        """on: False/0 off, True/1 events around the iteration, K2 and K5,
        "k5"/2 around K5 only (fewer stream markers inside a timed region)."""
        level = 2 if on == "k5" else int(on)
        check(lib.tritd_session_set_timing(self._s, level))

    def kernel_ms(self):
        a, b, c = C.c_double(0), C.c_double(0), C.c_double(0)
        n = _lib.i32(0)
        check(lib.tritd_session_kernel_ms(self._s, C.byref(a), C.byref(b), C.byref(c), C.byref(n)))
        return dict(fused_update=a.value, mode3=b.value, iteration=c.value, samples=n.value)

    def close(self):
        if self._s:
            lib.tritd_session_destroy(self._s)
            self._s = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class AlsSession:
    """Steppable device-resident triple_decomp_ALS on one mode-1 shard
    (bench; one process per GPU with ``comm``).  ``quiet`` drops the
    every-5-iterations progress line and its host synchronisation."""

    def __init__(self, r, opts, A0, B0, C0, *, n1, n2, n3, i0=0, i1=None, X=None,
                 x_device_ptr=None, ldX=None, device=0, comm=None, quiet=True):
        self._s = C.c_void_p()
        o = make_als_opts(opts)
        i1 = n1 if i1 is None else i1
        A0, B0, C0 = _fortran(A0), _fortran(B0), _fortran(C0)
        flags = 0
        if x_device_ptr is not None:
            xptr = C.c_void_p(int(x_device_ptr))
            flags |= _lib.SESSION_D_ON_DEVICE
            ldX = ldX if ldX is not None else (i1 - i0)
        else:
            X = _fortran(X)
            xptr = _ptr(X)
            ldX = ldX if ldX is not None else X.shape[0]
        self.n1, self.n2, self.n3, self.i0, self.i1, self.r = n1, n2, n3, i0, i1, r
        self.maxIter = o.maxIter
        check(lib.tritd_als_session_create(C.byref(self._s), int(device), xptr, int(ldX), n1, n2,
                                           n3, i0, i1, r, C.byref(o), _ptr(A0), _ptr(B0),
                                           _ptr(C0), comm.handle if comm is not None else None,
                                           flags, int(bool(quiet))))

    def run(self, iters):
        check(lib.tritd_als_session_run(self._s, int(iters)))

    def sync(self):
        d, s = _lib.i32(0), _lib.i32(0)
        check(lib.tritd_als_session_sync(self._s, C.byref(d), C.byref(s)))
        return d.value, bool(s.value)

    def flags(self):
        """TRITD_FLAG_* raised so far (read at each sync)."""
        f = C.c_uint32(0)
        check(lib.tritd_als_session_flags(self._s, C.byref(f)))
        return f.value

    def get(self):
        r, n1, n2, n3 = self.r, self.n1, self.n2, self.n3
        A = np.zeros((n1, r, r), order="F")
        B = np.zeros((r, n2, r), order="F")
        Cf = np.zeros((r, r, n3), order="F")
        eh = np.zeros(max(self.maxIter, 1))
        k = _lib.i32(0)
        check(lib.tritd_als_session_get(self._s, _ptr(A), _ptr(B), _ptr(Cf), _ptr(eh), C.byref(k)))
        _lib.warn_flags(self.flags(), "AlsSession")
        return dict(A=A, B=B, C=Cf, errHist=eh[: k.value].copy(), k=k.value)

    def set_timing(self, on=True):
        check(lib.tritd_als_session_set_timing(self._s, int(bool(on))))

    def kernel_ms(self):
        a, b, c = C.c_double(0), C.c_double(0), C.c_double(0)
        n = _lib.i32(0)
        check(lib.tritd_als_session_kernel_ms(self._s, C.byref(a), C.byref(b), C.byref(c),
                                              C.byref(n)))
        return dict(fit=a.value, mode3=b.value, iteration=c.value, samples=n.value)

    def close(self):
        if self._s:
            lib.tritd_als_session_destroy(self._s)
            self._s = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Comm:
    """RCCL communicator owned by libtritd (one process per GPU), or — with
    :meth:`host` — a host transport that hands every all-reduce to a Python
    function (tritd_comm_create_host)."""

    def __init__(self, unique_id: bytes, nranks, rank, device):
        self.handle = C.c_void_p()
        buf = C.create_string_buffer(bytes(unique_id), 128)
        check(lib.tritd_comm_create(C.byref(self.handle), buf, int(nranks), int(rank), int(device)))

    @classmethod
    def host(cls, fn, nranks, rank, device):
        """fn(buf, op) all-reduces the float64 numpy array `buf` in place over
        the ranks (op 0: sum, 1: max).  Every all-reduce of a session drains
        its stream first: a correctness transport (several ranks on one GPU,
        hosts with their own collectives), not the fast path."""
        self = cls.__new__(cls)
        self.handle = C.c_void_p()

        def cb(buf, count, op, user):
            try:
                if count > 0:
                    fn(np.ctypeslib.as_array(buf, shape=(int(count),)), int(op))
                return 0
            except Exception:  # reported to the library as a failed collective
                import traceback
                traceback.print_exc()
                return 1

        self._cb = _lib.ALLREDUCE_FN(cb)  # kept alive with the comm
        check(lib.tritd_comm_create_host(C.byref(self.handle), self._cb, None, int(nranks),
                                         int(rank), int(device)))
        return self

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        check(lib.tritd_comm_unique_id(buf))
        return buf.raw

    def info(self):
        """(nranks, rank, transport) as the communicator reports them
        (RCCL: ncclCommCount / ncclCommUserRank); transport 'rccl' or 'host'."""
        n, me, tr = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib.tritd_comm_info(self.handle, C.byref(n), C.byref(me), C.byref(tr)))
        return n.value, me.value, ("rccl" if tr.value == 0 else "host")

    def close(self):
        if self.handle:
            lib.tritd_comm_destroy(self.handle)
            self.handle = C.c_void_p()


__all__ = ["triple_decomp_ADMM", "triple_decomp_ADMM_outlier", "triple_decomp_ALS", "AlsSession",
           "triple_decomp_ncvx",
           "make_als_opts", "evaluate", "quality_ybz", "triple_product", "unfold",
           "soft_threshold", "buildF", "buildG", "buildH", "Session", "Comm", "TritdError",
           "make_opts", "initial_factors", "PinvToleranceWarning"]
