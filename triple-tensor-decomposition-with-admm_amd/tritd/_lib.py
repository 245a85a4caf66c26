"""ctypes binding of libtritd.so (include/tritd.h).

The library is the product: there is no CPU fallback.  If the shared object
is missing this module raises at import time; if no gfx950 device is visible
every compute entry point returns TRITD_ERR_NODEV and the Python wrappers
raise `TritdError`.
"""
from __future__ import annotations

import ctypes as C
import importlib.util
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TRITD_LIB", os.path.join(HERE, "libtritd.so"))

OK = 0
TRITD_ERR_HIP = 3
STATUS_NAMES = {0: "TRITD_OK", 1: "TRITD_ERR_ARG", 2: "TRITD_ERR_OPTS", 3: "TRITD_ERR_HIP",
                4: "TRITD_ERR_RCCL", 5: "TRITD_ERR_NOMEM", 6: "TRITD_ERR_NODEV",
                7: "TRITD_ERR_UNSUPPORTED", 8: "TRITD_ERR_STATE"}

OPT_MU, OPT_RHO, OPT_LAMBDA, OPT_LAMBDA2, OPT_MAXITER, OPT_TOL, OPT_DISP = (1 << i for i in range(7))
OPT_BITS = {"mu": OPT_MU, "rho": OPT_RHO, "lambda": OPT_LAMBDA, "lambda2": OPT_LAMBDA2,
            "maxIter": OPT_MAXITER, "tol": OPT_TOL, "disp": OPT_DISP}
MODELS = {"cp": 0, "qi": 1}  # opts.model: TRITD_MODEL_CP / TRITD_MODEL_QI (include/tritd.h)
SESSION_D_ON_DEVICE = 1
SESSION_F32 = 2
SESSION_PROBE = 4
FLAG_PINV_TOL = 1  # TRITD_FLAG_PINV_TOL (include/tritd.h)


class TritdError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


class PinvToleranceWarning(UserWarning):
    """TRITD_FLAG_PINV_TOL: a ridge Gram's smallest pivot came within 1e3x of
    MATLAB's pinv tolerance (triple_decomp_ADMM.m:78,86,93), where pinv could
    truncate singular values and the GPU's inverse does not — results may
    differ from the reference's beyond rounding."""


class Opts(C.Structure):
    _fields_ = [("mu", C.c_double), ("rho", C.c_double), ("lambda_", C.c_double),
                ("lambda2", C.c_double), ("tol", C.c_double), ("maxIter", C.c_int32),
                ("disp", C.c_int32), ("present", C.c_uint32), ("model", C.c_uint32)]


PRINT_FN = C.CFUNCTYPE(None, C.c_char_p, C.c_void_p)
# tritd_allreduce_fn: (buf, count, op 0 sum / 1 max, user) -> 0 on success
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int32, C.POINTER(C.c_double), C.c_int64, C.c_int32, C.c_void_p)

dp = C.POINTER(C.c_double)
vp = C.c_void_p
i64 = C.c_int64
i32 = C.c_int32

# name -> (restype, argtypes); every symbol declared in include/tritd.h
SIGNATURES = {
    "tritd_version": (C.c_char_p, []),
    "tritd_last_error": (C.c_char_p, []),
    "tritd_last_flags": (C.c_uint32, []),
    "tritd_session_flags": (C.c_int, [vp, C.POINTER(C.c_uint32)]),
    "tritd_als_session_flags": (C.c_int, [vp, C.POINTER(C.c_uint32)]),
    "tritd_set_print_callback": (None, [PRINT_FN, vp]),
    "tritd_device_count": (C.c_int, [C.POINTER(i32)]),
    "tritd_admm_f64": (C.c_int, [vp, i64, i64, i64, i32, C.POINTER(Opts), vp, vp, vp, vp, vp, vp,
                                 vp, vp, vp, C.POINTER(i32), i32]),
    "tritd_admm_f32": (C.c_int, [vp, i64, i64, i64, i32, C.POINTER(Opts), vp, vp, vp, vp, vp, vp,
                                 vp, vp, vp, C.POINTER(i32), i32]),
    "tritd_session_create": (C.c_int, [C.POINTER(vp), i32, vp, i64, i64, i64, i64, i64, i64, i32,
                                       C.POINTER(Opts), vp, vp, vp, vp, C.c_uint32]),
    "tritd_session_run": (C.c_int, [vp, i32]),
    "tritd_session_sync": (C.c_int, [vp, C.POINTER(i32), C.POINTER(i32)]),
    "tritd_session_get": (C.c_int, [vp, vp, vp, vp, vp, vp, i64, vp, C.POINTER(i32)]),
    "tritd_session_rre_parts": (C.c_int, [vp, vp, i64, dp, dp]),
    "tritd_session_get_f32": (C.c_int, [vp, vp, vp, vp, vp, vp, i64, vp, C.POINTER(i32)]),
    "tritd_session_rre_parts_f32": (C.c_int, [vp, vp, i64, dp, dp]),
    "tritd_session_set_timing": (C.c_int, [vp, i32]),
    "tritd_session_kernel_ms": (C.c_int, [vp, dp, dp, dp, C.POINTER(i32)]),
    "tritd_session_comm_ms": (C.c_int, [vp, dp, C.POINTER(i32)]),
    "tritd_session_probe": (C.c_int, [vp, dp, i32, C.POINTER(i32), C.POINTER(i32)]),
    "tritd_session_counters": (C.c_int, [vp, C.POINTER(i64), C.POINTER(i64)]),
    "tritd_session_k5_profile": (C.c_int, [vp, C.POINTER(i32), C.POINTER(i32)]),
    "tritd_session_destroy": (None, [vp]),
    "tritd_comm_unique_id": (C.c_int, [vp]),
    "tritd_comm_create": (C.c_int, [C.POINTER(vp), vp, i32, i32, i32]),
    "tritd_comm_create_host": (C.c_int, [C.POINTER(vp), ALLREDUCE_FN, vp, i32, i32, i32]),
    "tritd_comm_destroy": (None, [vp]),
    "tritd_comm_info": (C.c_int, [vp, C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]),
    "tritd_admm_sharded_virtual_f64": (C.c_int, [vp, i64, i64, i64, i32, C.POINTER(Opts), vp, vp,
                                                 vp, i32, vp, vp, vp, vp, vp, vp, C.POINTER(i32),
                                                 i32]),
    "tritd_set_devices": (C.c_int, [C.POINTER(i32), i32]),
    "tritd_shutdown": (None, []),
    "tritd_als_f64": (C.c_int, [vp, i64, i64, i64, i32, C.POINTER(Opts), vp, vp, vp, vp, vp, vp,
                                vp, C.POINTER(i32), i32]),
    "tritd_als_session_create": (C.c_int, [C.POINTER(vp), i32, vp, i64, i64, i64, i64, i64, i64,
                                           i32, C.POINTER(Opts), vp, vp, vp, vp, C.c_uint32, i32]),
    "tritd_als_session_run": (C.c_int, [vp, i32]),
    "tritd_als_session_sync": (C.c_int, [vp, C.POINTER(i32), C.POINTER(i32)]),
    "tritd_als_session_get": (C.c_int, [vp, vp, vp, vp, vp, C.POINTER(i32)]),
    "tritd_als_session_set_timing": (C.c_int, [vp, i32]),
    "tritd_als_session_kernel_ms": (C.c_int, [vp, dp, dp, dp, C.POINTER(i32)]),
    "tritd_als_session_destroy": (None, [vp]),
    "tritd_als_sharded_virtual_f64": (C.c_int, [vp, i64, i64, i64, i32, C.POINTER(Opts), vp, vp, vp,
                                                i32, vp, vp, vp, vp, C.POINTER(i32), i32]),
    "tritd_evaluate_f64": (C.c_int, [vp, i64, vp, i64, vp, dp, dp]),
    "tritd_quality_f64": (C.c_int, [vp, vp, i64, i64, i64, dp, dp, vp, vp]),
    "tritd_dev_evaluate_f64": (C.c_int, [vp, i64, vp, i64, vp, dp, dp, vp]),
    "tritd_dev_quality_f64": (C.c_int, [vp, vp, i64, i64, i64, dp, dp, vp, vp, vp]),
    "tritd_triple_product_f64": (C.c_int, [vp, vp, vp, i64, i64, i64, i32, vp]),
    "tritd_unfold_f64": (C.c_int, [vp, i64, i64, i64, i32, vp]),
    "tritd_soft_threshold_f64": (C.c_int, [vp, i64, C.c_double, vp]),
    "tritd_build_design_f64": (C.c_int, [C.c_char, vp, vp, i64, i64, i32, vp]),
    "tritd_dev_unfold_f64": (C.c_int, [vp, i64, i64, i64, i32, vp, vp]),
    "tritd_dev_soft_threshold_f64": (C.c_int, [vp, i64, C.c_double, vp, vp]),
    "tritd_dev_triple_product_f64": (C.c_int, [vp, vp, vp, i64, i64, i64, i32, vp, vp]),
    "tritd_triple_product_qi_f64": (C.c_int, [vp, vp, vp, i64, i64, i64, i32, vp]),
    "tritd_ncvx_f64": (C.c_int, [vp, i64, i64, i64, i32] + [C.c_double] * 6
                       + [i32, C.c_double, vp, vp, vp, vp, vp, vp, vp, vp, C.POINTER(i32), i32]),
    "tritd_dev_triple_product_qi_f64": (C.c_int, [vp, vp, vp, i64, i64, i64, i32, vp, vp]),
}


def _torch_lib_dir():
    """torch's bundled lib directory, without importing torch."""
    t = sys.modules.get("torch")
    if t is not None and getattr(t, "__file__", None):
        return os.path.join(os.path.dirname(t.__file__), "lib")
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return None
    return os.path.join(list(spec.submodule_search_locations)[0], "lib")


def mapped_libraries(stem):
    """Distinct files whose name starts with `stem` mapped into this process
    (/proc/self/maps), e.g. "libamdhip64", "libhsa-runtime64", "librccl"."""
    try:
        maps = open("/proc/self/maps").read()
    except OSError:
        return []
    return sorted(set(re.findall(r"(/\S*/%s\S*)" % re.escape(stem), maps)))


def hip_runtimes():
    """Distinct libamdhip64 files mapped into this process (/proc/self/maps)."""
    return mapped_libraries("libamdhip64")


def runtime_stack():
    """The HIP runtime, HSA runtime and RCCL copies this process has mapped:
    exactly one of each, from /opt/rocm, unless torch was imported first."""
    return {k: mapped_libraries(v) for k, v in (("hip", "libamdhip64"),
                                                 ("hsa", "libhsa-runtime64"),
                                                 ("rccl", "librccl"))}


def _preload_hip_runtime():
    """Choose the HIP runtime libtritd binds: ONE per process.

    libtritd.so is built against /opt/rocm's HIP and needs libamdhip64.so.7;
    by default the loader binds /opt/rocm's copy (RPATH) — the runtime the
    MATLAB/MEX drop-in uses.  torch ships its own copy (torch/lib, same
    soname), and a process holding both has two runtimes whose streams are not
    interchangeable (a torch stream in a tritd_dev_* call fails to launch;
    torch's device init can fail — round 4, tools/rounds/r4/dbg_bisect.sh).  So:
      * torch already imported (sys.modules): bind torch's copy, the one
        mapped already;
      * TRITD_HIP_RUNTIME=torch: bind torch's copy before torch is imported
        (a host that will import torch later);
      * otherwise (TRITD_HIP_RUNTIME unset / "system"): /opt/rocm's.
    A host that imports torch AFTER tritd on the system runtime gets two
    runtimes: check_one_runtime() (called by the device-pointer entry points
    of the Python API) then fails with a message saying so."""
    mode = os.environ.get("TRITD_HIP_RUNTIME", "auto")
    if mode not in ("auto", "torch", "system"):
        raise ImportError(f"TRITD_HIP_RUNTIME={mode!r}: expected 'torch' or 'system'")
    if mode == "system" or (mode == "auto" and "torch" not in sys.modules):
        return
    d = _torch_lib_dir()
    p = os.path.join(d, "libamdhip64.so") if d else None
    if p and os.path.exists(p):
        C.CDLL(p, mode=C.RTLD_GLOBAL)
    elif mode == "torch":
        raise ImportError("TRITD_HIP_RUNTIME=torch but torch's libamdhip64 was not found")


def check_one_runtime(where):
    """Fail loudly when the process maps two HIP runtimes (torch imported
    after tritd on the system runtime): device pointers and streams of one are
    not valid in the other."""
    rts = hip_runtimes()
    if len(rts) > 1:
        raise TritdError(TRITD_ERR_HIP, f"{where}: two HIP runtimes in this process ({', '.join(rts)}); "
                         "import torch before tritd, or set TRITD_HIP_RUNTIME=torch")


def _load():
    _preload_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libtritd.so not found at {LIB_PATH}: run __graft_entry__.build() "
                          "(or `make` in triple-tensor-decomposition-with-admm_amd/csrc)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()
# the libamdhip64 libtritd is bound to (recorded by bench.py's line)
HIP_RUNTIME = next((p for p in hip_runtimes()), None)


def check(status):
    if status != OK:
        raise TritdError(status, lib.tritd_last_error().decode(errors="replace"))


def warn_flags(flags, where):
    """Turn TRITD_FLAG_* bits into Python warnings (the call itself succeeded)."""
    if flags & FLAG_PINV_TOL:
        import warnings
        warnings.warn(f"{where}: a Gram's smallest pivot came within 1e3x of MATLAB's pinv "
                      "tolerance; pinv could have truncated there (results may differ from the "
                      "reference beyond rounding)", PinvToleranceWarning, stacklevel=3)


def check_flags(status, where):
    """check() for the one-shot solvers, then warn on tritd_last_flags()."""
    check(status)
    warn_flags(lib.tritd_last_flags(), where)


def device_count():
    n = i32(0)
    check(lib.tritd_device_count(C.byref(n)))
    return n.value


def set_devices(devices):
    """Device set of triple_decomp_ADMM (tritd_set_devices): more than one
    device shards D along mode 1 over them from this thread; one device
    repeated runs virtual shards on it; [] clears the set."""
    d = [int(x) for x in devices]
    arr = (i32 * max(len(d), 1))(*d)
    check(lib.tritd_set_devices(arr, len(d)))


def shutdown():
    lib.tritd_shutdown()


_printer_ref = None


def set_printer(fn):
    """Route opts.disp lines to `fn(str)` (None restores stdout)."""
    global _printer_ref
    if fn is None:
        _printer_ref = PRINT_FN(0)
    else:
        _printer_ref = PRINT_FN(lambda line, user: fn(line.decode()))
    lib.tritd_set_print_callback(_printer_ref, None)
