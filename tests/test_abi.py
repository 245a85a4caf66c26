"""The C-ABI boundary on a host without a GPU: libtritd.so loads, exports
every entry point include/tritd.h declares, validates arguments the way the
reference fails, and refuses to compute without a gfx950 device (there is
no CPU fallback in the product path)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "tritd.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(tritd_[a-z0-9_]+)\s*\(", src)) - {"tritd_print_fn"})


@pytest.fixture(scope="module")
def lib():
    from tritd import _lib
    return _lib


def test_header_and_binding_agree(lib):
    assert set(declared_symbols()) == set(lib.SIGNATURES)


def test_shared_object_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (tritd_\w+)", out))
    missing = set(declared_symbols()) - exported
    assert not missing, missing


def test_library_is_gfx950_code(lib):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", lib.LIB_PATH],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_version_and_device_count(lib):
    assert b"gfx950" in lib.lib.tritd_version()
    assert lib.device_count() >= 0


def _opts(lib, **kw):
    o = lib.Opts()
    o.mu, o.rho, o.lambda_, o.lambda2, o.tol, o.maxIter, o.disp = 1e-3, 1.25, 1.8, 1e-3, 1e-5, 5, 0
    o.present = kw.get("present", 0x7F)
    return o


def test_missing_opts_field_is_reported_like_matlab(lib):
    D = np.zeros((4, 4, 4), order="F")
    o = _opts(lib, present=0x7F & ~lib.OPT_LAMBDA2)
    buf = [np.zeros(64) for _ in range(3)]
    st = lib.lib.tritd_admm_f64(C.c_void_p(D.ctypes.data), 4, 4, 4, 2, C.byref(o),
                                *[C.c_void_p(b.ctypes.data) for b in buf], None, None, None, None,
                                None, None, None, -1)
    assert st == 2  # TRITD_ERR_OPTS
    assert lib.lib.tritd_last_error() == b"Reference to non-existent field 'lambda2'."


def test_python_api_raises_keyerror_for_missing_field():
    import tritd
    with pytest.raises(KeyError, match="non-existent field 'tol'"):
        tritd.triple_decomp_ADMM(np.zeros((3, 3, 3)), 1,
                                 dict(mu=1, rho=1, **{"lambda": 1}, lambda2=1, maxIter=1, disp=0))


def test_rank_above_the_kernels_is_unsupported(lib):
    """ADMM: r <= 16 in either precision (fp64 r = 9..16 on the padded-rank
    128/256 kernels); r = 17 is refused before any device work.  ALS keeps r <= 8."""
    D = np.zeros((4, 4, 4), order="F")
    o = _opts(lib)
    big = np.zeros(4 * 17 * 17 * 4)
    st = lib.lib.tritd_admm_f64(C.c_void_p(D.ctypes.data), 4, 4, 4, 17, C.byref(o),
                                *[C.c_void_p(big.ctypes.data)] * 3, None, None, None, None, None,
                                None, None, -1)
    assert st == 7  # TRITD_ERR_UNSUPPORTED
    st = lib.lib.tritd_als_f64(C.c_void_p(D.ctypes.data), 4, 4, 4, 9, C.byref(o),
                               *[C.c_void_p(big.ctypes.data)] * 3, None, None, None, None, None, -1)
    assert st == 7


def test_bad_unfold_mode_message(lib):
    X = np.zeros(8)
    st = lib.lib.tritd_unfold_f64(C.c_void_p(X.ctypes.data), 2, 2, 2, 4, C.c_void_p(X.ctypes.data))
    assert st == 1
    assert lib.lib.tritd_last_error() == b"Mode must be 1, 2, or 3."


def test_no_cpu_fallback_without_gpu(lib):
    import tritd
    if tritd.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(tritd.TritdError, match="NODEV"):
        tritd.soft_threshold(np.ones(4), 0.5)
    with pytest.raises(tritd.TritdError, match="NODEV"):
        from tritd import synth
        d = synth.low_rank_plus_outliers(4, 4, 4, 2)
        tritd.triple_decomp_ADMM(d["D"], 2, synth.TRAFFIC_OPTS, d["A0"], d["B0"], d["C0"])


def test_shard_range_validation(lib):
    o = _opts(lib)
    D = np.zeros(64)
    s = C.c_void_p()
    st = lib.lib.tritd_session_create(C.byref(s), 0, C.c_void_p(D.ctypes.data), 4, 4, 4, 4, 3, 2,
                                      2, C.byref(o), *[C.c_void_p(D.ctypes.data)] * 3, None, 0)
    assert st == 1  # i0 >= i1


def test_admm_sessions_accept_rank_16_in_fp64(lib):
    """tritd_session_create takes the one-shot solver's ADMM rank range (r <= 16)
    in fp64 too: r = 9 passes validation (without a GPU the call then fails
    for lack of a device, not for the rank); r = 17 is refused."""
    import tritd
    o = _opts(lib)
    D = np.zeros(4 * 4 * 4)
    F = np.zeros(4 * 17 * 17 * 4)
    for r, want in ((9, None), (17, 7)):
        s = C.c_void_p()
        st = lib.lib.tritd_session_create(C.byref(s), 0, C.c_void_p(D.ctypes.data), 4, 4, 4, 4, 0,
                                          4, r, C.byref(o), *[C.c_void_p(F.ctypes.data)] * 3,
                                          None, 0)
        if want is not None:
            assert st == want
        elif tritd.device_count() == 0:
            assert st == 6  # TRITD_ERR_NODEV, past the rank check
        else:
            assert st == 0
            lib.lib.tritd_session_destroy(s)


def test_last_flags_cleared_by_a_failed_call(lib):
    D = np.zeros((4, 4, 4), order="F")
    o = _opts(lib, present=0)
    st = lib.lib.tritd_admm_f64(C.c_void_p(D.ctypes.data), 4, 4, 4, 2, C.byref(o),
                                *[C.c_void_p(D.ctypes.data)] * 3, None, None, None, None, None,
                                None, None, -1)
    assert st == 2 and lib.lib.tritd_last_flags() == 0


def test_build_keeps_matlab_rounding_flags():
    """The elementwise statements must round like MATLAB's separate operators
    and the fixed-order reductions must stay bitwise reproducible: the build
    keeps -ffp-contract=off and never enables reassociation."""
    mk = open(os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd", "csrc",
                           "Makefile")).read()
    flags = re.search(r"^CXXFLAGS\s*:=(.*)$", mk, flags=re.M).group(1)
    assert "-ffp-contract=off" in flags
    for bad in ("-ffast-math", "-fassociative-math", "-Ofast", "-funsafe-math-optimizations",
                "-ffp-contract=fast", "-ffp-contract=on"):
        assert bad not in mk, bad


def test_make_tracks_every_header():
    """bench.py's ensure_built() trusts `make -q`: every header of csrc/ and the
    ABI header must be a prerequisite, so an edit to any of them (pinv.h,
    sweep.h, ...) marks the library out of date."""
    csrc = os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd", "csrc")
    if subprocess.run(["make", "-q", "-C", csrc], capture_output=True).returncode != 0:
        pytest.skip("library not built (or out of date) in this tree")
    hdrs = [f for f in os.listdir(csrc) if f.endswith(".h")] + ["../../include/tritd.h"]
    assert "pinv.h" in hdrs and "sweep.h" in hdrs
    for h in hdrs:
        p = subprocess.run(["make", "-q", "-W", h, "-C", csrc], capture_output=True)
        assert p.returncode == 1, "an edit to %s would not rebuild libtritd.so" % h


def test_product_reads_few_environment_knobs():
    """The product path reads a handful of environment knobs, each exercised
    by a test: TRITD_DENSE_E, TRITD_PROBE, TRITD_K5_TSPLIT,
    TRITD_FUSED, TRITD_SHOV.  No per-launch experiment switches."""
    csrc = os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd", "csrc")
    knobs = set()
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".h")):
            knobs |= set(re.findall(r'getenv\("(TRITD_\w+)"\)', open(os.path.join(csrc, f)).read()))
    assert knobs <= {"TRITD_DENSE_E", "TRITD_PROBE", "TRITD_K5_TSPLIT", "TRITD_FUSED", "TRITD_SHOV"}, knobs
    assert len(knobs) <= 8


_MAPS_CHILD = """
import re, sys, json
sys.path.insert(0, %(pkg)r)
order = %(order)r
if order == "torch_first":
    import torch
import tritd._lib as L
err = None
if order == "torch_after":
    import torch
    try:
        L.check_one_runtime("probe")
    except L.TritdError as e:
        err = str(e)
maps = open("/proc/self/maps").read()
libs = lambda name: sorted(set(re.findall(r"(/\\S*%%s\\S*)" %% name, maps)))
print(json.dumps({"hip": libs("libamdhip64"), "hsa": libs("libhsa-runtime64"),
                  "rccl": libs("librccl"), "bound": L.HIP_RUNTIME, "err": err}))
"""


def _maps(order):
    import json
    code = _MAPS_CHILD % {"pkg": os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"),
                          "order": order}
    env = {k: v for k, v in os.environ.items() if k != "TRITD_HIP_RUNTIME"}
    out = subprocess.run([os.sys.executable, "-c", code], capture_output=True, text=True,
                         check=True, timeout=300, env=env).stdout.strip().splitlines()[-1]
    return json.loads(out)


def test_hip_runtime_without_torch_is_the_system_one():
    """No torch in the process: libtritd binds /opt/rocm's HIP runtime (the one
    it is built against, and the MEX drop-in's), one copy each of the HIP, HSA
    and RCCL libraries."""
    m = _maps("no_torch")
    assert len(m["hip"]) == 1 and m["hip"][0].startswith("/opt/rocm"), m
    assert m["bound"] == m["hip"][0]
    assert len(m["hsa"]) == 1 and m["hsa"][0].startswith("/opt/rocm"), m
    assert len(m["rccl"]) == 1, m


def test_hip_runtime_with_torch_imported_first_is_torch_s():
    """torch imported first: libtritd binds torch's copy — still one runtime,
    so torch streams and memory are valid in tritd_dev_* calls."""
    m = _maps("torch_first")
    assert len(m["hip"]) == 1 and "torch" in m["hip"][0], m
    assert m["bound"] == m["hip"][0]
    # one HSA runtime and one RCCL too: libtritd's
    # ncclCommInitRank runs on whichever RCCL torch mapped
    assert len(m["hsa"]) == 1 and len(m["rccl"]) == 1, m


def test_torch_imported_after_tritd_fails_loudly():
    """torch imported after tritd (system runtime): two runtimes are mapped,
    and the device-pointer entry points refuse to run (check_one_runtime)."""
    m = _maps("torch_after")
    assert len(m["hip"]) == 2, m
    assert m["err"] and "two HIP runtimes" in m["err"], m


_KFD_CHILD = """
import os, sys
sys.path.insert(0, %(pkg)r)
from tritd import _lib
def kfd():
    for f in os.listdir('/proc/self/fd'):
        try:
            if os.readlink('/proc/self/fd/' + f) == '/dev/kfd':
                return True
        except OSError:
            pass
    return False
_lib.lib.tritd_version(); _lib.lib.tritd_last_error()
before = kfd()
n = _lib.device_count()
print(before, kfd(), n)
"""


@pytest.mark.gpu
def test_host_only_entry_points_do_not_initialise_hip():
    """an entry point that needs no GPU (tritd_version,
    tritd_last_error) leaves the HIP runtime uninitialised (no /dev/kfd
    open), so a host may query the library before it launches workers; the
    first device call initialises it."""
    code = _KFD_CHILD % {"pkg": os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd")}
    out = subprocess.run([os.sys.executable, "-c", code], capture_output=True, text=True,
                         check=True, timeout=300).stdout.split()
    assert out[0] == "False" and out[1] == "True" and int(out[2]) >= 1, out
