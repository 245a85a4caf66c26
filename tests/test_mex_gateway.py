"""The MEX gateway (matlab/tritd_mex.cpp) compiled against a mock mx runtime
(tests/mock_mex/) and driven through ctypes — MATLAB itself is absent
(SURVEY.md §4.5).  CPU: argument parsing and MATLAB-style errors.  GPU: a
full solve through the gateway matches the golden vectors."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT, load_golden, rel

MOCK = os.path.join(ROOT, "tests", "mock_mex")


@pytest.fixture(scope="module")
def gw(tmp_path_factory):
    out = tmp_path_factory.mktemp("mex") / "libmexmock.so"
    libdir = os.path.join(PKG, "tritd")
    subprocess.run(["g++", "-std=c++17", "-O1", "-shared", "-fPIC", "-I" + MOCK,
                    "-I" + os.path.join(ROOT, "include"),
                    os.path.join(PKG, "matlab", "tritd_mex.cpp"), os.path.join(MOCK, "mock_mex.cpp"),
                    "-L" + libdir, "-ltritd", "-Wl,-rpath," + libdir, "-o", str(out)], check=True)
    lib = C.CDLL(str(out))
    lib.mock_admm.restype = C.c_int
    lib.mock_als.restype = C.c_int
    return lib


def run(gw, g, names=None, vals=None, single=False, want_E=True):
    D = np.asfortranarray(g["D"], dtype=np.float32 if single else np.float64)
    n1, n2, n3 = D.shape
    r = g["r"]
    o = g["opts"]
    names = names or ["mu", "rho", "lambda", "lambda2", "maxIter", "tol", "disp"]
    vals = np.array(vals if vals is not None else [float(o[n]) for n in names])
    A = np.zeros((n1, r, r), order="F")
    B = np.zeros((r, n2, r), order="F")
    Cc = np.zeros((r, r, n3), order="F")
    O = np.zeros_like(D)
    E = np.zeros_like(D)
    eh = np.zeros(int(o["maxIter"]) + 1)
    k = C.c_int(0)
    err = C.create_string_buffer(1024)
    pr = C.create_string_buffer(4096)
    p = lambda a: C.c_void_p(a.ctypes.data)
    A0, B0, C0 = (np.asfortranarray(g[x]) for x in ("A0", "B0", "C0"))
    rc = gw.mock_admm(p(D), n1, n2, n3, r, ",".join(names).encode(), p(vals), p(A0), p(B0), p(C0),
                      p(A), p(B), p(Cc), p(O), p(E) if want_E else None, p(eh), C.byref(k), err,
                      1024, pr, 4096, int(single))
    return rc, err.value.decode(), dict(A=A, B=B, C=Cc, O=O, E=E, errHist=eh[: k.value], k=k.value,
                                        printed=pr.value.decode())


def test_gateway_missing_field_error(gw):
    g = load_golden("g12x10x8_r2")
    names = ["mu", "rho", "lambda", "maxIter", "tol", "disp"]
    rc, err, _ = run(gw, g, names, [float(g["opts"][n]) for n in names])
    assert rc == 1
    assert err == "MATLAB:nonExistentField|Reference to non-existent field 'lambda2'."


def test_gateway_reports_missing_gpu(gw):
    import tritd
    if tritd.device_count() > 0:
        pytest.skip("GPU visible")
    rc, err, _ = run(gw, load_golden("g12x10x8_r2"))
    assert rc == 1 and err.startswith("tritd:solver|") and "NODEV" not in err and "no HIP device" in err


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["g30_r3", "g12x10x8_r2_stop", "g54x4x96_r5_sensor"])
def test_gateway_solve_matches_golden(gw, name):
    import tritd_oracle as orc
    g = load_golden(name)
    rc, err, res = run(gw, g)
    assert rc == 0, err
    assert res["k"] == g["k"]
    assert rel(orc.triple_product(res["A"], res["B"], res["C"]),
               orc.triple_product(g["A"], g["B"], g["C"])) <= 1e-9
    assert rel(res["O"], g["O"]) <= 1e-9 and rel(res["E"], g["E"]) <= 1e-9
    np.testing.assert_allclose(res["errHist"], g["errHist"], rtol=1e-8, atol=1e-13)


@pytest.mark.gpu
def test_gateway_five_outputs_skip_E(gw):
    """[A,B,C,O,errHist] = triple_decomp_ADMM(...) (nargout 5, the drivers' call):
    no 6th output is created, the five match the golden."""
    g = load_golden("g30_r3")
    rc, err, res = run(gw, g, want_E=False)
    assert rc == 0, err
    assert res["k"] == g["k"] and rel(res["O"], g["O"]) <= 1e-9
    np.testing.assert_allclose(res["errHist"], g["errHist"], rtol=1e-8, atol=1e-13)


@pytest.mark.gpu
def test_gateway_disp_goes_through_mexPrintf(gw):
    g = load_golden("g30_r3")
    g["opts"] = dict(g["opts"], disp=1, maxIter=20)
    rc, err, res = run(gw, g)
    assert rc == 0, err
    assert res["printed"].splitlines()[0].startswith("Iter 10, errL=")


def devices(gw, idx):
    err = C.create_string_buffer(1024)
    v = np.asarray(idx, dtype=np.float64)
    rc = gw.mock_devices(C.c_void_p(v.ctypes.data) if len(v) else None, len(v), err, 1024)
    return rc, err.value.decode()


def test_gateway_devices_validates(gw):
    rc, err = devices(gw, [0.5])
    assert rc == 1 and err == "tritd:devices|device ordinals must be integers"
    rc, err = devices(gw, list(range(17)))
    assert rc == 1 and err == "tritd:devices|at most 16 devices"
    rc, err = devices(gw, [])  # clearing the set needs no GPU
    assert rc == 0, err
    assert gw.mock_clear() == 0  # the gateway registered tritd_shutdown with mexAtExit


@pytest.mark.gpu
def test_gateway_single_class_and_device_set(gw):
    """A single D goes through tritd_admm_f32 with single O/E; a device set of
    one GPU repeated twice runs the sharded schedule (virtual shards)."""
    import tritd_oracle as orc
    g = load_golden("g30_r3")
    rc, err, one = run(gw, g, single=True)
    assert rc == 0, err
    assert one["O"].dtype == np.float32 and one["k"] == g["k"]
    assert rel(orc.triple_product(one["A"], one["B"], one["C"]),
               orc.triple_product(g["A"], g["B"], g["C"])) <= 1e-4
    rc, err = devices(gw, [0, 0])
    assert rc == 0, err
    try:
        rc, err, two = run(gw, g)
        assert rc == 0, err
        assert two["k"] == g["k"]
        assert rel(two["O"], g["O"]) <= 1e-9
        np.testing.assert_allclose(two["errHist"], g["errHist"], rtol=1e-8, atol=1e-13)
    finally:
        assert devices(gw, [])[0] == 0


# ---------------------------------------------------------------------------
# 'als' command (matlab/triple_decomp_ALS.m -> tritd_als_f64)
# ---------------------------------------------------------------------------
def run_als(gw, g, names=("maxIter", "tol"), vals=None):
    X = np.asfortranarray(g["X"])
    n1, n2, n3 = X.shape
    r = g["r"]
    names = list(names)
    vals = np.array(vals if vals is not None else [float(g["opts"][n]) for n in names])
    A = np.zeros((n1, r, r), order="F")
    B = np.zeros((r, n2, r), order="F")
    Cc = np.zeros((r, r, n3), order="F")
    eh = np.zeros(int(g["opts"]["maxIter"]) + 1)
    k = C.c_int(0)
    err = C.create_string_buffer(1024)
    pr = C.create_string_buffer(4096)
    p = lambda a: C.c_void_p(a.ctypes.data)
    A0, B0, C0 = (np.asfortranarray(g[x]) for x in ("A0", "B0", "C0"))
    rc = gw.mock_als(p(X), n1, n2, n3, r, ",".join(names).encode(), p(vals), p(A0), p(B0), p(C0),
                     p(A), p(B), p(Cc), p(eh), C.byref(k), err, 1024, pr, 4096)
    return rc, err.value.decode(), dict(A=A, B=B, C=Cc, errHist=eh[: k.value], k=k.value,
                                        printed=pr.value.decode())


def test_gateway_als_missing_field_error(gw):
    g = load_golden("als12x10x8_r2")
    rc, err, _ = run_als(gw, g, names=("tol", "mu"), vals=[1e-5, 1.0])
    assert rc == 1
    assert err == "MATLAB:nonExistentField|Reference to non-existent field 'maxIter'."
    rc, err, _ = run_als(gw, g, names=("maxIter",), vals=[5.0])
    assert err == "MATLAB:nonExistentField|Reference to non-existent field 'tol'."


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["als30_r3", "als20x24x18_r5_stop"])
def test_gateway_als_matches_golden(gw, name):
    import tritd_oracle as orc
    g = load_golden(name)
    rc, err, res = run_als(gw, g)
    assert rc == 0, err
    assert res["k"] == g["k"]
    assert rel(orc.triple_product(res["A"], res["B"], res["C"]),
               orc.triple_product(g["A"], g["B"], g["C"])) <= 1e-9
    np.testing.assert_allclose(res["errHist"], g["errHist"], rtol=1e-9, atol=1e-14)
    lines = res["printed"].splitlines()
    assert lines == ["Iteration %d, relative error = %.4e" % (i, g["errHist"][i - 1])
                     for i in range(5, g["k"] + 1, 5)]


# ---------------------------------------------------------------------------
# opts.model = 'qi' and the nonconvex 'ncvx' command
# ---------------------------------------------------------------------------
def test_gateway_bad_model_is_refused(gw):
    g = load_golden("qi12x10x8_r2")
    names = ["mu", "rho", "lambda", "lambda2", "maxIter", "tol", "disp"]
    rc, err, _ = run(gw, g, names + ["model=tucker"], [float(g["opts"][n]) for n in names])
    assert rc == 1 and err == "tritd:opts|opts.model must be 'cp' or 'qi'"


@pytest.mark.gpu
def test_gateway_qi_matches_golden(gw):
    import tritd_oracle as orc
    g = load_golden("qi30_r3")
    names = ["mu", "rho", "lambda", "lambda2", "maxIter", "tol", "disp"]
    rc, err, res = run(gw, g, names + ["model=qi"], [float(g["opts"][n]) for n in names])
    assert rc == 0, err
    assert res["k"] == g["k"]
    L = orc.triple_product(res["A"], res["B"], res["C"], "qi")
    assert rel(L, orc.triple_product(g["A"], g["B"], g["C"], "qi")) <= 1e-9
    assert rel(res["O"], g["O"]) <= 1e-9


def run_ncvx(gw, g):
    X = np.asfortranarray(g["X"])
    n1, n2, n3 = X.shape
    r = g["r"]
    o = g["opts"]
    prm = np.array([o[n] for n in ("rho", "lambda", "gamma_A", "epsilon", "p", "theta",
                                   "maxIter", "tol")], dtype=np.float64)
    A = np.zeros((n1, r, r), order="F")
    B = np.zeros((r, n2, r), order="F")
    Cc = np.zeros((r, r, n3), order="F")
    O = np.zeros_like(X)
    eh = np.zeros(int(o["maxIter"]) + 1)
    k = C.c_int(0)
    err = C.create_string_buffer(1024)
    pr = C.create_string_buffer(1 << 16)
    p = lambda a: C.c_void_p(a.ctypes.data)
    A0, B0, C0 = (np.asfortranarray(g[x]) for x in ("A0", "B0", "C0"))
    rc = gw.mock_ncvx(p(X), n1, n2, n3, r, p(prm), p(A0), p(B0), p(C0), p(A), p(B), p(Cc), p(O),
                      p(eh), C.byref(k), err, 1024, pr, 1 << 16)
    return rc, err.value.decode(), dict(A=A, B=B, C=Cc, O=O, errHist=eh[: k.value], k=k.value,
                                        printed=pr.value.decode())


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["nc30_r3", "nc20x24x18_r3_stop"])
def test_gateway_ncvx_matches_golden(gw, name):
    import tritd_oracle as orc
    g = load_golden(name)
    rc, err, res = run_ncvx(gw, g)
    assert rc == 0, err
    assert res["k"] == g["k"]
    assert rel(orc.triple_product(res["A"], res["B"], res["C"]),
               orc.triple_product(g["A"], g["B"], g["C"])) <= 1e-9
    assert rel(res["O"], g["O"]) <= 1e-9
    np.testing.assert_allclose(res["errHist"], g["errHist"], rtol=1e-8, atol=1e-13)
    lines = [ln for ln in res["printed"].splitlines() if ln.startswith("Iteration ")]
    assert len(lines) == g["k"]  # test.m:63 prints every iteration
