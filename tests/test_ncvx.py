"""The nonconvex solver of fast_robust_triple_tensor/test.m (SURVEY.md §8f
rank 4): `triple_decomp_ADMM_outlier(X, r, rho, lambda, gamma_A, epsilon, p,
theta, maxIter, tol)`.  The reference has no caller, no tests and no data for
it; the golden vectors (tests/golden/nc*.npz) come from the oracle's line-by-
line restatement (`tritd_oracle.triple_decomp_ADMM_ncvx`, made by
tests/golden/make_golden.py with the parameters recorded in each file), so
parity is unpinned beyond the primitives it shares with the main solver
(buildF/G/H, triple_product, unfold: tests/test_oracle.py).

GPU tests (@gpu) run libtritd's fused path (k_als_fit<RP, true> + the shared
M1/M2/K2/solve kernels + k_ncvx_shrink) against the goldens:
A, B, C, O <= 1e-9 relative Frobenius (L = triple_product for the factors),
errHist rtol 1e-8, same k.  pow() in the reweighting may differ from libm by
an ulp, far inside these bounds.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, rel

import tritd_oracle as orc

PARAM_KEYS = ("rho", "lambda", "gamma_A", "epsilon", "p", "theta", "maxIter", "tol")


def _args(g):
    o = g["opts"]
    return [o[k] for k in PARAM_KEYS]


@pytest.mark.parametrize("name", golden_names("ncvx"))
def test_oracle_reproduces_ncvx_golden(name):
    g = load_golden(name)
    A, B, C, O, eh, k, tr = orc.triple_decomp_ADMM_ncvx(g["X"], g["r"], *_args(g), g["A0"], g["B0"],
                                                        g["C0"], printer=lambda s: None)
    assert k == g["k"] and len(eh) == len(g["errHist"])
    for key, X in (("A", A), ("B", B), ("C", C), ("O", O)):
        assert rel(X, g[key]) <= 1e-12, key
    np.testing.assert_allclose(eh, g["errHist"], rtol=1e-12, atol=1e-15)


def test_ncvx_stop_semantics():
    """test.m:65-71: on a break errHist is truncated and O is NOT advanced."""
    g = load_golden("nc20x24x18_r3_stop")
    k = g["k"]
    assert k < g["opts"]["maxIter"] and len(g["errHist"]) == k
    e = g["errHist"]
    assert abs(e[-1] - e[-2]) < g["opts"]["tol"] * e[-2]
    prm = _args(g)
    prm[6] = k - 1  # the same run stopped by maxIter one iteration earlier
    A, B, C, O, eh, kk, _ = orc.triple_decomp_ADMM_ncvx(g["X"], g["r"], *prm, g["A0"], g["B0"],
                                                        g["C0"], printer=lambda s: None)
    assert kk == k - 1
    np.testing.assert_array_equal(O, g["O"])  # the returned O is that of iteration k-1
    # and a run to maxIter keeps maxIter entries and the last O
    assert len(load_golden("nc30_r3")["errHist"]) == load_golden("nc30_r3")["opts"]["maxIter"]


def test_ncvx_factors_ignore_the_outlier_chain():
    """test.m:49-51 update A, B, C from X (not Y): with the shrink off
    (gamma_A = 0) and the ridges of test.m, the factor sequence is that of an
    ALS with ridge 1e-12 on A — independent of rho and lambda."""
    g = load_golden("nc12x10x8_r2")
    prm = _args(g)
    prm[2] = 0.0  # gamma_A
    prm[6] = 3
    a1 = orc.triple_decomp_ADMM_ncvx(g["X"], g["r"], *prm, g["A0"], g["B0"], g["C0"],
                                     printer=lambda s: None)
    prm[0], prm[1] = 3.0, 7.0
    a2 = orc.triple_decomp_ADMM_ncvx(g["X"], g["r"], *prm, g["A0"], g["B0"], g["C0"],
                                     printer=lambda s: None)
    for q in range(3):
        np.testing.assert_array_equal(a1[q], a2[q])


def test_ncvx_prints_every_iteration():
    g = load_golden("nc12x10x8_r2")
    prm = _args(g)
    prm[6] = 4
    lines = []
    orc.triple_decomp_ADMM_ncvx(g["X"], g["r"], *prm, g["A0"], g["B0"], g["C0"],
                                printer=lines.append)
    assert [ln.split(",")[0] for ln in lines] == ["Iteration %d" % k for k in (1, 2, 3, 4)]


# ---------------------------------------------------------------------------
# GPU (libtritd, HIP on gfx950)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def tritd():
    import tritd as t
    assert t.device_count() > 0, "no GPU visible: the HIP path must run, there is no CPU fallback"
    return t


def _check(got, g):
    A, B, C, O, eh, k = got
    assert k == g["k"] and len(eh) == len(g["errHist"])
    assert rel(orc.triple_product(A, B, C), orc.triple_product(g["A"], g["B"], g["C"])) <= 1e-9
    for key, X in (("A", A), ("B", B), ("C", C), ("O", O)):
        assert rel(X, g[key]) <= 1e-9, key
    np.testing.assert_allclose(eh, g["errHist"], rtol=1e-8, atol=1e-13)


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names("ncvx"))
def test_gpu_ncvx_matches_golden(tritd, name):
    g = load_golden(name)
    tritd.set_printer(lambda s: None)
    try:
        got = tritd.triple_decomp_ncvx(g["X"], g["r"], *_args(g), g["A0"], g["B0"], g["C0"],
                                       return_iters=True)
    finally:
        tritd.set_printer(None)
    _check(got, g)


@pytest.mark.gpu
def test_gpu_ncvx_first_iterations_and_alias(tritd):
    g = load_golden("nc12x10x8_r2")
    tritd.set_printer(lambda s: None)
    try:
        for it in (1, 2):
            prm = _args(g)
            prm[6] = it
            A, B, C, O, eh, k = tritd.triple_decomp_ADMM_outlier(g["X"], g["r"], *prm, g["A0"],
                                                                 g["B0"], g["C0"], return_iters=True)
            assert k == it
            for key, X in (("A", A), ("B", B), ("C", C), ("O", O)):
                assert rel(X, g[f"it{it}_{key}"]) <= 1e-11, (it, key)
    finally:
        tritd.set_printer(None)


@pytest.mark.gpu
@pytest.mark.parametrize("serial", [False, True])
def test_gpu_ncvx_device_set(tritd, serial, monkeypatch):
    """Mode-1 shards through tritd_set_devices (one GPU repeated): partial fit
    sums, [M2 | A^TA] and M3 all-reduced; O gathered per shard.  Default one
    host thread per shard; TRITD_SHOV=0 the phase-serial driver."""
    if serial:
        monkeypatch.setenv("TRITD_SHOV", "0")
    g = load_golden("nc30_r3")
    tritd.set_printer(lambda s: None)
    tritd.set_devices([0, 0, 0])
    try:
        got = tritd.triple_decomp_ncvx(g["X"], g["r"], *_args(g), g["A0"], g["B0"], g["C0"],
                                       return_iters=True)
    finally:
        tritd.set_devices([])
        tritd.set_printer(None)
    _check(got, g)


@pytest.mark.gpu
def test_gpu_ncvx_prints_like_reference(tritd):
    g = load_golden("nc12x10x8_r2")
    prm = _args(g)
    prm[6] = 3
    lines = []
    tritd.set_printer(lines.append)
    try:
        tritd.triple_decomp_ncvx(g["X"], g["r"], *prm, g["A0"], g["B0"], g["C0"])
    finally:
        tritd.set_printer(None)
    ref = []
    orc.triple_decomp_ADMM_ncvx(g["X"], g["r"], *prm, g["A0"], g["B0"], g["C0"], printer=ref.append)
    assert lines == ref
