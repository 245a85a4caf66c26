"""The oracle itself: pinned against the reference's own known answers, then
against the committed golden vectors; the C restatement against both.

Known answers taken from the reference:
  * buildF.m:5-16, buildG.m:5-16, buildH.m:5-16 — commented loop definitions
    must equal the vectorised code at :17-21;
  * fast_robust_triple_tensor/test.m:142-160 — explicit five-loop
    triple_product;
  * triple_decomp_ADMM.m:111-130 — reshape_*_from_* invert unfold;
  * MATLAB scalar semantics sign(0)=0, max(NaN,0)=0, pinv tolerance.
The solver loop itself has no reference-side pin (MATLAB is absent): the
golden vectors are regression vectors of this restatement ("parity
unpinned").
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, rel

import tritd_oracle as orc


@pytest.mark.parametrize("dims", [(5, 4, 3, 2), (3, 6, 4, 3), (4, 3, 5, 1)])
def test_design_matrices_match_loop_definitions(synth, dims):
    n1, n2, n3, r = dims
    A, B, C = synth.random_factors(n1, n2, n3, r, seed=11)
    np.testing.assert_array_equal(orc.buildF(B, C), orc.buildF_loops(B, C))
    np.testing.assert_array_equal(orc.buildG(A, C), orc.buildG_loops(A, C))
    np.testing.assert_array_equal(orc.buildH(A, B), orc.buildH_loops(A, B))


@pytest.mark.parametrize("dims", [(5, 4, 3, 2), (4, 6, 5, 3)])
def test_triple_product_matches_five_loop(synth, dims):
    A, B, C = synth.random_factors(*dims, seed=5)
    assert rel(orc.triple_product(A, B, C), orc.triple_product_loops(A, B, C)) < 1e-14


def test_triple_product_is_rank_r2_cp(synth):
    """L(i,j,t) = sum_pq A(i,p,q) B(p,j,q) C(p,q,t)."""
    A, B, C = synth.random_factors(6, 5, 4, 3, seed=2)
    L = np.einsum("ipq,pjq,pqt->ijt", A, B, C)
    assert rel(orc.triple_product(A, B, C), L) < 1e-14
    assert rel(synth.cp_full(*synth.hat_factors(A, B, C)), L) < 1e-14


def test_unfold_and_refold_roundtrip(synth):
    X = np.asfortranarray(np.random.default_rng(0).standard_normal((4, 3, 5)))
    assert orc.unfold(X, 1).shape == (4, 15)
    assert orc.unfold(X, 2)[2, 1 + 4 * 3] == X[1, 2, 3]
    assert orc.unfold(X, 3)[3, 1 + 4 * 2] == X[1, 2, 3]
    with pytest.raises(ValueError, match="Mode must be 1, 2, or 3."):
        orc.unfold(X, 4)
    A = synth.random_factors(4, 3, 5, 2, seed=1)[0]
    np.testing.assert_array_equal(orc.reshape_A_from_A1(orc.unfold(A, 1), 4, 2), A)
    B = synth.random_factors(4, 3, 5, 2, seed=1)[1]
    np.testing.assert_array_equal(orc.reshape_B_from_B2(orc.unfold(B, 2), 3, 2), B)
    C = synth.random_factors(4, 3, 5, 2, seed=1)[2]
    np.testing.assert_array_equal(orc.reshape_C_from_C3(orc.unfold(C, 3), 5, 2), C)


def test_matlab_scalar_semantics():
    x = np.array([0.0, -0.0, np.nan, 2.0, -3.0])
    np.testing.assert_array_equal(orc.matlab_sign(x), [0.0, 0.0, np.nan, 1.0, -1.0])
    np.testing.assert_array_equal(orc.matlab_max0(np.array([np.nan, -1.0, 2.0])), [0.0, 0.0, 2.0])
    np.testing.assert_array_equal(orc.soft_threshold(np.array([0.0, 1.0, -3.0, np.nan]), 1.5),
                                  [0.0, 0.0, -1.5, np.nan])
    assert orc.matlab_eps(1.0) == np.finfo(float).eps
    assert orc.matlab_eps(3.0) == 2 * np.finfo(float).eps


def test_pinv_truncates_with_matlab_tolerance():
    # exact singular values (permuted diagonal): tol = 6*eps(1) = 1.33e-15
    s = np.array([1e-14, 1.0, 1e-16, 0.5, 0.0, 1e-3])
    G = np.diag(s)
    P = orc.pinv(G)
    expect = np.diag([1e14, 1.0, 0.0, 2.0, 0.0, 1e3])
    assert rel(P, expect) < 1e-15
    # full rank: pinv == inverse
    U = np.linalg.qr(np.random.default_rng(3).standard_normal((6, 6)))[0]
    G2 = (U * np.array([3.0, 2, 1, 0.5, 0.2, 0.1])) @ U.T
    assert rel(orc.pinv(G2), np.linalg.inv(G2)) < 1e-12


def test_missing_opts_field_errors_like_matlab():
    with pytest.raises(KeyError, match="Reference to non-existent field 'lambda2'"):
        orc.check_opts(dict(mu=1, rho=1, **{"lambda": 1}, maxIter=1, tol=0, disp=0))


def test_mu_schedule_caps():
    mus = orc.mu_schedule(1e-3, 1.25, 100)
    assert mus[0] == 1e-3
    assert max(mus) == 1e-3 * 1e6
    assert mus.index(1e-3 * 1e6) == 62  # traffic opts cap at k ~ 62


@pytest.mark.parametrize("name", golden_names())
def test_oracle_reproduces_golden(name):
    g = load_golden(name)
    A, B, C, O, eh, E, k, tr = orc.triple_decomp_ADMM(g["D"], g["r"], g["opts"], g["A0"], g["B0"],
                                                      g["C0"], trace_iters=(1, 2))
    assert k == g["k"] and len(eh) == k
    for key, X in (("A", A), ("B", B), ("C", C), ("O", O), ("E", E)):
        assert rel(X, g[key]) <= 1e-12, key
    np.testing.assert_allclose(eh, g["errHist"], rtol=1e-12, atol=1e-15)
    for it in (1, 2):
        assert rel(tr[it]["A"], g[f"it{it}_A"]) <= 1e-13


def test_golden_stop_case_truncates():
    g = load_golden("g12x10x8_r2_stop")
    assert g["k"] < g["opts"]["maxIter"]
    assert len(g["errHist"]) == g["k"]
    e = g["errHist"]
    assert abs(e[-1] - e[-2]) < g["opts"]["tol"] * e[-2]


def test_synthetic_recovery_known_answer(synth):
    """outlier-corrupted rank-R tensor is recovered."""
    g = load_golden("g30_r3")
    L = orc.triple_product(g["A"], g["B"], g["C"])
    assert rel(L, g["Lstar"]) < 1e-6
    assert g["k"] == 100
    e = g["errHist"]
    assert e[-1] < 1e-7 and e[-1] < 1e-6 * e[0]  # geometric decay, stop test never fires


# ---------------------------------------------------------------------------
# C restatement (oracle/tritd_ref.c) against the goldens
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def cref():
    import os
    import subprocess
    here = os.path.dirname(os.path.abspath(orc.__file__))
    subprocess.run(["make", "-C", here], check=True, capture_output=True)  # no-op when current
    import tritd_ref
    return tritd_ref, tritd_ref.load()


@pytest.mark.parametrize("name", golden_names())
def test_c_restatement_matches_golden(cref, name):
    mod, lib = cref
    g = load_golden(name)
    A, B, C, O, eh, E, k = mod.admm(lib, g["D"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"])
    assert k == g["k"]
    L = orc.triple_product(A, B, C)
    assert rel(L, orc.triple_product(g["A"], g["B"], g["C"])) <= 1e-9
    assert rel(O, g["O"]) <= 1e-9
    assert rel(E, g["E"]) <= 1e-9
    np.testing.assert_allclose(eh, g["errHist"], rtol=1e-8, atol=1e-13)


def test_c_restatement_primitives(cref, synth):
    import ctypes as C
    mod, lib = cref
    A, B, Cf = synth.random_factors(7, 5, 6, 3, seed=9)
    X = np.zeros((7, 5, 6), order="F")
    p = lambda a: C.c_void_p(a.ctypes.data)
    lib.tritd_ref_triple_product(p(A), p(B), p(Cf), 7, 5, 6, 3, p(X))
    assert rel(X, orc.triple_product_loops(A, B, Cf)) < 1e-14
    for mode in (1, 2, 3):
        out = np.zeros(orc.unfold(X, mode).shape, order="F")
        lib.tritd_ref_unfold(p(X), 7, 5, 6, mode, p(out))
        np.testing.assert_array_equal(out, orc.unfold(X, mode))


@pytest.mark.parametrize("dims,iters", [((32, 24, 20, 3), 100), ((48, 40, 36, 4), 60),
                                        ((40, 24, 16, 5), 40)])
def test_lean_single_restatement_matches_c(cref, synth, dims, iters):
    """oracle/tritd_lean.py (the layout that runs config 5's 100-iteration
    horizon on a 64 GB host, tests/golden/make_c5_horizon.py) against the C
    restatement's single-class solver (tritd_ref_admm_f32) on the same
    inputs: both round to single at the same statements and accumulate their
    GEMMs in double, so the results agree to single rounding (measured:
    bitwise on these cases)."""
    import tritd_lean
    mod, lib = cref
    n1, n2, n3, r = dims
    d = synth.low_rank_plus_outliers_f32(n1, n2, n3, r, p_out=0.05, seed=0, init_seed=123)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=iters)
    ref = mod.admm(lib, d["D"], r, opts, d["A0"], d["B0"], d["C0"])
    A, B, C, O, E, eh, k = tritd_lean.admm_f32(lib, d["D"], r, opts, d["A0"], d["B0"], d["C0"],
                                               block=n1 * 4)
    assert k == ref[6]
    np.testing.assert_allclose(eh, ref[4], rtol=1e-6, atol=0)
    assert rel(orc.triple_product(A, B, C), orc.triple_product(*ref[:3])) <= 1e-6
    assert rel(O.astype(float), ref[3].astype(float)) <= 1e-6
    assert rel(E.astype(float), ref[5].astype(float)) <= 1e-6
    Lr = orc.triple_product(*ref[:3])
    want = np.linalg.norm(Lr - d["Lstar"]) / np.linalg.norm(d["Lstar"].astype(float))
    assert abs(tritd_lean.rre(lib, A, B, C, d["Lstar"]) - want) <= 1e-6 * want + 1e-15
    idx = np.array([0, 5, n1 * n2 * n3 - 1])
    np.testing.assert_allclose(tritd_lean.sample_L(A, B, C, idx),
                               orc.triple_product(A, B, C).reshape(-1, order="F")[idx], rtol=1e-12)


# ---------------------------------------------------------------------------
# triple_decomp_ALS (fast_robust_triple_tensor/triple_decomp_ALS.m)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", golden_names("als"))
def test_oracle_als_reproduces_golden(name):
    g = load_golden(name)
    A, B, C, eh, k = orc.triple_decomp_ALS(g["X"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"],
                                           printer=lambda s: None)
    assert k == g["k"] and len(eh) == k
    for key, X in (("A", A), ("B", B), ("C", C)):
        assert rel(X, g[key]) <= 1e-12, key
    np.testing.assert_allclose(eh, g["errHist"], rtol=1e-12, atol=1e-15)


@pytest.mark.parametrize("name", golden_names("als"))
def test_als_golden_stop_semantics(name):
    """:20-23: the stop test fires on the first k > 1 whose relative change is
    below tol, errHist is truncated to k; otherwise all maxIter entries."""
    g = load_golden(name)
    e, tol, k = g["errHist"], g["opts"]["tol"], g["k"]
    rel_change = np.abs(np.diff(e)) / e[:-1]
    fired = np.nonzero(rel_change < tol)[0]
    if k < g["opts"]["maxIter"]:
        assert len(fired) == 1 and fired[0] == k - 2
    else:
        assert len(fired) == 0 and k == g["opts"]["maxIter"]


def test_als_error_is_taken_before_the_update():
    """errHist(k) is the fit of the factors entering iteration k (:15-16), and
    a stop at k returns those factors un-updated (:22)."""
    g = load_golden("als20x24x18_r5_stop")
    k = g["k"]
    Xhat = orc.triple_product(g["A"], g["B"], g["C"])
    e_k = np.linalg.norm((g["X"] - Xhat).ravel()) / np.linalg.norm(g["X"].ravel())
    assert abs(e_k - g["errHist"][k - 1]) <= 1e-13 * e_k
    # one iteration: errHist(1) is the fit of the initial factors
    _, _, _, eh1, k1 = orc.triple_decomp_ALS(g["X"], g["r"], dict(maxIter=1, tol=1e-5), g["A0"],
                                             g["B0"], g["C0"], printer=lambda s: None)
    Xhat0 = orc.triple_product(g["A0"], g["B0"], g["C0"])
    assert k1 == 1
    assert abs(eh1[0] - np.linalg.norm((g["X"] - Xhat0).ravel()) / np.linalg.norm(g["X"].ravel())) < 1e-14


def test_als_recovers_exact_low_rank(synth):
    """Known answer: on an exactly rank-r^2 tensor (no outliers) ALS drives the
    relative error down by orders of magnitude, and the error never rises by
    more than rounding (each update is a ridge-1e-9 least-squares solve)."""
    A, B, C = synth.random_factors(14, 12, 10, 2, seed=3)
    X = orc.triple_product(A, B, C)
    A0, B0, C0 = synth.random_factors(14, 12, 10, 2, seed=4)
    _, _, _, eh, k = orc.triple_decomp_ALS(X, 2, dict(maxIter=200, tol=1e-12), A0, B0, C0,
                                           printer=lambda s: None)
    assert eh[-1] < 1e-9 * eh[0]
    assert np.all(np.diff(eh) <= 1e-9 * eh[:-1] + 1e-13)  # rounding floor ~1e-10


def test_als_opts_and_print():
    g = load_golden("als12x10x8_r2")
    with pytest.raises(KeyError, match="maxIter"):
        orc.triple_decomp_ALS(g["X"], 2, dict(tol=1e-5), g["A0"], g["B0"], g["C0"])
    with pytest.raises(KeyError, match="tol"):
        orc.triple_decomp_ALS(g["X"], 2, dict(maxIter=3), g["A0"], g["B0"], g["C0"])
    lines = []
    _, _, _, eh, k = orc.triple_decomp_ALS(g["X"], 2, dict(maxIter=12, tol=0.0, mu=1), g["A0"],
                                           g["B0"], g["C0"], printer=lines.append)
    assert k == 12
    assert lines == ["Iteration %d, relative error = %.4e" % (i, eh[i - 1]) for i in (5, 10)]


# ---------------------------------------------------------------------------
# Driver metrics: evaluate (traffic_triple_comparison.m:194-202), quality_ybz
# (psnr_index.m, ssim_index.m) — SURVEY.md §8f ranks 1, 3
# ---------------------------------------------------------------------------
def test_oracle_filter2_and_window():
    from scipy.signal import correlate2d
    w = orc.fspecial_gaussian(11, 1.5)
    assert w.shape == (11, 11) and abs(w.sum() - 1.0) < 1e-15
    assert np.array_equal(w, w.T) and np.array_equal(w, w[::-1, ::-1])
    assert w[5, 5] == w.max()
    img = np.random.default_rng(1).uniform(0, 255, (23, 19))
    np.testing.assert_allclose(orc.filter2_valid(w, img), correlate2d(img, w, mode="valid"),
                               rtol=1e-13)


def test_oracle_quality_known_answers():
    rng = np.random.default_rng(2)
    X = rng.uniform(0, 255, (20, 24, 3))
    p, s = orc.quality_ybz(X, X)
    assert p == np.inf and s == 1.0
    Y = X + 1.0  # mse = 1 -> psnr = 20 log10(255)
    p, _ = orc.quality_ybz(X, Y)
    assert abs(p - 20 * np.log10(255.0)) < 1e-12
    Z = X + rng.normal(0, 20, X.shape)
    assert abs(orc.ssim_index(X[:, :, 0], Z[:, :, 0]) - orc.ssim_index(Z[:, :, 0], X[:, :, 0])) < 1e-14
    assert orc.ssim_index(X[:10, :, 0], Z[:10, :, 0]) == -np.inf  # smaller than the window


def test_oracle_evaluate_masked_order():
    rng = np.random.default_rng(3)
    X = rng.standard_normal((5, 4, 3))
    Xh = X + 0.1 * rng.standard_normal(X.shape)
    mask = rng.random(X.shape) < 0.3
    gt = X[mask.ravel(order="F").reshape(X.shape, order="F")]  # any order of the same set...
    gt = X.ravel(order="F")[mask.ravel(order="F")]             # ...MATLAB's X(mask) is column-major
    rmse, nrmse = orc.evaluate(Xh.ravel(order="F")[mask.ravel(order="F")], gt)
    assert abs(rmse - np.linalg.norm((Xh - X)[mask])) < 1e-14
    assert abs(nrmse - rmse / np.linalg.norm(X[mask])) < 1e-14


def test_derived_yo_identity_in_the_restatement():
    """The identity K5's derived-Y_O mode relies on (k_admm.hip header):
    with muL == muO (:16-17), Y_L^(k) - Y_O^(k) = mu_k (E^(k) - E^(k-1)) for
    every k, up to rounding — checked on the restatement's own trace."""
    g = load_golden("g12x10x8_r2")
    *_, tr = orc.triple_decomp_ADMM(g["D"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"],
                                    trace_iters=(1, 2, 3, 7))
    mus = orc.mu_schedule(g["opts"]["mu"], g["opts"]["rho"], 10)
    E_prev = {1: np.zeros_like(tr[1]["E"]), 2: tr[1]["E"], 3: tr[2]["E"]}
    for k in (1, 2, 3):
        lhs = tr[k]["Y_L"] - tr[k]["Y_O"]
        rhs = mus[k - 1] * (tr[k]["E"] - E_prev[k])
        scale = np.abs(tr[k]["Y_L"]).max()
        assert np.abs(lhs - rhs).max() <= 1e-13 * scale, k
