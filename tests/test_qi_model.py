"""opts.model = 'qi' (SURVEY.md §8f rank 4): the ADMM loop of
fast_robust_triple_tensor/triple_decomp_ADMM.m with the Qi-model design
matrices of origin_triple_tensor/buildF.m:2-6, buildG.m:7-11, buildH.m:7-11
(Qi's 3-index triple product sum_{p,q,s} A(i,q,s) B(p,j,s) C(p,q,t)).

CPU part: the oracle's Qi builders against the reference's own definitions
(the loop comments of origin_triple_tensor/buildG.m:2-6 and buildH.m:2-6, the
explicit-Kronecker kronF.m, the sum origin_triple_tensor/triple_product.m:8-19
spells out), and the oracle against its committed qi*.npz goldens
(tests/golden/make_golden.py).  The reference never runs this model (its
solver shadows these files with local CP builders), so the loop is outside the
parity contract: parity unpinned beyond these primitive identities.

GPU part (@gpu): libtritd with opts.model='qi' against the same goldens at
the tolerances of tests/test_gpu_parity.py, sharded == unsharded, and the Qi
triple product against the oracle.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, rel

import tritd_oracle as orc

TOL_LOE = 1e-9
TOL_ABC = 1e-8


def _factors(n1, n2, n3, r, seed=0):
    rng = np.random.default_rng(seed)
    return (np.asfortranarray(rng.standard_normal((n1, r, r))),
            np.asfortranarray(rng.standard_normal((r, n2, r))),
            np.asfortranarray(rng.standard_normal((r, r, n3))))


@pytest.mark.parametrize("dims", [(5, 4, 3, 2), (3, 6, 4, 3), (4, 3, 5, 1)])
def test_qi_builders_match_reference_definitions(dims):
    n1, n2, n3, r = dims
    A, B, C = _factors(n1, n2, n3, r)
    np.testing.assert_allclose(orc.buildG_qi(A, C), orc.buildG_qi_loops(A, C), rtol=0, atol=1e-13)
    np.testing.assert_allclose(orc.buildH_qi(A, B), orc.buildH_qi_loops(A, B), rtol=0, atol=1e-13)
    # kronF.m orders the rows s+(q-1)r; buildF.m q+(s-1)r
    F, K = orc.buildF_qi(B, C), orc.kronF(B, C)
    perm = [s + q * r for s in range(r) for q in range(r)]  # buildF row q+s*r <- kron row s+q*r
    np.testing.assert_allclose(F, K[perm], rtol=0, atol=1e-13)


@pytest.mark.parametrize("dims", [(5, 4, 3, 2), (4, 6, 5, 3)])
def test_qi_triple_product_matches_loop_and_unfoldings(dims):
    n1, n2, n3, r = dims
    A, B, C = _factors(n1, n2, n3, r, seed=1)
    L = orc.triple_product(A, B, C, "qi")
    np.testing.assert_allclose(L, orc.triple_product_qi_loops(A, B, C), rtol=0, atol=1e-12)
    # every mode: X_k = (factor unfolding) * (design matrix), as update_A/B/C assume
    B2 = np.stack([B[:, j, :].reshape(-1, order="F") for j in range(n2)])
    C3 = np.stack([C[:, :, t].reshape(-1, order="F") for t in range(n3)])
    np.testing.assert_allclose(orc.unfold(L, 2), B2 @ orc.buildG_qi(A, C), atol=1e-12)
    np.testing.assert_allclose(orc.unfold(L, 3), C3 @ orc.buildH_qi(A, B), atol=1e-12)
    # and it is not the executed CP product
    assert rel(L, orc.triple_product(A, B, C)) > 0.1


def test_model_option_validation():
    assert orc.opts_model({}) == "cp" and orc.opts_model({"model": "QI"}) == "qi"
    with pytest.raises(ValueError):
        orc.opts_model({"model": "tucker"})
    from tritd import api
    assert api.model_code(None) == 0 and api.model_code("qi") == 1
    with pytest.raises(ValueError):
        api.model_code("tucker")
    o = api.make_opts(dict(mu=1e-3, rho=1.25, maxIter=3, tol=1e-5, disp=0, lambda2=1e-3,
                           model="qi", **{"lambda": 1.8}))
    assert o.model == 1


@pytest.mark.parametrize("name", golden_names("qi"))
def test_oracle_reproduces_qi_golden(name):
    g = load_golden(name)
    assert g["opts"]["model"] == "qi"
    A, B, C, O, eh, E, k, tr = orc.triple_decomp_ADMM(g["D"], g["r"], g["opts"], g["A0"], g["B0"],
                                                      g["C0"], trace_iters=(1, 2))
    assert k == g["k"] and len(eh) == k
    for key, X in (("A", A), ("B", B), ("C", C), ("O", O), ("E", E)):
        assert rel(X, g[key]) <= 1e-12, key
    np.testing.assert_allclose(eh, g["errHist"], rtol=1e-12, atol=1e-15)


def test_qi_recovery_and_stop_known_answers():
    g = load_golden("qi30_r3")  # outlier-corrupted Qi-model tensor is recovered
    assert rel(orc.triple_product(g["A"], g["B"], g["C"], "qi"), g["Lstar"]) < 1e-6
    s = load_golden("qi20x24x18_r3_video_stop")  # the stop test at :63 fires
    assert s["k"] < s["opts"]["maxIter"]
    e = s["errHist"]
    assert abs(e[-1] - e[-2]) < s["opts"]["tol"] * e[-2]


# ---------------------------------------------------------------------------
# GPU (libtritd, HIP on gfx950)
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def tritd():
    import tritd as t
    assert t.device_count() > 0, "no GPU visible: the HIP path must run, there is no CPU fallback"
    return t


def _check(got, ref):
    A, B, C, O, eh, E, k = got
    assert k == ref["k"] and len(eh) == k
    L = orc.triple_product(A, B, C, "qi")
    assert rel(L, orc.triple_product(ref["A"], ref["B"], ref["C"], "qi")) <= TOL_LOE
    assert rel(O, ref["O"]) <= TOL_LOE
    assert rel(E, ref["E"]) <= TOL_LOE
    for key, X in (("A", A), ("B", B), ("C", C)):
        assert rel(X, ref[key]) <= TOL_ABC, key
    np.testing.assert_allclose(eh, ref["errHist"], rtol=1e-8, atol=1e-11)


@pytest.mark.gpu
@pytest.mark.parametrize("name", golden_names("qi"))
def test_gpu_qi_matches_golden(tritd, name):
    g = load_golden(name)
    got = tritd.triple_decomp_ADMM(g["D"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"],
                                   return_E=True, return_iters=True)
    _check(got, g)


@pytest.mark.gpu
def test_gpu_qi_first_iterations(tritd):
    g = load_golden("qi12x10x8_r2")
    for it in (1, 2):
        opts = dict(g["opts"], maxIter=it)
        A, B, C, O, eh, k = tritd.triple_decomp_ADMM(g["D"], g["r"], opts, g["A0"], g["B0"], g["C0"],
                                                     return_iters=True)
        assert k == it
        for key, X in (("A", A), ("B", B), ("C", C)):
            assert rel(X, g[f"it{it}_{key}"]) <= 1e-11, (it, key)


@pytest.mark.gpu
@pytest.mark.parametrize("name,P", [("qi30_r3", 3), ("qi17x16x20_r8", 2)])
def test_gpu_qi_virtual_shards(tritd, name, P):
    """Mode-1 sharded schedule with the Qi kernels (partial M2 / A^TA / M3 sums)."""
    g = load_golden(name)
    got = tritd.triple_decomp_ADMM(g["D"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"],
                                   return_E=True, return_iters=True, virtual_shards=P)
    _check(got, g)


@pytest.mark.gpu
@pytest.mark.parametrize("n1,n2,n3,r", [(12, 10, 8, 2), (30, 31, 29, 3), (17, 16, 20, 8),
                                        (9, 7, 33, 12)])
def test_gpu_qi_triple_product(tritd, n1, n2, n3, r):
    A, B, C = _factors(n1, n2, n3, r, seed=3)
    got = tritd.triple_product(A, B, C, "qi")
    assert rel(got, orc.triple_product_qi_loops(A, B, C) if r <= 3 else
               orc.triple_product(A, B, C, "qi")) <= 1e-13


@pytest.mark.gpu
def test_gpu_qi_medium_against_oracle(tritd, synth):
    """A 96 x 80 x 64 r=4 Qi solve (several K5 workgroups and t-tiles) against the oracle."""
    d = synth.low_rank_plus_outliers(96, 80, 64, 4, model="qi")
    opts = dict(synth.TRAFFIC_OPTS, maxIter=30, model="qi")
    ref = orc.triple_decomp_ADMM(d["D"], 4, opts, d["A0"], d["B0"], d["C0"])
    A, B, C, O, eh, E, k = tritd.triple_decomp_ADMM(d["D"], 4, opts, d["A0"], d["B0"], d["C0"],
                                                    return_E=True, return_iters=True)
    assert k == ref[6]
    assert rel(orc.triple_product(A, B, C, "qi"), orc.triple_product(ref[0], ref[1], ref[2], "qi")) <= 1e-9
    assert rel(O, ref[3]) <= 1e-9 and rel(E, ref[5]) <= 1e-9
    np.testing.assert_allclose(eh, ref[4], rtol=1e-8, atol=1e-11)


@pytest.mark.gpu
def test_gpu_qi_rejects_single_and_bad_model(tritd):
    g = load_golden("qi12x10x8_r2")
    with pytest.raises(tritd.TritdError, match="UNSUPPORTED"):
        tritd.triple_decomp_ADMM(g["D"].astype(np.float32), g["r"], g["opts"], g["A0"], g["B0"],
                                 g["C0"])
    with pytest.raises(ValueError):
        tritd.triple_decomp_ADMM(g["D"], g["r"], dict(g["opts"], model="x"), g["A0"], g["B0"],
                                 g["C0"])
