"""GPU parity of triple_decomp_ALS (fast_robust_triple_tensor/triple_decomp_ALS.m,
SURVEY.md §8f rank 2) against the oracle restatement and its golden vectors.

Tolerances (fp64): A, B, C relative Frobenius <= 1e-8, triple_product(A,B,C)
<= 1e-9, errHist rtol 1e-9, same k.  The GPU computes the same algorithm with
the dimension-tree MTTKRPs, Hadamard Grams and a Gauss-Jordan inverse of the
ridge-1e-9 SPD Gram instead of buildF/G/H + pinv.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden, rel

pytestmark = pytest.mark.gpu

TOL_ABC = 1e-8
TOL_L = 1e-9
TOL_ERR = 1e-9


@pytest.fixture(scope="module")
def tritd():
    import tritd as t
    assert t.device_count() > 0, "no GPU visible: the HIP path must run, there is no CPU fallback"
    return t


@pytest.fixture(scope="module")
def orc():
    import tritd_oracle
    return tritd_oracle


def check(orc, got, A, B, C, eh, k):
    gA, gB, gC, geh, gk = got
    assert gk == k and len(geh) == k
    np.testing.assert_allclose(geh, eh, rtol=TOL_ERR, atol=1e-14)
    for name, x, y in (("A", gA, A), ("B", gB, B), ("C", gC, C)):
        assert rel(x, y) <= TOL_ABC, name
    assert rel(orc.triple_product(gA, gB, gC), orc.triple_product(A, B, C)) <= TOL_L


@pytest.mark.parametrize("name", golden_names("als"))
def test_als_matches_golden(tritd, orc, name):
    g = load_golden(name)
    got = tritd.triple_decomp_ALS(g["X"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"],
                                  return_iters=True)
    check(orc, got, g["A"], g["B"], g["C"], g["errHist"], g["k"])


@pytest.mark.parametrize("name,P", [("als30_r3", 2), ("als30_r3", 3), ("als17x16x20_r8", 4)])
def test_als_virtual_shards(tritd, orc, name, P):
    """Mode-1 sharded ALS (three reductions per iteration) as P shards on one GPU."""
    g = load_golden(name)
    got = tritd.triple_decomp_ALS(g["X"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"],
                                  return_iters=True, virtual_shards=P)
    check(orc, got, g["A"], g["B"], g["C"], g["errHist"], g["k"])


@pytest.mark.parametrize("name,P,serial", [("als30_r3", 3, False), ("als17x16x20_r8", 2, False),
                                           ("als30_r3", 3, True)])
def test_als_device_set(tritd, orc, name, P, serial, monkeypatch):
    """tritd_set_devices with one GPU repeated: one host thread per shard
    (api.cpp run_als_group, in-process all-reduces); TRITD_SHOV=0 keeps the
    phase-serial driver (run_als_group_serial)."""
    if serial:
        monkeypatch.setenv("TRITD_SHOV", "0")
    g = load_golden(name)
    tritd.set_devices([0] * P)
    try:
        got = tritd.triple_decomp_ALS(g["X"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"],
                                      return_iters=True)
    finally:
        tritd.set_devices([])
    check(orc, got, g["A"], g["B"], g["C"], g["errHist"], g["k"])


@pytest.mark.parametrize("shape,r", [((97, 80, 41), 8), ((64, 33, 50), 5), ((40, 48, 16), 1)])
def test_als_padded_shapes(tritd, orc, synth, shape, r):
    """Shapes that are not multiples of the 16-row tiles, every padded rank."""
    n1, n2, n3 = shape
    d = synth.low_rank_plus_outliers(n1=n1, n2=n2, n3=n3, r=r)
    opts = dict(maxIter=8, tol=0.0)
    ref = orc.triple_decomp_ALS(d["D"], r, opts, d["A0"], d["B0"], d["C0"], printer=lambda s: None)
    got = tritd.triple_decomp_ALS(d["D"], r, opts, d["A0"], d["B0"], d["C0"], return_iters=True)
    check(orc, got, *ref)


def test_als_print_and_opts(tritd, orc):
    g = load_golden("als12x10x8_r2")
    lines = []
    tritd.set_printer(lines.append)
    try:
        _, _, _, eh, k = tritd.triple_decomp_ALS(g["X"], 2, dict(maxIter=12, tol=0.0), g["A0"],
                                                 g["B0"], g["C0"], return_iters=True)
    finally:
        tritd.set_printer(None)
    assert k == 12
    assert lines == ["Iteration %d, relative error = %.4e" % (i, eh[i - 1]) for i in (5, 10)]
    with pytest.raises(KeyError, match="tol"):
        tritd.triple_decomp_ALS(g["X"], 2, dict(maxIter=3), g["A0"], g["B0"], g["C0"])
    # maxIter = 0: the loop never runs, the initial factors come back
    A, B, C, eh = tritd.triple_decomp_ALS(g["X"], 2, dict(maxIter=0, tol=1e-5), g["A0"], g["B0"],
                                          g["C0"])
    assert len(eh) == 0 and np.array_equal(A, g["A0"]) and np.array_equal(C, g["C0"])


def test_als_session_steps(tritd, orc):
    """The steppable session (bench path) gives the one-shot result."""
    g = load_golden("als17x16x20_r8")
    X = g["X"]
    s = tritd.AlsSession(g["r"], g["opts"], g["A0"], g["B0"], g["C0"], n1=X.shape[0],
                         n2=X.shape[1], n3=X.shape[2], X=X)
    for _ in range(5):
        s.run(5)
    out = s.get()
    s.close()
    check(orc, (out["A"], out["B"], out["C"], out["errHist"], out["k"]), g["A"], g["B"], g["C"],
          g["errHist"], g["k"])
