"""The pinv-tolerance warning (TRITD_FLAG_PINV_TOL) end to end.

MATLAB's pinv (triple_decomp_ADMM.m:78,86,93; triple_decomp_ALS.m:27,32,37)
drops singular values below max(size)*eps(max sigma); the GPU inverts the
ridge Gram, and where a Gram's smallest pivot comes within 1e3x of that
cutoff it computes pinv itself (pinv.h: Jacobi eigendecomposition with
MATLAB's tolerance).  When that pinv drops a value the device raises a flag,
which every ABI path reports (tritd_last_flags, tritd_session_flags,
tritd_als_session_flags) and the Python wrappers turn into a
PinvToleranceWarning.  The ill-conditioned case:
n2 = n3 = 2 with r = 3 makes (B^TB)o(C^TC) (rank <= 4 < R = 9) singular, so
its smallest pivots sit at the ridge, and large B0, C0 push max sigma to
where eps(max sigma) * R * 1e3 exceeds the ridge.  Also here: repeated solves
give bitwise-identical errHist (fixed-order reductions, no reassociation)."""
import warnings

import numpy as np
import pytest

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tritd():
    import tritd as t
    assert t.device_count() > 0, "no GPU visible: the HIP path must run, there is no CPU fallback"
    return t


def ill_conditioned(scale):
    rng = np.random.default_rng(11)
    n1, n2, n3, r = 6, 2, 2, 3
    X = np.asfortranarray(rng.standard_normal((n1, n2, n3)))
    A0 = rng.standard_normal((n1, r, r))
    B0 = scale * rng.standard_normal((r, n2, r))
    C0 = scale * rng.standard_normal((r, r, n3))
    return X, r, A0, B0, C0


def test_als_raises_pinv_flag(tritd):
    from tritd import _lib
    X, r, A0, B0, C0 = ill_conditioned(30.0)
    with pytest.warns(tritd.PinvToleranceWarning):
        tritd.triple_decomp_ALS(X, r, dict(maxIter=2, tol=0.0), A0, B0, C0)
    assert _lib.lib.tritd_last_flags() & _lib.FLAG_PINV_TOL
    s = tritd.AlsSession(r, dict(maxIter=2, tol=0.0), A0, B0, C0, n1=6, n2=2, n3=2, X=X, device=0)
    s.run(2)
    s.sync()
    assert s.flags() & _lib.FLAG_PINV_TOL
    s.close()


def test_admm_raises_pinv_flag(tritd):
    from tritd import _lib, synth
    X, r, A0, B0, C0 = ill_conditioned(1000.0)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=2)
    with pytest.warns(tritd.PinvToleranceWarning):
        tritd.triple_decomp_ADMM(X, r, opts, A0, B0, C0)
    assert _lib.lib.tritd_last_flags() & _lib.FLAG_PINV_TOL
    s = tritd.Session(r, opts, A0, B0, C0, n1=6, n2=2, n3=2, D=X, device=0)
    s.run(2)
    s.sync()
    assert s.flags() & _lib.FLAG_PINV_TOL
    with pytest.warns(tritd.PinvToleranceWarning):
        s.get()
    s.close()


# The truncated pinv itself (pinv.h): where the pivots come near MATLAB's
# cutoff the apply uses pinv(G) from a Jacobi eigendecomposition, dropping
# |lambda| <= R eps(max |lambda|) exactly as tritd_oracle.pinv (SVD) does.
# Cases are chosen so that every Gram they meet is either cleanly truncated
# (dropped eigenvalues <= 0.13 x the cutoff, kept ones >= 1e13 x) or
# well-conditioned enough for 1e-8 (cond <= 1e7): the ADMM case for its first
# iteration (update_A truncates 5 of 9 values; at iteration 2 its Gram is
# untruncated with cond 1.7e12, where any two pinv implementations part at
# the 1e-6 level), the ALS case for four (update_A truncates every time).

def _rel(a, b):
    return np.linalg.norm((a - b).ravel()) / np.linalg.norm(b.ravel())


@pytest.mark.parametrize("iters", [1])
def test_admm_truncated_pinv_matches_oracle(tritd, iters):
    import tritd_oracle as orc
    from tritd import synth
    X, r, A0, B0, C0 = ill_conditioned(1000.0)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=iters)
    rA, rB, rC, rO, reh, rE, rk, _ = orc.triple_decomp_ADMM(X, r, opts, A0, B0, C0)
    with pytest.warns(tritd.PinvToleranceWarning):
        A, B, C, O, eh, E, k = tritd.triple_decomp_ADMM(X, r, opts, A0, B0, C0, return_E=True,
                                                        return_iters=True)
    assert k == rk
    L, Lr = orc.triple_product(A, B, C), orc.triple_product(rA, rB, rC)
    assert _rel(L, Lr) <= 1e-8 and _rel(O, rO) <= 1e-8
    np.testing.assert_allclose(eh, reh, rtol=1e-8)
    # an inverse instead of pinv lands far away: the case really truncates
    Ginv_like = orc.triple_product(A0, B0, C0)
    assert _rel(L, Ginv_like) > 1e-3


@pytest.mark.parametrize("iters", [1, 2, 4])
def test_als_truncated_pinv_matches_oracle(tritd, iters):
    import tritd_oracle as orc
    X, r, A0, B0, C0 = ill_conditioned(30.0)
    opts = dict(maxIter=iters, tol=0.0)
    rA, rB, rC, reh, rk = orc.triple_decomp_ALS(X, r, opts, A0, B0, C0, printer=lambda s: None)
    with pytest.warns(tritd.PinvToleranceWarning):
        A, B, C, eh = tritd.triple_decomp_ALS(X, r, opts, A0, B0, C0)
    assert len(eh) == rk
    L, Lr = orc.triple_product(A, B, C), orc.triple_product(rA, rB, rC)
    assert _rel(L, Lr) <= 1e-8
    np.testing.assert_allclose(eh, reh, rtol=1e-8, atol=1e-11)


@pytest.mark.parametrize("name", golden_names()[:3])
def test_well_conditioned_goldens_raise_no_flag(tritd, name):
    from tritd import _lib
    g = load_golden(name)
    with warnings.catch_warnings():
        warnings.simplefilter("error", tritd.PinvToleranceWarning)
        tritd.triple_decomp_ADMM(g["D"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"])
    assert _lib.lib.tritd_last_flags() == 0


@pytest.mark.parametrize("name", ["g30_r3", "g54x4x96_r5_sensor"])
def test_repeated_solves_are_bitwise_identical(tritd, name):
    g = load_golden(name)
    runs = [tritd.triple_decomp_ADMM(g["D"], g["r"], g["opts"], g["A0"], g["B0"], g["C0"],
                                     return_E=True) for _ in range(3)]
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            np.testing.assert_array_equal(a, b)


# solve A of iteration k+1 runs beside K5 of iteration k, before
# k's stop test; the pinv fallback of that solve (and its flag) must wait for
# apply A, which runs only if the loop goes on.  With maxIter = 0 the loop
# stops before update_A(1), whose Gram (B0, C0 of the ill-conditioned case) is
# singular: MATLAB performs no pinv, so no flag.  Both the MFMA apply (fp64,
# r = 3) and the generic apply (single class) paths.
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_no_pinv_flag_for_an_update_the_loop_never_runs(tritd, dtype):
    from tritd import _lib, synth
    X, r, A0, B0, C0 = ill_conditioned(1000.0)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=0)
    with warnings.catch_warnings():
        warnings.simplefilter("error", tritd.PinvToleranceWarning)
        tritd.triple_decomp_ADMM(np.asfortranarray(X, dtype=dtype), r, opts, A0, B0, C0)
    assert (_lib.lib.tritd_last_flags() & _lib.FLAG_PINV_TOL) == 0
