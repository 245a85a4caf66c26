"""fp32 data path (D of MATLAB class single; SURVEY.md §8a row 1, §8b
tritd_admm_f32, §8d config 5) against the single-class C restatement
(oracle/tritd_ref.c: tritd_ref_admm_f32) on the same inputs.

Tolerances (stated here): both sides round to single at the
same statements but accumulate their GEMMs in different orders (the oracle
in double then rounded once, the GPU in single on MFMA), so the iterates
agree at single-precision level on well-conditioned problems (n_k >= R):
relative Frobenius error of L = triple_product(A,B,C), O, E <= 2e-5 and the
same iteration count.

errHist (errHist(k) = (||resL|| + ||resO||) / ||D||, :59) per iteration:
|eh_gpu(k) - eh_ref(k)| <= RHO * eh_ref(k) + EH_C * u32 * s, u32 = 2^-24
the unit roundoff of single and s = (||D|| + ||L|| + 2 ||O|| + ||E||) /
||D||: each element of resL = D - L - O and resO = O - E is formed in
single on both sides, so each residual norm carries an absolute rounding
error of order u32 (||D|| + ||L|| + ||O||), resp. u32 (||O|| + ||E||) — at
the fp32 floor (errHist ~1.3 u32) the two sides' norms are independent
rounding noise of that size, and the bound says that much; RHO covers the
iterates' own single-precision divergence (the L/O/E tolerance above) while
the residuals are far above the floor.  (Round 4 compared with an absolute
floor of 1e-4 errHist(1), ~1000x looser at the floor: VERDICT r4 weak 1b.)
Ill-conditioned Grams (n_k < R) amplify single rounding by their condition
number on any implementation and are not used for parity.
"""
import numpy as np
import pytest

from conftest import rel

pytestmark = pytest.mark.gpu

TOL = 2e-5
U32 = 2.0 ** -24
EH_C = 8.0  # errHist rounding-noise constant (module docstring)
RHO = 1e-5  # errHist relative divergence allowance, r <= 8 (module docstring)
# r = 16 (R = 256, config 5's rank): L is formed in f32 on MFMA over 256
# terms where the restatement forms it in double (the stated deviation of
# DESIGN.md §2); over the 100-iteration horizon at 256^3 the two errHist
# sequences drift apart by up to RHO_R16 relative while the residuals decay
RHO_R16 = 2e-3  # measured need 5.5e-4 (profiles/round5/f32_errhist_calibration.txt)


def eh_bound(D, L, O, E, eh_ref, rho=RHO):
    """Per-iteration errHist tolerance (module docstring)."""
    f = lambda x: np.linalg.norm(np.asarray(x, np.float64))  # noqa: E731
    nD = f(D)
    s = (nD + f(L) + 2 * f(O) + f(E)) / nD
    return rho * np.asarray(eh_ref) + EH_C * U32 * s, s


def check_errhist(eh, eh_ref, D, L, O, E, report=None, rho=RHO):
    eh, eh_ref = np.asarray(eh), np.asarray(eh_ref)
    b, s = eh_bound(D, L, O, E, eh_ref, rho)
    d = np.abs(eh - eh_ref)
    worst = float(np.max(d / b))
    if report is not None:  # calibration figures: what each term alone would need
        report.update(eh_worst=worst, eh_max_abs_over_u32s=float(np.max(d) / (U32 * s)),
                      rho_needed=float(np.max(np.maximum(d - EH_C * U32 * s, 0.0) / eh_ref)),
                      eh_max_rel=float(np.max(d / eh_ref)))
    assert worst <= 1.0, ("errHist outside the fp32 rounding bound", worst, report)
    return worst


@pytest.fixture(scope="module")
def tritd():
    import tritd as t
    assert t.device_count() > 0
    return t


@pytest.fixture(scope="module")
def cref():
    import os
    import subprocess
    import tritd_oracle
    here = os.path.dirname(os.path.abspath(tritd_oracle.__file__))
    subprocess.run(["make", "-C", here], check=True, capture_output=True)
    import tritd_ref
    return tritd_ref, tritd_ref.load()


def _compare(tritd, cref, D, r, opts, A0, B0, C0, tol=TOL):
    import tritd_oracle as orc
    mod, lib = cref
    ref = mod.admm(lib, D, r, opts, A0, B0, C0)
    A, B, C, O, eh, E, k = tritd.triple_decomp_ADMM(D, r, opts, A0, B0, C0, return_E=True,
                                                    return_iters=True)
    assert O.dtype == np.float32 and E.dtype == np.float32 and A.dtype == np.float64
    assert k == ref[6]
    L = orc.triple_product(A, B, C)
    Lr = orc.triple_product(ref[0], ref[1], ref[2])
    assert rel(L, Lr) <= tol
    assert rel(O.astype(np.float64), ref[3].astype(np.float64)) <= tol
    if np.any(ref[5]):
        assert rel(E.astype(np.float64), ref[5].astype(np.float64)) <= tol
    else:
        assert not np.any(E)
    check_errhist(eh, ref[4], D, Lr, ref[3], ref[5], {})
    return E


@pytest.mark.parametrize("shape,r,iters", [((24, 20, 18), 3, 30), ((80, 64, 96), 5, 40),
                                           ((128, 16, 64), 4, 40), ((96, 80, 72), 8, 30)])
def test_f32_vs_c_oracle(tritd, cref, shape, r, iters):
    from tritd import synth
    d = synth.low_rank_plus_outliers(*shape, r, seed=2, init_seed=7)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=iters)
    _compare(tritd, cref, d["D"].astype(np.float32), r, opts, d["A0"], d["B0"], d["C0"])


@pytest.mark.parametrize("shape,r,iters", [((96, 80, 72), 10, 12), ((80, 72, 64), 12, 10),
                                           ((64, 64, 48), 16, 10)])
def test_f32_large_rank_vs_c_oracle(tritd, cref, shape, r, iters):
    """r = 9..16 (padded rank 128 / 256, config 5's r = 16): the blocked R x R
    sweep (k_contract.hip k_solve_big) and the RP-general fp32 kernels."""
    from tritd import synth
    d = synth.low_rank_plus_outliers(*shape, r, seed=2, init_seed=7)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=iters)
    _compare(tritd, cref, d["D"].astype(np.float32), r, opts, d["A0"], d["B0"], d["C0"])


@pytest.mark.parametrize("P", [2, 3])
def test_f32_r16_sharded_vs_c_oracle(tritd, cref, P):
    """Config 5's rank (r = 16, padded rank 256) on the mode-1 sharded schedule
     — what the config-5 leg of an N > 1 bench runs on every
    rank: one GPU repeated P times as a device set (one host thread and one
    session per shard, all-reduces in shard order), shards of 32 | 32 and
    22 | 21 | 21 rows (straddling the 16-row tiles), against the C restatement
    at the fp32 tolerances of this module."""
    from tritd import synth
    d = synth.low_rank_plus_outliers_f32(64, 64, 48, 16, p_out=0.05, seed=2, init_seed=7)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=10)
    tritd.set_devices([0] * P)
    try:
        _compare(tritd, cref, d["D"], 16, opts, d["A0"], d["B0"], d["C0"])
    finally:
        tritd.set_devices([])


@pytest.mark.timeout(300)
def test_f32_r16_long_horizon_vs_c_oracle(tritd, cref, capsys):
    """Config 5's rank (r = 16, padded rank 256) over the whole 100-iteration
    horizon of the bench, at 256^3 (n_k >= R = 256: well-conditioned Grams)
    where the C restatement takes ~30 s.  The restatement follows MATLAB's
    class rules (L = triple_product of double factors, rounded to single where
    it meets D, triple_product.m:6, triple_decomp_ADMM.m:41,50); the GPU forms
    L and W on f32 MFMA with f32 accumulation.  This bounds
    what that deviation does to the solve over the bench's horizon: same k,
    errHist, L, O, E at the fp32 tolerance, and the driver's RRE against L*
    (traffic_triple_comparison.m:62-63) within 1e-6 + 2e-5 RRE."""
    import time

    import tritd_oracle as orc
    from tritd import synth
    mod, lib = cref
    n, r = 256, 16
    d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
    D = d["D"].astype(np.float32, order="F")
    opts = dict(synth.TRAFFIC_OPTS, maxIter=100)
    t0 = time.time()
    ref = mod.admm(lib, D, r, opts, d["A0"], d["B0"], d["C0"])
    tc = time.time() - t0
    A, B, C, O, eh, E, k = tritd.triple_decomp_ADMM(D, r, opts, d["A0"], d["B0"], d["C0"],
                                                    return_E=True, return_iters=True)
    L = orc.triple_product(A, B, C)
    Lr = orc.triple_product(ref[0], ref[1], ref[2])
    nL = np.linalg.norm(d["Lstar"])
    rre = np.linalg.norm(L - d["Lstar"]) / nL
    rre_c = np.linalg.norm(Lr - d["Lstar"]) / nL
    stats = dict(k=k, k_c=ref[6], rel_L=rel(L, Lr), rel_O=rel(O.astype(np.float64), ref[3].astype(np.float64)),
                 rel_E=rel(E.astype(np.float64), ref[5].astype(np.float64)), rre=rre, rre_c=rre_c,
                 d_rre=abs(rre - rre_c), eh_last=float(eh[-1]), eh_last_c=float(ref[4][-1]),
                 max_rel_eh=float(np.max(np.abs(eh - ref[4]) / ref[4])), c_seconds=round(tc, 1),
                 max_abs_eh_over_u32=float(np.max(np.abs(eh - ref[4])) / U32))
    with capsys.disabled():
        print("  r=16 fp32 long horizon:", stats, flush=True)
    assert k == ref[6] == 100
    assert stats["rel_L"] <= TOL and stats["rel_O"] <= TOL and stats["rel_E"] <= TOL
    rep = {}
    try:
        check_errhist(eh, ref[4], D, Lr, ref[3], ref[5], rep, rho=RHO_R16)
    finally:
        with capsys.disabled():
            print("  errHist vs bound:", rep, flush=True)
    assert stats["d_rre"] <= 1e-6 + 2e-5 * rre_c


@pytest.mark.parametrize("shape,r,tol,k_expected", [((96, 80, 72), 5, 1e-3, 13),
                                                    ((64, 64, 64), 4, 5e-4, 8)])
def test_f32_stop_fires_at_the_same_iteration(tritd, cref, capsys, shape, r, tol, k_expected):
    """The stop test (:63: |errHist(k) - errHist(k-1)| < tol errHist(k-1))
    fires before maxIter on an fp32 solve at the iteration the restatement
    stops at.  The cases stop in the slow phase of the first iterations,
    where the relative change first drops below tol by a clear margin (every
    earlier change is at least 2x tol): the same k is a parity statement
    there, not a coin flip at the fp32 floor (where single-precision noise
    decides any implementation's relative change)."""
    import tritd_oracle as orc
    from tritd import synth
    mod, lib = cref
    d = synth.low_rank_plus_outliers(*shape, r, seed=2, init_seed=7)
    D = d["D"].astype(np.float32)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=100, tol=tol)
    ref = mod.admm(lib, D, r, opts, d["A0"], d["B0"], d["C0"])
    A, B, C, O, eh, E, k = tritd.triple_decomp_ADMM(D, r, opts, d["A0"], d["B0"], d["C0"],
                                                    return_E=True, return_iters=True)
    kr, ehr = ref[6], np.asarray(ref[4])
    assert kr == k_expected < 100
    rc = np.abs(np.diff(ehr)) / ehr[:-1]  # rc[k-2]: the change tested at iteration k
    assert rc[-1] < tol and np.all(rc[:-1] >= 2 * tol)
    rep = {}
    try:
        Lr = orc.triple_product(ref[0], ref[1], ref[2])
        check_errhist(eh, ehr, D, Lr, ref[3], ref[5], rep)
    finally:
        with capsys.disabled():
            print("  tol=%g: k=%d (restatement %d), stop margin %.2fx tol; errHist %s"
                  % (tol, k, kr, (tol - rc[-1]) / tol, rep), flush=True)
    assert k == kr


@pytest.mark.parametrize("case", ["mixed_tiles", "all_dense"])
def test_f32_compact_e_overflow_tiles(tritd, cref, case):
    """Compact E in fp32: 64-word slots, more than 56 nonzeros of a 256-element
    tile go dense (k_admm32.hip)."""
    from tritd import synth
    n1, n2, n3, r = 64, 40, 64, 3
    d = synth.low_rank_plus_outliers(n1, n2, n3, r, p_out=0.05, seed=11, init_seed=5)
    D = d["D"].copy(order="F")
    opts = dict(synth.TRAFFIC_OPTS, maxIter=30)
    if case == "mixed_tiles":
        rng = np.random.default_rng(3)
        D[:16, :7, :40] += 8.0 * rng.standard_normal((16, 7, 40))
    else:
        opts["lambda"] = 1e-6
    E = _compare(tritd, cref, D.astype(np.float32), r, opts, d["A0"], d["B0"], d["C0"])
    nnz = np.count_nonzero(E) / E.size
    assert (nnz > 0.5) if case == "all_dense" else (0.02 < nnz < 0.5)


def test_f32_stepping_is_deterministic(tritd):
    from tritd import synth
    n, r = 64, 4
    d = synth.low_rank_plus_outliers(n, n, n, r, seed=0)
    D = d["D"].astype(np.float32)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=100)

    def session():
        return tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, D=D, device=0)

    s1 = session()
    s1.run(7)
    s1.run(8)
    r1 = s1.get()
    s1.close()
    s2 = session()
    s2.run(15)
    r2 = s2.get()
    s2.close()
    assert r1["k"] == r2["k"] == 15
    assert r1["O"].dtype == np.float32
    for key in ("A", "B", "C", "O", "E", "errHist"):
        np.testing.assert_array_equal(r1[key], r2[key])


def test_f32_zero_iterations(tritd):
    from tritd import synth
    d = synth.low_rank_plus_outliers(20, 18, 16, 2, seed=0)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=0)
    A, B, C, O, eh = tritd.triple_decomp_ADMM(d["D"].astype(np.float32), 2, opts, d["A0"],
                                              d["B0"], d["C0"])
    assert len(eh) == 0 and not np.any(O) and O.dtype == np.float32
    np.testing.assert_array_equal(A, d["A0"])


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_non_recovering_shape_rre_matches_oracle(tritd, cref, dtype):
    """At 256x256x32 r=4 the reference's ADMM does not recover L* within
    maxIter = 100 (RRE 0.24 in the C restatement, fp64 and fp32 alike): the
    config-5 bench's RRE of 0.10 is the algorithm's, not the kernels'.  The
    GPU reproduces the restatement's RRE to the stated tolerance."""
    import tritd_oracle as orc
    from tritd import synth
    d = synth.low_rank_plus_outliers(256, 256, 32, 4, p_out=0.05, seed=0, init_seed=123)
    opts = dict(synth.TRAFFIC_OPTS)
    mod, lib = cref
    D = d["D"].astype(dtype)
    ref = mod.admm(lib, D, 4, opts, d["A0"], d["B0"], d["C0"])
    A, B, C, O, eh = tritd.triple_decomp_ADMM(D, 4, opts, d["A0"], d["B0"], d["C0"])
    nL = np.linalg.norm(d["Lstar"])
    rre = np.linalg.norm(orc.triple_product(A, B, C) - d["Lstar"]) / nL
    rre_ref = np.linalg.norm(orc.triple_product(ref[0], ref[1], ref[2]) - d["Lstar"]) / nL
    assert len(eh) == ref[6] == 100
    assert rre_ref > 0.1
    assert abs(rre - rre_ref) <= (1e-9 if dtype == np.float64 else 1e-4) * rre_ref
