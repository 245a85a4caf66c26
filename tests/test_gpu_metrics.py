"""GPU parity of the driver metrics against the
oracle restatements: evaluate (traffic_triple_comparison.m:194-202) and
quality_ybz (psnr_index.m, ssim_index.m).  Tolerances: rmse/nrmse and PSNR
rtol 1e-12 (fixed-order sums vs numpy's), SSIM rtol 1e-11 (the 11x11 window
sums are accumulated in a different order than MATLAB's filter2)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tritd():
    import tritd as t
    assert t.device_count() > 0, "no GPU visible: the HIP path must run, there is no CPU fallback"
    return t


@pytest.fixture(scope="module")
def orc():
    import tritd_oracle
    return tritd_oracle


@pytest.mark.parametrize("shape,p", [((30, 30, 30), 0.1), ((54, 4, 1152), 0.1), ((7, 5, 3), 0.5),
                                     ((240, 320, 20), 0.05)])
def test_evaluate_masked_matches_oracle(tritd, orc, shape, p):
    rng = np.random.default_rng(5)
    X = np.asfortranarray(rng.standard_normal(shape))
    Xh = np.asfortranarray(X + 0.01 * rng.standard_normal(shape))
    mask = rng.random(shape) < p
    gt = X.ravel(order="F")[mask.ravel(order="F")]          # gt = X(mask_missing)
    rmse, nrmse = tritd.evaluate(Xh, gt, mask)
    r_ref, n_ref = orc.evaluate(Xh.ravel(order="F")[mask.ravel(order="F")], gt)
    assert rmse == pytest.approx(r_ref, rel=1e-12) and nrmse == pytest.approx(n_ref, rel=1e-12)
    # evaluate(X_hat, X, true(size(X))) -- the driver's RRE
    rmse, nrmse = tritd.evaluate(Xh, X)
    r_ref, n_ref = orc.evaluate(Xh, X)
    assert rmse == pytest.approx(r_ref, rel=1e-12) and nrmse == pytest.approx(n_ref, rel=1e-12)


def test_evaluate_size_mismatch_and_empty(tritd):
    X = np.ones((4, 4, 4))
    mask = np.zeros(X.shape, dtype=bool)
    mask[0, 0, 0] = mask[1, 2, 3] = True
    with pytest.raises(tritd.TritdError, match="incompatible sizes"):
        tritd.evaluate(X, np.ones(3), mask)
    r, n = tritd.evaluate(X, np.array([2.0, 1.0]), mask)
    assert r == 1.0 and n == pytest.approx(1.0 / np.sqrt(5.0), rel=1e-15)


def test_evaluate_more_true_entries_than_gt(tritd):
    """nnz(mask) > numel(gt): MATLAB's size error; the kernels read gt only below m."""
    mask = np.zeros((33, 40, 9), dtype=bool)
    mask.ravel()[::7] = True
    with pytest.raises(tritd.TritdError, match="incompatible sizes"):
        tritd.evaluate(np.ones(mask.shape), np.ones(5), mask)


@pytest.mark.parametrize("n,offset", [(1 << 20, 1), (100003, 3), (4097, 0), (15, 1)])
def test_evaluate_device_mask_unaligned_and_ragged(tritd, orc, n, offset):
    """tritd_dev_evaluate_f64 on device buffers: a mask pointer off the 16-byte
    grid (byte-load path) and lengths that end inside a 16-position group or a
    wave chunk."""
    import ctypes as C
    from tritd import _lib
    hip = C.CDLL("libamdhip64.so")  # the runtime libtritd.so already loaded
    hip.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    hip.hipFree.argtypes = [C.c_void_p]
    rng = np.random.default_rng(n)
    X = rng.standard_normal(n)
    mk = np.zeros(n + 16, dtype=np.uint8)
    mk[offset:offset + n] = rng.random(n) < 0.3
    gt = rng.standard_normal(int(mk.sum()))
    bufs = []

    def dev(a):
        p = C.c_void_p()
        assert hip.hipMalloc(C.byref(p), C.c_size_t(max(a.nbytes, 1))) == 0
        bufs.append(p)
        assert hip.hipMemcpy(p, a.ctypes.data_as(C.c_void_p), C.c_size_t(a.nbytes), 1) == 0  # H2D
        return p.value

    try:
        Xd, gd, mb = dev(X), dev(gt), dev(mk)
        rm, nr = C.c_double(0), C.c_double(0)
        st = _lib.lib.tritd_dev_evaluate_f64(C.c_void_p(Xd), n, C.c_void_p(gd), gt.size,
                                              C.c_void_p(mb + offset), C.byref(rm), C.byref(nr), None)
        assert hip.hipDeviceSynchronize() == 0
    finally:
        for p in bufs:
            hip.hipFree(p)
    assert st == 0
    mk = mk[offset:offset + n].astype(bool)
    r_ref, n_ref = orc.evaluate(X[mk], gt)
    assert rm.value == pytest.approx(r_ref, rel=1e-12) and nr.value == pytest.approx(n_ref, rel=1e-12)


@pytest.mark.parametrize("shape", [(40, 50, 4), (240, 320, 6), (11, 11, 2), (64, 17, 3)])
def test_quality_matches_oracle(tritd, orc, shape):
    rng = np.random.default_rng(6)
    X = np.asfortranarray(rng.uniform(0, 255, shape))
    Y = np.asfortranarray(np.clip(X + rng.normal(0, 12, shape), 0, 255))
    p, s, pf, sf = tritd.quality_ybz(X, Y, per_frame=True)
    for f in range(shape[2]):
        assert pf[f] == pytest.approx(orc.psnr_index(X[:, :, f], Y[:, :, f]), rel=1e-12)
        assert sf[f] == pytest.approx(orc.ssim_index(X[:, :, f], Y[:, :, f]), rel=1e-11)
    pr, sr = orc.quality_ybz(X, Y)
    assert p == pytest.approx(pr, rel=1e-12) and s == pytest.approx(sr, rel=1e-11)


def test_quality_edge_cases(tritd):
    X = np.asfortranarray(np.random.default_rng(7).uniform(0, 255, (10, 30, 2)))
    p, s = tritd.quality_ybz(X, X + 1.0)
    assert p == pytest.approx(20 * np.log10(255.0), rel=1e-14) and s == -np.inf
    p, s = tritd.quality_ybz(np.ones((12, 12, 1)), np.ones((12, 12, 1)))
    assert p == np.inf and s == 1.0


def test_quality_more_frames_than_one_launch(tritd, orc):
    """quality_ybz.m folds every trailing dimension into frames with no limit;
    the kernels launch frames in batches of 65535 (grid y/z), so 65535 + 2500
    frames cross a batch boundary.  Frames on both sides are checked against
    the oracle, and the batch-seam frames against a single-batch call."""
    nf = 65535 + 2500
    rng = np.random.default_rng(8)
    X = np.asfortranarray(rng.uniform(0, 255, (12, 11, nf)))
    Y = np.asfortranarray(np.clip(X + rng.normal(0, 9, X.shape), 0, 255))
    p, s, pf, sf = tritd.quality_ybz(X, Y, per_frame=True)
    for f in (0, 1, 65533, 65534, 65535, 65536, nf - 1):
        assert pf[f] == pytest.approx(orc.psnr_index(X[:, :, f], Y[:, :, f]), rel=1e-12)
        assert sf[f] == pytest.approx(orc.ssim_index(X[:, :, f], Y[:, :, f]), rel=1e-11)
    lo, hi = 65535 - 100, 65535 + 100
    _, _, pf2, sf2 = tritd.quality_ybz(X[:, :, lo:hi], Y[:, :, lo:hi], per_frame=True)
    np.testing.assert_array_equal(pf[lo:hi], pf2)
    np.testing.assert_array_equal(sf[lo:hi], sf2)
    assert p == pytest.approx(np.mean(pf), rel=1e-12) and s == pytest.approx(np.mean(sf), rel=1e-12)


def test_unfold_more_matrices_than_one_launch(tritd, orc):
    """unfold(X, 2) transposes n3 matrices (one per grid z); n3 > 65535 runs
    in batches."""
    X = np.asfortranarray(np.random.default_rng(9).standard_normal((3, 5, 70000)))
    np.testing.assert_array_equal(tritd.unfold(X, 2), orc.unfold(X, 2))
