"""Driver-side data path of the reference experiments.

The TRIPLE branches of the two driver scripts, on the GPU path:

    traffic_triple(X, ...)   traffic_triple_comparison.m:20-64   (completion, RRE)
    video_triple(X, ...)     video_triple_comparison.m:19-76     (background
                             separation: RMSE/NRMSE on the missing and observed
                             entries, total RRE, PSNR/SSIM of the low-rank part)
    load_dataset(path)       the `load(name + ".mat")` of both scripts (:20 / :20)

The solver, `triple_product`, `evaluate` and `quality_ybz` all run through
libtritd.so; only the mask draw, the `Y(mask) = 0` copy and the `X_hat + O`
sum are host numpy (the reference does them in MATLAB on the host too).
MATLAB's `randperm` stream cannot be reproduced, so the missing-entry mask
comes from a seeded numpy generator (same count, `round(ratio * numel)`).
"""
from __future__ import annotations

import os
import time

import numpy as np

from . import api

# traffic_triple_comparison.m:42-50 / video_triple_comparison.m:41-49
TRAFFIC_OPTS = dict(maxIter=100, tol=1e-5, mu=1e-3, **{"lambda": 1.8}, lambda2=1e-3, rho=1.25,
                    alphaA=1e-3, alphaB=1e-3, disp=1)
VIDEO_OPTS = dict(maxIter=100, tol=1e-5, mu=1e-2, **{"lambda": 1.8}, lambda2=1e-2, rho=1.2,
                  alphaA=1e-3, alphaB=1e-3, disp=1)


def load_dataset(path, kind="traffic"):
    """`load(name + ".mat")`: the traffic script reads variable T
    (traffic_triple_comparison.m:20-22, `X = double(T)`, taxi cut to 500
    slices at :23-25), the video script `gray_images` (video_triple_comparison.m:20-21).
    MAT v5/v7 files through scipy.io; a v7.3 (HDF5) file is refused with a
    message (h5py is not available here)."""
    from scipy.io import loadmat
    try:
        m = loadmat(path)
    except NotImplementedError as e:  # v7.3
        raise ValueError(f"{path}: MAT v7.3 (HDF5) files need h5py, which is not installed") from e
    var = "T" if kind == "traffic" else "gray_images"
    if var not in m:
        raise KeyError(f"{path}: variable '{var}' not found (have {sorted(k for k in m if not k.startswith('__'))})")
    X = np.asfortranarray(np.asarray(m[var], dtype=np.float64))
    if kind == "traffic" and os.path.basename(path).startswith("taxi"):
        X = np.asfortranarray(X[:, :, :500])
    return X


def missing_mask(shape, ratio, rng):
    """Step 1 of both scripts: `num_to_zero = round(ratio*numel)` distinct
    positions drawn uniformly (randperm), returned as a logical array."""
    total = int(np.prod(shape))
    num = int(np.floor(ratio * total + 0.5))  # MATLAB round (half away from zero, ratio >= 0)
    idx = rng.permutation(total)[:num]
    mask = np.zeros(total, dtype=bool)
    mask[idx] = True
    return mask.reshape(shape, order="F")


def _observe(X, mask):
    Y = np.array(X, dtype=np.float64, order="F", copy=True)
    Y[mask] = 0.0
    return Y


def traffic_triple(X, r=5, missing_ratio=0.15, *, opts=None, seed=0, A0=None, B0=None, C0=None,
                   printer=print, name="data"):
    """TRIPLE branch of traffic_triple_comparison.m (:26-64): mask, zero the
    missing entries, solve, `X_hat = triple_product(A,B,C)`, RRE over all
    entries with `evaluate(X_hat, X, true(size(X)))`, print as at :64."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    rng = np.random.default_rng(seed)
    mask = missing_mask(X.shape, missing_ratio, rng)
    printer("\n===== Dataset: %s Missing Radio %.3f=====" % (name, missing_ratio))
    Y = _observe(X, mask)
    o = dict(TRAFFIC_OPTS if opts is None else opts)
    t0 = time.perf_counter()
    A, B, C, O, errHist = api.triple_decomp_ADMM(Y, r, o, A0, B0, C0)
    timer = time.perf_counter() - t0
    X_hat = api.triple_product(A, B, C)
    rmse, nrmse = api.evaluate(X_hat, X)
    printer("TRIPLE ADMM - RRE: %.2f, Time: %.2f s" % (nrmse, timer))
    return dict(A=A, B=B, C=C, O=O, errHist=errHist, X_hat=X_hat, mask=mask, rmse=rmse,
                nrmse=nrmse, time=timer)


def video_triple(X, r=5, missing_ratio=0.0, *, opts=None, seed=0, A0=None, B0=None, C0=None,
                 printer=print, name="data", save_dir=None):
    """TRIPLE branch of video_triple_comparison.m (:26-76) through the
    `triple_decomp_ADMM_outlier` name the script calls (:54): RMSE/NRMSE of
    X_hat on the missing entries, of O on the observed ones, of X_hat + O on
    all of them, and PSNR/SSIM of X_hat against X (quality_ybz), printed as at
    :74-75.  With `save_dir` the observed tensor is saved as `<name>_raw.mat`
    (variable Y, :32, every ratio) and, when missing_ratio == plot_rate == 0
    (:58), the errHist / X_hat / O .mat files of :59-61."""
    X = np.asfortranarray(np.asarray(X, dtype=np.float64))
    rng = np.random.default_rng(seed)
    mask = missing_mask(X.shape, missing_ratio, rng)
    printer("\n===== Dataset: %s Missing Radio %.3f=====" % (name, missing_ratio))
    Y = _observe(X, mask)
    if save_dir is not None:  # save(sprintf("%s_raw.mat", name), 'Y')  (:32)
        from scipy.io import savemat
        savemat(os.path.join(save_dir, "%s_raw.mat" % name), {"Y": Y})
    gt = X.ravel(order="F")[mask.ravel(order="F")]       # X(mask_missing), column-major (:36)
    gt_2 = X.ravel(order="F")[~mask.ravel(order="F")]    # X(~mask_missing)              (:37)
    o = dict(VIDEO_OPTS if opts is None else opts)
    t0 = time.perf_counter()
    A, B, C, O, errHist = api.triple_decomp_ADMM_outlier(Y, r, o, A0, B0, C0)
    timer = time.perf_counter() - t0
    X_hat = api.triple_product(A, B, C)
    if save_dir is not None and missing_ratio == 0:
        from scipy.io import savemat
        savemat(os.path.join(save_dir, "%s_triple_re_errHist.mat" % name), {"errHist": errHist})
        savemat(os.path.join(save_dir, "%s_triple_re_Xhat.mat" % name), {"X_hat_re": X_hat})
        savemat(os.path.join(save_dir, "%s_triple_re_O.mat" % name), {"O": O})
    # with no missing entries gt is empty: norm([]) = 0 and nrmse = 0/0 = NaN, as in MATLAB
    rmse, nrmse = api.evaluate(X_hat, gt, mask)
    rmse2, nrmse2 = api.evaluate(O, gt_2, ~mask)
    rmse3, nrmse3 = api.evaluate(np.asfortranarray(X_hat + O), X)
    psnr, ssim = api.quality_ybz(X, X_hat)
    printer("TRIPLE ADMM - RMSE: %.4e, NRMSE: %.4e, SRMSE: %.4e, SNRMSE: %.4e, TRMSE: %.4e, "
            "TNRMSE: %.4e, PSNR: %.4e, SSIM: %.4e, Time: %.2f s"
            % (rmse, nrmse, rmse2, nrmse2, rmse3, nrmse3, psnr, ssim, timer))
    return dict(A=A, B=B, C=C, O=O, errHist=errHist, X_hat=X_hat, mask=mask, rmse=rmse,
                nrmse=nrmse, srmse=rmse2, snrmse=nrmse2, trmse=rmse3, tnrmse=nrmse3, psnr=psnr,
                ssim=ssim, time=timer)
