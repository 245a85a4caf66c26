"""Driver-side data path (tritd/drivers.py; traffic_triple_comparison.m,
video_triple_comparison.m — SURVEY.md §8f rank 3).  CPU: mask draw, dataset
loading.  GPU: the TRIPLE branches end to end against the oracle composition."""
import os

import numpy as np
import pytest

from conftest import rel


def test_missing_mask_count_and_determinism():
    from tritd import drivers
    m1 = drivers.missing_mask((54, 4, 96), 0.15, np.random.default_rng(0))
    m2 = drivers.missing_mask((54, 4, 96), 0.15, np.random.default_rng(0))
    assert m1.sum() == round(0.15 * m1.size) and np.array_equal(m1, m2)
    assert drivers.missing_mask((3, 3, 3), 0.0, np.random.default_rng(0)).sum() == 0


def test_load_dataset_variables(tmp_path):
    from scipy.io import savemat
    from tritd import drivers
    T = np.arange(2 * 3 * 600, dtype=np.float32).reshape((2, 3, 600), order="F")
    savemat(tmp_path / "taxi.mat", {"T": T})
    X = drivers.load_dataset(str(tmp_path / "taxi.mat"))
    assert X.dtype == np.float64 and X.shape == (2, 3, 500)  # taxi: X(:,:,1:500)
    savemat(tmp_path / "highway.mat", {"gray_images": np.ones((12, 13, 4), dtype=np.uint8)})
    assert drivers.load_dataset(str(tmp_path / "highway.mat"), "video").shape == (12, 13, 4)
    with pytest.raises(KeyError, match="gray_images"):
        drivers.load_dataset(str(tmp_path / "taxi.mat"), "video")


@pytest.mark.gpu
def test_traffic_triple_branch(synth):
    import tritd_oracle as orc
    from tritd import drivers
    d = synth.sensor_like(n1=54, n2=4, n3=96, r=5)
    lines = []
    opts = dict(drivers.TRAFFIC_OPTS, disp=0, maxIter=30)
    res = drivers.traffic_triple(d["D"], 5, 0.1, opts=opts, A0=d["A0"], B0=d["B0"], C0=d["C0"],
                                 printer=lines.append, name="sensor")
    Y = np.where(res["mask"], 0.0, d["D"])
    A, B, C, O, eh, E, k, _ = orc.triple_decomp_ADMM(Y, 5, opts, d["A0"], d["B0"], d["C0"])
    Xh = orc.triple_product(A, B, C)
    assert rel(res["X_hat"], Xh) <= 1e-9
    _, nrmse = orc.evaluate(Xh, d["D"])
    assert res["nrmse"] == pytest.approx(nrmse, rel=1e-8)
    assert lines[-1].startswith("TRIPLE ADMM - RRE: ")


@pytest.mark.gpu
def test_video_triple_branch(synth, tmp_path):
    import tritd_oracle as orc
    from tritd import drivers
    d = synth.video_like(n1=24, n2=32, n3=20, r=5)
    lines = []
    opts = dict(drivers.VIDEO_OPTS, disp=0, maxIter=20)
    res = drivers.video_triple(d["D"], 5, 0.0, opts=opts, A0=d["A0"], B0=d["B0"], C0=d["C0"],
                               printer=lines.append, name="highway", save_dir=str(tmp_path))
    A, B, C, O, eh, E, k, _ = orc.triple_decomp_ADMM(d["D"], 5, opts, d["A0"], d["B0"], d["C0"])
    Xh = orc.triple_product(A, B, C)
    p, s = orc.quality_ybz(d["D"], Xh)
    assert res["psnr"] == pytest.approx(p, rel=1e-8) and res["ssim"] == pytest.approx(s, rel=1e-8)
    _, tn = orc.evaluate(Xh + O, d["D"])
    assert res["tnrmse"] == pytest.approx(tn, rel=1e-6)
    assert np.isnan(res["nrmse"])  # no missing entries: 0/0 like MATLAB
    assert os.path.exists(tmp_path / "highway_triple_re_O.mat")
    from scipy.io import loadmat  # video_triple_comparison.m:32 save(..._raw.mat, 'Y')
    np.testing.assert_array_equal(loadmat(tmp_path / "highway_raw.mat")["Y"], d["D"])
    assert "PSNR: " in lines[-1] and "SSIM: " in lines[-1]
