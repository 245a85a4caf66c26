"""Roofline of the API-level kernels outside the ADMM loop (one MI355X):
unfold (K0, unfold.m), soft_threshold (K6, soft_threshold.m), triple_product
(k_tp, triple_product.m), evaluate (traffic_triple_comparison.m:194-202) and
quality_ybz (PSNR/SSIM) on device-resident inputs, timed with HIP events on
the stream the kernels are launched on.  Prints one JSON object.

    python tools/bench_prims.py [--n 512] [--reps 20]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM = 8000.0   # GB/s, MI355X_MICROARCH.md
F64_MFMA = 78.6  # TF/s dense f64 matrix


def timed(fn, reps, stream, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=512)
    ap.add_argument("--r", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import tritd
    from tritd._lib import check, lib
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)
    n, r = a.n, a.r
    N = n ** 3
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(N, dtype=torch.float64, device=dev, generator=g)
    Y = torch.empty_like(X)
    out = {"n": n, "r": r, "kernels": {}}

    def rec(name, ms, bytes_=None, flops=None):
        d = {"ms": ms}
        if bytes_ is not None:
            d["GBs"] = bytes_ / ms / 1e6
            d["hbm_frac"] = d["GBs"] / HBM
        if flops is not None:
            d["TFs"] = flops / ms / 1e9
            d["mfma_frac"] = d["TFs"] / F64_MFMA
        out["kernels"][name] = d

    p = lambda t: C.c_void_p(t.data_ptr())
    for mode in (2, 3, 2):  # mode 2 again: the first timed kernel of the process ran slow
        ms = timed(lambda: check(lib.tritd_dev_unfold_f64(p(X), n, n, n, mode, p(Y), sp)), a.reps, st)
        rec("unfold_mode%d" % mode, ms, 2 * N * 8)
    ms = timed(lambda: check(lib.tritd_dev_soft_threshold_f64(p(X), N, C.c_double(0.5), p(Y), sp)),
               a.reps, st)
    rec("soft_threshold", ms, 2 * N * 8)

    R = r * r
    A = torch.randn(n * R, dtype=torch.float64, device=dev, generator=g)
    B = torch.randn(R * n, dtype=torch.float64, device=dev, generator=g)
    Cc = torch.randn(R * n, dtype=torch.float64, device=dev, generator=g)
    ms = timed(lambda: check(lib.tritd_dev_triple_product_f64(p(A), p(B), p(Cc), n, n, n, r, p(Y),
                                                             sp)), a.reps, st)
    rec("triple_product", ms, N * 8, 2.0 * N * R)

    rm, nr = C.c_double(0), C.c_double(0)
    ms = timed(lambda: check(lib.tritd_dev_evaluate_f64(p(X), N, p(Y), N, None, C.byref(rm),
                                                       C.byref(nr), sp)), a.reps, st)
    rec("evaluate_full", ms, 2 * N * 8)
    mask = (torch.rand(N, device=dev, generator=g) < 0.1).to(torch.uint8)
    m = int(mask.sum().item())
    gt = torch.randn(m, dtype=torch.float64, device=dev, generator=g)
    ms = timed(lambda: check(lib.tritd_dev_evaluate_f64(p(X), N, p(gt), m, p(mask), C.byref(rm),
                                                       C.byref(nr), sp)), a.reps, st)
    # mask read twice (count + pairing), X at the true positions (counted as
    # all of X: at 10 % density most 64 B sectors hold one), gt once
    rec("evaluate_masked10", ms, 2 * N + N * 8 + m * 8)

    n1, n2, nf = 240, 320, 300  # the Highway video shape (config 3)
    V1 = torch.rand(n1 * n2 * nf, dtype=torch.float64, device=dev, generator=g) * 255
    V2 = torch.rand(n1 * n2 * nf, dtype=torch.float64, device=dev, generator=g) * 255
    ps, ss = C.c_double(0), C.c_double(0)
    ms = timed(lambda: check(lib.tritd_dev_quality_f64(p(V1), p(V2), n1, n2, nf, C.byref(ps),
                                                      C.byref(ss), None, None, sp)), a.reps, st)
    rec("quality_ybz_240x320x300", ms, 2 * 2 * n1 * n2 * nf * 8)  # sqdiff pass + SSIM pass
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
