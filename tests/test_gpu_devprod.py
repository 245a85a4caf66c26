"""Device-form triple products (tritd_dev_triple_product_f64 / _qi_f64): they
return without synchronising (include/tritd.h) and reuse per-stream scratch
(csrc/api.cpp scratch_set).  Back-to-back calls with different factors on one
stream, on two streams, on the null stream, and on a destroyed-and-recreated
stream must each give the host form's result (triple_product.m:6, checked
against the oracle in test_gpu_parity.py); so must a call that grows the
scratch while an earlier, smaller call may still be running."""
import ctypes as C

import numpy as np
import pytest

from conftest import rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def env():
    import torch
    import tritd
    from tritd._lib import check, lib
    assert tritd.device_count() > 0, "no GPU visible: the HIP path must run"
    return torch, tritd, check, lib


def _case(torch, n1, n2, n3, r, seed):
    from tritd import synth
    A, B, Cc = synth.random_factors(n1, n2, n3, r, seed=seed)
    dev = torch.device("cuda", 0)
    t = [torch.from_numpy(np.asarray(x).ravel(order="F").copy()).to(dev) for x in (A, B, Cc)]
    return (A, B, Cc), t


def _launch(lib, check, fn, t, dims, X, stream):
    p = lambda x: C.c_void_p(x.data_ptr())  # noqa: E731
    check(fn(p(t[0]), p(t[1]), p(t[2]), *dims, p(X), C.c_void_p(stream)))


@pytest.mark.parametrize("model", ["cp", "qi"])
def test_dev_products_unsynchronised(env, model):
    torch, tritd, check, lib = env
    fn = lib.tritd_dev_triple_product_qi_f64 if model == "qi" else lib.tritd_dev_triple_product_f64
    dev = torch.device("cuda", 0)
    # small then larger shapes (the second grows every scratch buffer), 8 cases
    shapes = [(30, 31, 29, 3), (64, 40, 50, 8), (17, 16, 20, 8), (96, 80, 70, 16)] * 2
    cases = [_case(torch, *s, seed=11 + q) for q, s in enumerate(shapes)]
    ref = [tritd.triple_product(*h, model=model) for h, _ in cases]
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    outs = []
    for q, ((h, t), s) in enumerate(zip(cases, shapes)):
        X = torch.empty(s[0] * s[1] * s[2], dtype=torch.float64, device=dev)
        st = (0, s1.cuda_stream, s2.cuda_stream)[q % 3]
        torch.cuda.synchronize(dev)  # the operands were made on the current stream
        _launch(lib, check, fn, t, s[:4], X, st)  # no synchronisation between calls
        outs.append(X)
    torch.cuda.synchronize(dev)
    for X, s, R in zip(outs, shapes, ref):
        got = X.cpu().numpy().reshape(s[:3], order="F")
        assert rel(got, R) <= 1e-13


def test_dev_product_recreated_stream(env):
    torch, tritd, check, lib = env
    dev = torch.device("cuda", 0)
    shapes = [(128, 96, 200, 8), (40, 30, 20, 4), (128, 96, 200, 8)]
    outs = []
    for q, s in enumerate(shapes):
        h, t = _case(torch, *s, seed=40 + q)
        torch.cuda.synchronize(dev)
        st = torch.cuda.Stream(dev)  # a stream per call (torch's pool repeats handles)
        X = torch.empty(s[0] * s[1] * s[2], dtype=torch.float64, device=dev)
        _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X, st.cuda_stream)
        outs.append((X, s, tritd.triple_product(*h), t))
    torch.cuda.synchronize(dev)
    for X, s, R, _ in outs:
        assert rel(X.cpu().numpy().reshape(s[:3], order="F"), R) <= 1e-13


def test_dev_product_after_shutdown(env):
    """tritd_shutdown frees the per-stream scratch (after the last product on
    it finishes); the next device-form call recreates it."""
    torch, tritd, check, lib = env
    dev = torch.device("cuda", 0)
    s = (64, 40, 50, 8)
    h, t = _case(torch, *s, seed=77)
    torch.cuda.synchronize(dev)
    X1 = torch.empty(s[0] * s[1] * s[2], dtype=torch.float64, device=dev)
    X2 = torch.empty_like(X1)
    _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X1, 0)
    lib.tritd_shutdown()  # no synchronisation before it
    _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X2, 0)
    torch.cuda.synchronize(dev)
    R = tritd.triple_product(*h)
    for X in (X1, X2):
        assert rel(X.cpu().numpy().reshape(s[:3], order="F"), R) <= 1e-13
