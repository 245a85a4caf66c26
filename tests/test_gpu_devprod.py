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
    import tritd
    from tritd import hip
    from tritd._lib import check, lib
    assert tritd.device_count() > 0, "no GPU visible: the HIP path must run"
    return hip, tritd, check, lib


def _case(hip, n1, n2, n3, r, seed):
    from tritd import synth
    A, B, Cc = synth.random_factors(n1, n2, n3, r, seed=seed)
    t = [hip.DeviceArray.from_host(np.asarray(x).ravel(order="F").copy()) for x in (A, B, Cc)]
    return (A, B, Cc), t


def _launch(lib, check, fn, t, dims, X, stream):
    p = lambda x: C.c_void_p(x.ptr)  # noqa: E731
    check(fn(p(t[0]), p(t[1]), p(t[2]), *dims, p(X), C.c_void_p(stream)))


def _host(X, s):
    out = np.empty(s[0] * s[1] * s[2])
    return X.to_host(out).reshape(s[:3], order="F")


@pytest.mark.parametrize("model", ["cp", "qi"])
def test_dev_products_unsynchronised(env, model):
    hip, tritd, check, lib = env
    fn = lib.tritd_dev_triple_product_qi_f64 if model == "qi" else lib.tritd_dev_triple_product_f64
    # small then larger shapes (the second grows every scratch buffer), 8 cases
    shapes = [(30, 31, 29, 3), (64, 40, 50, 8), (17, 16, 20, 8), (96, 80, 70, 16)] * 2
    cases = [_case(hip, *s, seed=11 + q) for q, s in enumerate(shapes)]
    ref = [tritd.triple_product(*h, model=model) for h, _ in cases]
    s1, s2 = hip.Stream(), hip.Stream()
    outs = []
    hip.synchronize()  # the operands' uploads
    for q, ((h, t), s) in enumerate(zip(cases, shapes)):
        X = hip.DeviceArray(s[0] * s[1] * s[2] * 8)
        st = (0, s1.handle, s2.handle)[q % 3]
        _launch(lib, check, fn, t, s[:4], X, st)  # no synchronisation between calls
        outs.append(X)
    hip.synchronize()
    for X, s, R in zip(outs, shapes, ref):
        assert rel(_host(X, s), R) <= 1e-13


def test_dev_product_recreated_stream(env):
    hip, tritd, check, lib = env
    shapes = [(128, 96, 200, 8), (40, 30, 20, 4), (128, 96, 200, 8)]
    outs = []
    for q, s in enumerate(shapes):
        h, t = _case(hip, *s, seed=40 + q)
        hip.synchronize()
        st = hip.Stream()  # a stream per call, destroyed after it (handles get reused)
        X = hip.DeviceArray(s[0] * s[1] * s[2] * 8)
        _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X, st.handle)
        st.close()
        outs.append((X, s, tritd.triple_product(*h), t))
    hip.synchronize()
    for X, s, R, _ in outs:
        assert rel(_host(X, s), R) <= 1e-13


def test_dev_product_after_shutdown(env):
    """tritd_shutdown frees the per-stream scratch (after the last product on
    it finishes); the next device-form call recreates it."""
    hip, tritd, check, lib = env
    s = (64, 40, 50, 8)
    h, t = _case(hip, *s, seed=77)
    hip.synchronize()
    X1 = hip.DeviceArray(s[0] * s[1] * s[2] * 8)
    X2 = hip.DeviceArray(X1.nbytes)
    _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X1, 0)
    lib.tritd_shutdown()  # no synchronisation before it
    _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X2, 0)
    hip.synchronize()
    R = tritd.triple_product(*h)
    for X in (X1, X2):
        assert rel(_host(X, s), R) <= 1e-13


_TORCH_CHILD = """
import sys, ctypes as C
sys.path.insert(0, %(pkg)r)
import numpy as np
import torch                      # first: tritd then binds torch's HIP runtime
import tritd
from tritd import synth
from tritd._lib import check, lib, hip_runtimes
assert len(hip_runtimes()) == 1, hip_runtimes()
dev = torch.device("cuda", 0)
A, B, Cc = synth.random_factors(64, 40, 50, 8, seed=5)
t = [torch.from_numpy(np.asarray(x).ravel(order="F").copy()).to(dev) for x in (A, B, Cc)]
X = torch.empty(64 * 40 * 50, dtype=torch.float64, device=dev)
st = torch.cuda.Stream(dev)
torch.cuda.synchronize(dev)
p = lambda x: C.c_void_p(x.data_ptr())
check(lib.tritd_dev_triple_product_f64(p(t[0]), p(t[1]), p(t[2]), 64, 40, 50, 8, p(X),
                                       C.c_void_p(st.cuda_stream)))
torch.cuda.synchronize(dev)
R = tritd.triple_product(A, B, Cc)
got = X.cpu().numpy().reshape(64, 40, 50, order="F")
err = np.linalg.norm(got - R) / np.linalg.norm(R)
assert err <= 1e-13, err
print("torch interop ok", hip_runtimes()[0])
"""


def test_dev_product_on_torch_memory_and_stream():
    """A torch host (torch imported first): tritd binds torch's HIP runtime,
    and a device-form product on torch tensors and a torch stream gives the
    host form's result.  In a child process: this suite's own process stays
    on /opt/rocm's runtime (tests/test_zz_runtime.py)."""
    import subprocess
    import sys
    from conftest import PKG
    r = subprocess.run([sys.executable, "-c", _TORCH_CHILD % {"pkg": PKG}], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "torch interop ok" in r.stdout and "torch" in r.stdout


def test_dev_products_on_more_streams_than_the_scratch_cap(env):
    """The per-(device, stream) scratch cache is bounded (api.cpp SCRATCH_CAP
    = 16): products on 24 streams, round-robin twice, evict and
    recreate entries while earlier products may still run, and each result is
    still the host form's."""
    hip, tritd, check, lib = env
    s = (48, 40, 36, 8)
    cases = [_case(hip, *s, seed=200 + q) for q in range(4)]
    refs = [tritd.triple_product(*h) for h, _ in cases]
    streams = [hip.Stream() for _ in range(24)]
    hip.synchronize()
    outs = []
    for rep in range(2):
        for q, st in enumerate(streams):
            h, t = cases[q % 4]
            X = hip.DeviceArray(s[0] * s[1] * s[2] * 8)
            _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X, st.handle)
            outs.append((X, q % 4))
    hip.synchronize()
    for X, c in outs:
        assert rel(_host(X, s), refs[c]) <= 1e-13
    for st in streams:
        st.close()


def test_products_after_destroyed_streams_leave_no_error(env):
    """Round 5's intermittent failure (profiles/round5/gpu_tests_null_stream_
    wait_failure.log.txt), its condition made deliberate: scratch entries whose
    `done` events were last recorded on streams that have since been destroyed
    fill the cache; then host-form products on the null stream (new entry:
    eviction; growing sizes: scratch regrow), device-form products on new
    streams (more evictions) and a tritd_shutdown.  On ROCm 7.2 a host wait on
    such an event (hipEventSynchronize) reads the freed stream object and, when
    that memory happens to read "capture active", returns
    hipErrorCapturedEvent — which an unchecked call left behind for the next
    launch check.  The library now never waits on those events from the host
    (api.cpp ScratchSet); every call must succeed and leave the thread's HIP
    error state clear."""
    import tritd_oracle as orc
    from tritd import synth
    hip, tritd, check, lib = env
    rt = hip.rt
    rt.hipPeekAtLastError.restype = C.c_int
    s = (40, 32, 30, 8)
    h, t = _case(hip, *s, seed=300)
    hip.synchronize()
    for rep in range(3):
        streams = [hip.Stream() for _ in range(20)]
        for st in streams:
            X = hip.DeviceArray(s[0] * s[1] * s[2] * 8)
            _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X, st.handle)
            X.free()
        for st in streams:  # destroyed with their entries still cached
            st.close()
        # churn the host heap where the stream objects were
        junk = [hip.Stream() for _ in range(8)]
        for st in junk:
            st.close()
        for q, n in enumerate((24, 48, 72)):  # null stream: new entry, then regrowth
            A, B, Cc = synth.random_factors(n, n - 4, n - 8, 8, seed=310 + q)
            L = tritd.triple_product(A, B, Cc)
            assert rt.hipPeekAtLastError() == 0
            assert rel(L, orc.triple_product(A, B, Cc)) <= 1e-13
        st2 = hip.Stream()
        X = hip.DeviceArray(s[0] * s[1] * s[2] * 8)
        _launch(lib, check, lib.tritd_dev_triple_product_f64, t, s, X, st2.handle)
        st2.synchronize()
        assert rel(_host(X, s), tritd.triple_product(*h)) <= 1e-13
        X.free()
        st2.close()
        assert rt.hipPeekAtLastError() == 0
        lib.tritd_shutdown()
        assert rt.hipPeekAtLastError() == 0
