"""Debug: the unsynchronised device-form products one call at a time, with the
HIP error state cleared and reported before and after each call."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tritd  # noqa: E402
from tritd import synth  # noqa: E402
from tritd._lib import lib  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipGetLastError.restype = C.c_int
dev = torch.device("cuda", 0)
shapes = [(30, 31, 29, 3), (64, 40, 50, 8), (17, 16, 20, 8), (96, 80, 70, 16)] * 2
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
print("stale before:", hip.hipGetLastError(), flush=True)
for q, s in enumerate(shapes):
    A, B, Cc = synth.random_factors(*s, seed=11 + q)
    t = [torch.from_numpy(np.asarray(x).ravel(order="F").copy()).to(dev) for x in (A, B, Cc)]
    X = torch.empty(s[0] * s[1] * s[2], dtype=torch.float64, device=dev)
    st = (0, s1.cuda_stream, s2.cuda_stream)[q % 3]
    torch.cuda.synchronize(dev)
    e0 = hip.hipGetLastError()
    p = lambda x: C.c_void_p(x.data_ptr())  # noqa: E731
    rc = lib.tritd_dev_triple_product_f64(p(t[0]), p(t[1]), p(t[2]), *s, p(X), C.c_void_p(st))
    msg = lib.tritd_last_error().decode() if rc else ""
    torch.cuda.synchronize(dev)
    ref = tritd.triple_product(A, B, Cc)
    got = X.cpu().numpy().reshape(s[:3], order="F")
    err = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    print(q, s, "stream", st, "stale", e0, "rc", rc, msg, "rel", err, flush=True)
