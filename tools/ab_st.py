"""Interleaved A/B of soft_threshold's loads per thread (TRITD_ST_U=4 / 8) at
512^3 on random data, 10 rounds of 20 launches each."""
import ctypes as C
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import torch
from tritd._lib import check, lib
N = 512 ** 3
g = torch.Generator(device="cuda").manual_seed(0)
X = torch.randn(N, dtype=torch.float64, device="cuda", generator=g)
Y = torch.empty_like(X)
st = torch.cuda.current_stream()
sp = C.c_void_p(st.cuda_stream)
res = {"4": [], "8": []}
for rnd in range(10):
    for u in ("4", "8"):
        os.environ["TRITD_ST_U"] = u
        for _ in range(3):
            check(lib.tritd_dev_soft_threshold_f64(C.c_void_p(X.data_ptr()), N, C.c_double(0.5), C.c_void_p(Y.data_ptr()), sp))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            check(lib.tritd_dev_soft_threshold_f64(C.c_void_p(X.data_ptr()), N, C.c_double(0.5), C.c_void_p(Y.data_ptr()), sp))
        e1.record(st)
        torch.cuda.synchronize()
        res[u].append(e0.elapsed_time(e1) / 20)
for u, v in res.items():
    print("U=%s median %.4f ms = %.2f TB/s (min %.4f)" % (u, np.median(v), 2 * N * 8 / np.median(v) / 1e9, min(v)))
