"""Where a one-shot config-4 solve spends its time: host-D session creation,
100 iterations, get (O only / O and E), and the host<->device copy rates
(pageable numpy vs pinned torch buffers) of a 1 GB tensor."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import tritd  # noqa: E402
from tritd import synth  # noqa: E402

n, r = 512, 8
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
D = d["D"]
opts = dict(synth.TRAFFIC_OPTS, maxIter=100)


def t(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, out


for rep in range(2):
    ms_c, s = t(lambda: tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, D=D,
                                       device=0, probe=False))
    ms_r, _ = t(lambda: (s.run(100), s.sync()))
    ms_g, res = t(lambda: s.get())
    s.close()
    ms_1, _ = t(lambda: tritd.triple_decomp_ADMM(D, r, opts, d["A0"], d["B0"], d["C0"], device=0))
    ms_2, _ = t(lambda: tritd.triple_decomp_ADMM(D, r, opts, d["A0"], d["B0"], d["C0"], device=0,
                                                 return_E=True))
    print("rep %d: create %.1f ms, 100 its %.1f ms, get(O,E) %.1f ms | one-shot O only %.1f ms, "
          "O and E %.1f ms" % (rep, ms_c, ms_r, ms_g, ms_1, ms_2), flush=True)
N = D.size
g = torch.empty(N, dtype=torch.float64, device="cuda")
h_page = np.empty(N)
h_pin = torch.empty(N, dtype=torch.float64, pin_memory=True)
for rep in range(2):
    ms, _ = t(lambda: g.copy_(torch.from_numpy(D.reshape(-1, order="F"))))
    print("H2D pageable %.1f ms = %.1f GB/s" % (ms, N * 8 / ms / 1e6))
    ms, _ = t(lambda: g.copy_(h_pin))
    print("H2D pinned   %.1f ms = %.1f GB/s" % (ms, N * 8 / ms / 1e6))
    ms, _ = t(lambda: torch.from_numpy(h_page).copy_(g))
    print("D2H pageable %.1f ms = %.1f GB/s" % (ms, N * 8 / ms / 1e6))
    ms, _ = t(lambda: h_pin.copy_(g))
    print("D2H pinned   %.1f ms = %.1f GB/s" % (ms, N * 8 / ms / 1e6))
    x = np.empty(N)
    ms, _ = t(lambda: np.copyto(x, h_pin.numpy()))
    print("host memcpy 1 thread %.1f ms = %.1f GB/s" % (ms, N * 8 / ms / 1e6), flush=True)
# host page population on this box (Python threads + libc madvise): the cost the
# library's populate_output pays before a 1 GB device-to-host copy
import ctypes
import threading
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.madvise.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
for huge in (False, True):
    for nt in (1, 16):
        a = np.zeros(N)
        p = a.ctypes.data
        s0 = (p + 4095) & ~4095
        e = (p + a.nbytes) & ~4095
        t0 = time.perf_counter()
        if huge:
            h0 = (p + (2 << 20) - 1) & ~((2 << 20) - 1)
            libc.madvise(h0, (e - h0) & ~((2 << 20) - 1), 14)
        ch = ((e - s0) // nt + (2 << 20) - 1) & ~((2 << 20) - 1)
        ths = [threading.Thread(target=lambda s=s: libc.madvise(s, min(ch, e - s), 23)) for s in range(s0, e, ch)]
        [t_.start() for t_ in ths]
        [t_.join() for t_ in ths]
        print("populate 1 GB: huge %s, %d threads: %.1f ms" % (huge, nt, (time.perf_counter() - t0) * 1e3))
