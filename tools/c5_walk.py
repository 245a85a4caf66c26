"""Config-5 fused update vs walk length: k5_f32s<256> on fp32 r = 16 tensors of
the same size N = 2^30 with n3 = 256 / 512 / 1024 (16 / 32 / 64 t-tiles per
wave walk, 4x / 2x / 1x the waves).  If K5's time per element falls with the
walk length, per-wave fixed costs (Khatri-Rao operand gather, first loads, W
epilogue, workgroup turnover) are a real share of config 5's K5.

    python tools/c5_walk.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402
import tritd  # noqa: E402
from tritd import synth  # noqa: E402

r = 16
shapes = [(2048, 2048, 256), (2048, 1024, 512), (1024, 1024, 1024)]
for (n1, n2, n3) in shapes:
    rng = np.random.default_rng(0)
    D = np.asfortranarray(rng.standard_normal((n1, n2, n3), dtype=np.float32))
    A0, B0, C0 = synth.random_factors(n1, n2, n3, r, 123)
    opts = dict(synth.TRAFFIC_OPTS, maxIter=40, tol=0.0)
    s = tritd.Session(r, opts, A0, B0, C0, n1=n1, n2=n2, n3=n3, D=D, device=0, dtype=np.float32)
    del D
    s.run(5)
    s.sync()
    s.set_timing(True)
    s.run(10)
    s.sync()
    km = s.kernel_ms()
    N = n1 * n2 * n3
    print("%dx%dx%d (t-tiles per walk %d): K5 %.3f ms  K2 %.3f ms  iteration %.3f ms  | K5 f32-MFMA frac %.3f"
          % (n1, n2, n3, n3 // 16, km["fused_update"], km["mode3"], km["iteration"],
             4.0 * N * r * r / (km["fused_update"] * 1e-3) / 1e12 / 157.3), flush=True)
    s.close()
