"""Dev helper: per-iteration E/O error vs the C restatement on the mixed
dense/compact tile case of tests/test_gpu_configs.py."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
import tritd
from tritd import synth
import subprocess
subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
import tritd_ref
lib = tritd_ref.load()
rel = lambda a, b: np.linalg.norm((a - b).ravel()) / max(np.linalg.norm(b.ravel()), 1e-300)
n1, n2, n3, r = 48, 20, 64, 3
d = synth.low_rank_plus_outliers(n1, n2, n3, r, p_out=0.05, seed=11, init_seed=5)
D = d["D"].copy(order="F")
rng = np.random.default_rng(3)
D[:16, :7, :40] += 8.0 * rng.standard_normal((16, 7, 40))
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 1, int(sys.argv[2]) if len(sys.argv) > 2 else 16):
    opts = dict(synth.TRAFFIC_OPTS, maxIter=it)
    ref = tritd_ref.admm(lib, D, r, opts, d["A0"], d["B0"], d["C0"])
    A, B, C, O, eh, E, k = tritd.triple_decomp_ADMM(D, r, opts, d["A0"], d["B0"], d["C0"], return_E=True, return_iters=True)
    rE = ref[5]
    t = (rE != 0).reshape(n1 // 16, 16, n2, n3 // 16, 16).sum(axis=(1, 4))
    print("it %2d k %d/%d: O %.1e E %.1e  nan %d  ref nnz %.3f  tiles>28 %d" % (
        it, k, ref[6], rel(O, ref[3]), rel(E, rE), np.isnan(E).sum(), (rE != 0).mean(), (t > 28).sum()), flush=True)
