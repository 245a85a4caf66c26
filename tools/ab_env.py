"""Dev helper: interleaved in-process A/B of an env knob read at session creation.
usage: python tools/ab_env.py VAR v1,v2[,..] reps [iters]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import synth
var, vals, reps = sys.argv[1], sys.argv[2].split(","), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 10
n, r = 512, 8
n1 = n2 = n3 = n
if os.environ.get("AB_CFG", "4") == "5":  # 2048x2048x256 r=16 fp32 (bench.py --config 5)
    n1, n2, n3, r = 2048, 2048, 256, 16
    dd = synth.low_rank_plus_outliers_f32(n1, n2, n3, r, p_out=0.05, seed=0, init_seed=123)
    D, A0, B0, C0 = dd["D"], dd["A0"], dd["B0"], dd["C0"]
    del dd
elif os.environ.get("AB_CFG", "4") == "3":  # 240x320x300 r=5 video stand-in (bench.py --config 3)
    n1, n2, n3, r = 240, 320, 300, 5
    dd = synth.video_like(n1, n2, n3, r, seed=0, init_seed=123)
    D, A0, B0, C0 = dd["D"], dd["A0"], dd["B0"], dd["C0"]
elif os.environ.get("AB_DATA", "bench") == "noise":  # E dense everywhere
    rng = np.random.default_rng(0)
    D = np.asfortranarray(rng.standard_normal((n, n, n)))
    A0, B0, C0 = synth.random_factors(n, n, n, r, 123)
else:  # the bench workload (low rank + 5 % outliers)
    dd = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
    D, A0, B0, C0 = dd["D"], dd["A0"], dd["B0"], dd["C0"]
opts = dict(synth.VIDEO_OPTS if os.environ.get("AB_CFG", "4") == "3" else synth.TRAFFIC_OPTS, maxIter=100)
res = {v: [] for v in vals}
for rep in range(reps):
    for v in vals:
        if v == "-":  # "-": the variable unset
            os.environ.pop(var, None)
        else:
            os.environ[var] = v
        s = tritd.Session(r, opts, A0, B0, C0, n1=n1, n2=n2, n3=n3, D=D, device=0, dtype=D.dtype)
        s.run(int(os.environ.get('AB_WARM', '15'))); s.sync(); s.set_timing(True); s.run(iters); s.sync()
        km = s.kernel_ms()
        res[v].append((km["iteration"], km["fused_update"], km["mode3"]))
        print("%s=%s rep %d: it %.3f k5 %.3f m3 %.3f" % (var, v, rep, km["iteration"], km["fused_update"], km["mode3"]), flush=True)
        s.close()
for v in vals:
    a = np.array(res[v])
    print("%s=%s median it %.3f k5 %.3f m3 %.3f | min it %.3f" % (var, v, *np.median(a, 0), a[:, 0].min()))
