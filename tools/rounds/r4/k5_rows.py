"""Dev helper: K5 time and placement-probe results vs the shard's row count
(config-4 problem, session over rows [0, rows)).
usage: python tools/rounds/r4/k5_rows.py rows[@i0][:ENV=V,ENV=V] ...  (env knobs set for that session only)"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import synth

n, r = 512, 8
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=200, tol=0.0)
for spec in sys.argv[1:]:
    rows, _, envs = spec.partition(":")
    rows, _, i0 = rows.partition("@")
    rows, i0 = int(rows), int(i0 or 0)
    kv = dict(e.split("=") for e in envs.split(",") if e)
    saved = {k: os.environ.get(k) for k in kv}
    os.environ.update(kv)
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, i0=i0, i1=i0 + rows,
                      D=np.asfortranarray(d["D"][i0:i0 + rows]), device=0)
    s.run(10); s.sync()
    s.set_timing(True); s.run(30); s.sync()
    km = s.kernel_ms()
    dense, per = s.counters()
    print("rows=%d@%d %s iteration %.4f ms  k5 %.4f  m3 %.4f  dense E tiles %d (of %d per launch, 40 launches)  probe %s" %
          (rows, i0, envs, km["iteration"], km["fused_update"], km["mode3"], dense, per,
           [round(x, 3) for x in s.probe()[0]]), flush=True)
    s.close()
    for k, v in saved.items():
        if v is None:
            os.environ.pop(k)
        else:
            os.environ[k] = v
