"""Dev helper: K5 / K2 time of a mode-1 shard of the config-4 problem as a
function of its row count (a shard of rows [0, i1), one-rank RCCL schedule).
usage: [ROWS_SKIP=10] python tools/rows_sweep.py i1 [i1 ...]"""
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
os.environ["TRITD_OVERLAP"] = "0"
os.environ["TRITD_SHOV"] = "1"
for i1 in [int(x) for x in sys.argv[1:]]:
    comm = tritd.Comm(tritd.Comm.unique_id(), 1, 0, 0)
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, i0=0, i1=i1,
                      D=np.asfortranarray(d["D"][:i1]), device=0, comm=comm)
    s.run(int(os.environ.get("ROWS_SKIP", "10"))); s.sync()
    d0, tpl = s.counters()
    s.set_timing(True); s.run(40); s.sync()
    d1, _ = s.counters()
    km = s.kernel_ms()
    print("rows=%d iteration %.4f ms  k5 %.4f (%.4f per 512 rows)  m3 %.4f  dense E tiles %.4f %%  probe %s" %
          (i1, km["iteration"], km["fused_update"], km["fused_update"] * 512 / i1, km["mode3"],
           100.0 * (d1 - d0) / 40 / tpl, s.probe()), flush=True)
    s.close()
    comm.close()
