"""Dev helper: placement-probe times of hipMalloc vs hipDeviceMallocContiguous
tensor pools (TRITD_CONTIG), alternating in one process at 512^3 r=8."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import tritd
from tritd import synth
n, r = 512, 8
d = synth.low_rank_plus_outliers(n, n, n, r, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=200, tol=0.0)
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for cg in ("0", "1"):
        os.environ["TRITD_CONTIG"] = cg
        try:
            s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n, n2=n, n3=n, D=d["D"], device=0)
        except Exception as e:
            print("contig=%s rep %d: %s" % (cg, rep, e), flush=True)
            continue
        s.run(5); s.sync(); s.set_timing(True); s.run(20); s.sync()
        ms, pick = s.probe()
        print("contig=%s rep %d: probe %s pick %d  k5 %.4f it %.4f" % (cg, rep, [round(x, 3) for x in ms], pick,
              s.kernel_ms()["fused_update"], s.kernel_ms()["iteration"]), flush=True)
        s.close()
