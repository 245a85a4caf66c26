"""Phase timings of a config-5 (2048x2048x256 fp32 r=16) solve from a host D:
session creation (probe, upload, TM conversion), run, get.  Prints a line per
phase and a heartbeat every 20 s (a long phase must not look hung)."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))
import numpy as np  # noqa: E402

t00 = time.time()


def say(m):
    print("[%7.1f s] %s" % (time.time() - t00, m), flush=True)


def beat():
    while True:
        time.sleep(20)
        say("...")


threading.Thread(target=beat, daemon=True).start()
import tritd  # noqa: E402
from tritd import synth  # noqa: E402

n1, n2, n3, r = 2048, 2048, 256, 16
iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
d = synth.low_rank_plus_outliers(n1, n2, n3, r, p_out=0.05, seed=0, init_seed=123)
D = d["D"].astype(np.float32, order="F")
del d["D"], d["Lstar"]
say("data ready")
opts = dict(synth.TRAFFIC_OPTS, maxIter=iters)
for probe in ("1", None):
    if probe:
        os.environ["TRITD_PROBE"] = probe
    else:
        os.environ.pop("TRITD_PROBE", None)
    t0 = time.time()
    s = tritd.Session(r, opts, d["A0"], d["B0"], d["C0"], n1=n1, n2=n2, n3=n3, D=D, device=0)
    say("probe=%s session created %.2f s (probe ms %s)" % (probe, time.time() - t0, s.probe()[0][:4]))
    t0 = time.time()
    s.run(iters)
    k, st = s.sync()
    say("run %d its %.2f s" % (k, time.time() - t0))
    t0 = time.time()
    out = s.get()
    say("get %.2f s flags %d errHist %s" % (time.time() - t0, s.flags(), out["errHist"]))
    s.close()
    del out
for probe in ("1", None, None):
    if probe:
        os.environ["TRITD_PROBE"] = probe
    else:
        os.environ.pop("TRITD_PROBE", None)
    t0 = time.time()
    res = tritd.triple_decomp_ADMM(D, r, opts, d["A0"], d["B0"], d["C0"], return_iters=True)
    say("one-shot probe=%s %.2f s k=%d" % (probe, time.time() - t0, res[-1]))
    del res
O = np.zeros((n1, n2, n3), order="F", dtype=np.float32)
t0 = time.time()
O[:] = 1.0
say("first touch of a 4.3 GB array %.2f s" % (time.time() - t0))
