"""One-shot triple_decomp_ADMM host to host (config 4, 100 iterations, with
and without E) for two libtritd builds, interleaved in child processes.
python tools/rounds/r5/e2e_ab.py libA.so libB.so [reps]"""
import os
import subprocess
import sys

CHILD = r'''
import os, sys, time
sys.path.insert(0, os.path.join(os.environ["ROOT"], "triple-tensor-decomposition-with-admm_amd"))
import numpy as np
import tritd
from tritd import synth
d = synth.low_rank_plus_outliers(512, 512, 512, 8, p_out=0.05, seed=0, init_seed=123)
opts = dict(synth.TRAFFIC_OPTS, maxIter=100)
out = []
for e in (False, True, False, True):
    t = time.perf_counter()
    tritd.triple_decomp_ADMM(d["D"], 8, opts, d["A0"], d["B0"], d["C0"], return_E=e)
    out.append("%s:%.1f" % ("E" if e else "-", (time.perf_counter() - t) * 1e3))
print(" ".join(out))
'''
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
libs = sys.argv[1:3]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
for rep in range(reps):
    for l in libs:
        env = dict(os.environ, ROOT=ROOT, TRITD_LIB=os.path.abspath(l))
        r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
        print(rep, l, r.stdout.strip() or r.stderr[-300:], flush=True)
