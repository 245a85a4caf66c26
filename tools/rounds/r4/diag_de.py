"""Dense-E K5 form (TRITD_DENSE_E=1) against the C restatement over a sweep of
shapes, 3 iterations each: which dimension breaks it.  Diagnostic.

    python tools/rounds/r4/diag_de.py
"""
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"), os.path.join(ROOT, "oracle")]


def main():
    import tritd
    from tritd import synth
    import tritd_ref
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    lib = tritd_ref.load()
    lib.tritd_ref_set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    shapes = [(32, 24, 18), (32, 24, 48), (32, 24, 64), (32, 24, 80), (32, 24, 300), (240, 24, 48),
              (240, 320, 32), (240, 320, 48), (240, 320, 64), (64, 320, 300), (240, 320, 300)]
    if os.environ.get("DIAG_SHAPES"):
        shapes = [tuple(int(x) for x in t.split("x")) for t in os.environ["DIAG_SHAPES"].split(",")]
    print("lib", os.environ.get("TRITD_LIB", "in-tree"), flush=True)
    for shp in shapes:
        d = synth.video_like(*shp, 5)
        opts = dict(synth.VIDEO_OPTS, maxIter=3)
        ref = tritd_ref.admm(lib, d["D"], 5, opts, d["A0"], d["B0"], d["C0"])
        out = {}
        for de in ("0", "1"):
            os.environ["TRITD_DENSE_E"] = de
            try:
                got = tritd.triple_decomp_ADMM(d["D"], 5, opts, d["A0"], d["B0"], d["C0"], return_E=True,
                                               return_iters=True)
            finally:
                os.environ.pop("TRITD_DENSE_E", None)
            eh = np.asarray(got[4])
            out[de] = " ".join("%.1e" % x for x in np.abs(eh - ref[4][:len(eh)]) / np.abs(ref[4][:len(eh)]))
        print("%-16s de=0: %s | de=1: %s" % (shp, out["0"], out["1"]), flush=True)


if __name__ == "__main__":
    main()
