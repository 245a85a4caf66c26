"""Config 3 (240x320x300 r=5, video opts) for a few iterations: errHist of the
HIP path under several session forms against the C restatement, iteration by
iteration.  A diagnostic for a divergence the full-size test reports.

    python tools/diag_c3.py [iters]
"""
import os
import subprocess
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"), os.path.join(ROOT, "oracle")]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 14
    import tritd
    from tritd import synth
    import tritd_ref
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    lib = tritd_ref.load()
    lib.tritd_ref_set_threads(int(os.environ.get("OMP_NUM_THREADS", "16")))
    d = synth.video_like(240, 320, 300, 5)
    opts = dict(synth.VIDEO_OPTS, maxIter=iters)
    ref = tritd_ref.admm(lib, d["D"], 5, opts, d["A0"], d["B0"], d["C0"])
    eh_ref = np.asarray(ref[4])
    print("ref k", ref[6], flush=True)
    forms = [("default", {}), ("dense_e=0", {"TRITD_DENSE_E": "0"}), ("dense_e=1", {"TRITD_DENSE_E": "1"}),
             ("fused=0", {"TRITD_FUSED": "0"}), ("fused=0,de=0", {"TRITD_FUSED": "0", "TRITD_DENSE_E": "0"})]
    for name, env in forms:
        saved = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            with warnings.catch_warnings(record=True) as wl:
                warnings.simplefilter("always")
                A, B, C, O, eh, E, k = tritd.triple_decomp_ADMM(d["D"], 5, opts, d["A0"], d["B0"], d["C0"],
                                                                return_E=True, return_iters=True)
        finally:
            for kk, v in saved.items():
                if v is None:
                    os.environ.pop(kk, None)
                else:
                    os.environ[kk] = v
        n = min(len(eh), len(eh_ref))
        relv = np.abs(np.asarray(eh[:n]) - eh_ref[:n]) / np.abs(eh_ref[:n])
        first = int(np.argmax(relv > 1e-8)) + 1 if np.any(relv > 1e-8) else None
        print("%-14s k %d warnings %s first-bad-iter %s rel %s" % (
            name, k, [type(w.message).__name__ for w in wl], first,
            " ".join("%.1e" % x for x in relv)), flush=True)


if __name__ == "__main__":
    main()
