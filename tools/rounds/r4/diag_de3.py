"""Where the dense-E K5 form differs from the compact form: E and O after a
few iterations on the same input, located by (i, j, t) and tile coordinates.
Diagnostic.

    python tools/rounds/r4/diag_de3.py [n1 n2 n3 iters]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path[:0] = [os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd")]


def run(tritd, d, opts, de):
    os.environ["TRITD_DENSE_E"] = de
    try:
        return tritd.triple_decomp_ADMM(d["D"], 5, opts, d["A0"], d["B0"], d["C0"], return_E=True,
                                        return_iters=True)
    finally:
        os.environ.pop("TRITD_DENSE_E", None)


def where(tag, X, Y):
    diff = np.abs(X - Y) > 1e-9 * (1 + np.abs(Y))
    idx = np.argwhere(diff)
    print("%s: %d of %d differ" % (tag, len(idx), X.size), flush=True)
    if len(idx) == 0:
        return
    i, j, t = idx[:, 0], idx[:, 1], idx[:, 2]
    for name, v in (("i%16", i % 16), ("i//16", i // 16), ("t%16", t % 16), ("t//16", t // 16),
                    ("j%8", j % 8), ("grp=(i//16+j*q)//4 %8", ((i // 16 + j * ((X.shape[0] + 15) // 16)) // 4) % 8)):
        u, c = np.unique(v, return_counts=True)
        print("   %-24s %s" % (name, " ".join("%d:%d" % (a, b) for a, b in zip(u[:24], c[:24]))), flush=True)
    print("   first", [tuple(x) for x in idx[:8]], flush=True)


def main():
    import tritd
    from tritd import synth
    a = [int(x) for x in sys.argv[1:]] or [240, 320, 64, 2]
    n1, n2, n3, iters = a
    d = synth.video_like(n1, n2, n3, 5)
    opts = dict(synth.VIDEO_OPTS, maxIter=iters)
    ref = run(tritd, d, opts, "0")
    for rep in range(3):
        got = run(tritd, d, opts, "1")
        where("rep %d E" % rep, got[5], ref[5])
        where("rep %d O" % rep, got[3], ref[3])
    ref2 = run(tritd, d, opts, "0")
    where("compact vs compact E", ref2[5], ref[5])


if __name__ == "__main__":
    main()
