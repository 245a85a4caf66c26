"""Generate the committed golden vectors under tests/golden/.

The reference is MATLAB-only and MATLAB/Octave are absent here (SURVEY.md
§8c), so the vectors come from the numpy restatement in
`oracle/tritd_oracle.py` (itself pinned against the reference's own loop
definitions, tests/test_oracle.py).  Run from the repo root:

    python tests/golden/make_golden.py

Each .npz holds inputs (D, A0, B0, C0, r, opts as JSON) and outputs
(A, B, C, O, E, errHist, k), plus the state after iterations 1 and 2 for the
small cases (to localise a divergence).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "triple-tensor-decomposition-with-admm_amd"))

import tritd_oracle as orc  # noqa: E402
from tritd import synth  # noqa: E402

CASES = {
    # name: (generator, kwargs, r, opts, keep full trace?)
    "g12x10x8_r2": (synth.low_rank_plus_outliers, dict(n1=12, n2=10, n3=8, r=2), 2,
                    dict(synth.TRAFFIC_OPTS, maxIter=30), True),
    "g30_r3": (synth.low_rank_plus_outliers, dict(n1=30, n2=30, n3=30, r=3), 3,
               dict(synth.TRAFFIC_OPTS), False),
    "g54x4x96_r5_sensor": (synth.sensor_like, dict(n1=54, n2=4, n3=96, r=5), 5,
                           dict(synth.TRAFFIC_OPTS), False),
    "g20x24x18_r5_video": (synth.video_like, dict(n1=20, n2=24, n3=18, r=5), 5,
                           dict(synth.VIDEO_OPTS, maxIter=40), False),
    # a large tol makes the stop test at :63 fire early (errHist truncation)
    "g12x10x8_r2_stop": (synth.low_rank_plus_outliers, dict(n1=12, n2=10, n3=8, r=2), 2,
                         dict(synth.TRAFFIC_OPTS, tol=0.2), False),
    # r=8 exercises the R=64 (full MFMA tile) code path at a small size
    "g17x16x20_r8": (synth.low_rank_plus_outliers, dict(n1=17, n2=16, n3=20, r=8), 8,
                     dict(synth.TRAFFIC_OPTS, maxIter=25), False),
    # fp64 r = 10, 12, 16: the padded-rank 128 / 256 kernels (K5 at one wave per
    # SIMD, K2 in 64-column passes, generic apply, blocked / big solves)
    "g20x18x16_r10": (synth.low_rank_plus_outliers, dict(n1=20, n2=18, n3=16, r=10), 10,
                      dict(synth.TRAFFIC_OPTS, maxIter=20), False),
    "g24x20x18_r12": (synth.low_rank_plus_outliers, dict(n1=24, n2=20, n3=18, r=12), 12,
                      dict(synth.TRAFFIC_OPTS, maxIter=15), False),
    "g24x22x20_r16": (synth.low_rank_plus_outliers, dict(n1=24, n2=22, n3=20, r=16), 16,
                      dict(synth.TRAFFIC_OPTS, maxIter=10), False),
    # opts.model = 'qi' (SURVEY.md §8f rank 4): Qi-model builders of
    # origin_triple_tensor/, data drawn from the Qi triple product
    "qi12x10x8_r2": (synth.low_rank_plus_outliers, dict(n1=12, n2=10, n3=8, r=2, model="qi"), 2,
                     dict(synth.TRAFFIC_OPTS, maxIter=30, model="qi"), True),
    "qi30_r3": (synth.low_rank_plus_outliers, dict(n1=30, n2=30, n3=30, r=3, model="qi"), 3,
                dict(synth.TRAFFIC_OPTS, model="qi"), False),
    "qi17x16x20_r8": (synth.low_rank_plus_outliers, dict(n1=17, n2=16, n3=20, r=8, model="qi"), 8,
                      dict(synth.TRAFFIC_OPTS, maxIter=25, model="qi"), False),
    "qi20x24x18_r3_video_stop": (synth.video_like, dict(n1=20, n2=24, n3=18, r=3), 3,
                                 dict(synth.VIDEO_OPTS, maxIter=60, tol=0.1, model="qi"), False),
}


# triple_decomp_ALS.m: reads only maxIter and tol
ALS_CASES = {
    "als12x10x8_r2": (synth.low_rank_plus_outliers, dict(n1=12, n2=10, n3=8, r=2), 2,
                      dict(maxIter=40, tol=1e-5)),
    "als30_r3": (synth.low_rank_plus_outliers, dict(n1=30, n2=30, n3=30, r=3), 3,
                 dict(maxIter=60, tol=1e-5)),
    "als17x16x20_r8": (synth.low_rank_plus_outliers, dict(n1=17, n2=16, n3=20, r=8), 8,
                       dict(maxIter=25, tol=1e-5)),
    # early stop (:20-23): the factors of the stopping iteration are returned un-updated
    "als20x24x18_r5_stop": (synth.video_like, dict(n1=20, n2=24, n3=18, r=5), 5,
                            dict(maxIter=50, tol=1e-2)),
}


# fast_robust_triple_tensor/test.m (nonconvex variant):
# positional parameters (rho, lambda, gamma_A, epsilon, p, theta, maxIter, tol);
# the reference has no caller, so these values are this build's choice
NCVX_PARAMS = dict(rho=1.0, **{"lambda": 0.5}, gamma_A=1e-3, epsilon=1e-2, p=0.5, theta=2.0 / 3.0)
NCVX_CASES = {
    "nc12x10x8_r2": (synth.low_rank_plus_outliers, dict(n1=12, n2=10, n3=8, r=2), 2,
                     dict(NCVX_PARAMS, maxIter=30, tol=1e-5)),
    "nc30_r3": (synth.low_rank_plus_outliers, dict(n1=30, n2=30, n3=30, r=3), 3,
                dict(NCVX_PARAMS, maxIter=60, tol=1e-5)),
    "nc17x16x20_r8": (synth.low_rank_plus_outliers, dict(n1=17, n2=16, n3=20, r=8), 8,
                      dict(NCVX_PARAMS, maxIter=25, tol=1e-5)),
    # the stop test fires: errHist truncated, O of the previous iteration returned
    "nc20x24x18_r3_stop": (synth.video_like, dict(n1=20, n2=24, n3=18, r=3), 3,
                           dict(NCVX_PARAMS, rho=0.5, maxIter=60, tol=2e-2)),
}


def make_ncvx(name):
    gen, kw, r, prm = NCVX_CASES[name]
    d = gen(**kw)
    A, B, C, O, eh, k, tr = orc.triple_decomp_ADMM_ncvx(
        d["D"], r, prm["rho"], prm["lambda"], prm["gamma_A"], prm["epsilon"], prm["p"],
        prm["theta"], prm["maxIter"], prm["tol"], d["A0"], d["B0"], d["C0"],
        printer=lambda s: None, trace_iters=(1, 2))
    out = dict(X=d["D"], A0=d["A0"], B0=d["B0"], C0=d["C0"], r=np.int64(r),
               opts=np.array(json.dumps(prm)), A=A, B=B, C=C, O=O, errHist=eh, k=np.int64(k))
    if name == "nc12x10x8_r2":  # the state after iterations 1 and 2 (localises a divergence)
        for it in (1, 2):
            for key in ("A", "B", "C", "O"):
                out[f"it{it}_{key}"] = tr[it][key]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    return k, eh[-1]


def make_als(name):
    gen, kw, r, opts = ALS_CASES[name]
    d = gen(**kw)
    A, B, C, eh, k = orc.triple_decomp_ALS(d["D"], r, opts, d["A0"], d["B0"], d["C0"],
                                           printer=lambda s: None)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), X=d["D"], A0=d["A0"], B0=d["B0"],
                        C0=d["C0"], r=np.int64(r), opts=np.array(json.dumps(opts)), A=A, B=B,
                        C=C, errHist=eh, k=np.int64(k))
    return k, eh[-1]


def make(name):
    gen, kw, r, opts, full = CASES[name]
    d = gen(**kw)
    res = orc.triple_decomp_ADMM(d["D"], r, opts, d["A0"], d["B0"], d["C0"], trace_iters=(1, 2))
    A, B, C, O, eh, E, k, trace = res
    out = dict(D=d["D"], A0=d["A0"], B0=d["B0"], C0=d["C0"], r=np.int64(r),
               opts=np.array(json.dumps(opts)), A=A, B=B, C=C, O=O, E=E, errHist=eh, k=np.int64(k))
    if "Lstar" in d:
        out["Lstar"] = d["Lstar"]
    for it in (1, 2):
        st = trace[it]
        for key in ("A", "B", "C"):
            out[f"it{it}_{key}"] = st[key]
        if full:
            for key in ("O", "E", "Y_L", "Y_O"):
                out[f"it{it}_{key}"] = st[key]
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    return k, eh[-1]


if __name__ == "__main__":
    # python tests/golden/make_golden.py [admm|qi|wide|als|ncvx]  (default: all)
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("all", "admm", "qi", "wide"):
        for n in CASES:
            if which == "qi" and not n.startswith("qi"):
                continue
            if which == "wide" and n not in ("g20x18x16_r10", "g24x20x18_r12", "g24x22x20_r16"):
                continue
            print(n, *make(n))
    if which in ("all", "als"):
        for n in ALS_CASES:
            print(n, *make_als(n))
    if which in ("all", "ncvx"):
        for n in NCVX_CASES:
            print(n, *make_ncvx(n))
