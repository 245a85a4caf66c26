"""Synthetic workloads for the TriTD-ADMM hot path.

The reference's datasets (`sensor.mat`, CDnet2014 videos) are not shipped
(SURVEY.md §2 #17), so benchmarks and parity tests run on seeded synthetic
tensors of the reference shapes.  Everything here is plain numpy data
generation in MATLAB (column-major) layout: it produces *inputs*, it is not
part of the accelerated path.

Recipe (SURVEY.md §8d "Synthetic generator"):
  A*, B*, C* ~ N(0,1) in the reference shapes (n1,r,r), (r,n2,r), (r,r,n3)
  L* = triple_product(A*, B*, C*)      (triple_product.m:6)
  S* : Bernoulli(p_out) support, values U(-10 sigma, 10 sigma), sigma = std(L*)
  D  = L* + S*
  A0, B0, C0 ~ N(0,1) (seed 123) — the initial factors the MATLAB wrapper would
  draw with randn (triple_decomp_ADMM.m:23).
"""
from __future__ import annotations

import numpy as np

# opts of the completion driver (traffic_triple_comparison.m:42-50)
TRAFFIC_OPTS = dict(maxIter=100, tol=1e-5, mu=1e-3, **{"lambda": 1.8}, lambda2=1e-3, rho=1.25, disp=0)
# opts of the video driver (video_triple_comparison.m:41-50)
VIDEO_OPTS = dict(maxIter=100, tol=1e-5, mu=1e-2, **{"lambda": 1.8}, lambda2=1e-2, rho=1.2, disp=0)


def hat_factors(A, B, C):
    """Reference factors -> CP factor matrices:
    Ahat(i,k)=A(i,p,q), Bhat(j,k)=B(p,j,q), Chat(t,k)=C(p,q,t), k=p+(q-1)r."""
    n1, r, _ = A.shape
    n2 = B.shape[1]
    n3 = C.shape[2]
    Ah = A.reshape((n1, r * r), order="F")
    Bh = np.transpose(B, (1, 0, 2)).reshape((n2, r * r), order="F")
    Ch = C.reshape((r * r, n3), order="F").T
    return Ah, Bh, Ch


def cp_full(Ah, Bh, Ch):
    """L(i,j,t) = sum_k Ah(i,k) Bh(j,k) Ch(t,k), column-major (n1,n2,n3)."""
    n1, R = Ah.shape
    n2 = Bh.shape[0]
    n3 = Ch.shape[0]
    # (n1 x R) @ (R x n2*n3) with KR(k, j + n2 t) = Bh(j,k) Ch(t,k)
    KR = (Bh[:, None, :] * Ch[None, :, :]).reshape((n2 * n3, R), order="F")
    return (Ah @ KR.T).reshape((n1, n2, n3), order="F")


def qi_full(A, B, C):
    """Qi-model triple product L(i,j,t) = sum_{p,q,s} A(i,q,s) B(p,j,s) C(p,q,t)
    (origin_triple_tensor/triple_product.m:8-19; opts.model='qi')."""
    return np.asfortranarray(np.einsum("iqs,pjs,pqt->ijt", A, B, C, optimize=True))


def random_factors(n1, n2, n3, r, seed):
    rng = np.random.default_rng(seed)
    A = np.asfortranarray(rng.standard_normal((n1, r, r)))
    B = np.asfortranarray(rng.standard_normal((r, n2, r)))
    C = np.asfortranarray(rng.standard_normal((r, r, n3)))
    return A, B, C


def low_rank_plus_outliers(n1, n2, n3, r, p_out=0.05, seed=0, init_seed=123, model="cp"):
    """Config 1/4/5 generator.  Returns dict(D, Lstar, A0, B0, C0).
    model='qi' draws L* from the Qi-model triple product instead."""
    rng = np.random.default_rng(seed)
    As = np.asfortranarray(rng.standard_normal((n1, r, r)))
    Bs = np.asfortranarray(rng.standard_normal((r, n2, r)))
    Cs = np.asfortranarray(rng.standard_normal((r, r, n3)))
    Lstar = qi_full(As, Bs, Cs) if model == "qi" else cp_full(*hat_factors(As, Bs, Cs))
    sigma = float(Lstar.std())
    support = rng.random((n1, n2, n3)) < p_out
    vals = rng.uniform(-10.0 * sigma, 10.0 * sigma, size=(n1, n2, n3))
    D = np.asfortranarray(Lstar + np.where(support, vals, 0.0))
    A0, B0, C0 = random_factors(n1, n2, n3, r, init_seed)
    return dict(D=D, Lstar=Lstar, A0=A0, B0=B0, C0=C0)


def low_rank_plus_outliers_f32(n1, n2, n3, r, p_out=0.05, seed=0, init_seed=123, chunk=64,
                               rows=None):
    """low_rank_plus_outliers(...) rounded to single (D and L* as float32,
    column-major) without its fp64 full-size temporaries: the same draws from
    the same generator streams, produced in chunks of mode-1 rows (the support
    and value draws are C-ordered with i slowest, so row chunks consume them
    in order; the value stream starts n1*n2*n3 draws later, where the
    one-shot recipe's second call starts).  Equal to
    `low_rank_plus_outliers(...)["D"].astype(np.float32)` except where
    sigma = std(L*), summed chunk-wise here, differs in its last fp64 bit
    (config 5: 2048x2048x256 in ~10 GB instead of ~35 GB).

    rows=(i0, i1): only the mode-1 rows i0..i1-1 of D and L* (a rank's shard,
    SURVEY.md §8e), identical to those rows of the full call: sigma still
    comes from every row of L* (computed, not kept), and both draw streams are
    advanced past the rows before i0 (one 64-bit draw per value, PCG64)."""
    import copy
    i0, i1 = (0, n1) if rows is None else (int(rows[0]), int(rows[1]))
    if not 0 <= i0 < i1 <= n1:
        raise ValueError("rows must satisfy 0 <= i0 < i1 <= n1")
    rng = np.random.default_rng(seed)
    As = np.asfortranarray(rng.standard_normal((n1, r, r)))
    Bs = np.asfortranarray(rng.standard_normal((r, n2, r)))
    Cs = np.asfortranarray(rng.standard_normal((r, r, n3)))
    Ah, Bh, Ch = hat_factors(As, Bs, Cs)
    R = Ah.shape[1]
    KR = (Bh[:, None, :] * Ch[None, :, :]).reshape((n2 * n3, R), order="F")
    L = np.empty((i1 - i0, n2, n3), dtype=np.float32, order="F")
    # std(L*) in one pass: per-chunk mean and centred sum of squares,
    # combined pairwise (Chan, Golub & LeVeque)
    cnt, mean, m2 = 0, 0.0, 0.0
    for c0 in range(0, n1, chunk):
        c1 = min(n1, c0 + chunk)
        blk = (Ah[c0:c1] @ KR.T).reshape((c1 - c0, n2, n3), order="F")
        nb = blk.size
        mb = float(blk.mean())
        m2b = float(np.square(blk - mb).sum())
        delta = mb - mean
        tot = cnt + nb
        mean += delta * nb / tot
        m2 += m2b + delta * delta * cnt * nb / tot
        cnt = tot
        lo, hi = max(c0, i0), min(c1, i1)
        if lo < hi:
            L[lo - i0:hi - i0] = blk[lo - c0:hi - c0]
    sigma = float(np.sqrt(m2 / cnt))
    N = n1 * n2 * n3
    skip = i0 * n2 * n3
    rs = rng
    bg = copy.deepcopy(rng.bit_generator)
    bg.advance(N + skip)
    rv = np.random.Generator(bg)
    if skip:
        rs.bit_generator.advance(skip)
    D = np.empty((i1 - i0, n2, n3), dtype=np.float32, order="F")
    for c0 in range(i0, i1, chunk):
        c1 = min(i1, c0 + chunk)
        c = c1 - c0
        sup = rs.random((c, n2, n3)) < p_out
        vals = rv.uniform(-10.0 * sigma, 10.0 * sigma, size=(c, n2, n3))
        blk = (Ah[c0:c1] @ KR.T).reshape((c, n2, n3), order="F")
        D[c0 - i0:c1 - i0] = blk + np.where(sup, vals, 0.0)
    A0, B0, C0 = random_factors(n1, n2, n3, r, init_seed)
    return dict(D=D, Lstar=L, A0=A0, B0=B0, C0=C0)


def sensor_like(n1=54, n2=4, n3=1152, r=5, missing=0.10, seed=0, init_seed=123):
    """Config 2 stand-in: smooth daily-periodic readings + noise, a seeded
    fraction zeroed (traffic_triple_comparison.m:27-35 zeroes missing entries)."""
    rng = np.random.default_rng(seed)
    t = np.arange(n3)
    base = rng.uniform(15.0, 25.0, size=(n1, n2, 1))
    amp = rng.uniform(1.0, 5.0, size=(n1, n2, 1))
    phase = rng.uniform(0, 2 * np.pi, size=(n1, n2, 1))
    X = base + amp * np.sin(2 * np.pi * t[None, None, :] / 144.0 + phase)
    X = X + 0.1 * rng.standard_normal((n1, n2, n3))
    X = np.asfortranarray(X)
    mask = rng.random((n1, n2, n3)) < missing
    Y = X.copy(order="F")
    Y[mask] = 0.0
    A0, B0, C0 = random_factors(n1, n2, n3, r, init_seed)
    return dict(D=Y, X=X, mask=mask, A0=A0, B0=B0, C0=C0)


def video_like(n1=240, n2=320, n3=300, r=5, seed=0, init_seed=123):
    """Config 3 stand-in: static background (rank-1 in time) + moving bright
    blobs + N(0,2) noise, clipped to 0..255 (video_triple_comparison.m:20-21
    loads uint8 frames as double)."""
    rng = np.random.default_rng(seed)
    bg = rng.uniform(40.0, 200.0, size=(n1, n2))
    X = np.repeat(bg[:, :, None], n3, axis=2)
    ii, jj = np.meshgrid(np.arange(n1), np.arange(n2), indexing="ij")
    for b in range(3):
        ci0, cj0 = rng.uniform(0, n1), rng.uniform(0, n2)
        vi, vj = rng.uniform(-1.0, 1.0), rng.uniform(0.5, 2.0)
        rad = max(2.0, min(n1, n2) / 12.0)
        for t in range(n3):
            ci = (ci0 + vi * t) % n1
            cj = (cj0 + vj * t) % n2
            blob = (ii - ci) ** 2 + (jj - cj) ** 2 < rad ** 2
            X[:, :, t][blob] = 250.0
    X = X + 2.0 * rng.standard_normal(X.shape)
    X = np.asfortranarray(np.clip(X, 0.0, 255.0))
    A0, B0, C0 = random_factors(n1, n2, n3, r, init_seed)
    return dict(D=X.copy(order="F"), X=X, A0=A0, B0=B0, C0=C0)
