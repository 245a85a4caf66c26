"""Mode-1 sharded restatement of the ADMM loop — TEST INFRASTRUCTURE ONLY.

This is the algebra libtritd runs across GPUs,
written in numpy with an injected `allreduce(np.ndarray) -> np.ndarray` so
the CPU tests can drive it with torch.distributed/gloo at world_size 2 and
compare against the unsharded line-by-line oracle (tritd_oracle.py).

Per iteration k on the shard rows [i0, i1):
  A  M1 = sum_j W(i,j,:) o B^(j,:)             (W = T x3 C^ from the previous pass)
     A^ = M1 inv((B^TB) o (C^TC) + l2 I)        update_A, triple_decomp_ADMM.m:73-81
     red1 = [ M2 = sum_i W(i,:,:) o A^(i,:) | A^TA ]           -> all-reduce
  B  B^ = M2 inv((A^TA) o (C^TC) + l2 I)        update_B, :83-88
     red2 = M3 = sum_ij T(i,j,:) A^(i,:) o B^(j,:)             -> all-reduce
  C  C^ = M3 inv((A^TA) o (B^TB) + 1e-9 I)      update_C, :90-95
     L, O, E, Y_L, Y_O (:38-53), T_next (:33), W_next = T_next x3 C^
     red3 = [sum resL^2, sum resO^2]                           -> all-reduce
  D  errHist / stop test (:59-65)
Y_O is not carried: like the fp64 fused update (k_admm.hip, derived Y_O) it
is rebuilt each iteration as Y_L^(k-1) - mu_(k-1) (E^(k-1) - E^(k-2)).

`sharded_als` is the same for triple_decomp_ALS.m (fit sum, [M2 | A^TA] and
M3 reduced; als.cpp).
"""
from __future__ import annotations

import numpy as np


def _hat(A0, B0, C0, r):
    n1 = A0.shape[0]
    n2 = B0.shape[1]
    n3 = C0.shape[2]
    R = r * r
    Ah = A0.reshape((n1, R), order="F").copy()
    Bh = np.transpose(B0, (1, 0, 2)).reshape((n2, R), order="F").copy()
    Ch = C0.reshape((R, n3), order="F").T.copy()
    return Ah, Bh, Ch


def sharded_admm(D_local, i0, i1, r, opts, A0, B0, C0, allreduce):
    """Run the sharded schedule on rows [i0, i1).  Returns dict with the local
    A rows, replicated B, C (reference layouts), local O, E and errHist."""
    D = np.asarray(D_local, dtype=np.float64)
    nl, n2, n3 = D.shape
    n1 = A0.shape[0]
    R = r * r
    Ah_full, Bh, Ch = _hat(A0, B0, C0, r)
    Ah = Ah_full[i0:i1].copy()
    mu0, rho = float(opts["mu"]), float(opts["rho"])
    lam, l2 = float(opts["lambda"]), float(opts["lambda2"])
    maxIter, tol = int(opts["maxIter"]), float(opts["tol"])
    mus = []
    mu = mu0
    for _ in range(maxIter + 1):
        mus.append(mu)
        mu = min(mu * rho, mu0 * 1e6)

    O = np.zeros_like(D)
    E = np.zeros_like(D)
    E_prev = np.zeros_like(D)
    YL = np.zeros_like(D)
    normD = float(np.sqrt(allreduce(np.array([np.sum(D * D)]))[0]))
    T = (D - O) + (1.0 / mus[0]) * YL
    W = np.einsum("ijt,tk->ijk", T, Ch)
    BtB, CtC = Bh.T @ Bh, Ch.T @ Ch
    errHist = []
    k = 0
    for k in range(1, maxIter + 1):
        M1 = np.einsum("ijk,jk->ik", W, Bh)
        Ah = M1 @ np.linalg.inv(BtB * CtC + l2 * np.eye(R))
        red1 = allreduce(np.concatenate([np.einsum("ijk,ik->jk", W, Ah).ravel(),
                                         (Ah.T @ Ah).ravel()]))
        M2, AtA = red1[: n2 * R].reshape(n2, R), red1[n2 * R:].reshape(R, R)
        Bh = M2 @ np.linalg.inv(AtA * CtC + l2 * np.eye(R))
        BtB = Bh.T @ Bh
        M3 = allreduce(np.einsum("ijt,ik,jk->tk", T, Ah, Bh))
        Ch = M3 @ np.linalg.inv(AtA * BtB + 1e-9 * np.eye(R))
        CtC = Ch.T @ Ch

        muL = muO = mus[k - 1]
        mu_prev = mus[k - 2] if k >= 2 else 0.0
        YO = YL - mu_prev * (E - E_prev)  # derived Y_O^(k-1) (k_admm.hip)
        L = np.einsum("ik,jk,tk->ijt", Ah, Bh, Ch)
        R1 = (D - L) + (1.0 / muL) * YL
        R2 = E - (1.0 / muO) * YO
        O = (muL * R1 + muO * R2) / (muL + muO)
        R3 = O + (1.0 / muO) * YO
        E_prev = E
        E = np.sign(R3) * np.fmax(np.abs(R3) - lam / muO, 0.0)
        resL = (D - L) - O
        resO = O - E
        YL = YL + muL * resL
        T = (D - O) + (1.0 / mus[k]) * YL
        W = np.einsum("ijt,tk->ijk", T, Ch)
        ss = allreduce(np.array([np.sum(resL * resL), np.sum(resO * resO)]))
        errHist.append(np.sqrt(ss[0]) / normD + np.sqrt(ss[1]) / normD)
        if k > 1 and abs(errHist[-1] - errHist[-2]) < tol * errHist[-2]:
            break

    A = np.zeros((n1, r, r), order="F")
    A.reshape((n1, R), order="F")[i0:i1] = Ah  # rows of this shard only
    A_loc = Ah.reshape((nl, r, r), order="F")
    B = np.transpose(Bh.reshape((n2, r, r), order="F"), (1, 0, 2)).copy(order="F")
    C = Ch.T.reshape((r, r, n3), order="F").copy(order="F")
    return dict(A_rows=A_loc, B=B, C=C, O=O, E=E, errHist=np.array(errHist), k=k)


def k5_workgroups(nl: int, n2: int, n3: int = 1, RP: int = 16) -> int:
    """K5's grid on a shard of nl rows (k_admm.hip k5_grid x k5_tsplit): one
    workgroup per 4 ij-tiles of 16 padded rows, ij-tile g = (j*n1p + i) // 16,
    times the chunks of a t-split walk (fp64, RP <= 64: fewer than 256 such
    workgroups are cut into t-chunks of >= 8 t-tiles, up to ~256 in all)."""
    n1p = -(-nl // 16) * 16
    wg = -(-(n1p * n2 // 16) // 4)
    ntt = -(-n3 // 16)
    split = 1
    if RP <= 64 and wg < 256:
        split = max(1, min(-(-256 // wg), ntt // 8))
    return wg * split


def library_admm(D_local, i0, i1, r, opts, A0, B0, C0, allreduce, allreduce_max,
                 clear_tail=True):
    """The schedule solver.cpp runs with a communicator (Session::iterate_fused,
    fp64 CP model), as opposed to the phase order of sharded_admm:

    * two all-reduces per iteration: red1 = [M2 | A^TA | norm tail] and M3;
    * K5's residual norms stay per workgroup (k5_workgroups pairs of
      [sum resL^2, sum resO^2]) in red1's tail, which is sized to the largest
      shard's grid (agree_counts: a max-all-reduce at session creation); the
      pairs past this rank's own stay zero because k_reduce_finish clears
      what it consumed (clear_tail=False models the bug that clearing fixes);
    * the stop test of iteration k-1 runs after M1 .. M2 of iteration k
      (speculative: they write only scratch and A^'s other parity buffer), so
      a stop returns the A^ of k-1, and B^, C^, O, E of k-1;
    * after the last iteration the pending norms are flushed alone.

    allreduce(x) sums over ranks; allreduce_max(x) takes the elementwise max.
    Returns the same dict as sharded_admm plus 'counts', the element count of
    every all-reduce this rank issued, in order (they must agree across ranks).
    """
    D = np.asarray(D_local, dtype=np.float64)
    nl, n2, n3 = D.shape
    n1 = A0.shape[0]
    R = r * r
    Ah_full, Bh, Ch = _hat(A0, B0, C0, r)
    AhB = [Ah_full[i0:i1].copy(), None]  # A^ by iteration parity (set_ah)
    mu0, rho = float(opts["mu"]), float(opts["rho"])
    lam, l2 = float(opts["lambda"]), float(opts["lambda2"])
    maxIter, tol = int(opts["maxIter"]), float(opts["tol"])
    mus = []
    mu = mu0
    for _ in range(maxIter + 2):
        mus.append(mu)
        mu = min(mu * rho, mu0 * 1e6)
    counts = []

    def ar(x):
        counts.append(int(x.size))
        return allreduce(x)

    nwg = k5_workgroups(nl, n2)
    tail_n = int(allreduce_max(np.array([float(nwg)]))[0])
    n1p = -(-nl // 16) * 16
    ii, jj = np.meshgrid(np.arange(nl), np.arange(n2), indexing="ij")
    wg_of = ((jj * n1p + ii) // 16) // 4  # K5 workgroup of each (i, j)
    tail = np.zeros((tail_n, 2))

    O = np.zeros_like(D)
    E = np.zeros_like(D)
    E_prev = np.zeros_like(D)
    YL = np.zeros_like(D)
    normD = float(np.sqrt(ar(np.array([np.sum(D * D)]))[0]))
    T = (D - O) + (1.0 / mus[0]) * YL
    W = np.einsum("ijt,tk->ijk", T, Ch)
    BtB, CtC = Bh.T @ Bh, Ch.T @ Ch
    errHist = []
    pending = 0  # iteration whose norm partials wait in the tail

    def finish(kk):
        nonlocal tail
        ss = tail.sum(axis=0)
        if clear_tail:
            tail = np.zeros_like(tail)
        errHist.append(np.sqrt(ss[0]) / normD + np.sqrt(ss[1]) / normD)
        return kk > 1 and abs(errHist[-1] - errHist[-2]) < tol * errHist[-2]

    k_done = 0
    stopped = False
    for k in range(1, maxIter + 1):
        # M1 .. M2 of iteration k (speculative while iteration k-1's test is pending)
        M1 = np.einsum("ijk,jk->ik", W, Bh)
        Ah_k = M1 @ np.linalg.inv(BtB * CtC + l2 * np.eye(R))
        red1 = np.concatenate([np.einsum("ijk,ik->jk", W, Ah_k).ravel(), (Ah_k.T @ Ah_k).ravel()])
        nred1 = red1.size
        if pending:
            red1 = ar(np.concatenate([red1, tail.ravel()]))
            tail = red1[nred1:].reshape(tail_n, 2).copy()
            stop = finish(pending)
            pending = 0
            if stop:  # every later kernel sees the stop flag
                stopped = True
                break
        else:
            red1 = ar(red1)
        AhB[k & 1] = Ah_k
        M2, AtA = red1[: n2 * R].reshape(n2, R), red1[n2 * R: nred1].reshape(R, R)
        Bh = M2 @ np.linalg.inv(AtA * CtC + l2 * np.eye(R))
        BtB = Bh.T @ Bh
        M3 = ar(np.einsum("ijt,ik,jk->tk", T, Ah_k, Bh))
        Ch = M3 @ np.linalg.inv(AtA * BtB + 1e-9 * np.eye(R))
        CtC = Ch.T @ Ch

        muL = muO = mus[k - 1]
        mu_prev = mus[k - 2] if k >= 2 else 0.0
        YO = YL - mu_prev * (E - E_prev)
        L = np.einsum("ik,jk,tk->ijt", Ah_k, Bh, Ch)
        R1 = (D - L) + (1.0 / muL) * YL
        R2 = E - (1.0 / muO) * YO
        O = (muL * R1 + muO * R2) / (muL + muO)
        R3 = O + (1.0 / muO) * YO
        E_prev = E
        E = np.sign(R3) * np.fmax(np.abs(R3) - lam / muO, 0.0)
        resL = (D - L) - O
        resO = O - E
        YL = YL + muL * resL
        T = (D - O) + (1.0 / mus[k]) * YL
        W = np.einsum("ijt,tk->ijk", T, Ch)
        # K5's per-workgroup partials into the first nwg pairs of the tail
        tail[:nwg, 0] = np.bincount(wg_of.ravel(), (resL * resL).sum(axis=2).ravel(), nwg)
        tail[:nwg, 1] = np.bincount(wg_of.ravel(), (resO * resO).sum(axis=2).ravel(), nwg)
        pending = k
        k_done = k
    if pending and not stopped:  # flush_norms: the last iteration's stop test
        tail = ar(tail.ravel()).reshape(tail_n, 2).copy()
        finish(pending)

    Ah = AhB[k_done & 1]
    A_loc = Ah.reshape((nl, r, r), order="F")
    B = np.transpose(Bh.reshape((n2, r, r), order="F"), (1, 0, 2)).copy(order="F")
    C = Ch.T.reshape((r, r, n3), order="F").copy(order="F")
    return dict(A_rows=A_loc, B=B, C=C, O=O, E=E, errHist=np.array(errHist), k=k_done,
                counts=np.array(counts))


def sharded_als(X_local, i0, i1, r, opts, A0, B0, C0, allreduce):
    """triple_decomp_ALS.m:1-40 on the shard rows [i0, i1) (als.cpp):
    fit sum -> all-reduce -> errHist / stop; A local; [M2 | A^TA] and M3
    all-reduced.  Returns the local A rows, replicated B, C, errHist, k."""
    X = np.asarray(X_local, dtype=np.float64)
    nl, n2, n3 = X.shape
    R = r * r
    Ah_full, Bh, Ch = _hat(A0, B0, C0, r)
    Ah = Ah_full[i0:i1].copy()
    maxIter, tol = int(opts["maxIter"]), float(opts["tol"])
    Xnorm = float(np.sqrt(allreduce(np.array([np.sum(X * X)]))[0]))
    ridge = 1e-9 * np.eye(R)
    errHist = []
    k = 0
    for k in range(1, maxIter + 1):
        L = np.einsum("ik,jk,tk->ijt", Ah, Bh, Ch)
        ss = allreduce(np.array([np.sum((X - L) ** 2)]))
        errHist.append(np.sqrt(ss[0]) / Xnorm)
        if k > 1 and abs(errHist[-1] - errHist[-2]) < tol * errHist[-2]:
            break
        W = np.einsum("ijt,tk->ijk", X, Ch)
        M1 = np.einsum("ijk,jk->ik", W, Bh)
        Ah = M1 @ np.linalg.inv((Bh.T @ Bh) * (Ch.T @ Ch) + ridge)
        red1 = allreduce(np.concatenate([np.einsum("ijk,ik->jk", W, Ah).ravel(),
                                         (Ah.T @ Ah).ravel()]))
        M2, AtA = red1[: n2 * R].reshape(n2, R), red1[n2 * R:].reshape(R, R)
        Bh = M2 @ np.linalg.inv(AtA * (Ch.T @ Ch) + ridge)
        M3 = allreduce(np.einsum("ijt,ik,jk->tk", X, Ah, Bh))
        Ch = M3 @ np.linalg.inv(AtA * (Bh.T @ Bh) + ridge)
    A_loc = Ah.reshape((nl, r, r), order="F")
    B = np.transpose(Bh.reshape((n2, r, r), order="F"), (1, 0, 2)).copy(order="F")
    C = Ch.T.reshape((r, r, n3), order="F").copy(order="F")
    return dict(A_rows=A_loc, B=B, C=C, errHist=np.array(errHist), k=k)
