"""Lean class-single restatement of triple_decomp_ADMM.m — TEST
INFRASTRUCTURE ONLY (tests/golden/make_c5_horizon.py, tests/test_oracle.py).

`tritd_ref_admm_f32` (oracle/tritd_ref.c) keeps the reference's operation
structure: permute copies and design matrices are materialised, in double.
At config 5 (2048x2048x256 r=16) that needs ~65 GB and ~40 s per iteration on
8 cores, so the full 100-iteration horizon was never run.
This module runs the SAME arithmetic rules (MATLAB's class rules for a single
D; statement order of triple_decomp_ADMM.m:33-63) in a
layout that fits a 64 GB host:

* T, O, E, Y_L, Y_O are single (as in MATLAB); the elementwise statements
  :33 and :41-53 run in C (`tritd_ref_lean_form_T`, `tritd_ref_lean_update`),
  statement for statement the loop body of `tritd_ref_admm_f32`;
* X_k*F' (single * double -> single, :78,86,93) is accumulated in double by
  BLAS GEMMs over row blocks and rounded to single once, as the C restatement
  does: X1*F.' through W = T x3 C^ (dimension tree, the same sums regrouped),
  X3*H' as T(:,:)' * (A^ (.) B^) block by block;
* the Grams F*F.' etc. use the Hadamard identity F*F.' = (B^'B^).*(C^'C^)
  (exact in real arithmetic; differs from the explicit product at double
  rounding, ~1e-16 relative — far below the single-precision results);
* pinv is MATLAB's SVD pinv with tolerance max(size)*eps(max sigma)
  (tritd_oracle.pinv); (X*F')*pinv(G) is formed in double and rounded to
  single, then stored into the double factors (reshape_*: zeros() + assignment);
* L = triple_product(A,B,C) is double (A, B, C are double, triple_product.m:6),
  formed one frontal slice at a time and rounded to single where it meets D;
* norm() of a single array: squares summed in double, the root rounded to
  single; errHist(k) = single(eL + eO) stored into the double errHist (:59).

`tests/test_oracle.py` checks this module against `tritd_ref_admm_f32` at
small sizes (same k, errHist, O, E, L to single rounding).
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

import tritd_oracle as orc

f32, f64 = np.float32, np.float64


def _p(a):
    return C.c_void_p(a.ctypes.data)


def _bind(lib):
    i64, vp, d = C.c_int64, C.c_void_p, C.c_double
    lib.tritd_ref_lean_form_T.argtypes = [vp, vp, vp, d, vp, i64]
    lib.tritd_ref_lean_sumsq.argtypes = [vp, i64]
    lib.tritd_ref_lean_sumsq.restype = d
    lib.tritd_ref_lean_update.argtypes = [vp, vp, vp, vp, vp, vp, i64, d, d, d, vp]
    lib.tritd_ref_lean_rre_parts.argtypes = [vp, vp, i64, vp]
    return lib


def hat(A, B, Cc):
    """reference factors -> CP factor matrices."""
    n1, r, _ = A.shape
    n2, n3 = B.shape[1], Cc.shape[2]
    Ah = np.ascontiguousarray(A.reshape((n1, r * r), order="F"))
    Bh = np.ascontiguousarray(np.transpose(B, (1, 0, 2)).reshape((n2, r * r), order="F"))
    Ch = np.ascontiguousarray(Cc.reshape((r * r, n3), order="F").T)
    return Ah, Bh, Ch


def unhat(Ah, Bh, Ch, r):
    n1, n2, n3 = Ah.shape[0], Bh.shape[0], Ch.shape[0]
    A = np.asfortranarray(Ah.reshape((n1, r, r), order="F"))
    B = np.asfortranarray(np.transpose(Bh.reshape((n2, r, r), order="F"), (1, 0, 2)))
    Cc = np.asfortranarray(Ch.T.reshape((r, r, n3), order="F"))
    return A, B, Cc


def single_solve(M, G):
    """(X*F') * pinv(G): the single MTTKRP result (accumulated in double,
    rounded once) times MATLAB's pinv of the double Gram, rounded to single and
    stored into a double factor."""
    Ms = M.astype(f32).astype(f64)
    return (Ms @ orc.pinv(G)).astype(f32).astype(f64)


def slice_L(Ah, Bh, ct):
    """L(:,:,t) = sum_k A^(i,k) B^(j,k) C^(t,k) in double, column-major n1 x n2
    (the memory of the (n2, n1) C-ordered product)."""
    return Bh @ (Ah * ct).T


def admm_f32(lib, D, r, opts, A0, B0, C0, block=65536, log=None, trace=None):
    """triple_decomp_ADMM(D, r, opts) for a single D (class-single rules).
    Returns (A, B, C, O, E, errHist, k).  `trace(k, state)` is called after
    every iteration with a dict of the scalars of that iteration."""
    lib = _bind(lib)
    D = np.asfortranarray(D, dtype=f32)
    n1, n2, n3 = D.shape
    N, plane, R = D.size, n1 * n2, r * r
    if block % n1:
        block = max(n1, block // n1 * n1)
    mu0 = float(opts["mu"])
    muL = muO = mu0
    rho = float(opts["rho"])
    lam, lam2 = float(opts["lambda"]), float(opts["lambda2"])
    maxIter, tol, disp = int(opts["maxIter"]), float(opts["tol"]), bool(opts["disp"])
    Ah, Bh, Ch = hat(np.asfortranarray(A0, dtype=f64), np.asfortranarray(B0, dtype=f64),
                     np.asfortranarray(C0, dtype=f64))
    O = np.zeros(D.shape, f32, order="F")
    E = np.zeros(D.shape, f32, order="F")
    YL = np.zeros(D.shape, f32, order="F")
    YO = np.zeros(D.shape, f32, order="F")
    T = np.empty(D.shape, f32, order="F")
    W = np.empty((plane, R), f64)  # W = T x3 C^, double
    normD = f32(np.sqrt(lib.tritd_ref_lean_sumsq(_p(D), N)))
    Tm = T.reshape((plane, n3), order="F")
    eh = np.zeros(max(maxIter, 1))
    sums = np.zeros(2)
    k = 0
    for k in range(1, maxIter + 1):
        t0 = time.perf_counter()
        lib.tritd_ref_lean_form_T(_p(D), _p(O), _p(YL), muL, _p(T), N)  # :33
        # update_A (:73-81): X1*F.' = sum_j W(i,j,:) .* B^(j,:)
        G = (Bh.T @ Bh) * (Ch.T @ Ch) + lam2 * np.eye(R)
        M1 = np.zeros((n1, R))
        for c0 in range(0, plane, block):
            c1 = min(plane, c0 + block)
            Wc = Tm[c0:c1].astype(f64) @ Ch
            W[c0:c1] = Wc
            j0, j1 = c0 // n1, c1 // n1
            M1 += np.einsum("ijk,jk->ik", Wc.reshape((j1 - j0, n1, R)).transpose(1, 0, 2),
                            Bh[j0:j1], optimize=True)
        Ah = single_solve(M1, G)
        # update_B (:83-88): X2*G' = sum_i W(i,j,:) .* A^(i,:) (new A, old C)
        G = (Ah.T @ Ah) * (Ch.T @ Ch) + lam2 * np.eye(R)
        M2 = np.zeros((n2, R))
        for c0 in range(0, plane, block):
            c1 = min(plane, c0 + block)
            j0, j1 = c0 // n1, c1 // n1
            M2[j0:j1] = np.einsum("jik,ik->jk", W[c0:c1].reshape((j1 - j0, n1, R)), Ah,
                                  optimize=True)
        Bh = single_solve(M2, G)
        # update_C (:90-95): X3*H' = sum_ij T(i,j,:)' A^(i,:) .* B^(j,:), ridge 1e-9
        G = (Ah.T @ Ah) * (Bh.T @ Bh) + 1e-9 * np.eye(R)
        M3 = np.zeros((n3, R))
        for c0 in range(0, plane, block):
            c1 = min(plane, c0 + block)
            j0, j1 = c0 // n1, c1 // n1
            KR = (Bh[j0:j1, None, :] * Ah[None, :, :]).reshape((c1 - c0, R))
            M3 += Tm[c0:c1].astype(f64).T @ KR
        Ch = single_solve(M3, G)
        # L = triple_product(A,B,C) (:38) and :41-53, one frontal slice at a time
        sL = sO = 0.0
        for t in range(n3):
            Lt = slice_L(Ah, Bh, Ch[t])
            sl = slice(t * plane, (t + 1) * plane)
            lib.tritd_ref_lean_update(_p(D.reshape(-1, order="F")[sl]),
                                      _p(O.reshape(-1, order="F")[sl]),
                                      _p(E.reshape(-1, order="F")[sl]),
                                      _p(YL.reshape(-1, order="F")[sl]),
                                      _p(YO.reshape(-1, order="F")[sl]), _p(Lt), plane, muL, muO,
                                      lam, _p(sums))
            sL += sums[0]
            sO += sums[1]
        muL = min(muL * rho, mu0 * 1e6)  # :56
        muO = min(muO * rho, mu0 * 1e6)  # :57
        eL = f32(f32(np.sqrt(sL)) / normD)
        eO = f32(f32(np.sqrt(sO)) / normD)
        eh[k - 1] = float(f32(eL + eO))  # :59
        if disp and k % 10 == 0:
            print("Iter %d, errL=%.2e, errO=%.2e" % (k, eL, eO))
        if log is not None:
            log("iter %d errHist %.9e (%.1f s)" % (k, eh[k - 1], time.perf_counter() - t0))
        if trace is not None:
            trace(k, dict(errHist=eh[k - 1], muL=muL))
        if k > 1 and abs(eh[k - 1] - eh[k - 2]) < tol * eh[k - 2]:  # :63
            break
    del W, T
    A, B, Cc = unhat(Ah, Bh, Ch, r)
    return A, B, Cc, O, E, eh[:k].copy(), k


def rre(lib, A, B, Cc, X):
    """‖triple_product(A,B,C) − X‖_F / ‖X‖_F (traffic_triple_comparison.m:62-63,
    evaluate :194-199) with L formed in double slice by slice, X single."""
    lib = _bind(lib)
    Ah, Bh, Ch = hat(A, B, Cc)
    X = np.asfortranarray(X, dtype=f32)
    n1, n2, n3 = X.shape
    plane = n1 * n2
    parts = np.zeros(2)
    num = den = 0.0
    flat = X.reshape(-1, order="F")
    for t in range(n3):
        Lt = slice_L(Ah, Bh, Ch[t])
        lib.tritd_ref_lean_rre_parts(_p(Lt), _p(flat[t * plane:(t + 1) * plane]), plane,
                                     _p(parts))
        num += parts[0]
        den += parts[1]
    return float(np.sqrt(num) / np.sqrt(den))


def sample_L(A, B, Cc, idx):
    """L at linear (column-major) indices idx, in double."""
    Ah, Bh, Ch = hat(A, B, Cc)
    n1, n2 = Ah.shape[0], Bh.shape[0]
    i = idx % n1
    j = (idx // n1) % n2
    t = idx // (n1 * n2)
    return np.einsum("sk,sk,sk->s", Ah[i], Bh[j], Ch[t])


def diff_parts(A, B, Cc, A2, B2, C2):
    """(||L - L2||^2, ||L2||^2) for L = triple_product(A,B,C), L2 =
    triple_product(A2,B2,C2), formed in double one frontal slice at a time:
    L(:,:,t) - L2(:,:,t) = [A^.*C^(t,:), A2^.*C2^(t,:)] [B^, -B2^]' (one GEMM)."""
    Ah, Bh, Ch = hat(A, B, Cc)
    Ah2, Bh2, Ch2 = hat(A2, B2, C2)
    Bcat = np.concatenate([Bh, -Bh2], axis=1)
    num = den = 0.0
    for t in range(Ch.shape[0]):
        Acat = np.concatenate([Ah * Ch[t], Ah2 * Ch2[t]], axis=1)
        dlt = Bcat @ Acat.T
        l2 = Bh2 @ (Ah2 * Ch2[t]).T
        num += float(np.vdot(dlt, dlt))
        den += float(np.vdot(l2, l2))
    return num, den
