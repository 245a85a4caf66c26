"""CPU oracle for the TriTD-ADMM hot path — TEST INFRASTRUCTURE ONLY.

This module is a line-by-line numpy restatement of the MATLAB reference
(`/root/reference/fast_robust_triple_tensor/`), kept under `oracle/` so that it
is only ever used as the *checker*: by `tests/`, by `__graft_entry__.smoke()`
and by `bench.py`'s `cpu_baseline` leg.  The product path (`libtritd.so`)
never imports, links or calls anything in this directory.

Parity status
-------------
* **Primitives pinned**: `buildF/buildG/buildH` are checked against the
  reference's own commented loop definitions (`buildF.m:5-16`,
  `buildG.m:5-16`, `buildH.m:5-16`) and `triple_product` against the explicit
  five-loop in `fast_robust_triple_tensor/test.m:142-160` (tests/test_oracle.py).
* **Solver loop: parity unpinned.**  The reference is MATLAB-only; MATLAB and
  Octave are absent from this image (probed with `command -v`), the reference
  ships no tests, no fixtures and no data.  The loop below
  therefore restates `triple_decomp_ADMM.m:15-68` statement by statement with
  MATLAB semantics, and the committed golden vectors (`tests/golden/`) are
  generated *from this restatement* by `tests/golden/make_golden.py`.

MATLAB semantics restated here
------------------------------
* column-major storage: every array is handled with ``order='F'``;
* ``pinv`` = SVD with tolerance ``max(size(A)) * eps(max(sigma))``;
* ``sign(0) = 0``, ``sign(NaN) = NaN``, ``max(NaN, 0) = 0``;
* expression order of every elementwise statement is kept (no fusion),
  e.g. ``D - O + (1/muL)*Y_L`` evaluates ``(D - O) + ((1/muL) * Y_L)``;
* ``randn`` (mt19937ar + Ziggurat) cannot be reproduced outside MATLAB, so the
  initial factors ``A0, B0, C0`` are explicit inputs.
"""
from __future__ import annotations

import numpy as np

REQUIRED_OPTS = ("mu", "rho", "lambda", "lambda2", "maxIter", "tol", "disp")


# ---------------------------------------------------------------------------
# L1 primitives (fast_robust_triple_tensor/*.m)
# ---------------------------------------------------------------------------
def size3(X):
    """`[n1,n2,n3] = size(X)` with MATLAB's trailing-singleton rule."""
    s = tuple(X.shape) + (1, 1, 1)
    if X.ndim > 3:
        # MATLAB folds trailing dims into n3; the reference then fails at
        # `D - O` (triple_decomp_ADMM.m:33).  We refuse up front.
        raise ValueError("D must have at most 3 dimensions")
    return s[0], s[1], s[2]


def as3(X):
    n1, n2, n3 = size3(X)
    return np.asarray(X, dtype=np.float64).reshape((n1, n2, n3), order="F")


def unfold(X, mode):
    """unfold.m:1-13 (identical to triple_decomp_ADMM.m:97-109)."""
    X = as3(X)
    n1, n2, n3 = X.shape
    if mode == 1:
        return X.reshape((n1, n2 * n3), order="F")
    if mode == 2:
        return np.transpose(X, (1, 0, 2)).reshape((n2, n1 * n3), order="F")
    if mode == 3:
        return np.transpose(X, (2, 0, 1)).reshape((n3, n1 * n2), order="F")
    raise ValueError("Mode must be 1, 2, or 3.")


def buildF(B, C):
    """buildF.m:17-21: F(q+(s-1)r, j+(t-1)n2) = B(q,j,s)*C(q,s,t)."""
    B = as3(B)
    C = as3(C)
    r, n2, _ = B.shape
    n3 = C.shape[2]
    B_unfold = unfold(B, 2).reshape((n2, r * r, 1), order="F")
    C_unfold = unfold(C, 3).T.reshape((1, r * r, n3), order="F")
    F = B_unfold * C_unfold
    F = F.reshape((n2, r, r, n3), order="F")
    return np.transpose(F, (1, 2, 0, 3)).reshape((r * r, n2 * n3), order="F")


def buildG(A, C):
    """buildG.m:17-21: G(p+(s-1)r, i+(t-1)n1) = A(i,p,s)*C(p,s,t)."""
    A = as3(A)
    C = as3(C)
    n1, r, _ = A.shape
    n3 = C.shape[2]
    A_unfold = unfold(A, 1).reshape((n1, r * r, 1), order="F")
    C_unfold = unfold(C, 3).T.reshape((1, r * r, n3), order="F")
    G = A_unfold * C_unfold
    G = G.reshape((n1, r, r, n3), order="F")
    return np.transpose(G, (1, 2, 0, 3)).reshape((r * r, n1 * n3), order="F")


def buildH(A, B):
    """buildH.m:17-21: H(p+(q-1)r, i+(j-1)n1) = A(i,p,q)*B(p,j,q)."""
    A = as3(A)
    B = as3(B)
    n1, r, _ = A.shape
    n2 = B.shape[1]
    A_unfold = unfold(A, 1).reshape((n1, r * r, 1), order="F")
    B_unfold = unfold(B, 2).T.reshape((1, r * r, n2), order="F")
    H = A_unfold * B_unfold
    H = H.reshape((n1, r, r, n2), order="F")
    return np.transpose(H, (1, 2, 0, 3)).reshape((r * r, n1 * n2), order="F")


# ---------------------------------------------------------------------------
# Qi-model design matrices (origin_triple_tensor/build{F,G,H}.m, SURVEY.md §8f
# rank 4): the 3-index triple product L(i,j,t) = sum_{p,q,s} A(i,q,s)
# B(p,j,s) C(p,q,t) that README line 43 describes ("single GEMM per mode").
# In the reference these files are shadowed by the local CP builders of
# origin_triple_tensor/triple_decomp_ADMM.m:166-194; here they back the opt-in
# opts.model = 'qi' (restated exactly as the RPAS reshape-permute-GEMM).
# ---------------------------------------------------------------------------
def buildF_qi(B, C):
    """origin_triple_tensor/buildF.m:2-6: F(q+(s-1)r, j+(t-1)n2) = sum_p B(p,j,s) C(p,q,t)."""
    B = as3(B)
    C = as3(C)
    r, n2, _ = B.shape
    n3 = C.shape[2]
    F = np.transpose(B, (1, 2, 0)).reshape((n2 * r, r), order="F") @ C.reshape((r, r * n3), order="F")
    F = np.transpose(F.reshape((n2, r, r, n3), order="F"), (2, 1, 0, 3))
    return F.reshape((r * r, n2 * n3), order="F")


def buildG_qi(A, C):
    """origin_triple_tensor/buildG.m:7-11: G(p+(s-1)r, i+(t-1)n1) = sum_q A(i,q,s) C(p,q,t)."""
    A = as3(A)
    C = as3(C)
    n1, r, _ = A.shape
    n3 = C.shape[2]
    G = (np.transpose(A, (0, 2, 1)).reshape((n1 * r, r), order="F")
         @ np.transpose(C, (1, 0, 2)).reshape((r, r * n3), order="F"))
    G = np.transpose(G.reshape((n1, r, r, n3), order="F"), (2, 1, 0, 3))
    return G.reshape((r * r, n1 * n3), order="F")


def buildH_qi(A, B):
    """origin_triple_tensor/buildH.m:7-11: H(p+(q-1)r, i+(j-1)n1) = sum_s A(i,q,s) B(p,j,s)."""
    A = as3(A)
    B = as3(B)
    n1, r, _ = A.shape
    n2 = B.shape[1]
    H = A.reshape((n1 * r, r), order="F") @ np.transpose(B, (2, 0, 1)).reshape((r, r * n2), order="F")
    H = np.transpose(H.reshape((n1, r, r, n2), order="F"), (2, 1, 0, 3))
    return H.reshape((r * r, n1 * n2), order="F")


def kronF(B, C):
    """origin_triple_tensor/kronF.m:1-7: the explicit-Kronecker form of the Qi F
    (rows ordered s+(q-1)r instead of buildF's q+(s-1)r)."""
    B = as3(B)
    C = as3(C)
    r, n2, _ = B.shape
    B1 = np.kron(np.eye(r), unfold(np.transpose(B, (2, 1, 0)), 1))
    C1 = np.kron(C.reshape((r * r, C.shape[2]), order="F"), np.eye(n2))
    return B1 @ C1


BUILDERS = {"cp": None, "qi": None}  # filled below (model -> (buildF, buildG, buildH))


def triple_product(A, B, C, model="cp"):
    """triple_product.m:1-7: Xhat = reshape(unfold(A,1)*buildF(B,C), n1,n2,n3).
    model='qi': the same statement with origin_triple_tensor/buildF.m, i.e. the
    3-index sum origin_triple_tensor/triple_product.m:8-19 intends."""
    A = as3(A)
    B = as3(B)
    C = as3(C)
    n1 = A.shape[0]
    n2 = B.shape[1]
    n3 = C.shape[2]
    X = unfold(A, 1) @ BUILDERS[model][0](B, C)
    return X.reshape((n1, n2, n3), order="F")


def soft_threshold(X, lam):
    """soft_threshold.m:2 — sign(X).*max(abs(X)-lam,0) with MATLAB NaN rules."""
    X = np.asarray(X, dtype=np.float64)
    return matlab_sign(X) * matlab_max0(np.abs(X) - lam)


# ---------------------------------------------------------------------------
# MATLAB scalar semantics
# ---------------------------------------------------------------------------
def matlab_sign(X):
    """sign(): 1, -1, 0 for zero, NaN for NaN."""
    return np.sign(X)  # numpy already returns 0 for +-0 and NaN for NaN


def matlab_max0(X):
    """max(X, 0): NaN entries are ignored, i.e. max(NaN,0) = 0."""
    return np.fmax(X, 0.0)


def matlab_eps(x):
    """eps(x) for x >= 0: distance from |x| to the next larger double."""
    return np.spacing(np.abs(np.float64(x)))


def pinv(A):
    """MATLAB pinv: SVD, drop sigma <= max(m,n)*eps(max sigma), V*diag(1/s)*U'."""
    A = np.asarray(A, dtype=np.float64)
    U, s, Vt = np.linalg.svd(A, full_matrices=False)
    if s.size == 0:
        return np.zeros(A.T.shape)
    tol = max(A.shape) * matlab_eps(s.max())
    keep = s > tol
    return (Vt[keep].T / s[keep]) @ U[:, keep].T


# ---------------------------------------------------------------------------
# Solver-local helpers (triple_decomp_ADMM.m:73-130)
# ---------------------------------------------------------------------------
def reshape_A_from_A1(A1, n1, r):
    """triple_decomp_ADMM.m:111-116: A(i,:,:) = reshape(A1(i,:), [r r])."""
    return A1.reshape((n1, r, r), order="F").copy(order="F")


def reshape_B_from_B2(B2, n2, r):
    """triple_decomp_ADMM.m:118-123: B(:,j,:) = reshape(B2(j,:), [r r])."""
    B = np.zeros((r, n2, r), order="F")
    for j in range(n2):
        B[:, j, :] = B2[j, :].reshape((r, r), order="F")
    return B


def reshape_C_from_C3(C3, n3, r):
    """triple_decomp_ADMM.m:125-130: C(:,:,t) = reshape(C3(t,:), [r r])."""
    C = np.zeros((r, r, n3), order="F")
    for t in range(n3):
        C[:, :, t] = C3[t, :].reshape((r, r), order="F")
    return C


def update_A(X, A, B, C, alphaA, model="cp"):
    """triple_decomp_ADMM.m:73-81."""
    X1 = unfold(X, 1)
    F = BUILDERS[model][0](B, C)
    G = F @ F.T + alphaA * np.eye(F.shape[0])
    A1 = (X1 @ F.T) @ pinv(G)
    return reshape_A_from_A1(A1, A.shape[0], A.shape[1])


def update_B(X, A, B, C, alphaB, model="cp"):
    """triple_decomp_ADMM.m:83-88."""
    X2 = unfold(X, 2)
    G = BUILDERS[model][1](A, C)
    B_old_unf = (X2 @ G.T) @ pinv(G @ G.T + alphaB * np.eye(G.shape[0]))
    return reshape_B_from_B2(B_old_unf, B.shape[1], B.shape[0])


def update_C(X, A, B, C, model="cp"):
    """triple_decomp_ADMM.m:90-95 (ridge hard-coded to 1e-9 at :93)."""
    X3 = unfold(X, 3)
    H = BUILDERS[model][2](A, B)
    C_old_unf = (X3 @ H.T) @ pinv(H @ H.T + 1e-9 * np.eye(H.shape[0]))
    return reshape_C_from_C3(C_old_unf, C.shape[2], C.shape[0])


# ---------------------------------------------------------------------------
# Solver (triple_decomp_ADMM.m:1-70)
# ---------------------------------------------------------------------------
def check_opts(opts):
    """triple_decomp_ADMM.m:16-20 reads exactly these fields; a missing one is
    a MATLAB error ('Reference to non-existent field'), extras are ignored."""
    for f in REQUIRED_OPTS:
        if f not in opts:
            raise KeyError(f"Reference to non-existent field '{f}'.")


def opts_model(opts):
    """Opt-in model switch (not read by the reference): absent or 'cp' = the
    executed code (rank-r^2 CP, fast_robust_triple_tensor/buildF.m); 'qi' =
    the Qi-model builders of origin_triple_tensor/ (SURVEY.md §8f rank 4)."""
    m = opts.get("model", "cp") if hasattr(opts, "get") else "cp"
    m = str(m).lower()
    if m not in BUILDERS:
        raise ValueError("opts.model must be 'cp' or 'qi'")
    return m


def triple_decomp_ADMM(D, r, opts, A0, B0, C0, trace_iters=(), printer=None):
    """Restatement of fast_robust_triple_tensor/triple_decomp_ADMM.m:1-70.

    Returns ``(A, B, C, O, errHist, E, k, trace)``.  The reference returns only
    the first five (`:1`); ``E`` and the iteration count are extra outputs
    (SURVEY.md §0.7).  ``trace`` maps iteration index (1-based) in
    ``trace_iters`` to a dict of the state after that iteration.
    """
    check_opts(opts)
    D = as3(D)
    n1, n2, n3 = D.shape                                             # :15
    muL = float(opts["mu"]); rhoL = float(opts["rho"]); muL_max = float(opts["mu"]) * 1e6   # :16
    muO = float(opts["mu"]); rhoO = float(opts["rho"]); muO_max = float(opts["mu"]) * 1e6   # :17
    lam = float(opts["lambda"])                                      # :18
    lambda2 = float(opts["lambda2"])                                 # :19
    maxIter = int(opts["maxIter"]); tol = float(opts["tol"]); disp = bool(opts["disp"])  # :20
    model = opts_model(opts)

    A = as3(A0).reshape((n1, r, r), order="F").copy(order="F")      # :23
    B = as3(B0).reshape((r, n2, r), order="F").copy(order="F")
    C = as3(C0).reshape((r, r, n3), order="F").copy(order="F")
    O = np.zeros((n1, n2, n3), order="F"); E = O.copy(order="F")    # :24
    Y_L = np.zeros((n1, n2, n3), order="F")                          # :25
    Y_O = np.zeros((n1, n2, n3), order="F")                          # :26

    normD = np.linalg.norm(D.ravel(order="F"))                       # :28
    errHist = np.zeros(maxIter)                                      # :29
    trace = {}

    k = 0
    for k in range(1, maxIter + 1):                                  # :31
        T = (D - O) + (1.0 / muL) * Y_L                               # :33
        A = update_A(T, A, B, C, lambda2, model)                      # :34
        B = update_B(T, A, B, C, lambda2, model)                      # :35
        C = update_C(T, A, B, C, model)                               # :36

        L = triple_product(A, B, C, model)                            # :38

        R1 = (D - L) + (1.0 / muL) * Y_L                              # :41
        R2 = E - (1.0 / muO) * Y_O                                    # :42
        O = (muL * R1 + muO * R2) / (muL + muO)                       # :43

        R3 = O + (1.0 / muO) * Y_O                                    # :46
        E = matlab_sign(R3) * matlab_max0(np.abs(R3) - lam / muO)     # :47

        resL = (D - L) - O                                            # :50
        resO = O - E                                                  # :51
        Y_L = Y_L + muL * resL                                        # :52
        Y_O = Y_O + muO * resO                                        # :53

        muL = min(muL * rhoL, muL_max)                                # :56
        muO = min(muO * rhoO, muO_max)                                # :57

        errL = np.linalg.norm(resL.ravel(order="F")) / normD
        errO = np.linalg.norm(resO.ravel(order="F")) / normD
        errHist[k - 1] = errL + errO                                  # :59
        if disp and k % 10 == 0:                                      # :60-62
            msg = "Iter %d, errL=%.2e, errO=%.2e" % (k, errL, errO)
            (printer or print)(msg)
        if k in trace_iters:
            trace[k] = dict(A=A.copy(order="F"), B=B.copy(order="F"), C=C.copy(order="F"),
                            O=O.copy(order="F"), E=E.copy(order="F"),
                            Y_L=Y_L.copy(order="F"), Y_O=Y_O.copy(order="F"), L=L.copy(order="F"))
        if k > 1 and abs(errHist[k - 1] - errHist[k - 2]) < tol * errHist[k - 2]:  # :63
            break

    errHist = errHist[:k]                                             # :68
    return A, B, C, O, errHist, E, k, trace


# ---------------------------------------------------------------------------
# Nonconvex variant: fast_robust_triple_tensor/test.m.
# The file defines `triple_decomp_ADMM_outlier(X, r, rho, lambda, gamma_A,
# epsilon, p, theta, maxIter, tol)` with its own local helpers (`:77-211`):
# a Y-split ADMM for the outliers O, while A, B, C follow an ALS on the data X
# itself with a reweighted (l_p-like) soft threshold on A.
# ---------------------------------------------------------------------------
def weighted_soft_threshold(X, tau, W):
    """test.m:97-101: sign(X).*max(abs(X) - tau.*W, 0)."""
    return matlab_sign(X) * matlab_max0(np.abs(X) - tau * W)


def ncvx_update_A(X, A, B, C, gamma_A, epsilon, p, theta):
    """test.m:77-92: ridge 1e-12, then the reweighted shrink of A1."""
    X1 = unfold(X, 1)
    F = buildF(B, C)
    A_old_unf = (X1 @ F.T) @ pinv(F @ F.T + 1e-12 * np.eye(F.shape[0]))      # :82
    W_A = 1.0 / ((np.abs(A_old_unf) + epsilon) ** (theta - p))                 # :86
    A_new_unf = weighted_soft_threshold(A_old_unf, gamma_A, W_A)               # :89
    return reshape_A_from_A1(A_new_unf, A.shape[0], A.shape[1])                # :92


def ncvx_update_B(X, A, B, C):
    """test.m:114-119 (ridge 1e-9 at :117)."""
    X2 = unfold(X, 2)
    G = buildG(A, C)
    B_old_unf = (X2 @ G.T) @ pinv(G @ G.T + 1e-9 * np.eye(G.shape[0]))
    return reshape_B_from_B2(B_old_unf, B.shape[1], B.shape[0])


def triple_decomp_ADMM_ncvx(X, r, rho, lam, gamma_A, epsilon, p, theta, maxIter, tol,
                            A0, B0, C0, printer=None, trace_iters=()):
    """Restatement of fast_robust_triple_tensor/test.m:1-73.

    Returns ``(A, B, C, O, errHist, k, trace)``; the reference returns the
    first five.  Semantics kept: T uses the factors from the start of the
    iteration (`:35`); the factor updates read X, never Y or O (`:49-51`);
    errHist(k) = ||X - Y_new - O_new||/||X|| (`:62`) is printed every
    iteration (`:63`); on the stop test (`:65-68`) errHist is truncated and
    the loop breaks BEFORE `O = O_new` (`:71`), so the returned O is that of
    iteration k-1 while A, B, C are those of iteration k; without a break
    errHist keeps all maxIter entries.  W_O is all ones (`:43`)."""
    X = as3(X)
    n1, n2, n3 = X.shape                                              # :19
    Xnorm = np.linalg.norm(X.ravel(order="F"))                        # :20
    A = as3(A0).reshape((n1, r, r), order="F").copy(order="F")       # :24-26
    B = as3(B0).reshape((r, n2, r), order="F").copy(order="F")
    C = as3(C0).reshape((r, r, n3), order="F").copy(order="F")
    O = np.zeros((n1, n2, n3), order="F")                             # :28
    Lam = np.zeros((n1, n2, n3), order="F")                           # :29
    Gam = np.zeros((n1, n2, n3), order="F")                           # :30
    errHist = np.zeros(int(maxIter))                                  # :32
    trace = {}
    k = 0
    for k in range(1, int(maxIter) + 1):                              # :34
        T = triple_product(A, B, C)                                   # :35
        Y_new = ((X - O) + rho * (T + Lam / rho)) / (1 + rho)         # :36
        W_O = np.ones(O.shape)                                        # :43
        O_new = weighted_soft_threshold((X - Y_new) + Gam / rho, lam / rho, W_O)   # :44
        Lam = Lam + rho * (T - Y_new)                                 # :47
        Gam = Gam + rho * ((X - Y_new) - O_new)                       # :48
        A = ncvx_update_A(X, A, B, C, gamma_A, epsilon, p, theta)     # :49
        B = ncvx_update_B(X, A, B, C)                                 # :50
        C = update_C(X, A, B, C)                                      # :51 (same ridge 1e-9, :124)
        errHist[k - 1] = np.linalg.norm(((X - Y_new) - O_new).ravel(order="F")) / Xnorm   # :62
        (printer or print)("Iteration %d, relative error = %.4e" % (k, errHist[k - 1]))  # :63
        if k in trace_iters:
            trace[k] = dict(A=A.copy(order="F"), B=B.copy(order="F"), C=C.copy(order="F"),
                            O=O_new.copy(order="F"), Lam=Lam.copy(order="F"),
                            Gam=Gam.copy(order="F"))
        if k > 1 and abs(errHist[k - 1] - errHist[k - 2]) < tol * errHist[k - 2]:  # :65
            errHist = errHist[:k]                                     # :66
            break                                                     # :67 (O keeps iteration k-1)
        O = O_new                                                     # :71
    return A, B, C, O, errHist, k, trace


def triple_decomp_ALS(X, r, opts, A0, B0, C0, printer=None):
    """Restatement of fast_robust_triple_tensor/triple_decomp_ALS.m:1-40.

    Returns ``(A, B, C, errHist, k)``; the reference returns the first four
    (`:1`).  Only ``opts.maxIter`` and ``opts.tol`` are read (`:2-3`).  The
    relative error is taken *before* the update of iteration k (`:15-16`), the
    stop test leaves the factors of that iteration unchanged (`:20-23`), every
    mode uses the hard-coded ridge 1e-9 (`:27,:32,:37`), and the progress line
    is printed every 5 iterations unconditionally (`:17-19`).  ``unfold`` and
    ``buildF/G/H`` resolve to the standalone files of
    ``fast_robust_triple_tensor/`` (the same definitions as the ADMM's
    locals); the ``reshape_*`` helpers are ALS-local copies (`:44-63`)
    identical to the ADMM's.
    """
    for f in ("maxIter", "tol"):
        if f not in opts:
            raise KeyError(f"Reference to non-existent field '{f}'.")
    maxIter = int(opts["maxIter"]); tol = float(opts["tol"])         # :2-3
    X = as3(X)
    n1, n2, n3 = X.shape                                             # :5
    Xnorm = np.linalg.norm(X.ravel(order="F"))                       # :6
    A = as3(A0).reshape((n1, r, r), order="F").copy(order="F")      # :8
    B = as3(B0).reshape((r, n2, r), order="F").copy(order="F")      # :9
    C = as3(C0).reshape((r, r, n3), order="F").copy(order="F")      # :10
    errHist = np.zeros(max(maxIter, 0))                              # :12
    ridge = 1e-9 * np.eye(r * r)
    k = 0
    for k in range(1, maxIter + 1):                                  # :14
        Xhat = triple_product(A, B, C)                                # :15
        errHist[k - 1] = np.linalg.norm(X.ravel(order="F") - Xhat.ravel(order="F")) / Xnorm  # :16
        if k % 5 == 0:                                                # :17-19
            (printer or print)("Iteration %d, relative error = %.4e" % (k, errHist[k - 1]))
        if k > 1 and abs(errHist[k - 1] - errHist[k - 2]) < tol * errHist[k - 2]:  # :20
            errHist = errHist[:k]                                     # :21
            return A, B, C, errHist, k                                # :22
        F = buildF(B, C)                                              # :25-28
        A = reshape_A_from_A1((unfold(X, 1) @ F.T) @ pinv(F @ F.T + ridge), n1, r)
        G = buildG(A, C)                                              # :30-33
        B = reshape_B_from_B2((unfold(X, 2) @ G.T) @ pinv(G @ G.T + ridge), n2, r)
        H = buildH(A, B)                                              # :35-38
        C = reshape_C_from_C3((unfold(X, 3) @ H.T) @ pinv(H @ H.T + ridge), n3, r)
    return A, B, C, errHist, k


def mu_schedule(mu0, rho, n):
    """The deterministic penalty sequence of :16 and :56 (muL == muO always)."""
    out = []
    mu = float(mu0)
    mu_max = float(mu0) * 1e6
    for _ in range(n):
        out.append(mu)
        mu = min(mu * float(rho), mu_max)
    return out


# ---------------------------------------------------------------------------
# Driver-side helpers (traffic_triple_comparison.m:194-202)
# ---------------------------------------------------------------------------
def evaluate(X, gt, mask=None):
    """evaluate(): rmse = norm(X_hat(mask)-gt(:)), nrmse = rmse/norm(gt(:))."""
    X = np.asarray(X, dtype=np.float64)
    gt = np.asarray(gt, dtype=np.float64)
    if mask is not None:
        X = X[mask]
    rmse = np.linalg.norm(X.ravel(order="F") - gt.ravel(order="F"))
    return rmse, rmse / np.linalg.norm(gt.ravel(order="F"))


def fspecial_gaussian(size=11, sigma=1.5):
    """MATLAB fspecial('gaussian', size, sigma) (Image Processing Toolbox
    semantics; the toolbox is not in the reference tree): exp(-(x^2+y^2)/2s^2)
    on a meshgrid, entries below eps*max zeroed, normalised to sum 1."""
    siz = (size - 1) / 2.0
    x, y = np.meshgrid(np.arange(-siz, siz + 1), np.arange(-siz, siz + 1))
    h = np.exp(-(x * x + y * y) / (2.0 * sigma * sigma))
    h[h < np.finfo(float).eps * h.max()] = 0.0
    sh = h.sum()
    return h / sh if sh != 0 else h


def filter2_valid(w, img):
    """filter2(w, img, 'valid'): 2-D correlation over the fully-overlapping positions."""
    H, W = w.shape
    M, N = img.shape
    out = np.zeros((M - H + 1, N - W + 1))
    for u in range(H):
        for v in range(W):
            out += w[u, v] * img[u:u + M - H + 1, v:v + N - W + 1]
    return out


def ssim_index(img1, img2):
    """other_methods/IPI_RTC_FCTN-main/lib/ssim_index.m with nargin == 2 (the copy
    `addpath(genpath(pwd))` resolves first; byte-identical to the one in
    Low-rank-.../ssim_index.m): Gaussian 11x11 sigma 1.5, K = [0.01 0.03],
    L = 255, mean2 of the 'valid' SSIM map; -Inf below 11x11."""
    img1 = np.asarray(img1, dtype=np.float64)
    img2 = np.asarray(img2, dtype=np.float64)
    M, N = img1.shape
    if M < 11 or N < 11:
        return -np.inf
    w = fspecial_gaussian(11, 1.5)
    w = w / w.sum(axis=0).sum()
    C1 = (0.01 * 255) ** 2
    C2 = (0.03 * 255) ** 2
    mu1 = filter2_valid(w, img1)
    mu2 = filter2_valid(w, img2)
    mu1_sq, mu2_sq, mu1_mu2 = mu1 * mu1, mu2 * mu2, mu1 * mu2
    sigma1_sq = filter2_valid(w, img1 * img1) - mu1_sq
    sigma2_sq = filter2_valid(w, img2 * img2) - mu2_sq
    sigma12 = filter2_valid(w, img1 * img2) - mu1_mu2
    ssim_map = ((2 * mu1_mu2 + C1) * (2 * sigma12 + C2)) / \
               ((mu1_sq + mu2_sq + C1) * (sigma1_sq + sigma2_sq + C2))
    return ssim_map.mean()


def psnr_index(x, y):
    """other_methods/Low-rank-.../psnr_index.m:1-4: 10*log10(255^2/mse(x-y))."""
    d = np.asarray(x, dtype=np.float64) - np.asarray(y, dtype=np.float64)
    with np.errstate(divide="ignore"):
        return 10.0 * np.log10(255.0 ** 2 / np.mean(d * d))


def quality_ybz(imagery1, imagery2):
    """other_methods/Low-rank-.../quality_ybz.m:1-33: mean over frames
    (trailing dims folded) of psnr_index and ssim_index."""
    X1 = np.asarray(imagery1, dtype=np.float64)
    X2 = np.asarray(imagery2, dtype=np.float64)
    n1, n2 = X1.shape[0], X1.shape[1]
    X1 = X1.reshape((n1, n2, -1), order="F")
    X2 = X2.reshape((n1, n2, -1), order="F")
    nf = X1.shape[2]
    ps = [psnr_index(X1[:, :, i], X2[:, :, i]) for i in range(nf)]
    ss = [ssim_index(X1[:, :, i], X2[:, :, i]) for i in range(nf)]
    return float(np.mean(ps)), float(np.mean(ss))


# ---------------------------------------------------------------------------
# Loop definitions quoted in the reference's comments (known-answer checks)
# ---------------------------------------------------------------------------
def buildF_loops(B, C):
    """buildF.m:5-16 (commented loop definition)."""
    r, n2, _ = B.shape
    n3 = C.shape[2]
    F = np.zeros((r * r, n2 * n3), order="F")
    for j in range(n2):
        for t in range(n3):
            col = j + t * n2
            for q in range(r):
                for s in range(r):
                    F[q + s * r, col] = B[q, j, s] * C[q, s, t]
    return F


def buildG_loops(A, C):
    """buildG.m:5-16 (commented loop definition)."""
    n1, r, _ = A.shape
    n3 = C.shape[2]
    G = np.zeros((r * r, n1 * n3), order="F")
    for i in range(n1):
        for t in range(n3):
            col = i + t * n1
            for p in range(r):
                for s in range(r):
                    G[p + s * r, col] = A[i, p, s] * C[p, s, t]
    return G


def buildH_loops(A, B):
    """buildH.m:5-16 (commented loop definition)."""
    n1, r, _ = A.shape
    n2 = B.shape[1]
    H = np.zeros((r * r, n1 * n2), order="F")
    for i in range(n1):
        for j in range(n2):
            col = i + j * n1
            for p in range(r):
                for q in range(r):
                    H[p + q * r, col] = A[i, p, q] * B[p, j, q]
    return H


def triple_product_loops(A, B, C):
    """fast_robust_triple_tensor/test.m:142-160 (explicit five-loop)."""
    n1 = A.shape[0]
    n2 = B.shape[1]
    n3 = C.shape[2]
    X = np.zeros((n1, n2, n3), order="F")
    for i in range(n1):
        for j in range(n2):
            for t in range(n3):
                s = 0.0
                for p in range(A.shape[1]):
                    for q in range(A.shape[2]):
                        s = s + A[i, p, q] * B[p, j, q] * C[p, q, t]
                X[i, j, t] = s
    return X


BUILDERS["cp"] = (buildF, buildG, buildH)
BUILDERS["qi"] = (buildF_qi, buildG_qi, buildH_qi)


def buildG_qi_loops(A, C):
    """origin_triple_tensor/buildG.m:2-6 (comment): G(p+(s-1)r, i+(t-1)n1) = sum_q A(i,q,s) C(p,q,t)."""
    n1, r, _ = A.shape
    n3 = C.shape[2]
    G = np.zeros((r * r, n1 * n3), order="F")
    for i in range(n1):
        for t in range(n3):
            for p in range(r):
                for s_ in range(r):
                    G[p + s_ * r, i + t * n1] = sum(A[i, q, s_] * C[p, q, t] for q in range(r))
    return G


def buildH_qi_loops(A, B):
    """origin_triple_tensor/buildH.m:2-6 (comment): H(p+(q-1)r, i+(j-1)n1) = sum_s A(i,q,s) B(p,j,s)."""
    n1, r, _ = A.shape
    n2 = B.shape[1]
    H = np.zeros((r * r, n1 * n2), order="F")
    for i in range(n1):
        for j in range(n2):
            for p in range(r):
                for q in range(r):
                    H[p + q * r, i + j * n1] = sum(A[i, q, s_] * B[p, j, s_] for s_ in range(r))
    return H


def triple_product_qi_loops(A, B, C):
    """origin_triple_tensor/triple_product.m:8-19: total += a(i,q,s)*b(p,j,s)*c(p,q,t)
    (the file indexes undefined lower-case a/b/c — a MATLAB error as written;
    this is the sum it spells out, with A, B, C)."""
    n1, r, _ = A.shape
    n2 = B.shape[1]
    n3 = C.shape[2]
    X = np.zeros((n1, n2, n3), order="F")
    for i in range(n1):
        for j in range(n2):
            for t in range(n3):
                tot = 0.0
                for p in range(r):
                    for q in range(r):
                        for s_ in range(r):
                            tot = tot + A[i, q, s_] * B[p, j, s_] * C[p, q, t]
                X[i, j, t] = tot
    return X
