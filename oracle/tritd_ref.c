/*
 * tritd_ref.c — C restatement of the MATLAB reference, TEST INFRASTRUCTURE ONLY.
 *
 * Used as (a) a second, independent oracle (checked against the committed
 * golden vectors, tests/test_oracle.py) and (b) the CPU baseline that
 * bench.py times on the GPU box's host cores (cpu_baseline.kind = "port").
 * The product (libtritd.so) never links or calls this file.
 *
 * It keeps the reference's operation structure on purpose — the statement-
 * by-statement elementwise passes of triple_decomp_ADMM.m:33-59, the
 * materialised permute copies of unfold.m:8,10, the materialised design
 * matrices of buildF/G/H.m:17-21, one GEMM per mode (:78,:86,:93), explicit
 * F*F.' Grams and an SVD-style pinv (:78,86,93) — so it measures what the
 * MATLAB algorithm costs on a CPU, parallelised with OpenMP.
 *
 * Parity status: the solver loop is "parity unpinned" (MATLAB is absent,
 * the reference ships no golden vectors — SURVEY.md §8c); the primitives
 * are pinned by the reference's own loop definitions (see tritd_oracle.py).
 *
 * Semantics restated: column-major arrays; pinv = symmetric eigen-
 * decomposition of the SPD Gram with MATLAB's tolerance
 * max(size)*eps(max sigma); sign(0)=0, sign(NaN)=NaN; max(NaN,0)=0.
 * Build: oracle/Makefile (gcc -O3 -fopenmp -ffp-contract=off).
 */
#include <float.h>
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef int64_t idx;

/* ---------------------------------------------------------------- helpers */
static double* dalloc(idx n) {
    double* p = (double*)aligned_alloc(64, (size_t)((n * 8 + 63) / 64 * 64));
    if (!p) {
        fprintf(stderr, "tritd_ref: out of memory (%lld doubles)\n", (long long)n);
        abort();
    }
    return p;
}

static double matlab_sign(double x) { return x > 0 ? 1.0 : (x < 0 ? -1.0 : (x == 0 ? 0.0 : x)); }

/* eps(x) = 2^(floor(log2 |x|) - 52) for normal x */
static double matlab_eps(double x) {
    x = fabs(x);
    if (x == 0) return DBL_MIN * DBL_EPSILON;
    int e;
    frexp(x, &e); /* x = f * 2^e, f in [0.5,1) -> floor(log2 x) = e-1 */
    return ldexp(1.0, e - 1 - 52);
}

/* ------------------------------------------------------------- unfold.m */
/* unfold.m:1-13 — materialised copies (mode 1 is a reshape: copy too) */
void tritd_ref_unfold(const double* X, idx n1, idx n2, idx n3, int mode, double* Xn) {
    if (mode == 1) {
        memcpy(Xn, X, (size_t)(n1 * n2 * n3) * 8);
    } else if (mode == 2) { /* Xn(j, i + n1 t) = X(i,j,t) */
#pragma omp parallel for collapse(2) schedule(static)
        for (idx t = 0; t < n3; ++t)
            for (idx j = 0; j < n2; ++j)
                for (idx i = 0; i < n1; ++i) Xn[j + n2 * (i + n1 * t)] = X[i + n1 * (j + n2 * t)];
    } else { /* mode 3: Xn(t, i + n1 j) = X(i,j,t) */
#pragma omp parallel for schedule(static)
        for (idx ij = 0; ij < n1 * n2; ++ij)
            for (idx t = 0; t < n3; ++t) Xn[t + n3 * ij] = X[ij + n1 * n2 * t];
    }
}

/* --------------------------------------------------------- buildF/G/H.m */
/* F(k, a + nA*b) = P(..)*Q(..), k = p + r*q (buildF.m:12, buildG.m:12, buildH.m:12) */
void tritd_ref_build(char which, const double* P, const double* Q, idx nP, idx nQ, int r,
                     double* out) {
    const int R = r * r;
#pragma omp parallel for schedule(static)
    for (idx col = 0; col < nP * nQ; ++col) {
        const idx a = col % nP, b = col / nP;
        for (int q = 0; q < r; ++q)
            for (int p = 0; p < r; ++p) {
                const int k = p + r * q;
                double x, y;
                if (which == 'F') { /* B(p,a,q) * C(p,q,b) */
                    x = P[p + r * (a + nP * q)];
                    y = Q[k + (idx)R * b];
                } else if (which == 'G') { /* A(a,p,q) * C(p,q,b) */
                    x = P[a + nP * k];
                    y = Q[k + (idx)R * b];
                } else { /* 'H': A(a,p,q) * B(p,b,q) */
                    x = P[a + nP * k];
                    y = Q[p + r * (b + nQ * q)];
                }
                out[k + (idx)R * col] = x * y;
            }
    }
}

/* ------------------------------------------------------------ dense BLAS */
/* M (m x R) = X (m x K, col-major) * F^T (F: R x K, col-major).
 * K is split over threads; each thread keeps a private m x R partial. */
static void gemm_x_ft(const double* X, idx m, idx K, const double* F, int R, double* M) {
    const int nt = omp_get_max_threads();
    double* part = dalloc((idx)nt * m * R);
    memset(part, 0, (size_t)(nt * m * R) * 8);
#pragma omp parallel
    {
        const int tid = omp_get_thread_num();
        double* acc = part + (idx)tid * m * R;
        const idx c0 = K * tid / nt, c1 = K * (tid + 1) / nt;
        const idx IB = 64;
        for (idx cb = c0; cb < c1; cb += 8) {
            const idx ce = cb + 8 < c1 ? cb + 8 : c1;
            for (idx ib = 0; ib < m; ib += IB) {
                const idx ie = ib + IB < m ? ib + IB : m;
                for (int k = 0; k < R; ++k) {
                    double* a = acc + (idx)k * m;
                    for (idx c = cb; c < ce; ++c) {
                        const double f = F[k + (idx)R * c];
                        const double* x = X + m * c;
                        for (idx i = ib; i < ie; ++i) a[i] = fma(x[i], f, a[i]);
                    }
                }
            }
        }
    }
    for (idx e = 0; e < m * R; ++e) {
        double s = 0;
        for (int t = 0; t < nt; ++t) s += part[(idx)t * m * R + e];
        M[e] = s;
    }
    free(part);
}

/* G (R x R) = F * F^T + alpha I (F: R x K col-major) */
static void gram_ffT(const double* F, int R, idx K, double alpha, double* G) {
    const int nt = omp_get_max_threads();
    double* part = dalloc((idx)nt * R * R);
    memset(part, 0, (size_t)(nt * R * R) * 8);
#pragma omp parallel
    {
        const int tid = omp_get_thread_num();
        double* acc = part + (idx)tid * R * R;
        const idx c0 = K * tid / nt, c1 = K * (tid + 1) / nt;
        for (idx c = c0; c < c1; ++c) {
            const double* f = F + (idx)R * c;
            for (int kk = 0; kk < R; ++kk) {
                const double v = f[kk];
                double* a = acc + (idx)kk * R;
                for (int k = 0; k < R; ++k) a[k] = fma(f[k], v, a[k]);
            }
        }
    }
    for (idx e = 0; e < (idx)R * R; ++e) {
        double s = 0;
        for (int t = 0; t < nt; ++t) s += part[(idx)t * R * R + e];
        G[e] = s;
    }
    free(part);  /* (leaked until round 4: found by the ASan build, tests/test_sanitizers.py) */
    for (int k = 0; k < R; ++k) G[k + (idx)R * k] += alpha;
}

/* MATLAB pinv of a symmetric matrix: cyclic Jacobi eigen-decomposition,
 * sigma = |lambda|, drop sigma <= n*eps(max sigma) */
static void pinv_sym(const double* G, int n, double* P) {
    double* a = dalloc((idx)n * n);
    double* v = dalloc((idx)n * n);
    memcpy(a, G, (size_t)n * n * 8);
    for (int i = 0; i < n * n; ++i) v[i] = 0;
    for (int i = 0; i < n; ++i) v[i + n * i] = 1;
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0, tot = 0;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) {
                const double x = a[i + n * j] * a[i + n * j];
                tot += x;
                if (i != j) off += x;
            }
        if (off <= 1e-30 * tot || off == 0) break;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = a[p + n * q];
                if (apq == 0) continue;
                const double app = a[p + n * p], aqq = a[q + n * q];
                const double theta = (aqq - app) / (2 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1));
                const double c = 1 / sqrt(t * t + 1), s = t * c;
                for (int k = 0; k < n; ++k) { /* A = A J (columns p, q) */
                    const double akp = a[k + n * p], akq = a[k + n * q];
                    a[k + n * p] = c * akp - s * akq;
                    a[k + n * q] = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) { /* A = J^T A (rows p, q) */
                    const double apk = a[p + n * k], aqk = a[q + n * k];
                    a[p + n * k] = c * apk - s * aqk;
                    a[q + n * k] = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = v[k + n * p], vkq = v[k + n * q];
                    v[k + n * p] = c * vkp - s * vkq;
                    v[k + n * q] = s * vkp + c * vkq;
                }
            }
    }
    double smax = 0;
    for (int i = 0; i < n; ++i) smax = fmax(smax, fabs(a[i + n * i]));
    const double tol = n * matlab_eps(smax);
    for (int i = 0; i < n * n; ++i) P[i] = 0;
    for (int e = 0; e < n; ++e) {
        const double lam = a[e + n * e];
        if (!(fabs(lam) > tol)) continue;
        const double w = 1.0 / lam;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < n; ++i) P[i + n * j] += v[i + n * e] * w * v[j + n * e];
    }
    free(a);
    free(v);
}

/* Y (m x R) = M (m x R) * P (R x R), all col-major */
static void small_mm(const double* M, idx m, int R, const double* P, double* Y) {
#pragma omp parallel for schedule(static)
    for (idx i = 0; i < m; ++i)
        for (int k = 0; k < R; ++k) {
            double s = 0;
            for (int q = 0; q < R; ++q) s = fma(M[i + m * q], P[q + (idx)R * k], s);
            Y[i + m * k] = s;
        }
}

/* -------------------------------------------------------- triple_product.m */
/* X = reshape(unfold(A,1) * buildF(B,C), n1,n2,n3)  (triple_product.m:6) */
static void triple_product_F(const double* A, idx n1, int R, const double* F, idx K, double* X) {
#pragma omp parallel for schedule(static)
    for (idx cb = 0; cb < K; cb += 8) {
        const idx ce = cb + 8 < K ? cb + 8 : K;
        for (idx c = cb; c < ce; ++c)
            for (idx i = 0; i < n1; ++i) X[i + n1 * c] = 0;
        for (int k = 0; k < R; ++k) {
            const double* a = A + n1 * k;
            for (idx c = cb; c < ce; ++c) {
                const double f = F[k + (idx)R * c];
                double* x = X + n1 * c;
                for (idx i = 0; i < n1; ++i) x[i] = fma(a[i], f, x[i]);
            }
        }
    }
}

void tritd_ref_triple_product(const double* A, const double* B, const double* C, idx n1, idx n2,
                              idx n3, int r, double* X) {
    const int R = r * r;
    double* F = dalloc((idx)R * n2 * n3);
    tritd_ref_build('F', B, C, n2, n3, r, F);
    triple_product_F(A, n1, R, F, n2 * n3, X);
    free(F);
}

/* ---------------------------------------------------------- reshape_*_from */
static void reshape_B_from_B2(const double* B2, idx n2, int r, double* B) {
    /* B(:,j,:) = reshape(B2(j,:), [r r])  (:118-123) */
    for (idx j = 0; j < n2; ++j)
        for (int q = 0; q < r; ++q)
            for (int p = 0; p < r; ++p) B[p + r * (j + n2 * q)] = B2[j + n2 * (p + r * q)];
}

static void reshape_C_from_C3(const double* C3, idx n3, int r, double* C) {
    /* C(:,:,t) = reshape(C3(t,:), [r r])  (:125-130) */
    const int R = r * r;
    for (idx t = 0; t < n3; ++t)
        for (int k = 0; k < R; ++k) C[k + (idx)R * t] = C3[t + n3 * k];
}

/* ------------------------------------------------------ triple_decomp_ADMM */
/* opts7 = {mu, rho, lambda, lambda2, maxIter, tol, disp}  (triple_decomp_ADMM.m:16-20)
 * returns k; errHist capacity maxIter.  Follows :15-68 statement by statement. */
int tritd_ref_admm(const double* D, idx n1, idx n2, idx n3, int r, const double* opts7,
                   const double* A0, const double* B0, const double* C0, double* A, double* B,
                   double* C, double* O, double* E, double* errHist, int max_iters_override) {
    const int R = r * r;
    const idx N = n1 * n2 * n3;
    double muL = opts7[0], rhoL = opts7[1], muL_max = opts7[0] * 1e6; /* :16 */
    double muO = opts7[0], rhoO = opts7[1], muO_max = opts7[0] * 1e6; /* :17 */
    const double lambda = opts7[2], lambda2 = opts7[3];
    int maxIter = (int)opts7[4];
    const double tol = opts7[5];
    const int disp = opts7[6] != 0;
    if (max_iters_override > 0 && max_iters_override < maxIter) maxIter = max_iters_override;

    memcpy(A, A0, (size_t)(n1 * R) * 8); /* :23 (explicit initial factors) */
    memcpy(B, B0, (size_t)(R * n2) * 8);
    memcpy(C, C0, (size_t)(R * n3) * 8);
    double *YL = dalloc(N), *YO = dalloc(N), *T = dalloc(N), *L = dalloc(N), *X2 = dalloc(N),
           *X3 = dalloc(N);
    idx fmax_cols = n2 * n3;
    if (n1 * n3 > fmax_cols) fmax_cols = n1 * n3;
    if (n1 * n2 > fmax_cols) fmax_cols = n1 * n2;
    double* F = dalloc((idx)R * fmax_cols);
    double *G = dalloc((idx)R * R), *Pi = dalloc((idx)R * R);
    idx nmax = n1 > n2 ? n1 : n2;
    if (n3 > nmax) nmax = n3;
    double *Mk = dalloc(nmax * R), *Yk = dalloc(nmax * R);
#pragma omp parallel for schedule(static)
    for (idx e = 0; e < N; ++e) O[e] = E[e] = YL[e] = YO[e] = 0; /* :24-26 */

    double ss = 0; /* normD = norm(D(:))  :28 */
#pragma omp parallel for reduction(+ : ss) schedule(static)
    for (idx e = 0; e < N; ++e) ss += D[e] * D[e];
    const double normD = sqrt(ss);

    int k = 0;
    for (k = 1; k <= maxIter; ++k) { /* :31 */
        const double invL = 1.0 / muL, invO = 1.0 / muO;
#pragma omp parallel for schedule(static)
        for (idx e = 0; e < N; ++e) T[e] = (D[e] - O[e]) + invL * YL[e]; /* :33 */

        /* update_A :73-81 — X1 = unfold(T,1) is T itself */
        tritd_ref_build('F', B, C, n2, n3, r, F);
        gram_ffT(F, R, n2 * n3, lambda2, G);
        pinv_sym(G, R, Pi);
        gemm_x_ft(T, n1, n2 * n3, F, R, Mk);
        small_mm(Mk, n1, R, Pi, A); /* A memory = A1 (reshape_A_from_A1) */

        /* update_B :83-88 */
        tritd_ref_unfold(T, n1, n2, n3, 2, X2);
        tritd_ref_build('G', A, C, n1, n3, r, F);
        gram_ffT(F, R, n1 * n3, lambda2, G);
        pinv_sym(G, R, Pi);
        gemm_x_ft(X2, n2, n1 * n3, F, R, Mk);
        small_mm(Mk, n2, R, Pi, Yk);
        reshape_B_from_B2(Yk, n2, r, B);

        /* update_C :90-95 (ridge 1e-9, :93) */
        tritd_ref_unfold(T, n1, n2, n3, 3, X3);
        tritd_ref_build('H', A, B, n1, n2, r, F);
        gram_ffT(F, R, n1 * n2, 1e-9, G);
        pinv_sym(G, R, Pi);
        gemm_x_ft(X3, n3, n1 * n2, F, R, Mk);
        small_mm(Mk, n3, R, Pi, Yk);
        reshape_C_from_C3(Yk, n3, r, C);

        /* L = triple_product(A,B,C)  :38 */
        tritd_ref_build('F', B, C, n2, n3, r, F);
        triple_product_F(A, n1, R, F, n2 * n3, L);

        const double den = muL + muO, thr = lambda / muO;
        double sL = 0, sO = 0;
#pragma omp parallel for reduction(+ : sL, sO) schedule(static)
        for (idx e = 0; e < N; ++e) {
            const double R1 = (D[e] - L[e]) + invL * YL[e];                 /* :41 */
            const double R2 = E[e] - invO * YO[e];                          /* :42 */
            const double On = (muL * R1 + muO * R2) / den;                  /* :43 */
            const double R3 = On + invO * YO[e];                            /* :46 */
            const double En = matlab_sign(R3) * fmax(fabs(R3) - thr, 0.0);  /* :47 */
            const double rL = (D[e] - L[e]) - On;                           /* :50 */
            const double rO = On - En;                                      /* :51 */
            YL[e] = YL[e] + muL * rL;                                       /* :52 */
            YO[e] = YO[e] + muO * rO;                                       /* :53 */
            O[e] = On;
            E[e] = En;
            sL += rL * rL;
            sO += rO * rO;
        }
        muL = fmin(muL * rhoL, muL_max); /* :56 */
        muO = fmin(muO * rhoO, muO_max); /* :57 */
        const double eL = sqrt(sL) / normD, eO = sqrt(sO) / normD;
        errHist[k - 1] = eL + eO; /* :59 */
        if (disp && k % 10 == 0) printf("Iter %d, errL=%.2e, errO=%.2e\n", k, eL, eO);
        if (k > 1 && fabs(errHist[k - 1] - errHist[k - 2]) < tol * errHist[k - 2]) break; /* :63 */
    }
    if (k > maxIter) k = maxIter;
    free(YL); free(YO); free(T); free(L); free(X2); free(X3); free(F);
    free(G); free(Pi); free(Mk); free(Yk);
    return k;
}


/* ------------------------------------------------- single-precision D */
/* triple_decomp_ADMM with D of class single, following MATLAB's class rules
 * (SURVEY.md §8a row 1): every array derived from D (T, O, E, Y_L, Y_O,
 * residuals) is single and each statement of :33,:41-53 is evaluated in
 * single, with the double scalars (1/mu, mu, lambda/mu, mu+mu) converted to
 * single where they meet a single array; L = triple_product(A,B,C) is double
 * (A, B, C are double) and converted to single where it meets D (:41,:50);
 * X_k*F' (single * double) is a single result: here accumulated in double and
 * rounded to single once (MATLAB's sgemm accumulates in single: a difference
 * at single rounding level); Grams and pinv are double; (X*F')*pinv(G) is
 * single again and reshaped into the double A/B/C (reshape_*: zeros() then
 * element assignment).  norm() of a single array is single: squares summed
 * in double, root rounded to single; errHist(k) = single(eL + eO) stored in
 * the double errHist.  The zero initial O, E, Y_L, Y_O are exact in either
 * class, so iteration 1 already runs in single. */
static void round_to_single(double* x, idx n) {
    for (idx e = 0; e < n; ++e) x[e] = (double)(float)x[e];
}

int tritd_ref_admm_f32(const float* D, idx n1, idx n2, idx n3, int r, const double* opts7,
                       const double* A0, const double* B0, const double* C0, double* A, double* B,
                       double* C, float* O, float* E, double* errHist, int max_iters_override) {
    const int R = r * r;
    const idx N = n1 * n2 * n3;
    double muL = opts7[0], rhoL = opts7[1], muL_max = opts7[0] * 1e6;
    double muO = opts7[0], rhoO = opts7[1], muO_max = opts7[0] * 1e6;
    const double lambda = opts7[2], lambda2 = opts7[3];
    int maxIter = (int)opts7[4];
    const double tol = opts7[5];
    const int disp = opts7[6] != 0;
    if (max_iters_override > 0 && max_iters_override < maxIter) maxIter = max_iters_override;

    memcpy(A, A0, (size_t)(n1 * R) * 8);
    memcpy(B, B0, (size_t)(R * n2) * 8);
    memcpy(C, C0, (size_t)(R * n3) * 8);
    float *YL = (float*)malloc((size_t)N * 4), *YO = (float*)malloc((size_t)N * 4);
    double *Td = dalloc(N), *L = dalloc(N), *X2 = dalloc(N), *X3 = dalloc(N);
    idx fmax_cols = n2 * n3;
    if (n1 * n3 > fmax_cols) fmax_cols = n1 * n3;
    if (n1 * n2 > fmax_cols) fmax_cols = n1 * n2;
    double* F = dalloc((idx)R * fmax_cols);
    double *G = dalloc((idx)R * R), *Pi = dalloc((idx)R * R);
    idx nmax = n1 > n2 ? n1 : n2;
    if (n3 > nmax) nmax = n3;
    double *Mk = dalloc(nmax * R), *Yk = dalloc(nmax * R);
#pragma omp parallel for schedule(static)
    for (idx e = 0; e < N; ++e) O[e] = E[e] = YL[e] = YO[e] = 0.0f;

    double ss = 0;
#pragma omp parallel for reduction(+ : ss) schedule(static)
    for (idx e = 0; e < N; ++e) ss += (double)D[e] * (double)D[e];
    const float normD = (float)sqrt(ss);

    int k = 0;
    for (k = 1; k <= maxIter; ++k) {
        const float invL = (float)(1.0 / muL), invO = (float)(1.0 / muO);
#pragma omp parallel for schedule(static)
        for (idx e = 0; e < N; ++e) {
            const float t = (D[e] - O[e]) + invL * YL[e]; /* :33 in single */
            Td[e] = (double)t;
        }
        /* update_A */
        tritd_ref_build('F', B, C, n2, n3, r, F);
        gram_ffT(F, R, n2 * n3, lambda2, G);
        pinv_sym(G, R, Pi);
        gemm_x_ft(Td, n1, n2 * n3, F, R, Mk);
        round_to_single(Mk, n1 * R); /* X1*F.' : single */
        small_mm(Mk, n1, R, Pi, A);
        round_to_single(A, n1 * R); /* (..)*pinv(G) : single, assigned into double A */
        /* update_B */
        tritd_ref_unfold(Td, n1, n2, n3, 2, X2);
        tritd_ref_build('G', A, C, n1, n3, r, F);
        gram_ffT(F, R, n1 * n3, lambda2, G);
        pinv_sym(G, R, Pi);
        gemm_x_ft(X2, n2, n1 * n3, F, R, Mk);
        round_to_single(Mk, n2 * R);
        small_mm(Mk, n2, R, Pi, Yk);
        round_to_single(Yk, n2 * R);
        reshape_B_from_B2(Yk, n2, r, B);
        /* update_C */
        tritd_ref_unfold(Td, n1, n2, n3, 3, X3);
        tritd_ref_build('H', A, B, n1, n2, r, F);
        gram_ffT(F, R, n1 * n2, 1e-9, G);
        pinv_sym(G, R, Pi);
        gemm_x_ft(X3, n3, n1 * n2, F, R, Mk);
        round_to_single(Mk, n3 * R);
        small_mm(Mk, n3, R, Pi, Yk);
        round_to_single(Yk, n3 * R);
        reshape_C_from_C3(Yk, n3, r, C);
        /* L = triple_product(A,B,C), double */
        tritd_ref_build('F', B, C, n2, n3, r, F);
        triple_product_F(A, n1, R, F, n2 * n3, L);

        const float fmuL = (float)muL, fmuO = (float)muO;
        const float den = (float)(muL + muO), thr = (float)(lambda / muO);
        double sL = 0, sO = 0;
#pragma omp parallel for reduction(+ : sL, sO) schedule(static)
        for (idx e = 0; e < N; ++e) {
            const float d = D[e], Lf = (float)L[e], yl = YL[e], yo = YO[e];
            const float R1 = (d - Lf) + invL * yl;                             /* :41 */
            const float R2 = E[e] - invO * yo;                                 /* :42 */
            const float On = (fmuL * R1 + fmuO * R2) / den;                    /* :43 */
            const float R3 = On + invO * yo;                                   /* :46 */
            const float sg = R3 > 0 ? 1.0f : (R3 < 0 ? -1.0f : (R3 == 0 ? 0.0f : R3));
            const float En = sg * fmaxf(fabsf(R3) - thr, 0.0f);                /* :47 */
            const float rL = (d - Lf) - On;                                    /* :50 */
            const float rO = On - En;                                          /* :51 */
            YL[e] = yl + fmuL * rL;                                            /* :52 */
            YO[e] = yo + fmuO * rO;                                            /* :53 */
            O[e] = On;
            E[e] = En;
            sL += (double)rL * (double)rL;
            sO += (double)rO * (double)rO;
        }
        muL = fmin(muL * rhoL, muL_max);
        muO = fmin(muO * rhoO, muO_max);
        const float eL = (float)sqrt(sL) / normD, eO = (float)sqrt(sO) / normD;
        errHist[k - 1] = (double)(eL + eO); /* :59 (single, stored into double) */
        if (disp && k % 10 == 0) printf("Iter %d, errL=%.2e, errO=%.2e\n", k, eL, eO);
        if (k > 1 && fabs(errHist[k - 1] - errHist[k - 2]) < tol * errHist[k - 2]) break;
    }
    if (k > maxIter) k = maxIter;
    free(YL); free(YO); free(Td); free(L); free(X2); free(X3); free(F);
    free(G); free(Pi); free(Mk); free(Yk);
    return k;
}

int tritd_ref_threads(void) { return omp_get_max_threads(); }
void tritd_ref_set_threads(int n) { omp_set_num_threads(n); }


/* ------------------------------------------- lean single-precision form */
/* Building blocks of oracle/tritd_lean.py: the same class-single solver as
 * tritd_ref_admm_f32 (every elementwise statement of :33,:41-53 evaluated in
 * single with the same single scalars, L double and rounded to single where
 * it meets D), organised so that a 2048x2048x256 r=16 problem fits a 64 GB
 * host: T, O, E, Y_L, Y_O stay single, the permute copies and design matrices
 * are never materialised (the MTTKRPs are BLAS GEMMs on row blocks, driven
 * from Python), and L is formed one frontal slice (fixed t) at a time.
 * TEST INFRASTRUCTURE ONLY. */

/* T = D - O + (1/muL)*Y_L in single (:33) */
void tritd_ref_lean_form_T(const float* D, const float* O, const float* YL, double muL, float* T,
                           idx N) {
    const float invL = (float)(1.0 / muL);
#pragma omp parallel for schedule(static)
    for (idx e = 0; e < N; ++e) T[e] = (D[e] - O[e]) + invL * YL[e];
}

/* sum of squares of a single array, in double (norm(D(:)) at :28) */
double tritd_ref_lean_sumsq(const float* X, idx N) {
    double s = 0;
#pragma omp parallel for reduction(+ : s) schedule(static)
    for (idx e = 0; e < N; ++e) s += (double)X[e] * (double)X[e];
    return s;
}

/* :41-53 on one slice of n elements, given L of that slice in double; the
 * slice's sums of resL^2 and resO^2 go to sums[0], sums[1] (statement for
 * statement the loop body of tritd_ref_admm_f32) */
void tritd_ref_lean_update(const float* D, float* O, float* E, float* YL, float* YO,
                           const double* L, idx n, double muL, double muO, double lambda,
                           double* sums) {
    const float invL = (float)(1.0 / muL), invO = (float)(1.0 / muO);
    const float fmuL = (float)muL, fmuO = (float)muO;
    const float den = (float)(muL + muO), thr = (float)(lambda / muO);
    double sL = 0, sO = 0;
#pragma omp parallel for reduction(+ : sL, sO) schedule(static)
    for (idx e = 0; e < n; ++e) {
        const float d = D[e], Lf = (float)L[e], yl = YL[e], yo = YO[e];
        const float R1 = (d - Lf) + invL * yl;                             /* :41 */
        const float R2 = E[e] - invO * yo;                                 /* :42 */
        const float On = (fmuL * R1 + fmuO * R2) / den;                    /* :43 */
        const float R3 = On + invO * yo;                                   /* :46 */
        const float sg = R3 > 0 ? 1.0f : (R3 < 0 ? -1.0f : (R3 == 0 ? 0.0f : R3));
        const float En = sg * fmaxf(fabsf(R3) - thr, 0.0f);                /* :47 */
        const float rL = (d - Lf) - On;                                    /* :50 */
        const float rO = On - En;                                          /* :51 */
        YL[e] = yl + fmuL * rL;                                            /* :52 */
        YO[e] = yo + fmuO * rO;                                            /* :53 */
        O[e] = On;
        E[e] = En;
        sL += (double)rL * (double)rL;
        sO += (double)rO * (double)rO;
    }
    sums[0] = sL;
    sums[1] = sO;
}

/* sum over a slice of (L - X)^2 and X^2 in double, X single (the driver's
 * evaluate, traffic_triple_comparison.m:194-199) */
void tritd_ref_lean_rre_parts(const double* L, const float* X, idx n, double* parts) {
    double a = 0, b = 0;
#pragma omp parallel for reduction(+ : a, b) schedule(static)
    for (idx e = 0; e < n; ++e) {
        const double x = X[e], d = L[e] - x;
        a += d * d;
        b += x * x;
    }
    parts[0] = a;
    parts[1] = b;
}
