/* ASan/UBSan driver for the host-side C restatement (oracle/tritd_ref.c):
 * a small synthetic ADMM solve in fp64 and fp32, triple_product, unfold and
 * the design builders, on one thread.  Test infrastructure only
 * (tests/test_sanitizers.py builds it with -fsanitize=address,undefined). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

int tritd_ref_admm(const double* D, int64_t n1, int64_t n2, int64_t n3, int r, const double* opts,
                   const double* A0, const double* B0, const double* C0, double* A, double* B,
                   double* C, double* O, double* E, double* errHist, int max_iters);
int tritd_ref_admm_f32(const float* D, int64_t n1, int64_t n2, int64_t n3, int r, const double* opts,
                       const double* A0, const double* B0, const double* C0, double* A, double* B,
                       double* C, float* O, float* E, double* errHist, int max_iters);
void tritd_ref_triple_product(const double* A, const double* B, const double* C, int64_t n1,
                              int64_t n2, int64_t n3, int r, double* X);
void tritd_ref_unfold(const double* X, int64_t n1, int64_t n2, int64_t n3, int mode, double* out);
void tritd_ref_build(char which, const double* P, const double* Q, int64_t nP, int64_t nQ, int r,
                     double* out);
void tritd_ref_set_threads(int n);

static uint64_t st = 88172645463325252ull;
static double rnd(void) {  /* xorshift64, uniform in (-1, 1) */
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return (double)(st >> 11) / 4503599627370496.0 - 1.0;
}

int main(void) {
    enum { n1 = 11, n2 = 9, n3 = 13, r = 3, R = 9 };
    const int64_t N = (int64_t)n1 * n2 * n3;
    tritd_ref_set_threads(1);
    double* A0 = malloc(sizeof(double) * n1 * R);
    double* B0 = malloc(sizeof(double) * n2 * R);
    double* C0 = malloc(sizeof(double) * n3 * R);
    double* A = malloc(sizeof(double) * n1 * R);
    double* B = malloc(sizeof(double) * n2 * R);
    double* C = malloc(sizeof(double) * n3 * R);
    double* D = malloc(sizeof(double) * N);
    double* O = malloc(sizeof(double) * N);
    double* E = malloc(sizeof(double) * N);
    float* Df = malloc(sizeof(float) * N);
    float* Of = malloc(sizeof(float) * N);
    float* Ef = malloc(sizeof(float) * N);
    double* X = malloc(sizeof(double) * N);
    double* U = malloc(sizeof(double) * N);
    double* F = malloc(sizeof(double) * R * n2 * n3);
    double eh[40];
    for (int i = 0; i < n1 * R; ++i) A0[i] = rnd();
    for (int i = 0; i < n2 * R; ++i) B0[i] = rnd();
    for (int i = 0; i < n3 * R; ++i) C0[i] = rnd();
    tritd_ref_triple_product(A0, B0, C0, n1, n2, n3, r, D);
    for (int64_t e = 0; e < N; ++e) {
        if (rnd() > 0.9) D[e] += 5.0 * rnd();  /* outliers */
        Df[e] = (float)D[e];
    }
    const double opts[7] = {1e-2, 1.2, 1e-1, 1e-3, 40, 1e-9, 0};
    int bad = 0;
    int k = tritd_ref_admm(D, n1, n2, n3, r, opts, A0, B0, C0, A, B, C, O, E, eh, 0);
    if (k < 1 || k > 40) bad = 1;
    for (int i = 0; i < k; ++i) bad |= !isfinite(eh[i]);
    int kf = tritd_ref_admm_f32(Df, n1, n2, n3, r, opts, A0, B0, C0, A, B, C, Of, Ef, eh, 0);
    if (kf < 1 || kf > 40) bad = 1;
    tritd_ref_triple_product(A, B, C, n1, n2, n3, r, X);
    for (int mode = 1; mode <= 3; ++mode) tritd_ref_unfold(X, n1, n2, n3, mode, U);
    tritd_ref_build('F', B, C, n2, n3, r, F);
    for (int64_t e = 0; e < N; ++e) bad |= !isfinite(X[e]) || !isfinite(U[e]);
    printf("ref_driver: k=%d k_f32=%d errHist[k-1]=%.3e %s\n", k, kf, eh[kf - 1], bad ? "BAD" : "ok");
    free(A0); free(B0); free(C0); free(A); free(B); free(C); free(D); free(O); free(E);
    free(Df); free(Of); free(Ef); free(X); free(U); free(F);
    return bad;
}
