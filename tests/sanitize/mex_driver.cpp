// ASan/UBSan driver for the MEX gateway (matlab/tritd_mex.cpp) over the mock
// mx runtime (tests/mock_mex/): the argument checks that run without a GPU —
// a missing opts field, bad device ordinals, clearing the set, mexAtExit.
// Test infrastructure only (tests/test_sanitizers.py).
#include <cstdio>
#include <cstring>
#include <vector>

extern "C" {
int mock_admm(const void* D, long n1, long n2, long n3, int r, const char* opt_names,
              const double* opt_vals, const double* A0, const double* B0, const double* C0,
              double* A, double* B, double* C, void* O, void* E, double* errHist, int* k,
              char* err, int errlen, char* printed, int printlen, int single);
int mock_devices(const double* devs, int n, char* err, int errlen);
int mock_clear(void);
}

int main() {
    const long n1 = 6, n2 = 5, n3 = 4;
    const int r = 2, R = 4;
    std::vector<double> D(n1 * n2 * n3, 0.5), A0(n1 * R, 0.1), B0(n2 * R, 0.2), C0(n3 * R, 0.3);
    std::vector<double> A(n1 * R), B(n2 * R), C(n3 * R), O(D.size()), E(D.size()), eh(8);
    char err[1024], pr[1024];
    int k = 0, bad = 0;
    // opts without lambda2 (triple_decomp_ADMM.m:16-20 reads it): MATLAB's error
    const double vals[6] = {1e-2, 1.1, 1e-1, 5, 1e-5, 0};
    int rc = mock_admm(D.data(), n1, n2, n3, r, "mu,rho,lambda,maxIter,tol,disp", vals, A0.data(),
                       B0.data(), C0.data(), A.data(), B.data(), C.data(), O.data(), E.data(),
                       eh.data(), &k, err, sizeof err, pr, sizeof pr, 0);
    bad |= rc != 1 || std::strstr(err, "lambda2") == nullptr;
    std::printf("missing field: rc=%d err=%s\n", rc, err);
    // the same in class single
    std::vector<float> Df(D.size(), 0.5f), Of(D.size()), Ef(D.size());
    rc = mock_admm(Df.data(), n1, n2, n3, r, "mu,rho,lambda,maxIter,tol,disp", vals, A0.data(),
                   B0.data(), C0.data(), A.data(), B.data(), C.data(), Of.data(), Ef.data(), eh.data(),
                   &k, err, sizeof err, pr, sizeof pr, 1);
    bad |= rc != 1;
    const double half = 0.5;
    rc = mock_devices(&half, 1, err, sizeof err);
    bad |= rc != 1;
    std::vector<double> many(17);
    for (int q = 0; q < 17; ++q) many[q] = q;
    rc = mock_devices(many.data(), 17, err, sizeof err);
    bad |= rc != 1;
    rc = mock_devices(nullptr, 0, err, sizeof err);
    bad |= rc != 0;
    bad |= mock_clear() != 0;
    std::printf("mex_driver: %s\n", bad ? "BAD" : "ok");
    return bad;
}
